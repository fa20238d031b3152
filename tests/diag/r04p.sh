# Round 4: full GPU suite + smoke + bench on the tree, then C2 three times
set -o pipefail
bash tests/diag/r04_tests.sh || exit 1
for r in 1 2 3; do
  echo "c2 $(timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'.'); import bench; r=bench.bench_c2(cpu=False); print(round(r['ms_per_image'],4), {k: round(v,4) for k,v in r['timing_ms'].items() if v})")" || exit 1
done
