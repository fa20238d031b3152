# Round 4: orientation wave form with the gathers one batch ahead and the smoothing across
# lanes -- parity/API/option tests (single images take this form), then C2 against the previous
# build (prev), alternating.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_options.py -m gpu -q -x \
  --timeout 250 --timeout-method thread > gpurun_out/r04o_t.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/r04o_t.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r04o_t.log | head; exit $rc; }
for r in 1 2 3; do
  for L in lib prev; do
    D=build_exp/$L; [ $L = lib ] && D=modify-sift-gpu_amd/lib
    echo "$L c2 $(LD_LIBRARY_PATH=$D timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'.'); import bench; r=bench.bench_c2(cpu=False); print(round(r['ms_per_image'],4), {k: round(v,4) for k,v in r['timing_ms'].items() if v})")" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 bash tests/profile_c2.sh r04o > gpurun_out/prof_c2_r04o.log 2>&1 && echo c2 trace ok
