# Round 4: stage events with a device-scope release -- full GPU suite on the tree, then C2 and
# the batch stages against the previous build (prev), alternating, and the C2 trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
for r in 1 2 3; do
  for L in lib prev; do
    D=build_exp/$L; [ $L = lib ] && D=modify-sift-gpu_amd/lib
    echo "$L c2 $(LD_LIBRARY_PATH=$D timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'.'); import bench; r=bench.bench_c2(cpu=False); print(round(r['ms_per_image'],4), {k: round(v,4) for k,v in r['timing_ms'].items() if v})")" || exit 1
  done
done
LIBS="lib prev" bash tests/diag/r04l.sh || exit 1
for r in 1 2; do
  for L in lib prev; do
    P=build_exp/$L/libsiftgpu.so; [ $L = lib ] && P=modify-sift-gpu_amd/lib/libsiftgpu.so
    echo "$L: $(SGPU_LIB_PATH=$P timeout -k 10 120 python -u tests/diag/match_time.py 50000 plain,rows_only | tr '\n' ' ')" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 bash tests/profile_c2.sh r04q > gpurun_out/prof_c2_r04q.log 2>&1 && echo c2 trace ok
