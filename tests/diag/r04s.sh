# Round 4: fewer event records (none around an absent upload, none before the matcher's
# uploads): the full GPU suite, then C2 / batch / C5 against the previous build (prev)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tests/microbench/event_gap > gpurun_out/event_gap.txt 2>&1; cat gpurun_out/event_gap.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
for r in 1 2 3; do
  for L in lib prev; do
    D=build_exp/$L; [ $L = lib ] && D=modify-sift-gpu_amd/lib
    echo "$L c2 $(LD_LIBRARY_PATH=$D timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'.'); import bench; r=bench.bench_c2(cpu=False); print(round(r['ms_per_image'],4))")" || exit 1
  done
done
for r in 1 2; do
  for L in lib prev; do
    P=build_exp/$L/libsiftgpu.so; [ $L = lib ] && P=modify-sift-gpu_amd/lib/libsiftgpu.so
    echo "$L: $(SGPU_LIB_PATH=$P timeout -k 10 120 python -u tests/diag/match_time.py 50000 plain | tr '\n' ' ')" || exit 1
  done
done
