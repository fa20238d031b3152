# Round 4 matcher: the k_match_raw chunk cost model (shipped lib) against the pipelined kernel
# with the old ~4096-workgroup split (m1) and the model's fixed cost at 1 tile (ovt1): matcher
# tests on the shipped lib, then alternating C5 timings.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "match" --timeout 120 --timeout-method thread \
  > gpurun_out/r04k_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04k_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for L in m1 lib ovt1; do
    P=build_exp/$L/libsiftgpu.so; [ $L = lib ] && P=modify-sift-gpu_amd/lib/libsiftgpu.so
    echo "$L: $(SGPU_LIB_PATH=$P timeout -k 10 120 python -u tests/diag/match_time.py 50000 plain,rows_only | tr '\n' ' ')" || exit 1
  done
done
