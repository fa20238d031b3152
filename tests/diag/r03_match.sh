# Matcher round-3 experiments on the GPU box: parity of the shipped build, the shipped kernel
# against the register-staged one in the same build, then alternating A/B against experiment
# builds (tests/build_variant.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py -k "match or c5 or dma" -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_match.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_match.log
[ $rc -eq 0 ] || exit $rc
echo "== LDS-DMA kernel vs register staging (same build)"
for r in 1 2; do
  timeout -k 10 200 python -u tests/diag/match_time.py 50000 plain,rows_only,plain_reg,rows_reg | tr '\n' ' ' || exit 1
  echo
done
for v in "$@"; do
  echo "== A = shipped, B = $v"
  timeout -k 10 400 bash tests/diag/ab_match.sh build_exp/$v/libsiftgpu.so 2 || exit 1
done
