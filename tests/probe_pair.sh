# Two-level Gaussian kernel check on the GPU box: parity tests, interleaved A/B timing against
# one launch per level (variant 1024), then a kernel trace of both.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "gaussian_levels or golden" > gpurun_out/t_pair.log 2>&1; rc=$?; tail -3 gpurun_out/t_pair.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tests/ab_variants.py 0 524288 --rounds 6 > gpurun_out/ab_pair.log 2>&1; rc=$?; cat gpurun_out/ab_pair.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_gauss" --output-format csv -d gpurun_out/kt_pair -o run -- python3 tests/ab_variants.py 0 524288 --rounds 4 > gpurun_out/kt_pair.log 2>&1; echo kt rc=$?
