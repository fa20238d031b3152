# Round 4: dual descriptor occupancy A/B: shipped (reference centres, <= 128 VGPRs) against the
# compiler's 132 VGPRs (build_exp/dual_w0) and the keypoint-relative weights (build_exp/dual_ref0)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -s -k "shipped_descriptor or golden_extract" > gpurun_out/pytest_c.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_c.log; grep -E "descriptor L2" gpurun_out/pytest_c.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash tests/diag/ab_bench.sh build_exp/dual_w0/libsiftgpu.so 2 && \
timeout -k 10 300 bash tests/diag/ab_bench.sh build_exp/dual_ref0/libsiftgpu.so 2
