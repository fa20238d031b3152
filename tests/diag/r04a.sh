# Round 4: pixel-major (dual-cell) descriptor -- accuracy of the shipped build (reference cell
# centres) and of the keypoint-relative variant against the exact kernel, then the timing A/B
# against the round-3 kernel (build_exp/desc_fast) and the variant.
set -o pipefail
mkdir -p gpurun_out
T="-m gpu -q --timeout 200 --timeout-method thread -s"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gauss.py $T -x -k "golden_extract or shipped_descriptor or options_vs_oracle or keypoints or levels" > gpurun_out/pytest_a.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_a.log; grep -E "descriptor L2" gpurun_out/pytest_a.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_a.log | head -20; exit $rc; }
SGPU_LIB_PATH=build_exp/dual_ref0/libsiftgpu.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py $T -k "shipped_descriptor" > gpurun_out/pytest_a0.log 2>&1
echo "ref0:"; grep -E "descriptor L2|passed|failed" gpurun_out/pytest_a0.log
timeout -k 10 300 bash tests/diag/ab_bench.sh build_exp/desc_fast/libsiftgpu.so 2 && \
timeout -k 10 300 bash tests/diag/ab_bench.sh build_exp/dual_ref0/libsiftgpu.so 1
