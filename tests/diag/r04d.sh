# Round 4: extremum over-fetch fix (rows past the segment clamped, >= 32-row segments above
# octave 0) -- parity, then A/B against HEAD before it (build_exp/r04_prev) and against 16-row
# segments (build_exp/ext_seg16); descriptor occupancy A/B (build_exp/dual_w0: 132 VGPRs,
# build_exp/dual_ref0: keypoint-relative weights); the copy-walk microbench variants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -s -k "candidates or golden_extract or options_vs_oracle or full_hd or shipped_descriptor" > gpurun_out/pytest_d.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_d.log; grep -E "descriptor L2" gpurun_out/pytest_d.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_d.log | head; exit $rc; }
timeout -k 10 300 bash tests/diag/ab_bench.sh build_exp/r04_prev/libsiftgpu.so 2 && \
timeout -k 10 200 bash tests/diag/ab_bench.sh build_exp/ext_seg16/libsiftgpu.so 1 && \
timeout -k 10 200 bash tests/diag/ab_bench.sh build_exp/dual_w0/libsiftgpu.so 1 && \
timeout -k 10 200 bash tests/diag/ab_bench.sh build_exp/dual_ref0/libsiftgpu.so 1 && \
timeout -k 10 120 ./tests/microbench/layout_bw > gpurun_out/layout_bw2.txt 2>&1; cat gpurun_out/layout_bw2.txt
