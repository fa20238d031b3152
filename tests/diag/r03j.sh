# Descriptor at 6 waves per SIMD (SGK_DESC_WPE=6: 80 VGPRs, 8 spilled) against the shipped 5.
set -o pipefail
mkdir -p gpurun_out
V=${1:-desc_w6}
SGPU_LIB_PATH=build_exp/$V/libsiftgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "shipped_descriptor or golden" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$V.log 2>&1; rc=$?
echo "parity rc=$rc"; tail -1 gpurun_out/pytest_$V.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash tests/diag/ab_bench.sh build_exp/$V/libsiftgpu.so 3
