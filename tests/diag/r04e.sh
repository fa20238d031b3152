# Round 4: 3-slot Gaussian ring (FW <= 17: 16 waves per CU instead of 12) -- bitwise pyramid
# tests, then A/B against the 4-slot ring (build_exp/lean_r32)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gauss.py tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -k "levels or golden_extract or first_octave or candidates" > gpurun_out/pytest_e.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_e.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_e.log | head; exit $rc; }
timeout -k 10 400 bash tests/diag/ab_bench.sh build_exp/lean_r32/libsiftgpu.so 3
