# Fused octave pyramid (opt-in variant 8388608) vs the shipped per-level kernels on the GPU box:
# parity tests, then an interleaved A/B timing (tests/ab_variants.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "gaussian or fused" > gpurun_out/t_fused.log 2>&1; rc=$?; tail -2 gpurun_out/t_fused.log
[ $rc -eq 0 ] && timeout -k 10 200 python tests/ab_variants.py 0 8388608 > gpurun_out/ab_fused.log 2>&1; cat gpurun_out/ab_fused.log
