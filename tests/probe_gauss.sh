# Per-level Gaussian kernel check on the GPU box: parity tests, then interleaved A/B timing.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "gaussian or golden or first_octave or fused" > gpurun_out/t_gauss.log 2>&1; rc=$?; tail -2 gpurun_out/t_gauss.log
[ $rc -eq 0 ] && timeout -k 10 200 python tests/ab_variants.py 0 128 --no-check > gpurun_out/ab_gauss.log 2>&1; cat gpurun_out/ab_gauss.log
