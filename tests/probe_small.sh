# Pair kernel parity (restored compiler-tracked loads), then A/B of the fused octave kernel on
# the small octaves only (variants 4194304: octaves >= 1, 2097152: octaves >= 2).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "pair or gaussian or golden or fused" > gpurun_out/t_small.log 2>&1; rc=$?; tail -3 gpurun_out/t_small.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tests/ab_variants.py 0 1024 4194304 2097152 > gpurun_out/ab_small.log 2>&1; rc=$?; cat gpurun_out/ab_small.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_gauss|k_octave" --output-format csv -d gpurun_out/kt_small -o run -- python3 tests/ab_variants.py 0 4194304 2097152 --rounds 3 > gpurun_out/kt_small.log 2>&1; echo kt rc=$?
