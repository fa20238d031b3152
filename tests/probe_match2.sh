# Pipelined matcher (variant 64): parity, C5 timing against the shipped kernel.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "match" > gpurun_out/t_match.log 2>&1; rc=$?; tail -2 gpurun_out/t_match.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tests/match_probe.py 50000 0 64 0 64 > gpurun_out/match_probe.log 2>&1; cat gpurun_out/match_probe.log
