# Matcher check on the GPU box: parity tests, the C5 timing probe, SQ counters of k_match_rows.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "match" > gpurun_out/t_match.log 2>&1; rc=$?; tail -2 gpurun_out/t_match.log
[ $rc -eq 0 ] && timeout -k 10 200 python tests/match_probe.py > gpurun_out/match_probe.log 2>&1; cat gpurun_out/match_probe.log
[ $rc -eq 0 ] && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex "k_match_rows" --output-format csv -d gpurun_out/pmc_match -o run -- python3 tests/match_probe.py > gpurun_out/pmc_match.log 2>&1; echo pmc rc=$?
