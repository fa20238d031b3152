# Round 6 short closing run (pruned matcher column side): matcher GPU tests, C5 A/B pruned vs
# unpruned, the bench line, smoke.
set -o pipefail
mkdir -p gpurun_out/r06q
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "match" > gpurun_out/r06q/pytest_match.log 2>&1; rc=$?; tail -2 gpurun_out/r06q/pytest_match.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do timeout -k 10 120 python -u tests/diag/match_time.py 50000 plain,plain_noprune,rows_only >> gpurun_out/r06q/match_time.log 2>&1 || exit 1; done
cat gpurun_out/r06q/match_time.log
timeout -k 10 300 python bench.py > gpurun_out/r06q/bench.json 2> gpurun_out/r06q/bench.err && echo bench ok || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06q/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r06q/smoke.log; exit $rc
