# Round 6 closing tree with the pruned matcher column side: matcher GPU tests, C5 A/B (pruned vs
# unpruned, same box, three rounds), kernel profile + HBM counters of the bench workload (the
# summary the bench line's traffic reads), the bench line, smoke, matcher SQ counters.
set -o pipefail
mkdir -p gpurun_out/r06p
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06p/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/r06p/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do timeout -k 10 120 python -u tests/diag/match_time.py 50000 plain,plain_noprune,rows_only >> gpurun_out/r06p/match_time.log 2>&1 || exit 1; done
cat gpurun_out/r06p/match_time.log
timeout -k 10 900 bash tests/profile_kernels.sh r06p && echo profile ok || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r06p/bench.json 2> gpurun_out/r06p/bench.err && echo bench ok || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06p/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r06p/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash tests/pmc_match.sh gpurun_out/pmc_match_r06p && python3 tests/pmc_match_summary.py gpurun_out/pmc_match_r06p gpurun_out/r06p_match_sq_counters.json && echo pmc match ok
