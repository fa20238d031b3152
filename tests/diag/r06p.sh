set -o pipefail
mkdir -p gpurun_out/r06p
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "match" > gpurun_out/r06p/pytest_match.log 2>&1; rc=$?; tail -3 gpurun_out/r06p/pytest_match.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do timeout -k 10 120 python -u tests/diag/match_time.py 50000 plain,plain_noprune,rows_only >> gpurun_out/r06p/match_time.log 2>&1 || exit 1; done
cat gpurun_out/r06p/match_time.log
