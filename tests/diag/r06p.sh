# Round 6 closing tree with the pruned matcher column side: C5 A/B (pruned vs unpruned, same box,
# three alternating rounds), then the round-end evidence (tests/gpu_round.sh).
set -o pipefail
mkdir -p gpurun_out/r06p
for r in 1 2 3; do timeout -k 10 120 python -u tests/diag/match_time.py 50000 plain,plain_noprune,rows_only >> gpurun_out/r06p/match_time.log 2>&1 || exit 1; done
cat gpurun_out/r06p/match_time.log
bash tests/gpu_round.sh r06p
