# A/B of the matcher between two environment settings of the same build, alternating processes:
#   bash tests/diag/ab_match_env.sh "SGPU_MATCH=reg" [rounds]   (A = no setting)
B=$1; R=${2:-3}
for r in $(seq $R); do
  echo "A: $(timeout -k 10 120 python -u tests/diag/match_time.py 50000 plain,rows_only | tr '\n' ' ')" || exit 1
  echo "B: $(env $B timeout -k 10 120 python -u tests/diag/match_time.py 50000 plain,rows_only | tr '\n' ' ')" || exit 1
done
