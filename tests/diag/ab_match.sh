# A/B of the matcher against an experiment build, alternating processes:
#   bash tests/diag/ab_match.sh build_exp/<name>/libsiftgpu.so [rounds]
B=$1; R=${2:-3}
for r in $(seq $R); do
  echo "A: $(timeout -k 10 120 python -u tests/diag/match_time.py 50000 plain,rows_only | tr '\n' ' ')" || exit 1
  echo "B: $(SGPU_LIB_PATH=$B timeout -k 10 120 python -u tests/diag/match_time.py 50000 plain,rows_only | tr '\n' ' ')" || exit 1
done
