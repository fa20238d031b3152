# Round-end evidence on the one-stream default (tests/gpu_round.sh), then alternating A/Bs against
# the stream layout (SGPU_STREAMS=multi): headline batch, host-in/host-out, C4, C2.
set -o pipefail
bash tests/gpu_round.sh r03g || exit 1
echo "== headline A/B"
timeout -k 10 400 bash tests/diag/ab_env.sh "SGPU_X=" "SGPU_STREAMS=multi" 2 || exit 1
echo "== e2e A/B"
R=1 timeout -k 10 300 bash tests/diag/ab_e2e_env.sh "SGPU_X=" "SGPU_STREAMS=multi" || exit 1
echo "== C4 A/B"
R=1 timeout -k 10 200 bash tests/diag/ab_c4.sh "SGPU_X=" "SGPU_STREAMS=multi" || exit 1
echo "== C2 A/B"
R=2 timeout -k 10 200 bash tests/diag/r03_c2.sh "SGPU_X=" "SGPU_STREAMS=multi"
