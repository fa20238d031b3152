# One stream per single-part batch as the default: GPU suite, then alternating A/Bs against the
# stream layout (SGPU_STREAMS=multi): headline batch, host-in/host-out stream, C4, C2.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_f.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_f.log
[ $rc -eq 0 ] || exit $rc
echo "== headline A/B"
timeout -k 10 500 bash tests/diag/ab_env.sh "SGPU_X=" "SGPU_STREAMS=multi" 3 || exit 1
echo "== e2e A/B"
R=2 timeout -k 10 500 bash tests/diag/ab_e2e_env.sh "SGPU_X=" "SGPU_STREAMS=multi" || exit 1
echo "== C4 A/B"
R=2 timeout -k 10 300 bash tests/diag/ab_c4.sh "SGPU_X=" "SGPU_STREAMS=multi" || exit 1
echo "== C2 A/B"
R=2 timeout -k 10 200 bash tests/diag/r03_c2.sh "SGPU_X=" "SGPU_STREAMS=multi"
