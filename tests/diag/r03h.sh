# Short-band A/B on the GPU box: default (levels <= 128 MB: bands down to one chunk, ~8,192 waves)
# against SGPU_GAUSS_BANDS=mid (r03g: <= 64 MB, ~2,048 waves) and =long (round 2).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gauss.py tests/test_gpu_workloads.py tests/test_gpu_parity.py -k "gauss or levels or golden or c4 or shard or one_stream or capacity" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_h.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_h.log
[ $rc -eq 0 ] || exit $rc
echo "== headline A/B"
timeout -k 10 400 bash tests/diag/ab_env.sh "SGPU_X=" "SGPU_GAUSS_BANDS=mid" 3 || exit 1
echo "== C4 A/B"
R=2 timeout -k 10 300 bash tests/diag/ab_c4.sh "SGPU_X=" "SGPU_GAUSS_BANDS=mid" || exit 1
echo "== C2 A/B"
R=2 timeout -k 10 200 bash tests/diag/r03_c2.sh "SGPU_X=" "SGPU_GAUSS_BANDS=mid" "SGPU_GAUSS_BANDS=long"
