# Two waves per feature for few features (C2), opt-in SGPU_DESC_HALF=1: the GPU suite with it on,
# then C2 A/B against the shipped one wave per feature.
set -o pipefail
mkdir -p gpurun_out
SGPU_DESC_HALF=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_k.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_k.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_k.log | head -20; exit $rc; }
R=3 timeout -k 10 200 bash tests/diag/r03_c2.sh "SGPU_X=" "SGPU_DESC_HALF=1"
