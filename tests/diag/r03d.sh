# Round 3 step d on the GPU box: full GPU suite (one-stream small batches, short bands on
# cache-resident levels), C2 A/B and trace, descriptor lane-layout A/B, stream and band A/Bs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_d.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_d.log
[ $rc -eq 0 ] || exit $rc
echo "== C2 A/B"
R=3 timeout -k 10 300 bash tests/diag/r03_c2.sh "SGPU_X=" "SGPU_STREAMS=multi" "SGPU_GAUSS_BANDS=long" || exit 1
timeout -k 10 200 bash tests/profile_c2.sh r03d > gpurun_out/prof_c2_d.log 2>&1 || exit 1
tail -1 gpurun_out/prof_c2_d.log
timeout -k 10 600 bash tests/diag/r03_desc.sh || exit 1
echo "== batch A/B: A = every stage on one stream, B = shipped (octave + feature streams)"
timeout -k 10 400 bash tests/diag/ab_env.sh "SGPU_STREAMS=one" "SGPU_STREAMS=" 2 || exit 1
echo "== C4 A/B: short bands on the cache-resident octaves vs long"
R=2 timeout -k 10 300 bash tests/diag/ab_c4.sh "SGPU_X=" "SGPU_GAUSS_BANDS=long"
