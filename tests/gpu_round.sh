# Round-end evidence on the GPU box: GPU test suite, smoke, bench line, kernel profile + HBM
# counters, matcher SQ counters, C2 trace.
#   bash tests/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"
tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && echo bench ok && \
timeout -k 10 900 bash tests/profile_kernels.sh "$TAG" && echo profile ok && \
timeout -k 10 300 bash tests/pmc_match.sh "gpurun_out/pmc_match_$TAG" && \
python3 tests/pmc_match_summary.py "gpurun_out/pmc_match_$TAG" "gpurun_out/${TAG}_match_sq_counters.json" && echo pmc match ok && \
timeout -k 10 300 bash tests/profile_c2.sh "$TAG" > gpurun_out/prof_c2.log 2>&1 && echo c2 ok
