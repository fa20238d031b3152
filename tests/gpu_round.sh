set -o pipefail
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" 
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && echo bench ok && \
timeout -k 10 900 bash tests/profile_kernels.sh r01 && echo profile ok
