# The exact final tree on the GPU box: GPU suite, smoke, one bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_final.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_final.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err && \
python3 -c "import json; d=json.loads(open('gpurun_out/bench_final.json').read().strip().splitlines()[-1]); print(round(d['value']), d['roofline']['frac'], d['c2']['ms_per_image'], d['match']['ms'], d['c4']['value'], d['end_to_end']['value'])"
