# Round 5, first GPU pass: the paired-level Gaussian kernel's parity tests, then A/B bench lines
# (duo on / off, alternating processes), then the whole GPU suite.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gauss.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05a_gauss.log 2>&1; rc=$?
echo "gauss rc=$rc"; tail -4 gpurun_out/r05a_gauss.log
[ $rc -eq 0 ] || exit $rc
H="--no-c4 --no-e2e --no-cpu-baseline --no-c2 --no-match"
for i in 1 2; do
  timeout -k 10 200 python bench.py $H > gpurun_out/r05a_on$i.json 2> gpurun_out/r05a_on$i.err || exit 1
  SGPU_DUO=off timeout -k 10 200 python bench.py $H > gpurun_out/r05a_off$i.json 2> gpurun_out/r05a_off$i.err || exit 1
done
python3 - <<'PY'
import json
for t in ("on1", "off1", "on2", "off2"):
    d = json.loads(open(f"gpurun_out/r05a_{t}.json").read().strip().splitlines()[-1])
    s = d["stage_ms_per_step"]
    print(t, round(d["value"]), "pyr %.3f frac %.3f det %.3f" % (s["pyramid"], d["roofline"]["frac"], s["detect"]), d["roofline"]["kernel"][-90:])
PY
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05a_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r05a_pytest.log
