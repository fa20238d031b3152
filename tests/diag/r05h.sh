# Round 5: the paired-level kernel shipped by default ((11, 13) pairs): the whole GPU suite, the
# bench line, then the kernel / counter profile of this tree (GPU box).
set -o pipefail
mkdir -p gpurun_out/r05h
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05h/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05h/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r05h/bench.json 2> gpurun_out/r05h/bench.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05h/bench.json").read().strip().splitlines()[-1])
print(round(d["value"]), d["ms_per_step"], "pyr", d["stage_ms_per_step"]["pyramid"], "frac", d["roofline"]["frac"], "c2", d["c2"]["ms_per_image"], "c4", d["c4"]["value"])
PY
bash tests/profile_kernels.sh r05h > gpurun_out/r05h/prof.log 2>&1 || exit 1
tail -5 gpurun_out/prof_r05h/summary.log
