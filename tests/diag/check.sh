# Round 5 check of a tree on the GPU box: the whole GPU suite, the bench line, the pyramid per
# launch, then the kernel / counter profile of this tree:  bash tests/diag/check.sh <tag>
set -o pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 - $OUT <<'PY'
import json, sys
d = json.loads(open(sys.argv[1] + "/bench.json").read().strip().splitlines()[-1])
print(round(d["value"]), d["ms_per_step"], "pyr", d["stage_ms_per_step"]["pyramid"], "frac", d["roofline"]["frac"], "c2", d["c2"]["ms_per_image"], "c4", d["c4"]["value"], "match", d.get("match", {}).get("ms"))
PY
bash tests/profile_kernels.sh $TAG > $OUT/prof.log 2>&1 || exit 1
python3 tests/kt_levels.py gpurun_out/prof_$TAG/trace/run_kernel_trace.csv
