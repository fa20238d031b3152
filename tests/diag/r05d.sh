# Round 5, second GPU pass: the whole GPU suite on the folded C2 launches and the stage-timing
# switch, then the paired-level kernel variants under a kernel trace (r05c's runs), then one bench.
set -o pipefail
mkdir -p gpurun_out/r05d
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05d/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05d/pytest.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  name=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05d/$name -o run \
    -- python3 tests/probe.py extract --reps 4 > gpurun_out/r05d/$name.log 2>&1 || return 1
  echo "== $name $*"; python3 tests/kt_levels.py gpurun_out/r05d/$name/run_kernel_trace.csv 15 | grep -E "duo|sum|lean<1[13], false|diag<2"
}
run off SGPU_DUO=off && run n7b1 SGPU_DUO=on SGPU_DUO_NIN=7 SGPU_DUO_BANDS=1 && run n5b1 SGPU_DUO=on SGPU_DUO_NIN=5 SGPU_DUO_BANDS=1 && \
run n7b2 SGPU_DUO=on SGPU_DUO_NIN=7 SGPU_DUO_BANDS=2 && run n7b3 SGPU_DUO=on SGPU_DUO_NIN=7 SGPU_DUO_BANDS=3 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r05d/bench.json 2> gpurun_out/r05d/bench.err || exit 1
tail -c 3000 gpurun_out/r05d/bench.json
