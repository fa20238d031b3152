# Round 5: the (17, 21) pair with decimation (SGPU_DUO_WIDE=1): parity tests, pyramid per launch
# against duo off and the (11, 13) pairs alone (GPU box).
set -o pipefail
mkdir -p gpurun_out/r05i
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gauss.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05i/gauss.log 2>&1; rc=$?
echo "gauss rc=$rc"; tail -2 gpurun_out/r05i/gauss.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  name=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05i/$name -o run \
    -- python3 tests/probe.py extract --reps 3 > gpurun_out/r05i/$name.log 2>&1 || return 1
  echo "== $name $*"; python3 tests/kt_levels.py gpurun_out/r05i/$name/run_kernel_trace.csv 15
}
run off SGPU_DUO=off && run on SGPU_DUO=on && run wide SGPU_DUO=on SGPU_DUO_WIDE=1 && run wide6k SGPU_DUO=on SGPU_DUO_WIDE=1 SGPU_DUO_WAVES=6144
