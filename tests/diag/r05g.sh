# Round 5: the u8 ingest pair (levels 0 and 1 from the image in one k_gauss_duo launch): its
# parity tests, then the pyramid per launch against duo off, for band targets (GPU box).
set -o pipefail
mkdir -p gpurun_out/r05g
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gauss.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05g/gauss.log 2>&1; rc=$?
echo "gauss rc=$rc"; tail -2 gpurun_out/r05g/gauss.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  name=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05g/$name -o run \
    -- python3 tests/probe.py extract --reps 3 > gpurun_out/r05g/$name.log 2>&1 || return 1
  echo "== $name $*"; python3 tests/kt_levels.py gpurun_out/r05g/$name/run_kernel_trace.csv 15
}
run off SGPU_DUO=off && run w4k SGPU_DUO=on SGPU_DUO_WAVES=4096 && run w6k SGPU_DUO=on SGPU_DUO_WAVES=6144 && \
run w3k SGPU_DUO=on SGPU_DUO_WAVES=3072
