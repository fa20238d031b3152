# Round 5: k_gauss_duo with 96-column strips -- its parity tests, then the pyramid per launch for
# band targets (SGPU_DUO_WAVES) and narrow / wide pairing, against duo off (GPU box).
set -o pipefail
mkdir -p gpurun_out/r05f
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gauss.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05f/gauss.log 2>&1; rc=$?
echo "gauss rc=$rc"; tail -2 gpurun_out/r05f/gauss.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  name=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05f/$name -o run \
    -- python3 tests/probe.py extract --reps 3 > gpurun_out/r05f/$name.log 2>&1 || return 1
  echo "== $name $*"; python3 tests/kt_levels.py gpurun_out/r05f/$name/run_kernel_trace.csv 15 | grep -E "duo|sum|lean<2|diag"
}
run off SGPU_DUO=off && run w4k SGPU_DUO=on SGPU_DUO_WAVES=4096 && run w6k SGPU_DUO=on SGPU_DUO_WAVES=6144 && \
run w8k SGPU_DUO=on SGPU_DUO_WAVES=8192 && run w12k SGPU_DUO=on SGPU_DUO_WAVES=12288 && run wide SGPU_DUO=on SGPU_DUO_WIDE=1
