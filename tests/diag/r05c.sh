# Round 5: paired-level kernel variants (DMA depth, bands) against one level per launch: per-launch
# kernel times of the 128 x 1080p pyramid (GPU box).
set -o pipefail
mkdir -p gpurun_out/r05c
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gauss.py -x -q --timeout 120 --timeout-method thread -k "duo or streams" > gpurun_out/r05c/gauss.log 2>&1; rc=$?
echo "gauss rc=$rc"; tail -2 gpurun_out/r05c/gauss.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  name=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05c/$name -o run \
    -- python3 tests/probe.py extract --reps 4 > gpurun_out/r05c/$name.log 2>&1 || return 1
  echo "== $name $*"; python3 tests/kt_levels.py gpurun_out/r05c/$name/run_kernel_trace.csv 15 | grep -E "duo|sum|lean<1[13], false|diag<2"
}
run off SGPU_DUO=off && run n7b1 SGPU_DUO=on SGPU_DUO_NIN=7 SGPU_DUO_BANDS=1 && run n5b1 SGPU_DUO=on SGPU_DUO_NIN=5 SGPU_DUO_BANDS=1 && \
run n7b2 SGPU_DUO=on SGPU_DUO_NIN=7 SGPU_DUO_BANDS=2 && run n5b2 SGPU_DUO=on SGPU_DUO_NIN=5 SGPU_DUO_BANDS=2 && run n7b3 SGPU_DUO=on SGPU_DUO_NIN=7 SGPU_DUO_BANDS=3
