# Round 5: what bounds k_gauss_duo -- variants (tests/build_variant.sh): sw32 / sw16 = strips of
# 96 / 112 columns (128-B / 64-B aligned rows), dexp2 / dexp2sw = no filter arithmetic (timing
# only, wrong levels); bands 1 and 3 (GPU box).
set -o pipefail
mkdir -p gpurun_out/r05e
export TMPDIR=/tmp
run() {  # name, env...
  name=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05e/$name -o run \
    -- python3 tests/probe.py extract --reps 3 > gpurun_out/r05e/$name.log 2>&1 || return 1
  echo "== $name $*"; python3 tests/kt_levels.py gpurun_out/r05e/$name/run_kernel_trace.csv 15 | grep -E "duo|sum"
}
for v in sw32 sw16 dexp2sw dexp2; do
  for b in 1 3; do
    run ${v}b$b SGPU_LIB_PATH=build_exp/$v/libsiftgpu.so SGPU_DUO=on SGPU_DUO_BANDS=$b || exit 1
  done
done
