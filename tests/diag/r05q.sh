# Round 5: band targets and DMA depth for the shipped paired levels (per-launch kernel times of
# the 128 x 1080p pyramid), alternating (GPU box).
set -o pipefail
OUT=gpurun_out/r05q
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, env...
  name=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run \
    -- python3 tests/probe.py extract --reps 3 > $OUT/$name.log 2>&1 || return 1
  echo "== $name $*"; python3 tests/kt_levels.py $OUT/$name/run_kernel_trace.csv | grep -E "duo|sum"
}
run base X=0 && run w3k SGPU_DUO_WAVES=3072 && run w6k SGPU_DUO_WAVES=6144 && run n5 SGPU_DUO_NIN=5 && run w2k SGPU_DUO_WAVES=2048 && run base2 X=0
