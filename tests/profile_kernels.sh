#!/bin/bash
# Kernel timing + HBM counters of the headline bench workload (run on the GPU box), then the
# summary:
#   tests/profile_kernels.sh <tag>   -> gpurun_out/prof_<tag>/{trace,fetch,write,c4}/...
#                                       profiles/<tag>_kernel_stats.csv, profiles/<tag>_summary.json,
#                                       profiles/<tag>_c4_kernel_stats.csv
# Separate passes: kernel trace + stats of the headline (C3 shard) bench, then FETCH_SIZE, then
# WRITE_SIZE (the guide's HBM recipe: counters in their own passes, never together with
# --sys-trace/--runtime-trace), then the kernel trace of the C4 workload.  The sub-measurements
# (C4, end-to-end, matcher, CPU baseline) are left out of the headline passes so that every
# extract in them is a 128 x 1080p batch.
set -e
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
H="--no-c4 --no-e2e --no-match --no-cpu-baseline --no-c2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
    -- python3 bench.py $H > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
    -- python3 bench.py --steps 3 --warmup 1 $H > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
    -- python3 bench.py --steps 3 --warmup 1 $H > "$OUT/write.log" 2>&1
python3 tests/pmc_summary.py "$OUT" "$TAG" > "$OUT/summary.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4" -o run \
    -- python3 bench.py --workload c4 $H > "$OUT/c4.log" 2>&1
cp "$OUT"/c4/run_kernel_stats.csv "profiles/${TAG}_c4_kernel_stats.csv"
