#!/bin/bash
# Kernel timing + HBM counters of the bench command (run on the GPU box), then the summary:
#   tests/profile_kernels.sh <tag>   -> gpurun_out/prof_<tag>/{trace,fetch,write}/...
#                                       profiles/<tag>_kernel_stats.csv, profiles/<tag>_summary.json
# Separate passes: kernel trace + stats of `bench.py` as the driver runs it, then FETCH_SIZE,
# then WRITE_SIZE (the guide's HBM recipe: counters in their own passes, never together with
# --sys-trace/--runtime-trace).
set -e
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
    -- python3 bench.py > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
    -- python3 bench.py --steps 3 --warmup 1 --no-match --no-cpu-baseline > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
    -- python3 bench.py --steps 3 --warmup 1 --no-match --no-cpu-baseline > "$OUT/write.log" 2>&1
python3 tests/pmc_summary.py "$OUT" "$TAG" > "$OUT/summary.log" 2>&1
