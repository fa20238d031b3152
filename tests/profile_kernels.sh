#!/bin/bash
# Kernel timing + HBM counters of one bench configuration (run on the GPU box).
#   tests/profile_kernels.sh <tag>      -> gpurun_out/prof_<tag>/{trace,fetch,write}/...
# Separate passes: kernel trace + stats, then FETCH_SIZE, then WRITE_SIZE (the guide's
# HBM recipe: counters in their own passes, never with --sys-trace/--runtime-trace).
set -e
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
    -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
    -- python3 bench.py $ARGS --no-match > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
    -- python3 bench.py $ARGS --no-match > "$OUT/write.log" 2>&1
find "$OUT" -name "*.csv" | head -20
