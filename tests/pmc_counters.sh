#!/bin/bash
# Ad-hoc counter passes on the bench command (GPU box): tests/pmc_counters.sh <tag> "<set1>" "<set2>" ...
set -e
TAG=$1; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
A="--steps 1 --warmup 0 --no-cpu-baseline --no-match"
i=0
for SET in "$@"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $SET --output-format csv -d $OUT/p$i -o run -- python3 bench.py $A > $OUT/p$i.log 2>&1
done
