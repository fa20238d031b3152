#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the GPU box (tests/microbench/pmc_calib.hip: 1 GiB
# streamed once per kernel at 16 / 8 / 4 bytes per lane), one counter per rocprofv3 pass as the
# guide prescribes, then the factors into profiles/<tag>_pmc_calibration.json.
#   tests/pmc_calib.sh <tag>
set -e
TAG=${1:-r03}
OUT=gpurun_out/pmc_calib_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
B=tests/microbench/pmc_calib
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- ./$B > "$OUT/fetch.log" 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- ./$B > "$OUT/write.log" 2>&1
timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- ./$B > "$OUT/trace.log" 2>&1
python3 tests/pmc_calib_summary.py "$OUT" "$TAG"
