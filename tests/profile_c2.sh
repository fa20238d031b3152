#!/bin/bash
# Kernel + memory-copy trace of config C2 (one 1920x1080 image through SiftGPU::RunSIFT, the
# speed.cpp protocol of bin/speed_replica), on the GPU box:
#   tests/profile_c2.sh <tag>  -> gpurun_out/prof_c2_<tag>/...
set -e
TAG=${1:-r03}
OUT=gpurun_out/prof_c2_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -c "
import sys; sys.path.insert(0, 'modify-sift-gpu_amd/python')
from sift_synth import synth_image
img = synth_image(1920, 1080, 2000)
open('$OUT/c2.pgm', 'wb').write(b'P5\n1920 1080\n255\n' + img.tobytes())"
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/trace" -o run \
    -- ./modify-sift-gpu_amd/bin/speed_replica 10 -- -i "$OUT/c2.pgm" -fo 0 -no 4 -d 3 > "$OUT/run.log" 2>&1
cat "$OUT/run.log"
