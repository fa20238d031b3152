# Config C2 (one 1920x1080 image through SiftGPU::RunSIFT, bin/speed_replica) under several
# environment settings, alternating, on the GPU box:
#   bash tests/diag/r03_c2.sh "SGPU_X=" "SGPU_STREAMS=multi" "SGPU_GAUSS_BANDS=long" ... (R=rounds)
R=${R:-3}
mkdir -p gpurun_out/c2ab
python3 -c "
import sys; sys.path.insert(0, 'modify-sift-gpu_amd/python')
from sift_synth import synth_image
img = synth_image(1920, 1080, 2000)
open('gpurun_out/c2ab/c2.pgm', 'wb').write(b'P5\n1920 1080\n255\n' + img.tobytes())" || exit 1
for r in $(seq $R); do
  for e in "$@"; do
    env $e timeout -k 10 60 ./modify-sift-gpu_amd/bin/speed_replica 30 -- -i gpurun_out/c2ab/c2.pgm -fo 0 -no 4 -d 3 > gpurun_out/c2ab/run.json || exit 1
    tail -1 gpurun_out/c2ab/run.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$e]', d['avg_ms'], d['features'], {k: round(v, 3) for k, v in d['timing_ms'].items() if v})"
  done
done
