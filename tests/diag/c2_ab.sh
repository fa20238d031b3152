# C2 (one 1080p image through SiftGPU::RunSIFT, bin/speed_replica) under library A/B settings,
# alternating processes:  bash tests/diag/c2_ab.sh  (GPU box)
set -o pipefail
OUT=gpurun_out/c2ab
mkdir -p $OUT
python3 -c "
import sys; sys.path.insert(0, 'modify-sift-gpu_amd/python')
from sift_synth import synth_image
img = synth_image(1920, 1080, 2000)
open('$OUT/c2.pgm', 'wb').write(b'P5\n1920 1080\n255\n' + img.tobytes())"
for i in 1 2 3; do
  for cfg in base:X=0 nohost:SGPU_HOST_OUTPUT=0 notime:X=0; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env ${envs//,/ } timeout -k 10 60 ./modify-sift-gpu_amd/bin/speed_replica 30 -- -i $OUT/c2.pgm -fo 0 -no 4 -d 3 > $OUT/$name$i.json || exit 1
    python3 -c "import json; d=json.load(open('$OUT/$name$i.json')); print('$name', d['avg_ms'], d['timed_avg_ms'], {k: round(v, 4) for k, v in d['timing_ms'].items() if v})"
  done
done
exit 0
python3 tests/kt_summary.py gpurun_out/prof_c2_r05/trace/run_kernel_trace.csv | head -40
