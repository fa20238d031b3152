# Round 6: C2 with 16-row tiles on the larger levels (SGPU_TILE_ROWS16_MB: levels of at least that
# many MB), alternating processes; tile parity of the 16-row form.   (GPU box)
set -o pipefail
OUT=gpurun_out/r06e
mkdir -p $OUT
SGPU_TILE_ROWS16_MB=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_gauss.py -k "tile" > $OUT/pytest16.log 2>&1
rc=$?; tail -2 $OUT/pytest16.log; [ $rc -eq 0 ] || exit $rc
python3 -c "
import sys; sys.path.insert(0, 'modify-sift-gpu_amd/python')
from sift_synth import synth_image
img = synth_image(1920, 1080, 2000)
open('$OUT/c2.pgm', 'wb').write(b'P5\n1920 1080\n255\n' + img.tobytes())"
for i in 1 2 3; do
  for cfg in th32:X=0 th16o0:SGPU_TILE_ROWS16_MB=4 th16o01:SGPU_TILE_ROWS16_MB=1; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env ${envs//,/ } timeout -k 10 60 ./modify-sift-gpu_amd/bin/speed_replica 30 -- -i $OUT/c2.pgm -fo 0 -no 4 -d 3 > $OUT/$name$i.json || exit 1
    python3 -c "import json; d=json.load(open('$OUT/$name$i.json')); print('$name', d['features'], round(d['avg_ms'], 4), round(d['timed_avg_ms'], 4), {k: round(v, 4) for k, v in d['timing_ms'].items() if v})"
  done
done
exit 0
