# Round 6: the flat descriptor's DPP neighbours (default) against the 4-gather form (build variant
# nb0: tests/build_variant.sh nb0 -DSGK_DESC_DPP_NB=0) on the batch and C2; descriptor parity.
set -o pipefail
OUT=gpurun_out/r06f
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_gauss.py tests/test_gpu_options.py \
    -k "descriptor or golden or full_hd or wide or dual or host_output or rejected or speed or c3_shard or streams or orientation or options" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
python3 -c "
import sys; sys.path.insert(0, 'modify-sift-gpu_amd/python')
from sift_synth import synth_image
img = synth_image(1920, 1080, 2000)
open('$OUT/c2.pgm', 'wb').write(b'P5\n1920 1080\n255\n' + img.tobytes())"
for i in 1 2 3; do
  for cfg in dpp:X=0 nb0:SGPU_LIB_PATH=build_exp/nb0/libsiftgpu.so; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-c4 --no-e2e --no-c2 --no-match --no-cpu-baseline > $OUT/b_$name$i.json 2> $OUT/b_$name$i.err || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/b_$name$i.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['stage_ms_per_step'].items() if v > 0.01})"
  done
done
for i in 1 2; do
  for cfg in dpp:X=0 nb0:LD_LIBRARY_PATH=build_exp/nb0 oriexp:LD_LIBRARY_PATH=build_exp/oriexp; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env $envs timeout -k 10 60 ./modify-sift-gpu_amd/bin/speed_replica 30 -- -i $OUT/c2.pgm -fo 0 -no 4 -d 3 > $OUT/c2_$name$i.json || exit 1
    python3 -c "import json; d=json.load(open('$OUT/c2_$name$i.json')); print('c2 $name', d['features'], round(d['avg_ms'], 4), {k: round(v, 4) for k, v in d['timing_ms'].items() if v})"
  done
done
exit 0
