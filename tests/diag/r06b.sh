# Round 6: tile extremum kernel + host output from the descriptor kernel (parity, C2 A/B) and the
# paired-level kernel at 4 workgroups per CU (SGPU_DUO_NIN=4) on the 128 x 1080p batch.
#   bash tests/diag/r06b.sh   (GPU box)
set -o pipefail
OUT=gpurun_out/r06b
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_gauss.py \
    -k "extrema_tile or wide or host_output or speed or simplesift or tile or alias or orientation or golden or full_hd" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
python3 -c "
import sys; sys.path.insert(0, 'modify-sift-gpu_amd/python')
from sift_synth import synth_image
img = synth_image(1920, 1080, 2000)
open('$OUT/c2.pgm', 'wb').write(b'P5\n1920 1080\n255\n' + img.tobytes())"
for i in 1 2 3; do
  for cfg in wave:SGPU_EXTREMA=wave tile:X=0; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env ${envs//,/ } timeout -k 10 60 ./modify-sift-gpu_amd/bin/speed_replica 30 -- -i $OUT/c2.pgm -fo 0 -no 4 -d 3 > $OUT/$name$i.json || exit 1
    python3 -c "import json; d=json.load(open('$OUT/$name$i.json')); print('$name', d['features'], round(d['avg_ms'], 4), round(d['timed_avg_ms'], 4), {k: round(v, 4) for k, v in d['timing_ms'].items() if v})"
  done
done
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
    -- ./modify-sift-gpu_amd/bin/speed_replica 10 -- -i $OUT/c2.pgm -fo 0 -no 4 -d 3 > $OUT/prof.log 2>&1 || exit 1
python3 tests/kt_summary.py $OUT/trace/run_kernel_trace.csv > $OUT/kt_summary.txt 2>&1
head -32 $OUT/kt_summary.txt
for i in 1 2; do
  for cfg in nin7:X=0 nin4:SGPU_DUO_NIN=4; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env ${envs//,/ } timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-c4 --no-e2e --no-c2 --no-match --no-cpu-baseline > $OUT/bench_$name$i.json 2> $OUT/bench_$name$i.err || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/bench_$name$i.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), d['ms_per_step'], d.get('roofline', {}).get('frac'), d.get('stage_ms_per_step'))"
  done
done
exit 0
