# Round 6: tile duos (two levels per launch for a single image's pyramid) parity + C2 A/B, and the
# wide descriptor's wave count / grid knobs.   bash tests/diag/r06c.sh   (GPU box)
set -o pipefail
OUT=gpurun_out/r06c
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_gauss.py tests/test_gpu_parity.py tests/test_gpu_api.py \
    -k "tile or wide or host_output or golden or full_hd or simplesift or levels or descriptor or c3_shard" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
python3 -c "
import sys; sys.path.insert(0, 'modify-sift-gpu_amd/python')
from sift_synth import synth_image
img = synth_image(1920, 1080, 2000)
open('$OUT/c2.pgm', 'wb').write(b'P5\n1920 1080\n255\n' + img.tobytes())"
for i in 1 2 3; do
  for cfg in single:SGPU_TILE_DUO=off duo:X=0 w8:SGPU_WIDE_DESC_WAVES=8 g800:SGPU_WIDE_DESC_GRID=800 g400:SGPU_WIDE_DESC_GRID=400; do
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
timeout -k 10 120 python tests/make_shard_fixtures.py $OUT/match_shard_states.npz || exit 1
exit 0
