# Conflict-free row-pair stores in k_gauss_lean (build variant stmap, SGK_GW_STMAP=1): the
# Gaussian parity tests on the variant, then alternating bench pairs (pyramid stage times).
#   bash tests/diag/r06l.sh   (GPU box)
set -o pipefail
OUT=gpurun_out/r06l
mkdir -p $OUT
SGPU_LIB_PATH=build_exp/stmap/libsiftgpu.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_gauss.py tests/test_gpu_parity.py -k "gauss or level or golden or pyramid" > $OUT/pytest_stmap.log 2>&1
rc=$?; tail -2 $OUT/pytest_stmap.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for cfg in base:X=0 stmap:SGPU_LIB_PATH=build_exp/stmap/libsiftgpu.so; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-e2e --no-c2 --no-match --no-cpu-baseline > $OUT/b_$name$i.json 2> $OUT/b_$name$i.err || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/b_$name$i.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['stage_ms_per_step'].items() if v > 0.01}, 'c4', d.get('c4', {}).get('value'), d.get('c4', {}).get('stage_ms_per_step', {}).get('pyramid'))"
  done
done
# 32-bit descriptor sums (build variant u32, SGK_FLAT_U32=1)
SGPU_LIB_PATH=build_exp/u32/libsiftgpu.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py -k "shipped_descriptor or wide or golden" > $OUT/pytest_u32.log 2>&1
rc=$?; tail -2 $OUT/pytest_u32.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for cfg in u64:X=0 u32:SGPU_LIB_PATH=build_exp/u32/libsiftgpu.so; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-c4 --no-e2e --no-match --no-cpu-baseline > $OUT/b_$name$i.json 2> $OUT/b_$name$i.err || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/b_$name$i.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['stage_ms_per_step'].items() if v > 0.01}, 'c2', d.get('c2', {}).get('ms_per_image'))"
  done
done
exit 0
