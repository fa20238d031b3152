# Round 6 closing evidence (tests/gpu_round.sh) followed by the 32-bit descriptor-sum A/B
# (build variant u32).   bash tests/diag/r06k.sh <tag>   (GPU box)
set -o pipefail
TAG=${1:-r06k}
bash tests/gpu_round.sh "$TAG" || exit $?
OUT=gpurun_out/r06h
mkdir -p $OUT
SGPU_LIB_PATH=build_exp/u32/libsiftgpu.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py -k "shipped_descriptor or wide or golden" > $OUT/pytest_u32.log 2>&1
rc=$?; tail -2 $OUT/pytest_u32.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for cfg in u64:X=0 u32:SGPU_LIB_PATH=build_exp/u32/libsiftgpu.so; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-c4 --no-e2e --no-c2 --no-match --no-cpu-baseline > $OUT/b_$name$i.json 2> $OUT/b_$name$i.err || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/b_$name$i.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['stage_ms_per_step'].items() if v > 0.01})"
  done
done
exit 0
