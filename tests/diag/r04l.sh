# Round 4 extremum experiment: grouped XCD order (x4, x2: 4 / 2 workgroups of neighbouring
# strips on one XCD), half the segments (s16k), both (x4s) against the shipped lib; alternating
# whole-bench processes, stage times.
set -o pipefail
mkdir -p gpurun_out
H="--no-c4 --no-e2e --no-match --no-cpu-baseline --no-c2 --steps 10 --warmup 3"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], round(d['value']), {k: round(v, 3) for k, v in s.items() if v > 0.05})" "$1" "$2"; }
for r in 1 2; do
  for L in ${LIBS:-lib x4 x2 s16k x4s}; do
    P=build_exp/$L/libsiftgpu.so; [ $L = lib ] && P=modify-sift-gpu_amd/lib/libsiftgpu.so
    SGPU_LIB_PATH=$P timeout -k 10 120 python3 bench.py $H > gpurun_out/r04l_$L.json 2>/dev/null || exit 1
    show gpurun_out/r04l_$L.json $L
  done
done
