# Alternating A/B of the headline bench (stage times) against an experiment build:
#   bash tests/diag/ab_bench.sh build_exp/<name>/libsiftgpu.so [rounds]
B=$1; R=${2:-2}
H="--no-c4 --no-e2e --no-match --no-cpu-baseline --no-c2 --steps 10 --warmup 3"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], round(d['value']), {k: round(v, 3) for k, v in s.items() if v > 0.05})" "$1" "$2"; }
for r in $(seq $R); do
  timeout -k 10 120 python3 bench.py $H > gpurun_out/ab_a.json 2>/dev/null || exit 1; show gpurun_out/ab_a.json A
  SGPU_LIB_PATH=$B timeout -k 10 120 python3 bench.py $H > gpurun_out/ab_b.json 2>/dev/null || exit 1; show gpurun_out/ab_b.json B
done
