# Host-in / host-out stream (bench.py end_to_end) A/B against an experiment build, alternating:
#   bash tests/diag/ab_e2e.sh build_exp/<name>/libsiftgpu.so [rounds]
B=$1; R=${2:-2}
H="--no-cpu-baseline --no-c4 --no-match --no-c2 --steps 3 --warmup 1"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['end_to_end']; print(sys.argv[2], round(d['value']), 'e2e', round(e['value']), round(e['ms_per_batch'], 3))" "$1" "$2"; }
for r in $(seq $R); do
  timeout -k 10 200 python3 bench.py $H > gpurun_out/e2e_a.json 2>/dev/null || exit 1; show gpurun_out/e2e_a.json A
  SGPU_LIB_PATH=$B timeout -k 10 200 python3 bench.py $H > gpurun_out/e2e_b.json 2>gpurun_out/e2e_b.err || { tail -3 gpurun_out/e2e_b.err; exit 1; }; show gpurun_out/e2e_b.json B
done
