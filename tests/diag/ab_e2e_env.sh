# Host-in / host-out stream (bench.py end_to_end) under several environment settings:
#   bash tests/diag/ab_e2e_env.sh "SGPU_PYR=serial" "SGPU_X=0" ...   (R= rounds)
R=${R:-1}
H="--no-cpu-baseline --no-c4 --no-match --no-c2 --steps 3 --warmup 1"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['end_to_end']; print(sys.argv[2], round(d['value']), 'e2e', round(e['value']), round(e['ms_per_batch'], 3))" "$1" "$2"; }
for r in $(seq $R); do
  for e in "$@"; do
    env $e timeout -k 10 200 python3 bench.py $H > gpurun_out/e2e_x.json 2>/dev/null || exit 1; show gpurun_out/e2e_x.json "[$e]"
  done
done
