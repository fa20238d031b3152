# C4 (16 x 4096x4096, -no 6) stage times under several environment settings, alternating:
#   bash tests/diag/ab_c4.sh "SGPU_PYR=serial" "SGPU_X=0" ... [rounds via R=]
R=${R:-2}
H="--workload c4 --no-c4 --no-e2e --no-match --no-cpu-baseline --no-c2 --steps 6 --warmup 2"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], round(d['value']), {k: round(v, 3) for k, v in s.items() if v > 0.05})" "$1" "$2"; }
for r in $(seq $R); do
  for e in "$@"; do
    env $e timeout -k 10 120 python3 bench.py $H > gpurun_out/ab_c4.json 2>/dev/null || exit 1; show gpurun_out/ab_c4.json "[$e]"
  done
done
