# Alternating A/B of the headline bench (stage times) between environment settings:
#   bash tests/diag/ab_env.sh <rounds> "name:VAR=value[,VAR=value]" "name:..." ...   (GPU box)
R=$1; shift
H="${AB_C4:---no-c4} --no-e2e --no-match --no-cpu-baseline --no-c2 --steps 10 --warmup 3 ${AB_FLAGS:-}"
mkdir -p gpurun_out/ab
for r in $(seq $R); do
  for cfg in "$@"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env ${envs//,/ } timeout -k 10 180 python3 bench.py $H > gpurun_out/ab/$name$r.json 2> gpurun_out/ab/$name$r.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], round(d['value']), {k: round(v, 3) for k, v in s.items() if v > 0.05}, 'frac', round(d['roofline']['frac'], 3), 'c4', d.get('c4', {}).get('value'), d.get('c4', {}).get('stage_ms_per_step', {}).get('pyramid'))" gpurun_out/ab/$name$r.json $name
  done
done
