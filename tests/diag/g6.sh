# C4 (16 x 4096^2): the paired-level grid's wave target; k_gauss_lean's conflict-free row-pair
# stores (build variant stmap, SGK_GW_STMAP=1) on both workloads.  (GPU box)
set -o pipefail
mkdir -p gpurun_out/g6
B="--workload c4 --no-c4 --no-e2e --no-match --no-cpu-baseline --no-c2 --steps 10 --warmup 3"
for r in 1 2; do
  for w in 2048 4096 8192; do
    SGPU_DUO_WAVES=$w timeout -k 10 200 python3 bench.py $B > gpurun_out/g6/c4_$w$r.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c4 waves', sys.argv[2], round(d['value']), round(d['stage_ms_per_step']['pyramid'],3), round(d['roofline']['frac'],3))" gpurun_out/g6/c4_$w$r.json $w
  done
done
AB_C4=" " bash tests/diag/ab_env.sh 2 "base:X=0" "stmap:SGPU_LIB_PATH=build_exp/stmap/libsiftgpu.so" || exit 1
