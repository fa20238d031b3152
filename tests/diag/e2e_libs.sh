# Host-in / host-out stream (bench.py end_to_end) for several builds, in turn:
#   bash tests/diag/e2e_libs.sh build_exp/a/libsiftgpu.so build_exp/b/libsiftgpu.so ...
H="--no-cpu-baseline --no-c4 --no-match --no-c2 --steps 3 --warmup 1"
for L in "$@"; do
  SGPU_LIB_PATH=$L timeout -k 10 200 python3 bench.py $H > gpurun_out/e2e_l.json 2>gpurun_out/e2e_l.err || { tail -3 gpurun_out/e2e_l.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['end_to_end']; print(sys.argv[2], round(d['value']), 'e2e', round(e['value']), round(e['ms_per_batch'], 3))" gpurun_out/e2e_l.json "$L"
done
