# Round 5: paired levels on octave 2 too (SGK_DUO_MIN_MB=32 build variant) against the shipped
# 128 MB minimum: pyramid per launch, alternating (GPU box).
set -o pipefail
OUT=gpurun_out/r05t
mkdir -p $OUT
export TMPDIR=/tmp
SGPU_LIB_PATH=build_exp/dm32/libsiftgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_gauss.py -x -q --timeout 200 --timeout-method thread > $OUT/dm32.log 2>&1 || { tail -5 $OUT/dm32.log; exit 1; }
for cfg in base:X=0 dm32:SGPU_LIB_PATH=build_exp/dm32/libsiftgpu.so base2:X=0 dm32b:SGPU_LIB_PATH=build_exp/dm32/libsiftgpu.so; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- python3 tests/probe.py extract --reps 3 > $OUT/$name.log 2>&1 || exit 1
  echo "== $name"; python3 tests/kt_levels.py $OUT/$name/run_kernel_trace.csv | tail -9
done
