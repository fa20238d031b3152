# Round 5: two build variants (tests/build_variant.sh): fw8 = k_descriptor_flat at 8 waves per
# SIMD (64 VGPRs), nst8 = the u8 level kernel with 8 chunks of loads in flight; parity tests of
# each, then kernel times against the shipped build, alternating (GPU box).
set -o pipefail
OUT=gpurun_out/r05r
mkdir -p $OUT
export TMPDIR=/tmp
SGPU_LIB_PATH=build_exp/fw8/libsiftgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "descriptor or golden" > $OUT/fw8.log 2>&1 || { tail -5 $OUT/fw8.log; exit 1; }
SGPU_LIB_PATH=build_exp/nst8/libsiftgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_gauss.py -x -q --timeout 200 --timeout-method thread > $OUT/nst8.log 2>&1 || { tail -5 $OUT/nst8.log; exit 1; }
echo "parity ok"
for cfg in base:X=0 fw8:SGPU_LIB_PATH=build_exp/fw8/libsiftgpu.so nst8:SGPU_LIB_PATH=build_exp/nst8/libsiftgpu.so base2:X=0 fw8b:SGPU_LIB_PATH=build_exp/fw8/libsiftgpu.so nst8b:SGPU_LIB_PATH=build_exp/nst8/libsiftgpu.so; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- python3 tests/probe.py extract --reps 3 > $OUT/$name.log 2>&1 || exit 1
  echo "== $name"; python3 tests/kt_summary.py $OUT/$name/run_kernel_trace.csv "descriptor_flat|lean<13, true" | head -4
done
