# Round 5: k_orientation at 6 waves per SIMD (build variant ori6, 80 VGPRs + 14 spilled) against
# the shipped build (90 VGPRs, 5 waves): parity of the variant, then alternating kernel times.
set -o pipefail
OUT=gpurun_out/r05u
mkdir -p $OUT
export TMPDIR=/tmp
SGPU_LIB_PATH=build_exp/ori6/libsiftgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/ori6.log 2>&1 || { tail -5 $OUT/ori6.log; exit 1; }
echo "parity ok"
for cfg in base:X=0 ori6:SGPU_LIB_PATH=build_exp/ori6/libsiftgpu.so base2:X=0 ori6b:SGPU_LIB_PATH=build_exp/ori6/libsiftgpu.so; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- python3 tests/probe.py extract --reps 3 > $OUT/$name.log 2>&1 || exit 1
  echo "== $name"; python3 tests/kt_summary.py $OUT/$name/run_kernel_trace.csv "orientation" | head -4
done
