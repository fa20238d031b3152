# Round 5: k_descriptor_flat with 64-bit fixed-point LDS sums: descriptor parity, then its kernel
# time per 128 x 1080p extract against the dual-cell kernel (GPU box).
set -o pipefail
OUT=gpurun_out/r05m
mkdir -p $OUT
export TMPDIR=/tmp
SGPU_LIB_PATH=build_exp/fw8/libsiftgpu.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py -x -q --timeout 200 --timeout-method thread -s -k "descriptor or c3 or golden or c4" > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "descriptor L2|passed|failed|Error" $OUT/pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
for cfg in flat:X=0 fw8:SGPU_LIB_PATH=build_exp/fw8/libsiftgpu.so flat2:X=0 fw8b:SGPU_LIB_PATH=build_exp/fw8/libsiftgpu.so; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- python3 tests/probe.py extract --reps 3 > $OUT/$name.log 2>&1 || exit 1
  echo "== $name"; python3 tests/kt_summary.py $OUT/$name/run_kernel_trace.csv descriptor | head -2
done
