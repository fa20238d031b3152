# Round 5: the pixel-parallel descriptor (k_descriptor_flat): parity + workload tests, then the
# descriptor kernel per extract against the dual-cell kernel (SGPU_DESC=dual), alternating (GPU box).
set -o pipefail
OUT=gpurun_out/r05k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py -x -q --timeout 200 --timeout-method thread -s -k "descriptor or c3 or golden or c4" > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "descriptor L2|passed|failed" $OUT/pytest.log | tail -6
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for cfg in flat:X=0 dual:SGPU_DESC=dual; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env $envs timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name$i -o run -- python3 tests/probe.py extract --reps 3 > $OUT/$name$i.log 2>&1 || exit 1
    echo "== $name$i"; python3 tests/kt_summary.py $OUT/$name$i/run_kernel_trace.csv descriptor | head -3
  done
done
