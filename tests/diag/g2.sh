# Octave pairs from the end ((13, 11) u8, (13, 17) decimating its second level, (21, 25)): parity
# tests, the full-size workloads, alternating bench runs (with C4) against the front pairs and the
# 32-bit descriptor sums, a kernel trace.  (GPU box)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_gauss.py -x -q --timeout 300 --timeout-method thread -k "trio or duo or streams" > gpurun_out/t_g2.log 2>&1; rc=$?; tail -3 gpurun_out/t_g2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_workloads.py -x -q --timeout 600 --timeout-method thread > gpurun_out/t_g2w.log 2>&1; rc=$?; tail -3 gpurun_out/t_g2w.log; [ $rc -eq 0 ] || exit $rc
AB_C4=" " bash tests/diag/ab_env.sh 2 "end:SGPU_DUO_PLAN=end" "front:SGPU_DUO_PLAN=front" "u32:SGPU_LIB_PATH=build_exp/u32/libsiftgpu.so" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g2 -o run -- python3 bench.py --no-e2e --no-match --no-cpu-baseline --no-c2 --no-c4 --steps 10 --warmup 3 > gpurun_out/prof_g2.log 2>&1 || exit 1
find gpurun_out/prof_g2 -name "*kernel_stats.csv"
