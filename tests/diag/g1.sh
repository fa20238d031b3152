# Three-level kernel: parity tests, then alternating bench runs against the paired-level
# schedule and two build variants, then a kernel trace of the trio schedule.  (GPU box)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gauss.py -x -q --timeout 300 --timeout-method thread -k "trio or duo" > gpurun_out/t_trio.log 2>&1; rc=$?; tail -3 gpurun_out/t_trio.log; [ $rc -eq 0 ] || exit $rc
bash tests/diag/ab_env.sh 2 "off:SGPU_TRIO=off" "trio:SGPU_TRIO=on" "w2:SGPU_LIB_PATH=build_exp/trio_w2/libsiftgpu.so" "n5:SGPU_LIB_PATH=build_exp/trio_n5/libsiftgpu.so" "tw1:SGPU_TRIO_WAVES=2560" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trio -o run -- python3 bench.py --no-c4 --no-e2e --no-match --no-cpu-baseline --no-c2 --steps 10 --warmup 3 > gpurun_out/prof_trio.log 2>&1 || exit 1
find gpurun_out/prof_trio -name "*kernel_stats.csv"
