# Round 4: diagonal pyramid schedule (octave o+1's levels 1, 2 in the launches of octave o's
# levels 4, 5) -- bitwise pyramid / keypoint tests, A/B against SGPU_PYR=serial, per-launch trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gauss.py tests/test_gpu_parity.py tests/test_gpu_workloads.py -m gpu -q --timeout 200 --timeout-method thread -k "levels or golden_extract or first_octave or candidates or streams or c4 or shard" > gpurun_out/pytest_f.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_f.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_f.log | head; exit $rc; }
timeout -k 10 400 bash tests/diag/ab_env.sh "SGPU_PYR=x" "SGPU_PYR=serial" 3 && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_f -o run -- python3 bench.py --no-c4 --no-e2e --no-match --no-cpu-baseline --no-c2 --steps 5 --warmup 2 > gpurun_out/kt_f.log 2>&1 && \
python3 tests/kt_levels.py $(ls gpurun_out/kt_f/*/run_kernel_trace.csv gpurun_out/kt_f/run_kernel_trace.csv 2>/dev/null | head -1) 15
