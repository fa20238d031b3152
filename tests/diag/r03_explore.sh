# Round-3 exploration on the GPU box: lean Gaussian + wave orientation parity, then A/B timings.
set -o pipefail
mkdir -p gpurun_out
echo "== pair kernel determinism (1080p, octave 0 level 5)"
timeout -k 10 120 python tests/diag/pair_diff2.py > gpurun_out/pair_diff2.log 2>&1 || exit 1
sed -n 1p gpurun_out/pair_diff2.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_gauss.py tests/test_gpu_parity.py -k "gauss or levels or golden or first_octave or orientation_wave or compacts" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_lean.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_lean.log
[ $rc -eq 0 ] || exit $rc
echo "== gauss A/B (single levels vs pairs)"
timeout -k 10 600 bash tests/diag/ab_env.sh "SGPU_GAUSS=lean" "SGPU_GAUSS=pair" 3 || exit 1
echo "== c2"
timeout -k 10 100 python -c "import bench, json; print(json.dumps(bench.bench_c2(cpu=False)))"
echo "== kernel trace (pairs)"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pair -o run -- python3 bench.py --no-c4 --no-e2e --no-match --no-cpu-baseline --no-c2 > gpurun_out/prof_pair.log 2>&1 || exit 1
python3 tests/kt_levels.py gpurun_out/prof_pair/run_kernel_trace.csv 12
echo "== matcher parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py -k "match or c5" -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_match.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_match.log
[ $rc -eq 0 ] || exit $rc
echo "== matcher A/B: A = tile-max fold (152 VGPR), B = round 2"
timeout -k 10 400 bash tests/diag/ab_match.sh build_exp/match_r2/libsiftgpu.so 2 || exit 1
echo "== matcher A/B: A = tile-max fold, B = capped at 4 waves/SIMD"
timeout -k 10 400 bash tests/diag/ab_match.sh build_exp/match_wpe4/libsiftgpu.so 2 || exit 1
