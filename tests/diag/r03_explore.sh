# Round-3 exploration on the GPU box: lean Gaussian + wave orientation parity, then A/B timings.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_gauss.py tests/test_gpu_parity.py -k "gauss or levels or golden or first_octave or orientation_wave or compacts" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_lean.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_lean.log
[ $rc -eq 0 ] || exit $rc
echo "== gauss A/B (wave vs lean)"
timeout -k 10 400 bash tests/diag/ab_env.sh "SGPU_GAUSS=wave" "SGPU_GAUSS=lean" 3 || exit 1
for v in desc_r2 desc_r1; do
  echo "== descriptor variant $v: parity"
  SGPU_LIB_PATH=build_exp/$v/libsiftgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "shipped_descriptor or golden_extract or keypoints_vs_oracle" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1; rc=$?
  tail -2 gpurun_out/pytest_$v.log
  [ $rc -eq 0 ] || exit $rc
  echo "== descriptor variant $v: A/B"
  timeout -k 10 300 bash tests/diag/ab_bench.sh build_exp/$v/libsiftgpu.so 2 || exit 1
done
echo "== c2"
timeout -k 10 100 python -c "import bench, json; print(json.dumps(bench.bench_c2(cpu=False)))"
