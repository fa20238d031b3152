# Round 4: XCD-aware extremum wave order -- keypoint parity, FETCH_SIZE of k_extrema_wave2 for the
# shipped build and the linear order (build_exp/ext_lin), alternating A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -k "candidates or golden_extract or full_hd" > gpurun_out/pytest_g.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_g.log
[ $rc -eq 0 ] || exit $rc
for L in main ext_lin; do
  if [ $L = main ]; then unset SGPU_LIB_PATH; else export SGPU_LIB_PATH=build_exp/$L/libsiftgpu.so; fi
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fetch_g_$L -o run -- python3 tests/probe.py extract --reps 2 > gpurun_out/fetch_g_$L.log 2>&1 || exit 1
  python3 tests/pmc_table.py gpurun_out/fetch_g_$L/run_counter_collection.csv "extrema" | sed "s/^/$L: /"
done
unset SGPU_LIB_PATH
timeout -k 10 300 bash tests/diag/ab_bench.sh build_exp/ext_lin/libsiftgpu.so 3
