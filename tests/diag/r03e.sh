# Descriptor LDS-histogram variant (SGK_DESC_LDSBIN=1) on the GPU box: parity, alternating bench
# A/B against the shipped build, SQ counters.
set -o pipefail
mkdir -p gpurun_out
V=${1:-desc_lds}
export SGPU_LIB_PATH=build_exp/$V/libsiftgpu.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -k "descriptor or golden or keypoints or save_sift" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$V.log 2>&1; rc=$?
echo "parity $V rc=$rc"; tail -2 gpurun_out/pytest_$V.log
[ $rc -eq 0 ] || exit $rc
unset SGPU_LIB_PATH
echo "== A = shipped, B = $V"
timeout -k 10 400 bash tests/diag/ab_bench.sh build_exp/$V/libsiftgpu.so 3 || exit 1
export TMPDIR=/tmp
for W in shipped $V; do
  [ $W = shipped ] && unset SGPU_LIB_PATH || export SGPU_LIB_PATH=build_exp/$W/libsiftgpu.so
  O=gpurun_out/pmc_desc_$W; mkdir -p $O
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 --output-format csv -d $O/p3 -o run -- python3 tests/probe.py extract --reps 2 > $O/p3.log 2>&1 || exit 1
  python3 tests/pmc_table.py $O/p3/run_counter_collection.csv "descriptor"
done
