# Descriptor lane-layout A/B on the GPU box: parity of the experiment builds
# (SGK_DESC_RSTEP 1 / 2 against the shipped 4), alternating bench processes, TCP/TA counters.
#   bash tests/diag/r03_desc.sh
set -o pipefail
mkdir -p gpurun_out
for V in desc_flat desc_r1; do
  echo "== parity $V"
  SGPU_LIB_PATH=build_exp/$V/libsiftgpu.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
      -k "shipped_descriptor or golden or keypoints" -x -q --timeout 200 --timeout-method thread \
      > gpurun_out/pytest_$V.log 2>&1; rc=$?
  tail -2 gpurun_out/pytest_$V.log
  [ $rc -eq 0 ] || exit $rc
done
for V in desc_flat desc_r1; do
  echo "== A = shipped (RSTEP 4), B = $V"
  timeout -k 10 300 bash tests/diag/ab_bench.sh build_exp/$V/libsiftgpu.so 2 || exit 1
done
export TMPDIR=/tmp
for V in shipped desc_flat desc_r1; do
  [ $V = shipped ] && unset SGPU_LIB_PATH || export SGPU_LIB_PATH=build_exp/$V/libsiftgpu.so
  O=gpurun_out/pmc_desc_$V; mkdir -p $O
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d $O/p1 -o run -- python3 tests/probe.py extract --reps 2 > $O/p1.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES --output-format csv -d $O/p2 -o run -- python3 tests/probe.py extract --reps 2 > $O/p2.log 2>&1 || exit 1
  for f in $O/p*/run_counter_collection.csv; do python3 tests/pmc_table.py $f "descriptor"; done > $O/table.txt
  echo "== counters $V"; cat $O/table.txt
done
