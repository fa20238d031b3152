# Round 4 matcher experiment: column terms read as v4i slots (m0) and the column-group
# software pipeline (m1) against the previous build (mbase): matcher tests per build, then
# alternating C5 timings.
set -o pipefail
mkdir -p gpurun_out
for L in m0 m1; do
  echo "== tests $L"
  SGPU_LIB_PATH=build_exp/$L/libsiftgpu.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "match" \
    --timeout 120 --timeout-method thread > gpurun_out/r04i_tests_$L.log 2>&1; rc=$?
  tail -3 gpurun_out/r04i_tests_$L.log; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2 3; do
  for L in mbase m0 m1; do
    echo "$L: $(SGPU_LIB_PATH=build_exp/$L/libsiftgpu.so timeout -k 10 120 python -u tests/diag/match_time.py 50000 plain,rows_only | tr '\n' ' ')" || exit 1
  done
done
