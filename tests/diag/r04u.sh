# Round 4: single-image extremum segments of >= 8 rows instead of 16 (e8) against the shipped
# lib: C2 alternating, then the extremum parity tests on e8
set -o pipefail
for r in 1 2 3; do
  for L in lib e8; do
    D=build_exp/$L; [ $L = lib ] && D=modify-sift-gpu_amd/lib
    echo "$L c2 $(LD_LIBRARY_PATH=$D timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'.'); import bench; r=bench.bench_c2(cpu=False); print(r['runs_ms_per_image'], round(r['timing_ms']['detection'], 4))")" || exit 1
  done
done
SGPU_LIB_PATH=build_exp/e8/libsiftgpu.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 250 --timeout-method thread > gpurun_out/r04u_t.log 2>&1; echo "e8 parity rc=$?"; tail -1 gpurun_out/r04u_t.log
