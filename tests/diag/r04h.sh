# Round 4: C2 path (single-workgroup scans, two waves per feature descriptor) -- parity, the C2
# bench line and its trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -q -s --timeout 200 --timeout-method thread -k "golden_extract or shipped_descriptor or options_vs_oracle or keypoints or speed_replica or rejected or simplesift" > gpurun_out/pytest_h.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_h.log; grep "descriptor L2" gpurun_out/pytest_h.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_h.log | head; exit $rc; }
for i in 1 2 3; do timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'.'); import bench; r=bench.bench_c2(cpu=False); print(round(r['ms_per_image'],4), {k: round(v,4) for k,v in r['timing_ms'].items() if v})"; done
timeout -k 10 300 bash tests/profile_c2.sh r04h > gpurun_out/prof_c2_r04h.log 2>&1 && echo c2 trace ok
