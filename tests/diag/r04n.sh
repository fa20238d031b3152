# Round 4: the two-wave descriptor splitting the bins (bins: every bin summed as the one-wave
# kernel, which walks unsplit) against the shipped row-group split: batch-vs-single and the
# descriptor parity tests on the bins build, then batch stage times and C2 per image.
set -o pipefail
mkdir -p gpurun_out
SGPU_LIB_PATH=build_exp/bins/libsiftgpu.so timeout -k 10 400 python -u -m pytest tests/test_gpu_workloads.py tests/test_gpu_parity.py -m gpu -q -x -s \
  -k "c3_shard_128_full_hd or shipped_descriptor or golden_extract or keypoints" --timeout 250 --timeout-method thread > gpurun_out/r04n_t.log 2>&1; rc=$?
echo "bins tests rc=$rc"; tail -1 gpurun_out/r04n_t.log; grep "descriptor L2" gpurun_out/r04n_t.log; [ $rc -eq 0 ] || exit $rc
H="--no-c4 --no-e2e --no-match --no-cpu-baseline --no-c2 --steps 10 --warmup 3"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], round(d['value']), {k: round(v, 3) for k, v in s.items() if v > 0.05})" "$1" "$2"; }
for r in 1 2; do
  for L in lib bins; do
    P=build_exp/$L/libsiftgpu.so; [ $L = lib ] && P=modify-sift-gpu_amd/lib/libsiftgpu.so
    SGPU_LIB_PATH=$P timeout -k 10 120 python3 bench.py $H > gpurun_out/r04n_$L.json 2>/dev/null || exit 1
    show gpurun_out/r04n_$L.json $L
  done
done
for r in 1 2 3; do
  for L in lib bins; do
    D=build_exp/$L; [ $L = lib ] && D=modify-sift-gpu_amd/lib
    echo "$L c2 $(LD_LIBRARY_PATH=$D timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'.'); import bench; r=bench.bench_c2(cpu=False); print(round(r['ms_per_image'],4), round(r['timing_ms'].get('descriptor', 0), 4))")" || exit 1
  done
done
