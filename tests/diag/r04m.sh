# Round 4: descriptor forms that give a batch the single image's descriptors bit for bit --
# split1 (one wave walks the pair's two row groups in turn), d2w (two waves per feature always,
# 128-thread workgroups) -- and c2w (128-thread pairs for few features only): the batch-vs-single
# test per build, batch stage times, C2 per image.
set -o pipefail
mkdir -p gpurun_out
for L in split1 d2w; do
  SGPU_LIB_PATH=build_exp/$L/libsiftgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_workloads.py -m gpu -q -x \
    -k "c3_shard_128_full_hd" --timeout 250 --timeout-method thread > gpurun_out/r04m_t_$L.log 2>&1; echo "$L test rc=$?"; tail -1 gpurun_out/r04m_t_$L.log
done
H="--no-c4 --no-e2e --no-match --no-cpu-baseline --no-c2 --steps 10 --warmup 3"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], round(d['value']), {k: round(v, 3) for k, v in s.items() if v > 0.05})" "$1" "$2"; }
for r in 1 2; do
  for L in ${LIBS:-lib split1 d2w}; do
    P=build_exp/$L/libsiftgpu.so; [ $L = lib ] && P=modify-sift-gpu_amd/lib/libsiftgpu.so
    SGPU_LIB_PATH=$P timeout -k 10 120 python3 bench.py $H > gpurun_out/r04m_$L.json 2>/dev/null || exit 1
    show gpurun_out/r04m_$L.json $L
  done
done
for r in 1 2 3; do
  for L in lib c2w d2w split1; do
    D=build_exp/$L; [ $L = lib ] && D=modify-sift-gpu_amd/lib
    echo "$L c2 $(LD_LIBRARY_PATH=$D timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'.'); import bench; r=bench.bench_c2(cpu=False); print(round(r['ms_per_image'],4), round(r['timing_ms'].get('descriptor', 0), 4))")" || exit 1
  done
done
