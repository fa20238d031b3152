# Round 4: do the stage events cost C2 time?  notime = stage events without timing (the
# _timing slots read 0) against the shipped lib, alternating, and the notime C2 trace
set -o pipefail
for r in 1 2 3; do
  for L in lib notime; do
    D=build_exp/$L; [ $L = lib ] && D=modify-sift-gpu_amd/lib
    echo "$L c2 $(LD_LIBRARY_PATH=$D timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'.'); import bench; r=bench.bench_c2(cpu=False); print(round(r['ms_per_image'],4))")" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LD_LIBRARY_PATH=build_exp/notime timeout -k 10 300 bash tests/profile_c2.sh r04r > gpurun_out/prof_c2_r04r.log 2>&1 && echo c2 trace ok
