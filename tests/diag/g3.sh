# C4 (16 x 4096^2, -no 6) kernel traces under both octave pair plans.  (GPU box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for plan in front end; do
  SGPU_DUO_PLAN=$plan timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_c4_$plan -o run -- python3 bench.py --workload c4 --no-c4 --no-e2e --no-match --no-cpu-baseline --no-c2 --steps 5 --warmup 2 > gpurun_out/prof_c4_$plan.log 2>&1 || exit 1
done
ls gpurun_out/prof_c4_front gpurun_out/prof_c4_end
