# Round 5: per-launch kernel times of the pyramid with the paired-level kernel on / off, and SQ
# counters of the duo launches (GPU box).
set -o pipefail
mkdir -p gpurun_out/r05b
export TMPDIR=/tmp
for cfg in on:0 off:32768; do
  name=${cfg%%:*}; fl=${cfg##*:}
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05b/kt_$name -o run \
    -- python3 tests/probe.py extract --reps 4 --flags $fl > gpurun_out/r05b/kt_$name.log 2>&1 || exit 1
done
for name in on off; do
  echo "== $name"; python3 tests/kt_levels.py gpurun_out/r05b/kt_$name/run_kernel_trace.csv 15
done
bash tests/pmc_gauss.sh r05b 0 && cat gpurun_out/pmcg_r05b/table.txt | grep duo
