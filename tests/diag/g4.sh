# Timing-only: the paired-level kernel's row-pair DMA as 16-B-per-lane loads (build variants x4a,
# x4m: wrong levels) against the shipped dword DMAs; kernel stats per variant.  (GPU box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--no-c4 --no-e2e --no-match --no-cpu-baseline --no-c2 --steps 10 --warmup 3"
for cfg in base:X=0 base4:SGPU_DUO_NIN=4 x4a:SGPU_LIB_PATH=build_exp/x4a/libsiftgpu.so,SGPU_DUO_NIN=4 x4m:SGPU_LIB_PATH=build_exp/x4m/libsiftgpu.so; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env ${envs//,/ } timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g4_$name -o run -- python3 bench.py $B > gpurun_out/g4_$name.log 2>&1 || exit 1
done
ls gpurun_out/g4_base
