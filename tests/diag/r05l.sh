# Round 5: k_descriptor_flat histogram copies (8 shipped, 16, 32; fna = plain stores, timing only)
# against the dual-cell kernel: descriptor kernel time per 128 x 1080p extract (GPU box).
set -o pipefail
OUT=gpurun_out/r05l
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in fi32:SGPU_LIB_PATH=build_exp/fi32/libsiftgpu.so fi64:SGPU_LIB_PATH=build_exp/fi64/libsiftgpu.so fc1:SGPU_LIB_PATH=build_exp/fc1/libsiftgpu.so; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- python3 tests/probe.py extract --reps 3 > $OUT/$name.log 2>&1 || exit 1
  echo "== $name"; python3 tests/kt_summary.py $OUT/$name/run_kernel_trace.csv descriptor | head -2
done
