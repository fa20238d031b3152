# The paired-level kernel's 16-B row DMA (SGK_DUO_X4=1, shipped build) against the dword DMA
# (build variant x0): parity, kernel stats, alternating bench pairs.  (GPU box)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_gauss.py -x -q --timeout 300 --timeout-method thread -k "duo or streams or trio" > gpurun_out/t_g5.log 2>&1; rc=$?; tail -3 gpurun_out/t_g5.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
B="--no-c4 --no-e2e --no-match --no-cpu-baseline --no-c2 --steps 10 --warmup 3"
for cfg in x4:X=0 x0:SGPU_LIB_PATH=build_exp/x0/libsiftgpu.so; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env ${envs//,/ } timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g5_$name -o run -- python3 bench.py $B > gpurun_out/g5_$name.log 2>&1 || exit 1
done
AB_C4=" " bash tests/diag/ab_env.sh 2 "x4:X=0" "x0:SGPU_LIB_PATH=build_exp/x0/libsiftgpu.so" || exit 1
