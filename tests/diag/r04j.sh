# Round 4 matcher experiment: workgroups per launch (chunk count) with the pipelined raw kernel,
# alternating C5 timings, plus the kernel trace of m1 and w5000.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for L in m1 w5000 w1900 w2500; do
    echo "$L: $(SGPU_LIB_PATH=build_exp/$L/libsiftgpu.so timeout -k 10 120 python -u tests/diag/match_time.py 50000 plain,rows_only | tr '\n' ' ')" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for L in m1 w5000; do
  SGPU_LIB_PATH=build_exp/$L/libsiftgpu.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r04j_$L -o run -- python3 tests/diag/match_time.py 50000 plain > /dev/null 2>&1 || exit 1
done
