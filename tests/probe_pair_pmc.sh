# SQ counters of the two-level Gaussian kernel (variant 1024) and the per-level kernel.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-include-regex "k_gauss" --output-format csv -d gpurun_out/pmc_pair4 -o run -- python3 tests/ab_variants.py 0 1024 --rounds 2 > gpurun_out/pmc_pair4.log 2>&1; echo pmc rc=$?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_BUSY_CU_CYCLES SQ_INSTS_SMEM --kernel-include-regex "k_gauss" --output-format csv -d gpurun_out/pmc_pair5 -o run -- python3 tests/ab_variants.py 0 1024 --rounds 2 > gpurun_out/pmc_pair5.log 2>&1; echo pmc2 rc=$?
