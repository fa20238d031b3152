# SQ counters of the extraction kernels (descriptor, orientation, extremum, Gaussian) on the box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex "k_descriptor|k_orientation|k_extrema_wave|k_gauss_pk2" --output-format csv -d gpurun_out/pmc_stages -o run -- python3 tests/ab_variants.py 0 --rounds 2 > gpurun_out/pmc_stages.log 2>&1; echo pmc rc=$?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD TA_BUSY_avr TD_BUSY_avr --kernel-include-regex "k_descriptor|k_orientation|k_extrema_wave" --output-format csv -d gpurun_out/pmc_stages2 -o run -- python3 tests/ab_variants.py 0 --rounds 2 > gpurun_out/pmc_stages2.log 2>&1; echo pmc2 rc=$?
