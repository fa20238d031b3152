#!/bin/bash
set -e
OUT=gpurun_out/pmc1
mkdir -p $OUT
export TMPDIR=/tmp
A="--steps 1 --warmup 0 --no-cpu-baseline --no-match"
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES --output-format csv -d $OUT/a -o run -- python3 bench.py $A > $OUT/a.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/b -o run -- python3 bench.py $A > $OUT/b.log 2>&1
ls $OUT/a $OUT/b
