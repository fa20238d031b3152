#!/bin/bash
# Counter passes on the descriptor (and the other feature kernels) of the 128 x 1080p batch
# (GPU box):  bash tests/pmc_desc.sh <tag>  -> gpurun_out/pmc_<tag>/p*/..., table.txt
# One pass per hardware block limit (8 SQ, 4 TCP, 2 TA, 2 TD per pass).
set -e
TAG=$1
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P="tests/probe.py extract --reps 2"
i=0
for SET in \
  "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD" \
  "SQ_INSTS_VALU_TRANS_F32 SQ_IFETCH SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INSTS_SALU" \
  "TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_REQUEST TCP_PENDING_STALL_CYCLES TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL" \
  "TCP_TCC_READ_REQ TCP_TOTAL_CACHE_ACCESSES TCP_TCP_LATENCY TCP_TCC_READ_REQ_LATENCY GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $SET --output-format csv -d $OUT/p$i -o run -- python3 $P > $OUT/p$i.log 2>&1
done
for f in $OUT/p*/run_counter_collection.csv; do
  python3 tests/pmc_table.py $f "descriptor|orientation|extrema"
done > $OUT/table.txt
