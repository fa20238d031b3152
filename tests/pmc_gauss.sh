#!/bin/bash
# SQ counter passes on the Gaussian level kernels of the 128 x 1080p batch (GPU box):
#   bash tests/pmc_gauss.sh <tag> [debug flags]  -> gpurun_out/pmcg_<tag>/p*/..., table.txt
set -e
TAG=$1
FLAGS=${2:-0}
OUT=gpurun_out/pmcg_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P="tests/probe.py extract --reps 2 --flags $FLAGS"
i=0
for SET in \
  "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS" \
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM" \
  "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE GRBM_COUNT" ; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $SET --output-format csv -d $OUT/p$i -o run -- python3 $P > $OUT/p$i.log 2>&1
done
for f in $OUT/p*/run_counter_collection.csv; do
  python3 tests/pmc_table.py $f "gauss"
done > $OUT/table.txt
