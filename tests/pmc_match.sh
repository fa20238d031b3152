# SQ counters of the matcher (C5 50k x 50k), the shipped mutual path ("plain": row side and the
# matched columns' side) or another tests/diag/match_time.py path, two counter passes plus a
# kernel trace for the durations:
#   bash tests/pmc_match.sh <outdir> [path = plain]
set -o pipefail
OUT=${1:-gpurun_out/pmc_match}
PATHNAME=${2:-plain}
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU SQ_WAVES"
timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d "$OUT/p1" -o run -- python3 tests/diag/match_time.py 50000 $PATHNAME > "$OUT/p1.log" 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d "$OUT/p2" -o run -- python3 tests/diag/match_time.py 50000 $PATHNAME > "$OUT/p2.log" 2>&1 && \
timeout -k 10 90 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o run -- python3 tests/diag/match_time.py 50000 $PATHNAME > "$OUT/kt.log" 2>&1
