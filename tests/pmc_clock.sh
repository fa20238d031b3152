#!/bin/bash
# Effective clock per kernel (GRBM_GUI_ACTIVE / 8 / duration) from one counter pass with the
# kernel trace (GPU box):  bash tests/pmc_clock.sh <tag>
set -e
TAG=$1
OUT=gpurun_out/clk_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT -o run -- python3 tests/probe.py extract --reps 2 > $OUT/run.log 2>&1
python3 - "$OUT" > $OUT/clock.txt <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
cc = list(csv.DictReader(open(glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0])))
kt = list(csv.DictReader(open(glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0])))
dur = {r["Dispatch_Id"]: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in kt}
agg = collections.defaultdict(lambda: [0.0, 0.0, 0])
for r in cc:
    if r["Counter_Name"] != "GRBM_GUI_ACTIVE" or r["Dispatch_Id"] not in dur:
        continue
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    a = agg[name]
    a[0] += float(r["Counter_Value"]) / 8.0
    a[1] += dur[r["Dispatch_Id"]]
    a[2] += 1
for k, (cyc, ns, n) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{k:60s} n={n:3d} ms={ns / n * 1e-6:8.3f} GHz={cyc / ns:6.3f}")
PY
