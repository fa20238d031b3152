"""SQ counters of the matcher from tests/pmc_match.sh (two counter passes + a kernel trace),
per kernel averaged over its dispatches, and the MFMA-busy fraction of one match call
(GPU-box output -> profiles/<tag>_match_sq_counters.json):
  python tests/pmc_match_summary.py <pmc dir> <out.json> [clock GHz = 2.4]

mfma_busy_frac = sum over the call's kernels of SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over
the SIMDs; MI355X_MICROARCH.md: 32 x N for a 32x32x16 MFMA) / (the kernels' summed duration x
clock x 1,024 SIMDs) -- the share of the matrix pipes' cycles spent in MFMAs while the call's
kernels run; at the peak clock it is a lower bound when the clock runs below 2.4 GHz.  Beside it
the operation count's share of the dense i8 peak over the same kernel time."""
import csv
import glob
import json
import statistics
import sys
from collections import defaultdict

src, out = sys.argv[1], sys.argv[2]
clock = float(sys.argv[3]) * 1e9 if len(sys.argv) > 3 else 2.4e9


def short(n):
    return n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]


acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))   # kernel -> counter -> dispatch
for p in ("p1", "p2"):
    for r in csv.DictReader(open(glob.glob(f"{src}/{p}/**/*counter_collection.csv", recursive=True)[0])):
        if "k_match" not in r["Kernel_Name"] and "k_prep" not in r["Kernel_Name"]:
            continue
        acc[short(r["Kernel_Name"])][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
kt = list(csv.DictReader(open(glob.glob(f"{src}/kt/**/*kernel_trace.csv", recursive=True)[0])))
dur = defaultdict(list)
for r in kt:
    n = short(r["Kernel_Name"])
    if n in acc:
        dur[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
calls = 11   # match_time.py: one warm-up + 10 timed calls of the path
per_kernel = {}
busy = 0.0
t_sum = 0.0
mfma = 0.0
for k, cnt in acc.items():
    c = {name: sum(v.values()) / len(v) for name, v in cnt.items()}
    n_disp = len(next(iter(cnt.values())))
    per_call = n_disp / calls
    # the kernel's time per call: all its dispatches (e.g. k_match_raw's row and column sides)
    # over the calls of the trace run
    d = sum(dur[k]) / calls / per_call if dur.get(k) else None
    per_kernel[k] = {"dispatches_per_call": per_call, "mean_duration_ms": d * 1e3 if d else None,
                     "median_duration_ms": statistics.median(dur[k]) * 1e3 if dur.get(k) else None,
                     "counters_per_dispatch": c}
    if c.get("SQ_INSTS_MFMA"):
        per_kernel[k]["valu_insts_per_mfma"] = c.get("SQ_INSTS_VALU", 0) / c["SQ_INSTS_MFMA"]
    if c.get("SQ_WAVE_CYCLES"):
        for q in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            per_kernel[k][q.lower().replace("sq_", "") + "_frac_of_wave_cycles"] = c.get(q, 0) / c["SQ_WAVE_CYCLES"]
    if d:
        busy += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) * per_call
        mfma += c.get("SQ_INSTS_MFMA", 0) * per_call
        t_sum += d * per_call
res = {"command": "bash tests/pmc_match.sh (rocprofv3 --pmc, two passes, + a kernel trace, over "
                  "tests/diag/match_time.py 50000 <path>)",
       "path": "plain mutual matching (shipped C5 path: row side + matched columns' side)",
       "dense_i8_ops_per_call": 2.0 * 128 * 50000 * 50000,
       "clock_GHz_assumed": clock / 1e9, "simds": 1024,
       "kernels": per_kernel,
       "per_call": {"kernel_ms": t_sum * 1e3, "mfma_busy_cycles": busy, "mfma_insts": mfma,
                    "mfma_busy_frac": busy / (t_sum * clock * 1024) if t_sum else None,
                    "dense_i8_frac_of_5POPS": 2.0 * 128 * 50000 * 50000 / t_sum / 5e15 if t_sum else None}}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res["per_call"]))
