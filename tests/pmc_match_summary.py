"""SQ counters of the matcher's row kernel from tests/pmc_match.sh's two passes, averaged over
the dispatches, with the derived ratios (GPU-box output -> profiles/<tag>_match_sq_counters.json):
  python tests/pmc_match_summary.py <pmc dir> <kernel substring> <out.json>"""
import csv
import json
import sys
from collections import defaultdict

src, kern, out = sys.argv[1], sys.argv[2], sys.argv[3]
acc = defaultdict(lambda: defaultdict(float))   # counter -> dispatch -> value
name = None
for p in ("p1", "p2"):
    for r in csv.DictReader(open(f"{src}/{p}/run_counter_collection.csv")):
        if kern not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].split("(")[0]
        acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
c = {k: sum(v.values()) / len(v) for k, v in acc.items()}
d = {}
if c.get("SQ_INSTS_MFMA"):
    d["valu_insts_per_mfma"] = c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"]
    d["lds_insts_per_mfma"] = c["SQ_INSTS_LDS"] / c["SQ_INSTS_MFMA"]
if c.get("SQ_WAVE_CYCLES"):
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        d[k.lower().replace("sq_", "") + "_frac_of_wave_cycles"] = c[k] / c["SQ_WAVE_CYCLES"]
json.dump({"kernel": name, "dispatches": len(next(iter(acc.values()))) if acc else 0,
           "command": "bash tests/pmc_match.sh (rocprofv3 --pmc, two passes over "
                      "tests/diag/match_time.py 50000 rows_only)",
           "counters": c, "derived": d}, open(out, "w"), indent=1)
print(json.dumps(d))
