"""Per-kernel means of rocprofv3 counter-collection CSVs (one row per kernel name and grid).
Usage: python tests/pmc_table.py <run_counter_collection.csv> [name-regex]"""
import collections
import csv
import re
import sys

pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"]
    if not pat.search(name):
        continue
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    key = (name, r.get("Grid_Size", r.get("Grid_Size_X")))
    agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[key].add(r["Dispatch_Id"])
for key, v in sorted(agg.items()):
    n = len(disp[key])
    print(f"{key[0]} grid={key[1]} n={n}: " + " ".join(f"{c}={v[c] / n:.4g}" for c in sorted(v)))
