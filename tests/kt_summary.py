"""Median per-kernel durations from a rocprofv3 kernel-trace CSV, grouped by kernel and grid.
Usage: python tests/kt_summary.py <run_kernel_trace.csv> [name-regex]"""
import collections
import csv
import re
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
d = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"]
    if not pat.search(name):
        continue
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    d[(name, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in sorted(d.items(), key=lambda x: -statistics.median(x[1])):
    print(f"{statistics.median(v):9.1f} us  n={len(v):3d}  {k[0]}  grid={k[1]}")
