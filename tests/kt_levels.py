"""Median duration of each Gaussian launch position within an extract (rocprofv3 kernel trace):
  python tests/kt_levels.py <run_kernel_trace.csv> [ignored launch count, kept for old scripts]
An extract's pyramid is the run of k_gauss launches before its extremum launch; launch k of an
extract is (octave, level) in the pyramid's launch order.  Extracts with the most common launch
count are kept (the probe's smaller warm-up shapes drop out)."""
import csv
import statistics
import sys
from collections import Counter

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
runs, cur = [], []
for r in rows:
    n = r["Kernel_Name"]
    if "k_gauss" in n:
        cur.append(r)
    elif "k_extrema" in n and cur:
        runs.append(cur)
        cur = []
per = Counter(len(x) for x in runs).most_common(1)[0][0]
runs = [x for x in runs if len(x) == per]
tot = 0.0
for k in range(per):
    m = statistics.median((int(x[k]["End_Timestamp"]) - int(x[k]["Start_Timestamp"])) / 1000 for x in runs)
    tot += m
    name = runs[0][k]["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    print(f"{k:2d} {m:8.1f} us  {name}")
print(f"sum {tot:.1f} us over {len(runs)} extracts")
