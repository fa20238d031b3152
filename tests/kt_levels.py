"""Median duration of each Gaussian launch position within an extract (rocprofv3 kernel trace):
  python tests/kt_levels.py <run_kernel_trace.csv> [launches_per_extract=21] [octave sizes...]
Launch k of an extract is (octave, level) in the pyramid's launch order."""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
per = int(sys.argv[2]) if len(sys.argv) > 2 else 21
g = [r for r in rows if "k_gauss" in r["Kernel_Name"]]
g = g[len(g) % per:]
pos = [[] for _ in range(per)]
for i, r in enumerate(g):
    pos[i % per].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
names = [g[i]["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
         for i in range(per)]
tot = 0.0
for k in range(per):
    m = statistics.median(pos[k])
    tot += m
    print(f"{k:2d} {m:8.1f} us  {names[k]}")
print(f"sum {tot:.1f} us over {len(g) // per} extracts")
