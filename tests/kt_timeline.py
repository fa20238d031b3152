"""Timeline of the Gaussian launches of the last extract in a rocprofv3 kernel trace (start and
end relative to the first launch, microseconds), to see which launches overlap:
  python tests/kt_timeline.py <run_kernel_trace.csv> [launches_per_extract=21]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
per = int(sys.argv[2]) if len(sys.argv) > 2 else 21
g = [r for r in rows if "k_gauss" in r["Kernel_Name"]][-per:]
t0 = int(g[0]["Start_Timestamp"])
end = max(int(r["End_Timestamp"]) for r in g)
for r in g:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{s / 1000:8.1f} {e / 1000:8.1f} {(e - s) / 1000:7.1f}  {name}  grid={r.get('Grid_Size', '')}")
print(f"span {(end - t0) / 1000:.1f} us")
