"""Summarise a tests/profile_kernels.sh run into profiles/<tag>_summary.json (+ copies of the
rocprofv3 kernel stats) -- the kernel-level evidence behind bench.py's roofline.

  python tests/pmc_summary.py <prof dir, e.g. gpurun_out/prof_r01> <tag>

Per bench step (one extract of the batch): the Gaussian family's kernel time from the trace,
and its HBM bytes from FETCH_SIZE + WRITE_SIZE (kB units -> bytes).  The guide's gfx950 note
(FETCH_SIZE = half the bytes of 16-B-per-lane streaming reads) does not apply to these kernels'
4-B-per-lane loads: undoubled FETCH_SIZE already equals the bytes the Gaussian kernels must read
(each input row once plus the strip halo), so no factor is applied.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _one(pattern):
    f = sorted(glob.glob(pattern, recursive=True))
    if not f:
        raise SystemExit(f"missing {pattern}")
    return f[0]


def family(name):
    base = name.replace("void ", "").replace("sgk::(anonymous namespace)::", "")
    return base.split("(")[0].split("<")[0]


def main():
    src, tag = sys.argv[1], sys.argv[2]
    trace = _one(os.path.join(src, "trace", "**", "*kernel_trace.csv"))
    stats = _one(os.path.join(src, "trace", "**", "*kernel_stats.csv"))
    rows = list(csv.DictReader(open(trace)))
    # one k_image_offsets launch per extract (per batch part: the bench runs one part)
    n_steps = sum(1 for r in rows if "k_image_offsets" in r["Kernel_Name"])
    per_family = defaultdict(lambda: [0.0, 0])
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6   # ms
        f = family(r["Kernel_Name"])
        per_family[f][0] += d
        per_family[f][1] += 1
    gauss = [f for f in per_family if f.startswith("k_gauss")]
    out = {
        "tag": tag,
        "gauss_family": gauss,
        "extract_calls": n_steps,
        "ms_per_extract": {f: v[0] / n_steps for f, v in per_family.items() if v[1] >= n_steps},
        "launches_per_extract": {f: v[1] / n_steps for f, v in per_family.items() if v[1] >= n_steps},
    }
    for kind, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        pat = os.path.join(src, kind, "**", "*counter_collection.csv")
        files = sorted(glob.glob(pat, recursive=True))
        if not files:
            continue
        acc = defaultdict(float)
        calls = 0
        for r in csv.DictReader(open(files[0])):
            if r["Counter_Name"] != counter:
                continue
            acc[family(r["Kernel_Name"])] += float(r["Counter_Value"]) * 1024.0   # kB -> B
            if "k_image_offsets" in r["Kernel_Name"]:
                calls += 1
        out[f"{kind}_bytes_per_extract"] = {f: v / max(calls, 1) for f, v in acc.items()}
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    with open(os.path.join(prof, f"{tag}_summary.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
