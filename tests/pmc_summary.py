"""Summarise a tests/profile_kernels.sh run into profiles/<tag>_summary.json (+ copies of the
rocprofv3 kernel stats) -- the kernel-level evidence behind bench.py's roofline.

  python tests/pmc_summary.py <prof dir, e.g. gpurun_out/prof_r01> <tag>

Per bench step (one extract of the batch): the Gaussian family's kernel time from the trace,
and its HBM bytes from FETCH_SIZE + WRITE_SIZE (kB units -> bytes), raw and corrected.  The
correction (MI355X_MICROARCH.md, HBM section: FETCH_SIZE counts 1/2 of the bytes of a 16-B-per-lane
streaming read) uses the factors measured by tests/pmc_calib.sh on a known byte count at each
access width (profiles/*_pmc_calibration.json), applied to every kernel (factors()).
"""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _one(pattern):
    f = sorted(glob.glob(pattern, recursive=True))
    if not f:
        raise SystemExit(f"missing {pattern}")
    return f[0]


def family(name):
    base = name.replace("void ", "").replace("sgk::(anonymous namespace)::", "")
    return base.split("(")[0].split("<")[0]


def calibration():
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_calibration.json")))
    if not files:
        return None, None
    return json.load(open(files[-1]))["factor"], os.path.basename(files[-1])


def factors(name, cal):
    """(read factor, write factor) of a kernel from the calibration record.  The record measured
    FETCH_SIZE at 1/2 of the bytes for 4-, 8- and 16-byte-per-lane reads alike (and WRITE_SIZE
    exact), so the read factor of the kernel's access width applies to every kernel: the level
    kernels' 16-B (f32) or 4-B (u8 level 0) rows, the extremum kernel's 8-B row pairs, the
    feature kernels' 4- and 16-B gathers (round 3 corrected only the k_gauss family and left
    the other kernels at half their read bytes)."""
    if cal is None:
        return 1.0, 1.0
    u8 = re.search(r"k_gauss_(wave|lean)<\s*\d+\s*,\s*true", name) is not None
    if u8:
        r = cal.get("read4")
    elif "k_extrema" in name:
        r = cal.get("read8")
    else:
        r = cal.get("read16")
    return r or 1.0, cal.get("write8") or 1.0


def main():
    src, tag = sys.argv[1], sys.argv[2]
    cal, cal_src = calibration()
    trace = _one(os.path.join(src, "trace", "**", "*kernel_trace.csv"))
    stats = _one(os.path.join(src, "trace", "**", "*kernel_stats.csv"))
    rows = list(csv.DictReader(open(trace)))
    # one k_expand launch per extract (per batch part: the bench runs one part)
    n_steps = sum(1 for r in rows if "k_expand" in r["Kernel_Name"])
    per_family = defaultdict(lambda: [0.0, 0])
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6   # ms
        f = family(r["Kernel_Name"])
        per_family[f][0] += d
        per_family[f][1] += 1
    gauss = [f for f in per_family if f.startswith("k_gauss")]
    from prof_common import box_name, source_digest
    out = {
        "tag": tag,
        "source_digest": source_digest(),   # bench.py uses the counters only for this tree
        "box": box_name(),
        "gauss_family": gauss,
        "extract_calls": n_steps,
        "ms_per_extract": {f: v[0] / n_steps for f, v in per_family.items() if v[1] >= n_steps},
        "launches_per_extract": {f: v[1] / n_steps for f, v in per_family.items() if v[1] >= n_steps},
    }
    hbm = defaultdict(float)
    for kind, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        pat = os.path.join(src, kind, "**", "*counter_collection.csv")
        files = sorted(glob.glob(pat, recursive=True))
        if not files:
            continue
        acc = defaultdict(float)
        cor = defaultdict(float)
        calls = 0
        for r in csv.DictReader(open(files[0])):
            if r["Counter_Name"] != counter:
                continue
            b = float(r["Counter_Value"]) * 1024.0   # kB -> B
            fr, fw = factors(r["Kernel_Name"], cal)
            acc[family(r["Kernel_Name"])] += b
            cor[family(r["Kernel_Name"])] += b * (fr if kind == "fetch" else fw)
            if "k_expand" in r["Kernel_Name"]:
                calls += 1
        out[f"{kind}_bytes_per_extract"] = {f: v / max(calls, 1) for f, v in acc.items()}
        for f, v in cor.items():
            hbm[f] += v / max(calls, 1)
    if cal is not None:
        out["hbm_bytes_per_extract"] = dict(hbm)
        out["calibration"] = cal_src
        out["calibrated_all_kernels"] = True
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    # profiles/ on the GPU box does not come back (gpurun merges gpurun_out/ only): a copy beside
    # the traces, to be moved into profiles/ after the call
    for path in (os.path.join(prof, f"{tag}_summary.json"), os.path.join(src, "summary.json")):
        with open(path, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
