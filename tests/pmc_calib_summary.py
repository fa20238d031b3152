"""profiles/<tag>_pmc_calibration.json from a tests/pmc_calib.sh run: for each access width,
the known bytes (1 GiB) over the counter's bytes -- the factor that turns FETCH_SIZE /
WRITE_SIZE of a kernel with that access pattern into HBM bytes.

  python tests/pmc_calib_summary.py gpurun_out/pmc_calib_<tag> <tag>
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KNOWN = float(1 << 30)


def width(name):
    if "k_read" in name or "k_write" in name:
        kind = "read" if "k_read" in name else "write"
        head = name.split("(")[0] if "<" not in name else name.split(">")[0]
        w = 16 if "(4)" in head or "vector(4" in name.split(">")[0] else \
            8 if "(2)" in head or "vector(2" in name.split(">")[0] else 4
        return f"{kind}{w}"
    return None


def main():
    src, tag = sys.argv[1], sys.argv[2]
    out = {"tag": tag, "known_bytes": KNOWN, "counters": {}, "factor": {},
           "note": "factor = known bytes / (counter kB x 1024); multiply a kernel's counter by "
                   "the factor of its access width to get HBM bytes"}
    for kind, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        f = sorted(glob.glob(os.path.join(src, kind, "**", "*counter_collection.csv"), recursive=True))
        if not f:
            continue
        for r in csv.DictReader(open(f[0])):
            if r["Counter_Name"] != counter:
                continue
            k = width(r["Kernel_Name"])
            if k is None:
                continue
            b = float(r["Counter_Value"]) * 1024.0
            out["counters"][f"{counter}:{k}"] = b
            if (kind == "fetch") == k.startswith("read"):
                out["factor"][k] = KNOWN / b if b > 0 else None
    json.dump(out, open(os.path.join(ROOT, "profiles", f"{tag}_pmc_calibration.json"), "w"),
              indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
