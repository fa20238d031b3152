"""In-process A/B timing of kernel variants (sgpu_debug_set_variant), interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Usage: python tests/ab_variants.py v0 v1 ... [--batch B]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "modify-sift-gpu_amd", "python"))
import numpy as np  # noqa: E402

import sgpu  # noqa: E402
from sgpu_types import default_options  # noqa: E402
from sift_synth import synth_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", type=int, nargs="+")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--no-check", action="store_true", help="timing probes that change results")
    args = ap.parse_args()
    imgs = synth_batch(args.batch, 1920, 1080, 3000, unique=16)
    ctx = sgpu.SiftContext(0, default_options(octave_num=4))
    ctx.stage(imgs)
    res = {v: [] for v in args.variants}
    ref_total = None
    for r in range(args.rounds):
        for v in args.variants:
            sgpu.lib().sgpu_debug_set_variant(v)
            ctx.extract_staged()
            t = ctx.timing()
            if r > 0:
                res[v].append(t)
            tot = ctx.total()
            ref_total = tot if ref_total is None else ref_total
            assert args.no_check or tot == ref_total, (v, tot, ref_total)
    sgpu.lib().sgpu_debug_set_variant(0)
    for v in args.variants:
        keys = res[v][0].keys()
        med = {k: float(np.median([t[k] for t in res[v]])) for k in keys}
        print(f"variant {v}: " + " ".join(f"{k}={med[k]:.3f}" for k in
                                           ["pyramid", "detect", "orientation", "descriptor", "total"]))


if __name__ == "__main__":
    main()
