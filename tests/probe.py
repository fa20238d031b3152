"""Timing probes for the GPU box (run directly or under rocprofv3):
  python tests/probe.py extract [--batch 128] [--reps 5] [--w 1920 --h 1080 --octaves 4]
  python tests/probe.py match [--n 50000] [--reps 5]
Prints per-call stage times (HIP events inside the library) as one line per repetition."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "modify-sift-gpu_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import sgpu  # noqa: E402
from sgpu_types import default_options  # noqa: E402
from sift_synth import quantize, synth_batch_fast, synth_descriptors, synth_guided_scene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["extract", "match"])
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--octaves", type=int, default=4)
    ap.add_argument("--n", type=int, default=50000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--flags", type=int, default=0, help="sgpu_debug_set_flags")
    a = ap.parse_args()
    ctx = sgpu.SiftContext(0, default_options(octave_num=a.octaves))
    ctx.set_debug_flags(a.flags)
    if a.what == "extract":
        imgs = synth_batch_fast(a.batch, a.w, a.h, 3000)
        ctx.stage(imgs)
        ctx.extract_staged()
        for r in range(a.reps):
            t0 = time.perf_counter()
            ctx.extract_staged()
            wall = (time.perf_counter() - t0) * 1e3
            t = ctx.timing()
            print(f"rep {r}: wall {wall:.3f} ms " + " ".join(f"{k}={v:.3f}" for k, v in t.items()
                                                        if k != "match") +
                  f" features={ctx.total()}", flush=True)
    else:
        d1 = synth_descriptors(a.n, 5000)
        d2 = synth_descriptors(a.n, 5001, base=d1, n_dup=min(20000, a.n // 2))
        q1, q2 = quantize(d1), quantize(d2)
        g1, g2, l1, l2, H, F = synth_guided_scene(a.n, a.n, 5002)
        for name, fn in [("plain", lambda: ctx.match(q1, q2)),
                         ("plain_nombm", lambda: ctx.match(q1, q2, mbm=0)),
                         ("guided", lambda: ctx.match_guided(g1, g2, l1, l2, H, F))]:
            fn()
            ts = []
            for _ in range(a.reps):
                m = fn()
                ts.append(ctx.timing()["match"])
            print(f"{name}: min {min(ts):.3f} ms median {sorted(ts)[len(ts) // 2]:.3f} ms, "
                  f"{len(m)} matches", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
