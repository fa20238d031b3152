"""Quick GPU-vs-oracle diagnostic (run on the GPU box): prints where the HIP path and the oracle
first differ, stage by stage.  Not a test; tests/test_gpu_parity.py holds the asserts."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "modify-sift-gpu_amd", "python"))

import numpy as np  # noqa: E402

import oracle_py as O  # noqa: E402
import sgpu  # noqa: E402
from sgpu_types import default_options  # noqa: E402
from sift_synth import synth_image, synth_descriptors, quantize  # noqa: E402


def main():
    w, h = (640, 480) if len(sys.argv) < 2 else map(int, sys.argv[1].split("x"))
    img = synth_image(w, h, 1000)
    opts = default_options()
    ctx = sgpu.SiftContext(0, opts)
    t = time.time()
    ctx.extract(img)
    print("extract", time.time() - t, "count", ctx.count(0), ctx.timing(), flush=True)
    geo = ctx.geometry()
    print("geometry", geo)
    for o in range(len(geo)):
        for k in range(6):
            g = ctx.gaussian(0, o, k)
            r = O.gaussian(img, o, k, opts)
            nd = int(np.sum(g.view(np.uint32) != r.view(np.uint32)))
            if nd:
                print(f"gauss o{o} k{k}: {nd} diffs, max abs {np.max(np.abs(g - r))}", flush=True)
    print("gaussian compared", flush=True)
    gi, gf = ctx.candidates()
    ri, rf = O.candidates(img, opts)
    print("candidates gpu", gi.shape, "oracle", ri.shape)
    n = min(len(gi), len(ri))
    same = np.all(gi[:n, :3] == ri[:n, :3], axis=1)
    if not same.all() or len(gi) != len(ri):
        bad = np.where(~same)[0]
        print("first candidate mismatch", bad[:5], gi[bad[:5]] if len(bad) else None,
              ri[bad[:5]] if len(bad) else None)
    else:
        fd = np.sum(gf[:n, :3].view(np.uint32) != rf[:n, :3].view(np.uint32))
        print("candidate positions identical; dx/dy/ds bit diffs:", int(fd))
    k, d = ctx.features(0)
    rk, rd = O.extract(img, opts)
    print("features gpu", k.shape, "oracle", rk.shape)
    if k.shape == rk.shape:
        kd = np.sum(k.view(np.uint32) != rk.view(np.uint32), axis=0)
        print("key bit diffs per column", kd)
        l2 = np.linalg.norm(d - rd, axis=1)
        print("descriptor L2 max", l2.max(), "bitwise equal rows", int(np.sum(np.all(d == rd, axis=1))))
    # matcher
    d1 = synth_descriptors(3000, 5000)
    d2 = synth_descriptors(2500, 5001, base=d1, n_dup=1000)
    q1, q2 = quantize(d1), quantize(d2)
    t = time.time()
    m = ctx.match(q1, q2)
    print("match gpu", m.shape, time.time() - t)
    rm = O.match(q1, q2)
    print("match oracle", rm.shape, "equal", m.shape == rm.shape and bool(np.all(m == rm)))
    # 1080p timing
    img2 = np.stack([synth_image(1920, 1080, 2000 + i) for i in range(4)])
    opts4 = default_options(octave_num=4)
    ctx.set_options(opts4)
    for it in range(3):
        t = time.time()
        ctx.extract(img2)
        print("1080p x4", time.time() - t, ctx.total(), ctx.timing(), flush=True)


if __name__ == "__main__":
    main()
