"""Pattern of the pair-kernel difference at 1080p octave 0 level 5 (diagnostic)."""
import os, sys
sys.path.insert(0, 'tests'); sys.path.insert(0, 'modify-sift-gpu_amd/python')
import numpy as np, sgpu
from sift_synth import synth_batch
ctx = sgpu.SiftContext(0)
img = synth_batch(1, 1920, 1080, 5)[0]
out = {}
for name, fl in (("single", 0), ("pair", ctx.DEBUG_GAUSS_PAIR), ("pair2", ctx.DEBUG_GAUSS_PAIR)):
    ctx.set_debug_flags(fl)
    ctx.extract(img)
    w, h, wa = ctx.geometry()[0]
    out[name] = ctx.gaussian(0, 0, 5).reshape(h, wa).copy()
a, b, c = out["single"], out["pair"], out["pair2"]
d = a.view(np.uint32) != b.view(np.uint32)
print(os.environ.get("SGPU_LIB_PATH", "main"), "diffs", d.sum(), "pair vs pair2 diffs", (b.view(np.uint32) != c.view(np.uint32)).sum())
for r in range(0, 48):
    print(f"{r:3d}", "".join("x" if d[r, cc] else "." for cc in range(64, 192)))
idx = np.argwhere(d)[:5]
for r, cc in idx:
    print(r, cc, a[r, cc], b[r, cc])
