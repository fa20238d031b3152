"""Where do the two-level launches differ from single-level ones? (diagnostic)"""
import sys
sys.path.insert(0, 'tests'); sys.path.insert(0, 'modify-sift-gpu_amd/python')
import numpy as np, sgpu
from sgpu_types import default_options
from sift_synth import synth_image, synth_batch
ctx = sgpu.SiftContext(0)
for (w, h) in ((203, 97), (640, 480), (1920, 1080)):
    img = synth_image(w, h, 2) if w < 1000 else synth_batch(1, w, h, 5)[0]
    res = {}
    for name, fl in (("single", ctx.DEBUG_GAUSS_SINGLE), ("pair", 0)):
        ctx.set_debug_flags(fl)
        ctx.extract(img)
        geo = ctx.geometry()
        res[name] = [[ctx.gaussian(0, o, l).reshape(geo[o][1], geo[o][2]).copy() for l in range(6)] for o in range(len(geo))]
    for o in range(len(res["single"])):
        for l in range(6):
            a, b = res["single"][o][l], res["pair"][o][l]
            d = np.argwhere(a.view(np.uint32) != b.view(np.uint32))
            if len(d):
                print(w, h, "octave", o, "level", l, "diffs", len(d), "rows", np.unique(d[:, 0])[:20], "cols", np.unique(d[:, 1])[:40])
            else:
                print(w, h, "octave", o, "level", l, "same")
