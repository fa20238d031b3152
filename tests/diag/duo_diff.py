"""Where k_gauss_duo's levels differ from one level per launch (GPU box, diagnosis only):
  python tests/diag/duo_diff.py  -> per case: the first differing level, rows / columns of the
  differences."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "modify-sift-gpu_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import sgpu  # noqa: E402
from sgpu_types import default_options  # noqa: E402
from sift_synth import synth_batch, synth_image  # noqa: E402

ctx = sgpu.SiftContext(0, default_options())
DUO, OFF = ctx.DEBUG_DUO_ALWAYS, ctx.DEBUG_DUO_OFF


def levels(img_idx, opts):
    return [[ctx.gaussian(img_idx, o, l).copy() for l in range(opts.dog_level_num + 3)]
            for o in range(len(ctx.geometry()))]


for (n, w, h, seed, rows) in [(1, 104, 33, 5, 0), (1, 640, 480, 1000, 0), (1, 104, 33, 5, 0), (1, 640, 480, 1000, 0), (1, 640, 480, 1000, 8), (2, 640, 480, 7, 0),
                              (1, 1920, 1080, 5, 0), (1, 960, 480, 5, 0), (1, 576, 480, 5, 0),
                              (1, 640, 1080, 5, 0)]:
    imgs = synth_batch(n, w, h, seed) if n > 1 else synth_image(w, h, seed)
    opts = default_options()
    ctx.set_options(opts)
    # the paired run first, on buffers laid out for the previous case's size
    ctx.set_debug_flags((rows << sgpu.SiftContext.DEBUG_BAND_SHIFT) | DUO)
    ctx.extract(imgs)
    got = levels(0, opts)
    ctx.set_debug_flags(OFF)
    ctx.extract(imgs)
    ref = levels(0, opts)
    msg = "ok"
    for o, (la, lb) in enumerate(zip(ref, got)):
        for l, (x, y) in enumerate(zip(la, lb)):
            if not np.array_equal(x.view(np.uint32), y.view(np.uint32)):
                wa = ctx.geometry()[o][2]
                d = np.argwhere((x.view(np.uint32) != y.view(np.uint32)).reshape(-1, wa))
                msg = (f"level ({o},{l}) {x.shape}: {len(d)} px differ, rows {d[:, 0].min()}..{d[:, 0].max()}, "
                       f"cols {d[:, 1].min()}..{d[:, 1].max()}; first {d[:5].tolist()}")
                break
        if msg != "ok":
            break
    print(f"n={n} {w}x{h} rows={rows}: {msg}", flush=True)
ctx.set_debug_flags(0)
