"""Diagnostic (GPU box): features whose shipped (relaxed) descriptor differs from the bit-exact
one by more than a threshold, with the bins that differ."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "modify-sift-gpu_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import sgpu  # noqa: E402
from sgpu_types import default_options  # noqa: E402
from sift_synth import synth_image  # noqa: E402

img = synth_image(400, 300, 31)
ctx = sgpu.SiftContext(0, default_options(octave_min=-1, dog_level_num=4))
ctx.extract(img)
kf, df = ctx.features(0)
with ctx.exact_descriptors():
    ctx.extract(img)
    ke, de = ctx.features(0)
assert np.array_equal(kf.view(np.uint32), ke.view(np.uint32))
l2 = np.linalg.norm(df.astype(np.float64) - de, axis=1)
print("n", len(kf), "max", l2.max(), "median", np.median(l2), "n>1e-5", (l2 > 1e-5).sum())
for i in np.argsort(-l2)[:5]:
    diff = np.abs(df[i] - de[i])
    bins = np.argsort(-diff)[:6]
    print(i, "key", kf[i].tolist(), "l2", l2[i])
    print("   bins", bins.tolist(), "fast", df[i][bins].tolist(), "exact", de[i][bins].tolist())
