"""Generates tests/golden/*.npz from the CPU oracle (the reference itself cannot run here).

Each fixture holds the seeded input and the oracle's full outputs; tests/test_oracle.py pins the
oracle to them (regression) and the GPU parity tests compare the HIP path against them.
Run: python tests/make_golden.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "modify-sift-gpu_amd", "python"))

import numpy as np  # noqa: E402

import oracle_py as O  # noqa: E402
from sgpu_types import default_options  # noqa: E402
from sift_synth import synth_image, synth_descriptors, quantize  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")

CASES = [
    # name, w, h, seed, option overrides
    ("extract_160x120_s1", 160, 120, 1, {}),
    ("extract_203x97_s2", 203, 97, 2, {}),              # width not a multiple of 4 (truncation)
    ("extract_256x200_m1", 256, 200, 3, {"max_orientation": 1}),
    ("extract_256x200_ofix", 256, 200, 3, {"fixed_orientation": 1}),
    ("extract_240x180_no2_d4", 240, 180, 4, {"octave_num": 2, "dog_level_num": 4}),
    ("extract_200x150_circ_unn", 200, 150, 5, {"circular_window": 1, "normalized": 0}),
    ("extract_320x240_s6", 320, 240, 6, {}),
]


def main():
    os.makedirs(GOLDEN, exist_ok=True)
    for name, w, h, seed, over in CASES:
        img = synth_image(w, h, seed)
        opts = default_options(**over)
        k, d = O.extract(img, opts)
        names = np.array(list(over.keys()) or ["subpixel"])
        vals = np.array(list(over.values()) or [1], np.int64)
        np.savez_compressed(os.path.join(GOLDEN, name + ".npz"), image=img, keys=k, desc=d,
                            opt_names=names, opt_values=vals)
        print(name, k.shape)
    d1 = synth_descriptors(300, 5000)
    d2 = synth_descriptors(260, 5001, base=d1, n_dup=120)
    q1, q2 = quantize(d1), quantize(d2)
    pairs = O.match(q1, q2)
    np.savez_compressed(os.path.join(GOLDEN, "match_small.npz"), q1=q1, q2=q2, pairs=pairs)
    print("match_small", pairs.shape)


if __name__ == "__main__":
    main()
