"""The C++ oracle against the independent float64 NumPy restatement (tests/ref_numpy.py).

Different arithmetic (float64, libm) and different structure on the other side, so agreement here
pins the oracle's *algorithm* to the reference's, not to the HIP kernels.  Tolerances are float32
rounding of the oracle's computation; set membership near a threshold may differ by a few
candidates, which the tests bound explicitly.
"""
import math

import numpy as np
import pytest

import oracle_py as O
import ref_numpy as R
from sgpu_types import default_options
from sift_synth import synth_image

# (name, width, height, seed, oracle option overrides): the default case; config C2's 1080p
# image; the circular orientation window (ProgramCU-0.cu:834); -fo -1 (the upsampled first
# octave); -d 5 (other level sigmas and filter widths)
CASES = [
    ("default", 320, 240, 21, {}),
    ("c2_1080p", 1920, 1080, 2000, {"octave_num": 4}),
    ("circular", 320, 240, 22, {"circular_window": 1}),
    ("fo_m1", 320, 240, 23, {"octave_min": -1, "octave_num": 4}),
    ("d5", 320, 240, 24, {"dog_level_num": 5}),
]
# at most this many features per case go through the per-feature float64 loops
MAX_FEATS = 400


@pytest.fixture(scope="module", params=CASES, ids=[c[0] for c in CASES])
def case(request):
    name, w, h, seed, over = request.param
    img = synth_image(w, h, seed)
    opts = default_options(**over)
    S = R.schedule(d=opts.dog_level_num, octave_min=opts.octave_min)
    G = R.pyramid(img, S, octave_num=opts.octave_num, octave_min=opts.octave_min)
    return img, S, G, opts


def _sample(n):
    step = max(1, n // MAX_FEATS)
    return range(0, n, step)


def test_pyramid_levels(case):
    img, S, G, opts = case
    for o, lv in enumerate(G):
        for k, g64 in enumerate(lv):
            g32 = O.gaussian(img, o, k, opts).reshape(g64.shape)
            assert np.max(np.abs(g32 - g64)) < 2e-5, (o, k)


def test_candidates(case):
    img, S, G, opts = case
    cand64 = R.detect(G, S)
    ints, fl = O.candidates(img, opts)
    d = S["d"]
    ours = {}
    for (c, r, lid, _), f in zip(ints, fl):
        ours[(lid // d, lid % d, c, r)] = f[:3]
    ref = {}
    for (o, j), lst in cand64.items():
        for c, r, dx, dy, ds, _ in lst:
            ref[(o, j, c, r)] = np.array([dx, dy, ds])
    common = sorted(set(ours) & set(ref))
    union = set(ours) | set(ref)
    assert len(ours) > 100
    assert len(common) / len(union) > 0.97, (len(ours), len(ref), len(common))
    # The 3x3 solve (ProgramCU.cu:631-667) amplifies the oracle's float32 rounding of the
    # Gaussian levels by |A^-1| where the curvature is small, so the offsets are held to a
    # conditioning-aware bound: |err| <= 16 |A^-1|_2 max|G| 2^-24 for every common candidate
    # (observed: median 1.2, max 9.5 of that unit, at 320x240 and at 1080p alike), plus the
    # absolute bounds (95 % within 1e-3 -- -d 5's smaller DoG values are the worst conditioned,
    # 96 % -- and all within 2e-2).
    err = np.array([np.max(np.abs(ours[k] - ref[k])) for k in common])
    unit = np.array([_solve_unit(G, S, k) for k in common])
    assert np.all(err <= 16 * unit), np.sort(err / unit)[-5:]
    assert np.mean(err < 1e-3) > 0.95 and err.max() < 2e-2, np.sort(err)[-5:]


def _solve_unit(G, S, key):
    """|A^-1|_2 * max|G| * 2^-24 at a candidate (octave o, DoG level j, column c, row r): the
    offset error that one float32 rounding of the levels around it causes through the solve."""
    o, j, c, r = key
    lv = G[o]
    P, C, N = (lv[j + 1] - lv[j], lv[j + 2] - lv[j + 1], lv[j + 3] - lv[j + 2])
    v = C[r, c]
    fxx = C[r, c - 1] + C[r, c + 1] - 2 * v
    fyy = C[r - 1, c] + C[r + 1, c] - 2 * v
    fxy = 0.25 * (C[r + 1, c + 1] + C[r - 1, c - 1] - C[r + 1, c - 1] - C[r - 1, c + 1])
    fss = N[r, c] + P[r, c] - 2 * v
    fxs = 0.25 * (N[r, c + 1] + P[r, c - 1] - N[r, c - 1] - P[r, c + 1])
    fys = 0.25 * (N[r + 1, c] + P[r - 1, c] - N[r - 1, c] - P[r + 1, c])
    A = np.array([[fxx, fxy, fxs], [fxy, fyy, fys], [fxs, fys, fss]])
    gmax = max(abs(lv[m][r - 1:r + 2, c - 1:c + 2]).max() for m in range(j, j + 4))
    return np.linalg.norm(np.linalg.inv(A), 2) * gmax * 2.0 ** -24


def test_orientations(case):
    img, S, G, opts = case
    feat, lvl = O.features_oct(img, opts)
    d = S["d"]
    grads = {}
    hits = n = 0
    for i in _sample(len(feat)):
        (x, y, s, o), lid = feat[i], lvl[i]
        oc, j = lid // d, lid % d
        if (oc, j) not in grads:
            grads[(oc, j)] = R.gradient(G[oc][1 + j])
        mag, ang = grads[(oc, j)]
        angs = R.orientation(mag, ang, float(x), float(y), float(s),
                             circular=bool(opts.circular_window))
        diff = [abs((float(o) - a + math.pi) % (2 * math.pi) - math.pi) for a in angs]
        hits += bool(diff) and min(diff) < 2e-3
        n += 1
    assert n > 100
    assert hits / n > 0.97, (hits, n)


def test_descriptors(case):
    img, S, G, opts = case
    feat, lvl = O.features_oct(img, opts)
    _, desc = O.extract(img, opts)
    d = S["d"]
    errs = []
    grads = {}
    for i in _sample(len(feat)):
        (x, y, s, o), lid, dd = feat[i], lvl[i], desc[i]
        oc, j = lid // d, lid % d
        if (oc, j) not in grads:
            grads[(oc, j)] = R.gradient(G[oc][1 + j])
        mag, ang = grads[(oc, j)]
        ref = R.descriptor(mag, ang, float(x), float(y), float(s), float(o))
        errs.append(np.linalg.norm(ref - dd))
    errs = np.array(errs)
    assert len(errs) > 100
    assert np.median(errs) < 1e-4, np.median(errs)
    assert np.mean(errs < 1e-3) > 0.99, np.sort(errs)[-5:]


def test_unnormalized_descriptors(case):
    img, S, G, opts = case
    opts = default_options(**{f: getattr(opts, f) for f, _ in opts._fields_})
    opts.normalized = 0
    feat, lvl = O.features_oct(img, opts)
    _, desc = O.extract(img, opts)
    d = S["d"]
    rel = []
    grads = {}
    for i in list(_sample(len(feat)))[:200]:
        (x, y, s, o), lid, dd = feat[i], lvl[i], desc[i]
        oc, j = lid // d, lid % d
        if (oc, j) not in grads:
            grads[(oc, j)] = R.gradient(G[oc][1 + j])
        mag, ang = grads[(oc, j)]
        ref = R.descriptor(mag, ang, float(x), float(y), float(s), float(o), normalize=False)
        rel.append(np.linalg.norm(ref - dd) / max(np.linalg.norm(ref), 1e-12))
    assert np.median(rel) < 1e-4
