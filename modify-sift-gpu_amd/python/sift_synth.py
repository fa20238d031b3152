"""Deterministic synthetic inputs for tests and bench.py ("Synthetic inputs").

Images: background 128, anisotropic Gaussian blobs, rotated rectangles, Gaussian noise, rounded and
clamped to u8.  Descriptor sets: SIFT-like (|N(0,1)| with 60 % zeros, normalize, clip 0.2,
renormalize) with planted near-duplicates so the ratio test fires.  Everything is a pure function
of the seed (numpy PCG64).
"""
from __future__ import annotations

import numpy as np


def synth_image(w: int, h: int, seed: int, n_blobs: int = 400, n_rects: int = 200,
                noise: float = 4.0) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    img = np.full((h, w), 128.0, dtype=np.float64)
    scale = min(w, h) / 1080.0
    for _ in range(n_blobs):
        cx, cy = rng.uniform(0, w), rng.uniform(0, h)
        amp = rng.uniform(-96, 96)
        sx, sy = rng.uniform(2, 40) * max(scale, 0.15), rng.uniform(2, 40) * max(scale, 0.15)
        th = rng.uniform(0, np.pi)
        r = 4.0 * max(sx, sy)
        x0, x1 = int(max(0, cx - r)), int(min(w, cx + r + 1))
        y0, y1 = int(max(0, cy - r)), int(min(h, cy + r + 1))
        if x0 >= x1 or y0 >= y1:
            continue
        yy, xx = np.mgrid[y0:y1, x0:x1]
        dx, dy = xx - cx, yy - cy
        c, s = np.cos(th), np.sin(th)
        u, v = c * dx + s * dy, -s * dx + c * dy
        img[y0:y1, x0:x1] += amp * np.exp(-0.5 * ((u / sx) ** 2 + (v / sy) ** 2))
    for _ in range(n_rects):
        cx, cy = rng.uniform(0, w), rng.uniform(0, h)
        step = rng.uniform(-64, 64)
        hw, hh = rng.uniform(3, 60) * max(scale, 0.15), rng.uniform(3, 60) * max(scale, 0.15)
        th = rng.uniform(0, np.pi)
        r = np.hypot(hw, hh) + 1
        x0, x1 = int(max(0, cx - r)), int(min(w, cx + r + 1))
        y0, y1 = int(max(0, cy - r)), int(min(h, cy + r + 1))
        if x0 >= x1 or y0 >= y1:
            continue
        yy, xx = np.mgrid[y0:y1, x0:x1]
        dx, dy = xx - cx, yy - cy
        c, s = np.cos(th), np.sin(th)
        u, v = c * dx + s * dy, -s * dx + c * dy
        img[y0:y1, x0:x1] += step * ((np.abs(u) <= hw) & (np.abs(v) <= hh))
    img += rng.normal(0.0, noise, size=img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


_SYNTH_LIB = None


def _synth_lib():
    """tests/synth/libsynth.so (built here with gcc when missing)."""
    global _SYNTH_LIB
    if _SYNTH_LIB is None:
        import ctypes
        import os
        import subprocess
        d = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                         "tests", "synth")
        so = os.path.join(d, "libsynth.so")
        if not os.path.exists(so):
            subprocess.check_call(["gcc", "-O3", "-fopenmp", "-shared", "-fPIC", "-o", so,
                                   os.path.join(d, "synth.c"), "-lm"])
        L = ctypes.CDLL(so)
        L.synth_batch_u8.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_uint64, ctypes.c_int]
        _SYNTH_LIB = L
    return _SYNTH_LIB


def synth_batch_fast(n: int, w: int, h: int, seed0: int, threads: int | None = None) -> np.ndarray:
    """n distinct images [n, h, w] from seeds seed0 .. seed0 + n - 1, the synth_image recipe in C
    (tests/synth/synth.c; its own generator, so not the NumPy images), on up to 16 threads."""
    import os
    if threads is None:
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
    out = np.empty((n, h, w), np.uint8)
    _synth_lib().synth_batch_u8(out.ctypes.data, n, w, h, seed0, threads)
    return out


def synth_batch(n: int, w: int, h: int, seed0: int, unique: int | None = None) -> np.ndarray:
    """n images [n, h, w]; with `unique` set, only that many distinct images are generated and
    the batch cycles through them (generation cost only; every image is still processed)."""
    k = n if unique is None else max(1, min(unique, n))
    base = [synth_image(w, h, seed0 + i) for i in range(k)]
    return np.stack([base[i % k] for i in range(n)])


def synth_descriptors(n: int, seed: int, base: np.ndarray | None = None,
                      n_dup: int = 0, dup_noise: float = 0.02) -> np.ndarray:
    """n float SIFT-like descriptors [n, 128].  With `base`, the first n_dup rows are noisy
    copies of base rows (planted near-duplicates)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    d = np.abs(rng.normal(size=(n, 128)))
    d[rng.uniform(size=(n, 128)) < 0.6] = 0.0
    if base is not None and n_dup > 0:
        d[:n_dup] = base[:n_dup] + rng.normal(0.0, dup_noise, size=(n_dup, 128))
        d[:n_dup] = np.abs(d[:n_dup])
    d /= np.maximum(np.linalg.norm(d, axis=1, keepdims=True), 1e-12)
    d = np.minimum(d, 0.2)
    d /= np.maximum(np.linalg.norm(d, axis=1, keepdims=True), 1e-12)
    return d.astype(np.float32)


def quantize(d: np.ndarray) -> np.ndarray:
    """(unsigned char)int(512*d + 0.5) of SiftMatchCU.cpp:96-99 (float product, double add,
    truncation, modulo-256 narrowing)."""
    v = (np.float32(512.0) * d.astype(np.float32)).astype(np.float64) + 0.5
    return (np.trunc(v).astype(np.int64) & 0xFF).astype(np.uint8)


def synth_guided_scene(n1: int, n2: int, seed: int, n_dup: int | None = None,
                       n_exact: int = 8, width: float = 1920.0, height: float = 1080.0):
    """Two descriptor sets with locations for guided matching (SiftMatchGPU::GetGuidedSiftMatch).

    Set 2's first n_dup features are near-duplicates of set 1's that sit at H x1 (plus < 1 px),
    every third of those is then moved far away (a descriptor match the geometry must reject),
    and n_exact exact copies give dots above 2^18 (the reference's max(dot - 2^18, 0) branch).
    H is a similarity-plus-perspective homography; F = [e]_x H, so x2' F x1 = 0 for x2 = H x1.
    Returns (q1, q2, loc1, loc2, H, F) with u8 descriptors and float32 [n][2] locations."""
    rng = np.random.Generator(np.random.PCG64(seed))
    n_dup = min(n1, n2, n_dup if n_dup is not None else min(n1, n2) // 2)
    d1 = synth_descriptors(n1, seed * 7 + 1)
    d2 = synth_descriptors(n2, seed * 7 + 2, base=d1, n_dup=n_dup)
    q1, q2 = quantize(d1), quantize(d2)
    k = min(n_exact, n_dup)
    q2[:k] = q1[:k]
    loc1 = np.stack([rng.uniform(0, width, n1), rng.uniform(0, height, n1)], 1)
    a = rng.uniform(-0.2, 0.2)
    s = rng.uniform(0.9, 1.1)
    H = np.array([[s * np.cos(a), -s * np.sin(a), rng.uniform(-50, 50)],
                  [s * np.sin(a), s * np.cos(a), rng.uniform(-50, 50)],
                  [rng.uniform(-1e-5, 1e-5), rng.uniform(-1e-5, 1e-5), 1.0]])
    e = np.array([rng.uniform(-1, 1), rng.uniform(-1, 1), 1e-3])
    ex = np.array([[0, -e[2], e[1]], [e[2], 0, -e[0]], [-e[1], e[0], 0]])
    F = ex @ H
    F /= np.linalg.norm(F)
    loc2 = np.stack([rng.uniform(0, width, n2), rng.uniform(0, height, n2)], 1)
    x1 = np.concatenate([loc1[:n_dup], np.ones((n_dup, 1))], 1) @ H.T
    loc2[:n_dup] = x1[:, :2] / x1[:, 2:] + rng.uniform(-0.5, 0.5, (n_dup, 2))
    loc2[2:n_dup:3] += rng.uniform(200, 400, (len(range(2, n_dup, 3)), 2))
    return (q1, q2, loc1.astype(np.float32), loc2.astype(np.float32), H.astype(np.float32),
            F.astype(np.float32))


def synth_tie_scene(n1: int, n2: int, seed: int, col_pairs, row_pairs=()):
    """Descriptor sets with exact ties at row maxima: for each (c_a, c_b) in col_pairs one row of
    set 1 (self dot < 2^18, so distances stay > 0) is copied to set-2 columns c_a and c_b; for each
    (r_a, r_b) in row_pairs rows r_a and r_b of set 1 copy one set-2 column (a column-side tie).
    Matches on ties are accepted only with ratiomax > 1.  Returns (q1, q2, tied rows of set 1)."""
    q1 = quantize(synth_descriptors(n1, seed))
    q2 = quantize(synth_descriptors(n2, seed + 1))
    used = {r for pair in row_pairs for r in pair}
    rows = [i for i in range(n1) if i not in used and
            int((q1[i].astype(np.int64) ** 2).sum()) < 262144][:len(col_pairs)]
    for i, (ca, cb) in zip(rows, col_pairs):
        q2[ca] = q1[i]
        q2[cb] = q1[i]
    for k, (ra, rb) in enumerate(row_pairs):
        c = (k * 7919 + 11) % n2
        q1[ra] = q2[c]
        q1[rb] = q2[c]
    return q1, q2, rows


def tie_winner(ca: int, cb: int) -> int:
    """RowMatch_Kernel's choice between two equal maxima: lowest column mod 32, then lowest."""
    return min((ca, cb), key=lambda c: (c % 32, c))
