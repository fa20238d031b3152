"""GPU parity: the HIP path (through the C ABI, libsiftgpu.so) against the CPU oracle and the
committed golden fixtures.  Bar: keypoints (x, y, scale, orientation) bit-identical,
descriptors bit-identical (the test asserts the looser L2 < 1e-4 of the north star and reports
bitwise equality), matches identical.

Mirrors the reference's own checks: TestWin/SimpleSIFT.cpp's extract -> match flow (run here
through our SiftGPU.h with a compiled replica), SpeedSIFT's repeated extraction on one image
(determinism), and the option paths of ParseParam (-m, -ofix, -d, -no, -unn, circular window).
At sizes the oracle cannot finish quickly (full HD batches, 12 MP) the tests use
size-independent properties instead: repeatability, batch == single-image results, bounds.
"""
import glob
import os
import subprocess

import numpy as np
import pytest

import oracle_py as O
import sgpu
from sgpu_types import default_options
from sift_synth import (synth_batch, synth_descriptors, synth_guided_scene, synth_image,
                        synth_tie_scene, tie_winner, quantize)

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
DESC_L2_TOL = 1e-4   # BASELINE.json north_star: descriptor L2 < 1e-4
# C++ replicas that compare with the oracle bit for bit (or through matches of quantised
# descriptors) run the bit-exact descriptor kernel (sgpu.h SGPU_DEBUG_EXACT_DESCRIPTOR)
EXACT_ENV = dict(os.environ, SGPU_EXACT_DESCRIPTOR="1")


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _assert_features_equal(k, d, rk, rd, what=""):
    assert k.shape == rk.shape, f"{what}: {k.shape} features vs oracle {rk.shape}"
    if len(k) == 0:
        return
    diff = _bits(k) != _bits(rk)
    assert not diff.any(), f"{what}: keypoint bits differ at rows {np.where(diff.any(1))[0][:8]}"
    if d is not None and rd is not None:
        l2 = np.linalg.norm(d.astype(np.float64) - rd.astype(np.float64), axis=1)
        assert l2.max() < DESC_L2_TOL, f"{what}: descriptor L2 {l2.max()}"


def _golden_cases():
    return sorted(glob.glob(os.path.join(GOLDEN, "extract_*.npz")))


@pytest.mark.parametrize("path", _golden_cases(), ids=lambda p: os.path.basename(p)[:-4])
def test_golden_extract(gpu_ctx, path):
    z = np.load(path)
    opts = default_options(**{k: int(v) for k, v in zip(z["opt_names"], z["opt_values"])})
    gpu_ctx.set_options(opts)
    gpu_ctx.extract(z["image"])
    k, d = gpu_ctx.features(0)
    _assert_features_equal(k, d, z["keys"], z["desc"], os.path.basename(path))
    # the bit-exact descriptor kernel: bitwise, which is what the shared deterministic math gives
    with gpu_ctx.exact_descriptors():
        gpu_ctx.extract(z["image"])
        k, d = gpu_ctx.features(0)
    assert np.array_equal(_bits(k), _bits(z["keys"]))
    assert np.array_equal(_bits(d), _bits(z["desc"]))


def test_golden_match(gpu_ctx):
    z = np.load(os.path.join(GOLDEN, "match_small.npz"))
    m = gpu_ctx.match(z["q1"], z["q2"])
    assert np.array_equal(m, z["pairs"])


@pytest.mark.parametrize("w,h,seed", [(203, 97, 2), (320, 240, 6), (640, 480, 1000)])
def test_gaussian_levels_bitwise(gpu_ctx, w, h, seed):
    img = synth_image(w, h, seed)
    opts = default_options()
    gpu_ctx.set_options(opts)
    gpu_ctx.extract(img)
    geo = gpu_ctx.geometry()
    for o in range(len(geo)):
        for lvl in range(opts.dog_level_num + 3):
            g = gpu_ctx.gaussian(0, o, lvl)
            r = O.gaussian(img, o, lvl, opts)
            assert np.array_equal(_bits(g), _bits(r)), (o, lvl)


@pytest.mark.parametrize("fo,w,h", [(1, 203, 97), (-1, 203, 97), (-1, 96, 64), (2, 321, 241)])
def test_first_octave_levels_bitwise(gpu_ctx, fo, w, h):
    """-fo != 0: the resampled first octave (SampleImageD / UpsampleKernel) and its levels."""
    img = synth_image(w, h, 17 + fo)
    opts = default_options(octave_min=fo)
    gpu_ctx.set_options(opts)
    gpu_ctx.extract(img)
    geo = gpu_ctx.geometry()
    for o in range(min(len(geo), 2)):
        for lvl in range(opts.dog_level_num + 3):
            g = gpu_ctx.gaussian(0, o, lvl)
            r = O.gaussian(img, o, lvl, opts)
            assert np.array_equal(_bits(g), _bits(r)), (o, lvl)


@pytest.mark.parametrize("fo", [-2, -3])
def test_first_octave_nan_pyramid_has_no_features(gpu_ctx, fo):
    """-fo -2 / -3: the reference's initial smoothing sigma is 0 and its filter taps NaN
    (SiftGPU.cpp:446-452, ProgramCU.cu:391-398); no keypoint of the NaN pyramid gets an
    orientation, so the run succeeds with 0 features -- as the oracle."""
    imgs = np.stack([synth_image(96, 64, 5), synth_image(96, 64, 6)])
    opts = default_options(octave_min=fo)
    gpu_ctx.set_options(opts)
    gpu_ctx.extract(imgs)
    assert gpu_ctx.total() == 0 and gpu_ctx.count(1) == 0
    rk, _ = O.extract(imgs[0], opts)
    assert len(rk) == 0
    gpu_ctx.set_options(default_options())


def test_first_octave_on_a_batch(gpu_ctx):
    """-fo 1 and -fo -1 on a batch equal the single-image results (u8 and f32 input)."""
    imgs = np.stack([synth_image(256, 192, 40 + i) for i in range(3)])
    for fo in (1, -1):
        opts = default_options(octave_min=fo)
        gpu_ctx.set_options(opts)
        gpu_ctx.extract(imgs)
        batch = [gpu_ctx.features(i) for i in range(3)]
        for i in range(3):
            rk, rd = O.extract(imgs[i], opts)
            _assert_features_equal(batch[i][0], batch[i][1], rk, rd, f"fo{fo} image {i}")
        gpu_ctx.extract(imgs.astype(np.float32) / np.float32(255.0))
        k, d = gpu_ctx.features(1)
        _assert_features_equal(k, d, batch[1][0], batch[1][1], f"fo{fo} f32")


@pytest.mark.parametrize("w,h,seed", [(160, 120, 1), (640, 480, 1000), (333, 251, 9)])
def test_candidates_bitwise(gpu_ctx, w, h, seed):
    img = synth_image(w, h, seed)
    gpu_ctx.set_options(default_options())
    gpu_ctx.extract(img)
    gi, gf = gpu_ctx.candidates()
    ri, rf = O.candidates(img)
    assert np.array_equal(gi, ri)
    assert np.array_equal(_bits(gf[:, :3]), _bits(rf[:, :3]))   # column 3 is padding


OPTION_CASES = [
    {},
    {"max_orientation": 1},
    {"fixed_orientation": 1},
    {"dog_level_num": 4, "octave_num": 3},
    {"dog_level_num": 2},
    {"subpixel": 0},
    {"circular_window": 1},
    {"normalized": 0},
    {"keep_extremum_sign": 1},
    {"lowe_origin": 1},
    {"edge_threshold": 5},
    {"filter_width_factor": 3},
    {"descriptor_window_factor": 2},
    {"octave_min": 1},
    {"octave_min": 2},
    {"octave_min": -1},
    {"octave_min": -1, "dog_level_num": 4},
]


@pytest.mark.parametrize("over", OPTION_CASES, ids=lambda o: "-".join(f"{k}{v}" for k, v in o.items()) or "default")
def test_options_vs_oracle(gpu_ctx, over):
    img = synth_image(400, 300, 31)
    opts = default_options(**over)
    gpu_ctx.set_options(opts)
    gpu_ctx.extract(img)
    k, d = gpu_ctx.features(0)
    rk, rd = O.extract(img, opts)
    _assert_features_equal(k, d, rk, rd, str(over))
    with gpu_ctx.exact_descriptors():
        gpu_ctx.extract(img)
        k, d = gpu_ctx.features(0)
    assert np.array_equal(_bits(k), _bits(rk)) and np.array_equal(_bits(d), _bits(rd)), over


@pytest.mark.parametrize("over,n", [({}, 4), ({"normalized": 0}, 4), ({"descriptor_window_factor": 2}, 4),
                                    ({"octave_min": -1}, 4), ({"dog_level_num": 5}, 4), ({}, 24)],
                         ids=lambda o: ("-".join(f"{k}{v}" for k, v in o.items()) or "default")
                         if isinstance(o, dict) else f"n{o}")
def test_shipped_descriptor_vs_exact(gpu_ctx, over, n):
    """The shipped relaxed-order descriptor kernel against the bit-exact one on n HD images:
    same keypoints bit for bit, descriptors within L2 1e-5 (relative to |d| for -unn), i.e. 10x
    inside the north star's 1e-4.  Both counts run the same one-wave-per-feature kernel
    (k_descriptor_dual); the 4-image case (~5k features) is kept deliberately as the small-grid
    check (the grid is sized from the previous call's count), the 24-image one (~30k) as the
    full-occupancy check."""
    from sift_synth import synth_batch_fast
    imgs = synth_batch_fast(n, 1280, 720, 510)
    opts = default_options(**over)
    gpu_ctx.set_options(opts)
    gpu_ctx.extract(imgs)
    gpu_ctx.extract(imgs)   # the second call sizes its grids from the first one's counts
    fast = [gpu_ctx.features(i) for i in range(n)]
    with gpu_ctx.exact_descriptors():
        gpu_ctx.extract(imgs)
        exact = [gpu_ctx.features(i) for i in range(n)]
    kf = np.concatenate([f[0] for f in fast])
    ke = np.concatenate([e[0] for e in exact])
    df = np.concatenate([f[1] for f in fast]).astype(np.float64)
    de = np.concatenate([e[1] for e in exact]).astype(np.float64)
    assert len(kf) > 4000 and np.array_equal(_bits(kf), _bits(ke))
    l2 = np.linalg.norm(df - de, axis=1)
    if not opts.normalized:
        l2 = l2 / np.maximum(np.linalg.norm(de, axis=1), 1e-30)
    print(f"descriptor L2 fast vs exact over {len(kf)} features: max {l2.max():.3g}, "
          f"median {np.median(l2):.3g}")
    assert l2.max() < 1e-5
    gpu_ctx.set_options(default_options())


def test_no_descriptors_option(gpu_ctx):
    img = synth_image(300, 200, 8)
    opts = default_options(descriptors=0)
    gpu_ctx.set_options(opts)
    gpu_ctx.extract(img)
    k, _ = gpu_ctx.features(0, descriptors=False)
    rk, _ = O.extract(img, opts)
    _assert_features_equal(k, None, rk, None, "-sd")


@pytest.mark.parametrize("w,h", [(16, 16), (33, 17), (64, 48), (97, 1203), (1203, 97)])
def test_ragged_and_tiny_sizes(gpu_ctx, w, h):
    img = synth_image(w, h, w * 7 + h)
    gpu_ctx.set_options(default_options())
    gpu_ctx.extract(img)
    k, d = gpu_ctx.features(0)
    rk, rd = O.extract(img)
    _assert_features_equal(k, d, rk, rd, f"{w}x{h}")


def test_flat_image_has_no_features(gpu_ctx):
    gpu_ctx.set_options(default_options())
    gpu_ctx.extract(np.full((240, 320), 128, np.uint8))
    assert gpu_ctx.count(0) == 0 and gpu_ctx.total() == 0
    k, d = gpu_ctx.features(0)
    assert k.shape == (0, 4)


def test_float_input_matches_u8(gpu_ctx):
    # GL_FLOAT luminance (GLTexImage.cpp:981-1006) holding u8/255 gives the u8 path's bits
    img = synth_image(320, 240, 12)
    gpu_ctx.set_options(default_options())
    gpu_ctx.extract(img)
    k8, d8 = gpu_ctx.features(0)
    gpu_ctx.extract(img.astype(np.float32) / np.float32(255.0))
    kf, df = gpu_ctx.features(0)
    assert np.array_equal(_bits(k8), _bits(kf)) and np.array_equal(_bits(d8), _bits(df))


def _synth_color(w, h, seed, ch):
    rng = np.random.default_rng(seed)
    base = synth_image(w, h, seed).astype(np.int32)
    img = np.stack([np.clip(base + rng.integers(-40, 41, (h, w)), 0, 255) for _ in range(ch)], -1)
    return img.astype(np.uint8)


@pytest.mark.parametrize("fmt", ["rgb", "bgr", "rgba", "bgra"])
def test_color_ingest_vs_oracle(gpu_ctx, fmt):
    """Device luminance conversion (GLTexImage.cpp:834-858) then the float-input pipeline,
    against the oracle run on the host-converted luminance."""
    ch = 3 if fmt in ("rgb", "bgr") else 4
    imgs = np.stack([_synth_color(322, 241, 60 + i, ch) for i in range(2)])
    gpu_ctx.set_options(default_options())
    gpu_ctx.extract_color(imgs, fmt)
    for i in range(2):
        k, d = gpu_ctx.features(i)
        rk, rd = O.extract_f32(O.gray_from_color(imgs[i], fmt))
        _assert_features_equal(k, d, rk, rd, f"{fmt} image {i}")
    # -fo 1 on color input: luminance and the 2x sampling of -prep (DownSamplePixelDataI2F,
    # GLTexImage.cpp:928-1009)
    opts = default_options(octave_min=1)
    gpu_ctx.set_options(opts)
    gpu_ctx.extract_color(imgs[:1], fmt)
    k, d = gpu_ctx.features(0)
    rk, rd = O.extract_f32(O.gray_from_color(imgs[0], fmt), opts)
    _assert_features_equal(k, d, rk, rd, f"{fmt} -fo 1")
    gpu_ctx.set_options(default_options())


def test_float_input_vs_oracle(gpu_ctx):
    """Float luminance that is not u8 / 255 (GL_FLOAT input)."""
    rng = np.random.default_rng(3)
    img = (synth_image(300, 200, 5).astype(np.float32) / 300.0 +
           rng.uniform(0, 0.1, (200, 300)).astype(np.float32))
    gpu_ctx.set_options(default_options())
    gpu_ctx.extract(img)
    k, d = gpu_ctx.features(0)
    rk, rd = O.extract_f32(img)
    _assert_features_equal(k, d, rk, rd, "f32")


def test_batch_equals_single_images(gpu_ctx):
    imgs = np.stack([synth_image(256, 192, 500 + i) for i in range(5)])
    gpu_ctx.set_options(default_options())
    gpu_ctx.extract(imgs)
    batch = [gpu_ctx.features(i) for i in range(5)]
    assert gpu_ctx.total() == sum(len(b[0]) for b in batch)
    for i in range(5):
        rk, rd = O.extract(imgs[i])
        _assert_features_equal(batch[i][0], batch[i][1], rk, rd, f"image {i}")


def test_staged_input_matches_host_input(gpu_ctx):
    imgs = synth_batch(3, 320, 240, 77)
    gpu_ctx.set_options(default_options())
    gpu_ctx.extract(imgs)
    host = [gpu_ctx.features(i) for i in range(3)]
    gpu_ctx.stage(imgs).extract_staged()
    for i in range(3):
        k, d = gpu_ctx.features(i)
        assert np.array_equal(_bits(k), _bits(host[i][0]))
        assert np.array_equal(_bits(d), _bits(host[i][1]))


def test_full_hd_batch_properties(gpu_ctx):
    """BASELINE configs[1] shape (1920x1080, 4 octaves) on a batch of 8: repeatable to the
    bit, image 0 of the batch equals image 0 alone, features lie inside the image, descriptors
    are unit length with components <= 0.2 before renormalisation."""
    imgs = synth_batch(8, 1920, 1080, 3000, unique=8)
    opts = default_options(octave_num=4)
    gpu_ctx.set_options(opts)
    gpu_ctx.extract(imgs)
    first = [gpu_ctx.features(i) for i in range(8)]
    total = gpu_ctx.total()
    assert total > 8 * 500
    gpu_ctx.extract(imgs)
    assert gpu_ctx.total() == total
    for i in range(8):
        k, d = gpu_ctx.features(i)
        assert np.array_equal(_bits(k), _bits(first[i][0])) and np.array_equal(_bits(d), _bits(first[i][1]))
        assert (k[:, 0] >= 0).all() and (k[:, 0] < 1920).all()
        assert (k[:, 1] >= 0).all() and (k[:, 1] < 1080).all()
        assert (k[:, 3] >= 0).all() and (k[:, 3] <= 2 * np.pi + 1e-6).all()
        n = np.linalg.norm(d, axis=1)
        assert np.allclose(n, 1.0, atol=1e-3)
    gpu_ctx.extract(imgs[:1])
    k, d = gpu_ctx.features(0)
    assert np.array_equal(_bits(k), _bits(first[0][0]))


@pytest.mark.parametrize("seed", [4242, 2000])
def test_full_hd_single_vs_oracle(gpu_ctx, seed):
    """One 1080p image (-no 4) against the oracle key by key; seed 2000 is bench.py's C2 image."""
    img = synth_image(1920, 1080, seed)
    opts = default_options(octave_num=4)
    gpu_ctx.set_options(opts)
    gpu_ctx.extract(img)
    k, d = gpu_ctx.features(0)
    rk, rd = O.extract(img, opts)
    _assert_features_equal(k, d, rk, rd, "1080p")


def test_large_image_properties(gpu_ctx):
    # 4000 x 3000 (12 MP) with the default octave count: repeatable, in bounds
    img = synth_image(4000, 3000, 99, n_blobs=3000, n_rects=1500)
    gpu_ctx.set_options(default_options())
    gpu_ctx.extract(img)
    k1, d1 = gpu_ctx.features(0)
    gpu_ctx.extract(img)
    k2, d2 = gpu_ctx.features(0)
    assert len(k1) > 1000
    assert np.array_equal(_bits(k1), _bits(k2)) and np.array_equal(_bits(d1), _bits(d2))


# ---- matcher (SiftMatchGPU::GetSiftMatch) ----------------------------------------------------

@pytest.mark.parametrize("n1,n2,dup", [(1, 1, 0), (1, 700, 0), (700, 1, 0), (257, 1000, 100),
                                       (3000, 2500, 1000), (4096, 4096, 2000), (5000, 129, 50)])
def test_match_vs_oracle(gpu_ctx, n1, n2, dup):
    d1 = synth_descriptors(n1, 10 * n1 + n2)
    d2 = synth_descriptors(n2, 10 * n2 + n1 + 1, base=d1, n_dup=min(dup, n1, n2))
    q1, q2 = quantize(d1), quantize(d2)
    assert np.array_equal(gpu_ctx.match(q1, q2), O.match(q1, q2))


@pytest.mark.parametrize("distmax,ratiomax,mbm", [(0.7, 0.8, 1), (0.7, 0.8, 0), (0.5, 0.6, 1),
                                                  (1.0, 1.0, 0), (0.9, 0.95, 1)])
def test_match_thresholds(gpu_ctx, distmax, ratiomax, mbm):
    d1 = synth_descriptors(1500, 71)
    d2 = synth_descriptors(1800, 72, base=d1, n_dup=700)
    q1, q2 = quantize(d1), quantize(d2)
    a = gpu_ctx.match(q1, q2, distmax, ratiomax, mbm)
    b = O.match(q1, q2, distmax, ratiomax, mbm)
    assert np.array_equal(a, b)


def test_match_ties_and_duplicates(gpu_ctx):
    # identical rows in set 2: the best and second best tie -> ratio test rejects (reference's
    # strict '<' on the ratio), exactly as the oracle
    base = quantize(synth_descriptors(400, 5))
    q2 = np.concatenate([base, base[:200]])
    assert np.array_equal(gpu_ctx.match(base, q2), O.match(base, q2))
    zeros = np.zeros((50, 128), np.uint8)
    assert np.array_equal(gpu_ctx.match(zeros, zeros), O.match(zeros, zeros))


@pytest.mark.parametrize("n1,n2,cols", [
    (70, 100, [(5, 34), (40, 66), (3, 99), (31, 32), (7, 39)]),
    # across 128-column tiles (same and different col % 32) and across column chunks
    (3000, 9000, [(200, 129), (130, 2), (4000, 33), (8999, 1), (640, 4064), (7000, 5000)]),
])
def test_match_exact_ties(gpu_ctx, n1, n2, cols):
    """ratiomax > 1 accepts exact ties, so the winner's index shows: RowMatch_Kernel's order on
    the row side, the first row on the column side (oracle pinned by test_oracle)."""
    q1, q2, rows = synth_tie_scene(n1, n2, n1 + n2, cols, [(60, 61), (1, n1 - 5)])
    for mbm in (0, 1):
        a = gpu_ctx.match(q1, q2, distmax=2.0, ratiomax=1.5, mbm=mbm)
        b = O.match(q1, q2, distmax=2.0, ratiomax=1.5, mbm=mbm)
        assert np.array_equal(a, b), mbm
    pairs = dict(map(tuple, gpu_ctx.match(q1, q2, distmax=2.0, ratiomax=1.5, mbm=0).tolist()))
    assert [pairs.get(i) for i in rows] == [tie_winner(x, y) for x, y in cols]


@pytest.mark.parametrize("ratiomax", [0.8, 1.0])
def test_keyless_match_equals_keyed(gpu_ctx, ratiomax):
    """With ratiomax <= 1 plain matching folds raw values (no tie-order keys) and recovers the
    winning column afterwards; pairs must equal the keyed epilogue's (SGPU_DEBUG_KEYED_MATCH),
    on a large planted-duplicate set and on exact-tie scenes (a tied maximum is rejected)."""
    d1 = synth_descriptors(20000, 5000)
    d2 = synth_descriptors(20000, 5001, base=d1, n_dup=8000)
    q1, q2 = quantize(d1), quantize(d2)
    q1t, q2t, _ = synth_tie_scene(3000, 9000, 23, [(200, 129), (130, 2), (4000, 33), (8999, 1)],
                                  [(60, 61), (1, 2995)])
    base = quantize(synth_descriptors(400, 5))
    dup2 = np.concatenate([base, base[:200]])
    cases = [(q1, q2), (q1t, q2t), (base, dup2)]
    for mbm in (0, 1):
        raw = [gpu_ctx.match(a, b, 0.9, ratiomax, mbm) for a, b in cases]
        try:
            gpu_ctx.set_debug_flags(gpu_ctx.DEBUG_KEYED_MATCH)
            keyed = [gpu_ctx.match(a, b, 0.9, ratiomax, mbm) for a, b in cases]
        finally:
            gpu_ctx.set_debug_flags(0)
        for r, k in zip(raw, keyed):
            assert np.array_equal(r, k), mbm
    assert len(raw[0]) > 5000


def test_dma_matcher_equals_register_staged(gpu_ctx):
    """The keyless matcher's LDS-DMA kernel (k_match_raw: three staged tiles, swizzled image,
    precomputed column terms, columns past the set neutralised by a -2^22 - 2^21 column term
    instead of zeroed bytes) against the register-staged k_match_rows<..., RAW>
    (SGPU_DEBUG_MATCH_REGSTAGE): identical pairs for ragged sizes (one column, one partial tile,
    chunk ends inside a tile), exact ties, and rows whose dots are all 0 with the largest
    possible row term (the case a badly neutralised padding column would win)."""
    d1 = synth_descriptors(20000, 5000)
    d2 = synth_descriptors(20000, 5001, base=d1, n_dup=8000)
    q1t, q2t, _ = synth_tie_scene(3000, 9000, 23, [(200, 129), (130, 2), (4000, 33), (8999, 1)],
                                  [(60, 61), (1, 2995)])
    base = quantize(synth_descriptors(400, 5))
    ortho1 = np.zeros((300, 128), np.uint8)
    ortho1[:, :64] = 255
    ortho2 = np.zeros((129, 128), np.uint8)
    ortho2[:, 64:] = 255
    ortho2[5] = ortho1[0]
    cases = [(quantize(d1), quantize(d2)), (q1t, q2t), (base, base[:1].copy()),
             (base[:1].copy(), base), (base, np.concatenate([base, base[:200]])),
             (quantize(synth_descriptors(700, 8)), quantize(synth_descriptors(129, 9))),
             (quantize(synth_descriptors(5000, 11)), quantize(synth_descriptors(16385, 12))),
             (ortho1, ortho2)]
    for mbm in (0, 1):
        for ratiomax in (0.8, 1.0):
            dma = [gpu_ctx.match(a, b, 0.9, ratiomax, mbm) for a, b in cases]
            try:
                gpu_ctx.set_debug_flags(gpu_ctx.DEBUG_MATCH_REGSTAGE)
                reg = [gpu_ctx.match(a, b, 0.9, ratiomax, mbm) for a, b in cases]
            finally:
                gpu_ctx.set_debug_flags(0)
            for i, (x, y) in enumerate(zip(dma, reg)):
                assert np.array_equal(x, y), (mbm, ratiomax, i)
    assert len(dma[0]) > 5000
    # the last pass (mbm 1, ratiomax 1.0) against the oracle on the ragged and orthogonal cases
    for i in (5, 7):
        assert np.array_equal(dma[i], O.match(*cases[i], 0.9, 1.0, 1)), i


def test_matched_columns_equal_full_columns(gpu_ctx):
    """Mutual matching decides only the columns some row matched (a device-side list; the
    column GEMM takes its rows and their count from it).  Pairs must equal deciding every column
    (SGPU_DEBUG_FULL_COLUMNS), keyed and keyless, with ratiomax above 1, and where no row or
    every row matches."""
    d1 = synth_descriptors(20000, 5000)
    d2 = synth_descriptors(20000, 5001, base=d1, n_dup=8000)
    q1t, q2t, _ = synth_tie_scene(3000, 9000, 23, [(200, 129), (130, 2), (4000, 33), (8999, 1)],
                                  [(60, 61), (1, 2995)])
    base = quantize(synth_descriptors(400, 5))
    cases = [(quantize(d1), quantize(d2)), (q1t, q2t),
             (base, np.concatenate([base, base[:200]])),            # many rows -> one column
             (base[:130], base[:130].copy()),                       # every row matches
             (quantize(synth_descriptors(700, 8)), quantize(synth_descriptors(129, 9))),
             (base[:1], base.copy()), (base.copy(), base[:1])]
    for flags, ratiomax in ((0, 0.8), (0, 1.0), (gpu_ctx.DEBUG_KEYED_MATCH, 0.8), (0, 1.5)):
        try:
            gpu_ctx.set_debug_flags(flags)
            got = [gpu_ctx.match(a, b, 0.9, ratiomax, 1) for a, b in cases]
            gpu_ctx.set_debug_flags(flags | gpu_ctx.DEBUG_FULL_COLUMNS)
            full = [gpu_ctx.match(a, b, 0.9, ratiomax, 1) for a, b in cases]
        finally:
            gpu_ctx.set_debug_flags(0)
        for i, (g, f) in enumerate(zip(got, full)):
            assert np.array_equal(g, f), (flags, ratiomax, i)
        assert len(got[0]) > 5000 and len(got[3]) == 130, (flags, ratiomax)


def test_pruned_column_side_equals_unpruned(gpu_ctx):
    """Plain mutual matching with ratiomax <= 1 decides the listed columns over the rows of set 1
    whose largest dot reaches tau, the smallest second value that fails the ratio test against
    the weakest passing row maximum (k_match_finish bisects the distance table; k_prune_set
    compacts the rows; the column GEMM takes their count from the device).  Pairs must equal the
    unpruned column side (sgpu_debug_set_match_prune(0)) and the oracle: planted duplicates among
    random rows (most rows pruned), distmax / ratiomax that let weak rows pass (tau low, nothing
    pruned), exact copies (dots above 2^18), tie scenes, many rows on one column, no row and
    every row matching, ragged sizes."""
    d1 = synth_descriptors(20000, 6000)
    d2 = synth_descriptors(20000, 6001, base=d1, n_dup=8000)
    q1t, q2t, _ = synth_tie_scene(3000, 9000, 29, [(200, 129), (130, 2), (4000, 33), (8999, 1)],
                                  [(60, 61), (1, 2995)])
    g1, g2, _, _, _, _ = synth_guided_scene(3000, 2000, 31)
    base = quantize(synth_descriptors(400, 5))
    cases = [(quantize(d1), quantize(d2)), (q1t, q2t), (g1, g2),
             (base, np.concatenate([base, base[:200]])),
             (base[:130], base[:130].copy()),
             (quantize(synth_descriptors(700, 8)), quantize(synth_descriptors(129, 9))),
             (base[:1], base.copy()), (base.copy(), base[:1])]
    for distmax, ratiomax in ((0.7, 0.8), (0.9, 1.0), (2.0, 1.0), (0.9, 0.5), (2.0, 0.99)):
        got = [gpu_ctx.match(a, b, distmax, ratiomax, 1) for a, b in cases]
        try:
            gpu_ctx.set_match_prune(False)
            full = [gpu_ctx.match(a, b, distmax, ratiomax, 1) for a, b in cases]
        finally:
            gpu_ctx.set_match_prune(True)
        for i, (g, f) in enumerate(zip(got, full)):
            assert np.array_equal(g, f), (distmax, ratiomax, i)
        assert len(got[0]) > 5000 and len(got[4]) == 130, (distmax, ratiomax)
        for i in (2, 5):
            assert np.array_equal(got[i], O.match(*cases[i], distmax, ratiomax, 1)), (distmax, ratiomax, i)


@pytest.mark.parametrize("n1,n2,dup",[(1, 700, 0), (700, 1, 0), (257, 1000, 100),
                                       (3000, 2500, 1000), (4096, 4096, 2000), (5000, 129, 50)])
def test_fused_match_vs_oracle(gpu_ctx, n1, n2, dup):
    """The one-GEMM mutual matcher (row decisions and per-panel column partials from the same
    accumulators, SGPU_DEBUG_FUSED_MATCH) gives the oracle's pairs, ties included."""
    d1 = synth_descriptors(n1, 10 * n1 + n2)
    d2 = synth_descriptors(n2, 10 * n2 + n1 + 1, base=d1, n_dup=min(dup, n1, n2))
    q1, q2 = quantize(d1), quantize(d2)
    try:
        gpu_ctx.set_debug_flags(gpu_ctx.DEBUG_FUSED_MATCH)
        assert np.array_equal(gpu_ctx.match(q1, q2), O.match(q1, q2))
        q1t, q2t, _ = synth_tie_scene(3000, 9000, 17, [(200, 129), (130, 2), (4000, 33), (8999, 1)],
                                      [(60, 61), (1, 2995)])
        a = gpu_ctx.match(q1t, q2t, distmax=2.0, ratiomax=1.5, mbm=1)
        assert np.array_equal(a, O.match(q1t, q2t, distmax=2.0, ratiomax=1.5, mbm=1))
    finally:
        gpu_ctx.set_debug_flags(0)


def test_match_max_match_truncates(gpu_ctx):
    d1 = synth_descriptors(1000, 81)
    d2 = synth_descriptors(1000, 82, base=d1, n_dup=900)
    q1, q2 = quantize(d1), quantize(d2)
    full = O.match(q1, q2)
    assert len(full) > 100
    assert np.array_equal(gpu_ctx.match(q1, q2, max_match=100), O.match(q1, q2, max_match=100))


def test_extract_then_match_pipeline(gpu_ctx):
    """SimpleSIFT flow through the Python binding: two views, extract, quantize, match."""
    img = synth_image(640, 480, 55)
    shifted = np.roll(img, (7, 11), axis=(0, 1))
    gpu_ctx.set_options(default_options())
    gpu_ctx.extract(np.stack([img, shifted]))
    _, d1 = gpu_ctx.features(0)
    _, d2 = gpu_ctx.features(1)
    q1, q2 = sgpu.quantize(d1), sgpu.quantize(d2)
    assert np.array_equal(q1, quantize(d1))
    m = gpu_ctx.match(q1, q2)
    assert np.array_equal(m, O.match(q1, q2))
    assert len(m) > 50


# ---- the drop-in C++ API, driven like TestWin/SimpleSIFT.cpp -----------------------------------

def _write_pgm(path, img):
    h, w = img.shape
    with open(path, "wb") as f:
        f.write(f"P5\n{w} {h}\n255\n".encode())
        f.write(np.ascontiguousarray(img, np.uint8).tobytes())


def _read_sift_ascii(path):
    with open(path) as f:
        tok = f.read().split()
    n, dim = int(tok[0]), int(tok[1])
    vals = tok[2:]
    keys = []
    for i in range(n):
        row = vals[i * (4 + dim):(i + 1) * (4 + dim)]
        keys.append([float(v) for v in row[:4]])
    return np.array(keys, np.float64).reshape(n, 4)


def test_simplesift_replica(tmp_path):
    lib = os.path.join(ROOT, "modify-sift-gpu_amd", "lib", "libsiftgpu.so")
    exe = tmp_path / "simple_sift"
    r = subprocess.run(["g++", "-std=c++11", "-O1", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "abi", "simple_sift_replica.cpp"),
                        "-o", str(exe), "-ldl"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    img1 = synth_image(640, 480, 61)
    img2 = np.roll(img1, (5, 9), axis=(0, 1))
    p1, p2 = tmp_path / "a.pgm", tmp_path / "b.pgm"
    _write_pgm(p1, img1)
    _write_pgm(p2, img2)
    s1, s2 = tmp_path / "a.sift", tmp_path / "b.sift"
    r = subprocess.run([str(exe), lib, str(p1), str(p2), str(s1), str(s2)], capture_output=True,
                       text=True, timeout=300, env=EXACT_ENV)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.strip().splitlines()
    res = [l for l in lines if l.startswith("RESULT ")]
    assert len(res) == 1, r.stdout
    num1, num2, nm = map(int, res[0].split()[1:])
    rk1, rd1 = O.extract(img1)
    rk2, rd2 = O.extract(img2)
    assert (num1, num2) == (len(rk1), len(rk2))
    pairs = np.array([list(map(int, l.split()[1:])) for l in lines if l.startswith("PAIR ")],
                     np.int32).reshape(-1, 2)
    ref_pairs = O.match(quantize(rd1), quantize(rd2))
    assert nm == len(ref_pairs) and np.array_equal(pairs, ref_pairs)
    # SaveSIFT writes Lowe's format: y, x, scale, orientation (SiftGPU.cpp:1107-1140)
    k1 = _read_sift_ascii(s1)
    assert k1.shape == (num1, 4)
    assert np.allclose(k1[:, 0], rk1[:, 1], atol=1e-2) and np.allclose(k1[:, 1], rk1[:, 0], atol=1e-2)


@pytest.mark.parametrize("flags", [1, 2])
def test_batch_parts_match_single_part(gpu_ctx, flags):
    """The batch split into 2 / 4 parts on separate streams (sgpu_capi.cpp extract_impl) gives
    the single-part results image by image, including the gathered device arrays."""
    imgs = np.stack([synth_image(320, 240, 900 + i) for i in range(7)])
    gpu_ctx.set_options(default_options())
    gpu_ctx.extract(imgs)
    ref = [gpu_ctx.features(i) for i in range(7)]
    ref_c = gpu_ctx.candidates()
    try:
        gpu_ctx.set_debug_flags(flags)   # SGPU_DEBUG_PARTS2 / SGPU_DEBUG_PARTS4
        gpu_ctx.extract(imgs)
        got = [gpu_ctx.features(i) for i in range(7)]
        got_c = gpu_ctx.candidates()
    finally:
        gpu_ctx.set_debug_flags(0)
    for (k, d), (rk, rd) in zip(got, ref):
        assert np.array_equal(_bits(k), _bits(rk)) and np.array_equal(_bits(d), _bits(rd))
    assert np.array_equal(got_c[0], ref_c[0])
    assert gpu_ctx.total() == sum(len(k) for k, _ in ref)


def test_rccl_single_rank_collectives(gpu_ctx):
    """The RCCL communicator inside libsiftgpu (sgpu_comm_*), exercised with one rank on the
    one-GPU box: the all-gather returns the send buffer, the all-reduces the values."""
    uid = sgpu.comm_unique_id()
    assert len(uid) == 128
    gpu_ctx.comm_init(1, 0, uid)
    counts = np.arange(37, dtype=np.int32) * 3
    assert np.array_equal(gpu_ctx.allgather_i32(counts, 1), counts)
    assert gpu_ctx.allreduce_f64([1.5, -2.0], op_max=True).tolist() == [1.5, -2.0]
    assert gpu_ctx.allreduce_f64(4.25, op_max=False).tolist() == [4.25]


# ---- caller-supplied keypoints (SiftGPU::RunSIFT(num, keys, keys_have_orientation)) ----------

def _synth_keys(w, h, n, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    k = np.zeros((n, 4), np.float32)
    k[:, 0] = rng.uniform(0, w, n)
    k[:, 1] = rng.uniform(0, h, n)
    k[:, 2] = np.exp(rng.uniform(np.log(0.5), np.log(60.0), n))   # below the first / above the last level too
    k[:, 3] = rng.uniform(0, 2 * np.pi, n)
    return k


@pytest.mark.parametrize("has_orientation", [True, False])
@pytest.mark.parametrize("over", [{}, {"fixed_orientation": 1}, {"max_orientation": 1},
                                  {"normalized": 0, "lowe_origin": 1}])
def test_keypoints_vs_oracle(gpu_ctx, has_orientation, over):
    img = synth_image(480, 360, 71)
    opts = default_options(**over)
    keys = _synth_keys(480, 360, 300, 72)
    gpu_ctx.set_options(opts)
    gpu_ctx.extract(img)
    gpu_ctx.extract_keypoints(keys, has_orientation)
    assert gpu_ctx.count(0) == len(keys) and gpu_ctx.total() == len(keys)
    k, d = gpu_ctx.features(0)
    rk, rd = O.describe_keys(img, keys, has_orientation, opts)
    _assert_features_equal(k, d, rk, rd, "keypoints")
    with gpu_ctx.exact_descriptors():
        gpu_ctx.extract(img)
        gpu_ctx.extract_keypoints(keys, has_orientation)
        k, d = gpu_ctx.features(0)
    assert np.array_equal(_bits(k), _bits(rk))
    assert np.array_equal(_bits(d), _bits(rd))


def _synth_rects(w, h, n, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    k = np.zeros((n, 4), np.float32)
    k[:, 2] = np.exp(rng.uniform(np.log(4.0), np.log(300.0), n))     # width
    k[:, 3] = k[:, 2] * rng.uniform(0.3, 3.0, n).astype(np.float32)  # height
    k[:, 0] = rng.uniform(-20, w, n)                                 # left (may leave the image)
    k[:, 1] = rng.uniform(-20, h, n)
    return k


@pytest.mark.parametrize("over", [{}, {"normalized": 0}, {"octave_min": 1}])
def test_rect_keypoints_vs_oracle(gpu_ctx, over):
    """keys_have_orientation == -1: rectangle descriptors (ComputeDescriptorRECT_Kernel)."""
    img = synth_image(480, 360, 73)
    opts = default_options(**over)
    keys = _synth_rects(480, 360, 250, 74)
    gpu_ctx.set_options(opts)
    gpu_ctx.extract(img)
    gpu_ctx.extract_keypoints(keys, -1)
    k, d = gpu_ctx.features(0)
    rk, rd = O.describe_keys(img, keys, -1, opts)
    assert np.array_equal(_bits(k), _bits(keys)) and np.array_equal(_bits(rk), _bits(keys))
    _assert_features_equal(k, d, rk, rd, "rect")
    with gpu_ctx.exact_descriptors():
        gpu_ctx.extract(img)
        gpu_ctx.extract_keypoints(keys, -1)
        k, d = gpu_ctx.features(0)
    assert np.array_equal(_bits(d), _bits(rd))
    gpu_ctx.set_options(default_options())


@pytest.mark.parametrize("n,w,h,over", [(1, 1920, 1080, {}), (3, 640, 480, {}), (2, 203, 97, {}),
                                        (1, 4096, 4096, dict(octave_num=6)),
                                        (2, 517, 389, dict(dog_level_num=1)),
                                        (2, 517, 389, dict(dog_level_num=2)),
                                        (2, 517, 389, dict(dog_level_num=5)),
                                        (1, 641, 479, dict(octave_min=-1)),
                                        (1, 641, 479, dict(octave_min=1)),
                                        (2, 640, 480, dict(subpixel=0))])
def test_extrema_tile_equals_wave(gpu_ctx, n, w, h, over):
    """The tile extremum kernel (k_extrema_tile: a workgroup's 64 x 16-pixel window of every
    Gaussian plane loaded at once, DoG planes in LDS, the pre-filter and ComputeKEY per lane)
    against the wave-streaming k_extrema_wave2 (SGPU_DEBUG_EXTREMA_TILE_OFF): the same
    candidates in the same order and every key bit for bit, for 1 .. 6 DoG levels per octave."""
    imgs = synth_batch(n, w, h, 820 + w % 17)
    opts = default_options(**over)
    gpu_ctx.set_options(opts)
    try:
        gpu_ctx.set_debug_flags(gpu_ctx.DEBUG_EXTREMA_TILE_OFF)
        gpu_ctx.extract(imgs)
        ci, cf = gpu_ctx.candidates()
        ref = [gpu_ctx.features(i, descriptors=False)[0] for i in range(n)]
        gpu_ctx.set_debug_flags(gpu_ctx.DEBUG_GAUSS_TILE_ALWAYS)
        gpu_ctx.extract(imgs)
        ti, tf = gpu_ctx.candidates()
        assert len(ci) > 0 and np.array_equal(ci, ti) and np.array_equal(_bits(cf), _bits(tf))
        for i in range(n):
            k = gpu_ctx.features(i, descriptors=False)[0]
            assert k.shape == ref[i].shape and np.array_equal(_bits(k), _bits(ref[i])), i
    finally:
        gpu_ctx.set_debug_flags(0)
        gpu_ctx.set_options(default_options())


@pytest.mark.parametrize("normalized", [1, 0])
def test_dual_descriptor_vs_exact(gpu_ctx, normalized):
    """The round-4 dual-cell descriptor kernel (SGPU_DEBUG_DESC_DUAL, kept for A/B) against the
    bit-exact kernel: same keys, descriptors within L2 1e-5 (relative for -unn) -- the bound the
    shipped kernel meets (test_shipped_descriptor_vs_exact)."""
    from sift_synth import synth_batch_fast
    imgs = synth_batch_fast(4, 1280, 720, 515)
    opts = default_options(normalized=normalized)
    gpu_ctx.set_options(opts)
    try:
        gpu_ctx.set_debug_flags(gpu_ctx.DEBUG_DESC_DUAL)
        gpu_ctx.extract(imgs)
        dual = [gpu_ctx.features(i) for i in range(4)]
        gpu_ctx.set_debug_flags(gpu_ctx.DEBUG_EXACT_DESCRIPTOR)
        gpu_ctx.extract(imgs)
        exact = [gpu_ctx.features(i) for i in range(4)]
    finally:
        gpu_ctx.set_debug_flags(0)
        gpu_ctx.set_options(default_options())
    kd = np.concatenate([f[0] for f in dual])
    ke = np.concatenate([f[0] for f in exact])
    assert len(kd) > 3000 and np.array_equal(_bits(kd), _bits(ke))
    dd = np.concatenate([f[1] for f in dual]).astype(np.float64)
    de = np.concatenate([f[1] for f in exact]).astype(np.float64)
    l2 = np.linalg.norm(dd - de, axis=1)
    if not normalized:
        l2 = l2 / np.maximum(np.linalg.norm(de, axis=1), 1e-30)
    assert l2.max() < 1e-5, l2.max()


@pytest.mark.parametrize("n,w,h", [(1, 1920, 1080), (6, 640, 480)])
def test_wide_descriptor_equals_flat(gpu_ctx, n, w, h):
    """k_descriptor_wide (a workgroup of 4 waves per feature, each wave every fourth 64-pixel step
    of the window, the histograms' 64-bit integer sums merged by wave 0; the shipped form for few
    features) against k_descriptor_flat (one wave per feature): every descriptor bit for bit, in
    a single image and in a batch, normalised and -unn."""
    imgs = synth_batch(n, w, h, 710 + n)
    for opts in (default_options(), default_options(normalized=0)):
        gpu_ctx.set_options(opts)
        try:
            gpu_ctx.set_debug_flags(gpu_ctx.DEBUG_DESC_WIDE_OFF)
            gpu_ctx.extract(imgs)
            ref = [gpu_ctx.features(i) for i in range(n)]
            gpu_ctx.set_debug_flags(gpu_ctx.DEBUG_DESC_WIDE_ALWAYS)
            gpu_ctx.extract(imgs)
            got = [gpu_ctx.features(i) for i in range(n)]
            total = 0
            for (ka, da), (kb, db) in zip(ref, got):
                assert np.array_equal(_bits(ka), _bits(kb))
                assert np.array_equal(_bits(da), _bits(db))
                total += len(ka)
            assert total > 500
        finally:
            gpu_ctx.set_debug_flags(0)
            gpu_ctx.set_options(default_options())


@pytest.mark.parametrize("over", [{}, {"max_orientation": 1}, {"fixed_orientation": 1},
                                  {"circular_window": 1}, {"keep_extremum_sign": 1},
                                  {"subpixel": 0}, {"octave_min": -1}])
def test_orientation_wave_equals_quad(gpu_ctx, over):
    """Orientation one wave per candidate (the few-candidates form, SGPU_DEBUG_ORIENT_WAVE)
    against the quad form on a batch with more candidates than the wave form's automatic limit
    (so the unflagged run takes the quad form): every key bit for bit, and the oracle on one
    image."""
    imgs = synth_batch(20, 1280, 720, 610)
    opts = default_options(**over)
    gpu_ctx.set_options(opts)
    try:
        gpu_ctx.set_debug_flags(0)
        gpu_ctx.extract(imgs)
        gpu_ctx.extract(imgs)   # the candidate-count hint of this batch: above the wave limit
        assert len(gpu_ctx.candidates()[0]) > 16384
        quad = [gpu_ctx.features(i, descriptors=False)[0] for i in range(len(imgs))]
        gpu_ctx.set_debug_flags(gpu_ctx.DEBUG_ORIENT_WAVE)
        gpu_ctx.extract(imgs)
        wave = [gpu_ctx.features(i, descriptors=False)[0] for i in range(len(imgs))]
        for i, (a, b) in enumerate(zip(quad, wave)):
            assert a.shape == b.shape and np.array_equal(_bits(a), _bits(b)), i
        rk, _ = O.extract(imgs[3], opts)
        assert np.array_equal(_bits(wave[3]), _bits(rk))
    finally:
        gpu_ctx.set_debug_flags(0)
        gpu_ctx.set_options(default_options())


def test_keypoints_outside_the_image(gpu_ctx):
    """Caller keys far outside the image, with huge, tiny and negative scales: every sample box
    is clamped to the plane (the relaxed descriptor's loads stay inside it too), the results are
    the oracle's, and the context keeps working."""
    img = synth_image(320, 240, 75)
    keys = np.array([[1e6, 100, 3, 0.5], [100, -1e6, 3, 1.0], [-5e4, -5e4, 2, 2.0],
                     [3e9, 3e9, 40, 0.1], [160, 120, 1e6, 0.3], [160, 120, 1e20, 4.0],
                     [160, 120, 1e-8, 1.0], [160, 120, -3, 1.0], [319.9, 239.9, 900, 6.0],
                     [-1, -1, 0.7, 3.0], [2e9, 120, 1e7, 2.5]], np.float32)
    keys = np.concatenate([keys, _synth_keys(320, 240, 20, 76)])
    gpu_ctx.set_options(default_options())
    for ho in (True, False, -1):
        gpu_ctx.extract(img)
        gpu_ctx.extract_keypoints(keys, ho)
        k, d = gpu_ctx.features(0)
        rk, rd = O.describe_keys(img, keys, ho)
        # an empty orientation window gives NaN (0/0 in the peak interpolation) on both sides;
        # NaN payloads are not compared
        same = (_bits(k) == _bits(rk)) | (np.isnan(k) & np.isnan(rk))
        assert same.all(), ho
        ok = np.isfinite(rd).all(1)
        assert np.array_equal(np.isfinite(d).all(1), ok), ho
        assert np.linalg.norm(d[ok].astype(np.float64) - rd[ok], axis=1).max() < DESC_L2_TOL, ho
    gpu_ctx.extract(img)
    k, _ = gpu_ctx.features(0)
    assert np.array_equal(_bits(k), _bits(O.extract(img)[0]))


def test_detected_keypoints_fed_back(gpu_ctx):
    """Keys from the detector itself, described again as a caller-supplied list."""
    img = synth_image(400, 300, 73)
    gpu_ctx.set_options(default_options())
    gpu_ctx.extract(img)
    keys, _ = gpu_ctx.features(0)
    gpu_ctx.extract_keypoints(keys, True)
    k, d = gpu_ctx.features(0)
    rk, rd = O.describe_keys(img, keys, True)
    assert np.array_equal(_bits(k), _bits(keys))
    _assert_features_equal(k, d, rk, rd, "fed back")
    with gpu_ctx.exact_descriptors():
        gpu_ctx.extract(img)
        gpu_ctx.extract_keypoints(keys, True)
        k, d = gpu_ctx.features(0)
    assert np.array_equal(_bits(d), _bits(rd))


def test_keypoints_on_batch_image(gpu_ctx):
    imgs = np.stack([synth_image(320, 240, 80 + i) for i in range(3)])
    keys = _synth_keys(320, 240, 50, 83)
    gpu_ctx.set_options(default_options())
    gpu_ctx.extract(imgs)
    gpu_ctx.extract_keypoints(keys, False, image=2)
    assert [gpu_ctx.count(i) for i in range(3)] == [0, 0, 50]
    k, d = gpu_ctx.features(2)
    rk, rd = O.describe_keys(imgs[2], keys, False)
    _assert_features_equal(k, d, rk, rd, "batch image")
    with gpu_ctx.exact_descriptors():
        gpu_ctx.extract(imgs)
        gpu_ctx.extract_keypoints(keys, False, image=2)
        k, d = gpu_ctx.features(2)
    assert np.array_equal(_bits(k), _bits(rk)) and np.array_equal(_bits(d), _bits(rd))


def test_keypoint_api_replica(tmp_path):
    """SiftGPU::RunSIFT(num, keys, 1) and SetKeypointList + RunSIFT(image) through the C++ API."""
    lib = os.path.join(ROOT, "modify-sift-gpu_amd", "lib", "libsiftgpu.so")
    exe = tmp_path / "keypoint_replica"
    r = subprocess.run(["g++", "-std=c++11", "-O1", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "abi", "keypoint_replica.cpp"),
                        "-o", str(exe), "-ldl"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    img = synth_image(512, 384, 91)
    _write_pgm(tmp_path / "a.pgm", img)
    keys = _synth_keys(512, 384, 120, 92)
    keys.tofile(tmp_path / "keys.f32")
    r = subprocess.run([str(exe), lib, str(tmp_path / "a.pgm"), str(tmp_path / "keys.f32"),
                        str(len(keys)), str(tmp_path / "A.f32"), str(tmp_path / "B.f32")],
                       capture_output=True, text=True, timeout=300, env=EXACT_ENV)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    n = len(keys)
    for name, has_o in (("A.f32", True), ("B.f32", False)):
        raw = np.fromfile(tmp_path / name, np.float32)
        k, d = raw[: 4 * n].reshape(n, 4), raw[4 * n:].reshape(n, 128)
        rk, rd = O.describe_keys(img, keys, has_o)
        assert np.array_equal(_bits(k), _bits(rk)), name
        assert np.array_equal(_bits(d), _bits(rd)), name


# ---- guided matching (SiftMatchGPU::SetFeautreLocation + GetGuidedSiftMatch) -----------------
@pytest.mark.parametrize("n1,n2,hd,fd,mbm", [(1, 1, 32.0, 16.0, 1), (7, 9, 1e3, 1e3, 1),
                                             (300, 250, 32.0, 16.0, 1), (301, 257, 8.0, 1.0, 0),
                                             (1000, 1300, 32.0, 16.0, 1),
                                             (4097, 3001, 16.0, 4.0, 1)])
def test_match_guided_vs_oracle(gpu_ctx, n1, n2, hd, fd, mbm):
    q1, q2, l1, l2, H, F = synth_guided_scene(n1, n2, n1 * 3 + n2)
    for Hm, Fm in ((H, F), (H, None), (None, F)):
        a = gpu_ctx.match_guided(q1, q2, l1, l2, Hm, Fm, hdistmax=hd, fdistmax=fd, mbm=mbm)
        b = O.match_guided(q1, q2, l1, l2, Hm, Fm, hdistmax=hd, fdistmax=fd, mbm=mbm)
        assert np.array_equal(a, b), (Hm is None, Fm is None, len(a), len(b))
    if n1 >= 300:
        assert len(b) > 10


def test_match_guided_block_rule(gpu_ctx):
    """The 8-row block rule of MultiplyDescriptorG_Kernel (see test_oracle's planted case)."""
    q1, q2, l1, l2, H, F = synth_guided_scene(64, 40, 9, n_dup=0)
    self_dot = (q1.astype(np.int64) ** 2).sum(1)
    r = int(next(i for i in range(1, 64) if self_dot[i] > 262144 and i % 8))
    mate, j = r - r % 8 + (0 if r % 8 else 1), 17
    q2[j] = q1[r]
    x = H.astype(np.float64) @ np.array([l1[mate, 0], l1[mate, 1], 1.0])
    l2[j] = (x[:2] / x[2]).astype(np.float32)
    for dm, rm, mbm in ((2.0, 1.0, 0), (2.0, 1.0, 1), (0.7, 0.8, 1)):
        a = gpu_ctx.match_guided(q1, q2, l1, l2, H, F, distmax=dm, ratiomax=rm, mbm=mbm)
        b = O.match_guided(q1, q2, l1, l2, H, F, distmax=dm, ratiomax=rm, mbm=mbm)
        assert np.array_equal(a, b)
        if mbm == 0:
            assert [r, j] in a.tolist()


def test_match_guided_accept_all_is_plain_match(gpu_ctx):
    """Size-independent property at 8k x 8k: an all-accepting geometry (identity, 1e20) and no
    geometry at all both give exactly the plain matches (SiftMatch.cpp:663-677)."""
    q1, q2, l1, l2, H, F = synth_guided_scene(8192, 8000, 77)
    plain = gpu_ctx.match(q1, q2)
    assert len(plain) > 1000
    assert np.array_equal(gpu_ctx.match_guided(q1, q2, l1, l2, None, None), plain)
    eye = np.eye(3, dtype=np.float32)
    assert np.array_equal(gpu_ctx.match_guided(q1, q2, l1, l2, eye, None, hdistmax=1e20), plain)
    g = gpu_ctx.match_guided(q1, q2, l1, l2, H, F)
    assert 0 < len(g) < len(plain)


def test_guided_api_replica(tmp_path):
    """SetDescriptors + SetFeatureLocation (gap 2) + GetGuidedSiftMatch through our SiftGPU.h."""
    lib = os.path.join(ROOT, "modify-sift-gpu_amd", "lib", "libsiftgpu.so")
    exe = tmp_path / "guided_replica"
    r = subprocess.run(["g++", "-std=c++11", "-O1", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "abi", "guided_replica.cpp"),
                        "-o", str(exe), "-ldl"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    n1, n2 = 700, 650
    q1, q2, l1, l2, H, F = synth_guided_scene(n1, n2, 41)
    k1 = np.concatenate([l1, np.ones((n1, 2), np.float32)], 1)   # SiftKeypoint (x, y, s, o)
    k2 = np.concatenate([l2, np.ones((n2, 2), np.float32)], 1)
    th = np.array([0.7, 0.8, 32.0, 16.0], np.float32)
    with open(tmp_path / "scene.bin", "wb") as f:
        f.write(np.array([n1, n2], np.int32).tobytes())
        for a in (q1, q2, k1, k2, H, F, th):
            f.write(np.ascontiguousarray(a).tobytes())
        f.write(np.array([1], np.int32).tobytes())
    r = subprocess.run([str(exe), lib, str(tmp_path / "scene.bin")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    cases, cur = [], None
    for line in r.stdout.splitlines():
        if line.startswith("CASE"):
            cur = []
            cases.append(cur)
        elif line.startswith("PAIR"):
            cur.append([int(v) for v in line.split()[1:]])
    assert len(cases) == 4
    for got, (Hm, Fm) in zip(cases, ((H, F), (H, None), (None, F), (None, None))):
        want = O.match_guided(q1, q2, l1, l2, Hm, Fm)
        assert np.array_equal(np.array(got, np.int32).reshape(-1, 2), want)


@pytest.mark.parametrize("fused", [0, 1])
@pytest.mark.parametrize("bounds", [[0, 5000], [0, 1234, 1235, 3100, 5000], [0, 0, 2500, 5000]])
def test_sharded_match_equals_full(gpu_ctx, bounds, fused):
    """Sharded matcher on the device: sgpu_match_shard_begin per shard, the
    column states merged by sgpu_match_shard_end; the concatenated pairs equal sgpu_match and
    the oracle, ties between rows of different shards included."""
    d1 = synth_descriptors(5000, 7000)
    d2 = synth_descriptors(4100, 7001, base=d1, n_dup=2000)
    q1, q2 = quantize(d1), quantize(d2)
    q1[4000] = q1[17]
    q1[2600] = q1[1300]
    gpu_ctx.set_debug_flags(gpu_ctx.DEBUG_FUSED_MATCH if fused else 0)
    full = gpu_ctx.match(q1, q2)
    np.testing.assert_array_equal(full, O.match(q1, q2))
    shards = list(zip(bounds[:-1], bounds[1:]))
    begun = [gpu_ctx.match_shard_begin(q1[a:b], a, q2) for a, b in shards]
    gpu_ctx.set_debug_flags(0)
    allc = np.stack([c for _, c in begun])
    got = np.concatenate([sgpu.match_shard_end(allc, r, a) for (a, _), (r, _) in zip(shards, begun)])
    np.testing.assert_array_equal(got, full)
    # the convenience call: column states all-gathered by RCCL (one rank on this box)
    gpu_ctx.comm_init(1, 0, sgpu.comm_unique_id())
    np.testing.assert_array_equal(gpu_ctx.match_sharded(q1, 0, q2), full)


def test_float_input_compacts_caller_rows(tmp_path):
    """RunSIFT(w, h, float*, GL_LUMINANCE, GL_FLOAT) with w % 4 != 0 leaves the caller's buffer
    with its rows compacted to the truncated width (GLTexImage.cpp:994-1006), and the features
    are the oracle's for the float input."""
    lib = os.path.join(ROOT, "modify-sift-gpu_amd", "lib", "libsiftgpu.so")
    exe = tmp_path / "float_input"
    r = subprocess.run(["g++", "-std=c++11", "-O1", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "abi", "float_input_replica.cpp"),
                        "-o", str(exe), "-ldl"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    w, h = 331, 251
    img = (synth_image(w, h, 81).astype(np.float32) / 255.0).astype(np.float32)
    src = tmp_path / "img.f32"
    img.tofile(src)
    after, keys = tmp_path / "after.f32", tmp_path / "keys.f32"
    r = subprocess.run([str(exe), lib, str(src), str(w), str(h), str(after), str(keys)],
                       capture_output=True, text=True, timeout=120, env=EXACT_ENV)
    assert r.returncode == 0, r.stdout + r.stderr
    num = int([l for l in r.stdout.splitlines() if l.startswith("RESULT ")][0].split()[1])
    tw = w & ~3
    want = img.reshape(-1).copy()
    for i in range(1, h):
        want[i * tw:(i + 1) * tw] = img[i, :tw]
    assert np.array_equal(np.fromfile(after, np.float32), want)
    k = np.fromfile(keys, np.float32).reshape(-1, 4)
    rk, _ = O.extract_f32(img)
    assert num == len(rk) and np.array_equal(_bits(k), _bits(rk))
