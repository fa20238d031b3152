"""CPU tests of the oracle: the reference's own known-answer values, the deterministic math it
shares with the kernels, independent restatements of the list order and the matcher, and the
committed golden fixtures."""
import ctypes
import math
import os

import numpy as np
import pytest

import oracle_py as O
from sgpu_types import default_options
from sift_synth import (synth_image, synth_descriptors, quantize, synth_guided_scene,
                        synth_tie_scene, tie_winner)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _schedule(d=3):
    s0, sk = ctypes.c_float(), ctypes.c_float()
    sig = np.zeros(16, np.float32)
    wd = np.zeros(16, np.int32)
    O.lib().oracle_schedule(d, ctypes.byref(s0), ctypes.byref(sk), sig.ctypes.data,
                            wd.ctypes.data)
    return s0.value, sk.value, sig, wd


def test_sigma_schedule_kat():
    # SiftGPU.cpp:459-497 (comments state the default values)
    s0, sk, sig, wd = _schedule(3)
    assert np.float32(s0) == np.float32(2.0158737)
    assert np.float32(sk) == np.float32(1.5198685)
    np.testing.assert_array_equal(sig[:5], np.array([1.2262735, 1.5450078, 1.9465880, 2.4525471,
                                                     3.0900161], np.float32))
    # filter widths: initial 13, then {11, 13, 17, 21, 25} (SURVEY.md §4 KAT list)
    assert list(wd[:6]) == [13, 11, 13, 17, 21, 25]
    assert np.float32(0.02) / np.float32(3) == np.float32(0.0066666664)   # dog threshold, SiftGPU.cpp:495


def test_octave_geometry_kat():
    # PyramidCU.cpp:985: 800*600---400*300--200*150--100*75--52*37--28*18
    dims = np.zeros(48, np.int32)
    n = O.lib().oracle_geometry(800, 600, -1, dims.ctypes.data, 16, 0)
    got = [(dims[3 * i + 2], dims[3 * i + 1]) for i in range(n)]
    assert got == [(800, 600), (400, 300), (200, 150), (100, 75), (52, 37), (28, 18)]
    # 1080p with -no 4 (config C2): sum of wa*h = 2,754,000
    n = O.lib().oracle_geometry(1920, 1080, 4, dims.ctypes.data, 16, 0)
    assert n == 4
    assert sum(int(dims[3 * i + 2]) * int(dims[3 * i + 1]) for i in range(n)) == 2754000
    # 4096^2 with -no 6 (config C4): 22,364,160 px
    n = O.lib().oracle_geometry(4096, 4096, 6, dims.ctypes.data, 16, 0)
    assert sum(int(dims[3 * i + 2]) * int(dims[3 * i + 1]) for i in range(n)) == 22364160


def test_histopyramid_widths_kat():
    # PyramidCU.cpp:346-348 / 773: width 800 -> 200, 50, 13, 4, 1 (5 levels)
    w = np.zeros(16, np.int32)
    n = O.lib().oracle_hist_widths(800, 800, 600, w.ctypes.data, 16)
    assert list(w[:n]) == [200, 50, 13, 4, 1]


@pytest.mark.parametrize("name,fn,ref,lo,hi", [
    ("exp", "oracle_exp", np.exp, -100.0, 80.0),
    ("log", "oracle_log", np.log, 1e-30, 1e30),
])
def test_det_math_unary(name, fn, ref, lo, hi):
    rng = np.random.default_rng(7)
    xs = rng.uniform(lo, hi, 20000) if name == "exp" else np.exp(rng.uniform(math.log(lo), math.log(hi), 20000))
    f = getattr(O.lib(), fn)
    got = np.array([f(float(x)) for x in xs.astype(np.float32)], np.float64)
    want = ref(xs.astype(np.float32).astype(np.float64))
    ok = np.isfinite(want) & (np.abs(want) > 1e-37)
    rel = np.abs(got[ok] - want[ok]) / np.abs(want[ok])
    assert rel.max() < 4e-7, (name, rel.max())


def test_det_math_atan2_sincos():
    rng = np.random.default_rng(8)
    ys = rng.normal(size=20000).astype(np.float32)
    xs = rng.normal(size=20000).astype(np.float32)
    got = np.array([O.lib().oracle_atan2(float(y), float(x)) for y, x in zip(ys, xs)])
    want = np.arctan2(ys.astype(np.float64), xs.astype(np.float64))
    assert np.max(np.abs(got - want)) < 5e-7
    assert O.lib().oracle_atan2(0.0, -1.0) == np.float32(np.pi)
    assert O.lib().oracle_atan2(0.0, 1.0) == 0.0
    s, c = ctypes.c_float(), ctypes.c_float()
    for x in rng.uniform(-7, 7, 5000).astype(np.float32):
        O.lib().oracle_sincos(float(x), ctypes.byref(s), ctypes.byref(c))
        assert abs(s.value - math.sin(float(x))) < 3e-7
        assert abs(c.value - math.cos(float(x))) < 3e-7


def test_candidate_list_is_raster_order():
    # the histogram pyramid (ListGen_Kernel) must produce row-major order per level
    img = synth_image(320, 240, 11)
    ints, _ = O.candidates(img)
    assert len(ints) > 20
    for lv in np.unique(ints[:, 2]):
        sel = ints[ints[:, 2] == lv]
        key = sel[:, 1].astype(np.int64) * 100000 + sel[:, 0]
        assert np.all(np.diff(key) > 0)
    assert np.all(np.diff(ints[:, 2]) >= 0)   # level-major


def test_extract_deterministic_and_sane():
    img = synth_image(320, 240, 12)
    k1, d1 = O.extract(img)
    k2, d2 = O.extract(img)
    assert k1.shape[0] > 30
    np.testing.assert_array_equal(k1, k2)
    np.testing.assert_array_equal(d1, d2)
    assert np.all((k1[:, 0] >= 0) & (k1[:, 0] < 320) & (k1[:, 1] >= 0) & (k1[:, 1] < 240))
    assert np.all((k1[:, 3] >= 0) & (k1[:, 3] < 2 * np.pi + 1e-6))
    np.testing.assert_allclose(np.linalg.norm(d1, axis=1), 1.0, atol=1e-5)
    assert np.all(d1 <= 0.2 / np.float32(0.2 * np.sqrt(1) ) + 1)   # finite


def _np_top(dm, distmax, ratiomax, mod32=False):
    """Row/column decision on a dense value matrix: maximum from (0, -1, 0), second = the largest
    remaining value.  Equal maxima: the first index (ColMatch order), or with mod32 the index
    lowest mod 32, then lowest (RowMatch_Kernel's 32 strided threads + tree reduction,
    ProgramCU.cu:1803-1835)."""
    arg = np.argmax(dm, axis=1)
    mx = dm[np.arange(dm.shape[0]), arg]
    if mod32:
        cols = np.arange(dm.shape[1])
        rank = np.where(dm == mx[:, None], (cols % 32) * dm.shape[1] + cols, np.iinfo(np.int64).max)
        arg = np.argmin(rank, axis=1)
    srt = np.sort(dm, axis=1)
    sec = srt[:, -2] if dm.shape[1] > 1 else np.zeros_like(mx)
    mx, sec = np.maximum(mx, 0), np.maximum(sec, 0)
    dist = lambda v: np.arccos(np.minimum((np.minimum(v, 262144).astype(np.float32) * np.float32(2 ** -18)).astype(np.float64), 1.0)).astype(np.float32)
    d1, d2 = dist(mx), dist(sec)
    ok = (d1 < np.float32(distmax)) & (d1 < d2 * np.float32(ratiomax))
    return np.where(ok & (mx > 0), arg, -1)


def _np_pairs(r, c, mbm):
    out = [(i, j) for i, j in enumerate(r) if j >= 0 and (not mbm or c[j] == i)]
    return np.array(out, np.int32).reshape(-1, 2)


def _numpy_match(q1, q2, distmax=0.7, ratiomax=0.8, mbm=1):
    """Independent float64 restatement of RowMatch/ColMatch + GetBestMatch."""
    dot = q1.astype(np.int64) @ q2.astype(np.int64).T
    return _np_pairs(_np_top(dot, distmax, ratiomax, True), _np_top(dot.T, distmax, ratiomax), mbm)


@pytest.mark.parametrize("mbm", [1, 0])
def test_matcher_oracle_vs_numpy(mbm):
    d1 = synth_descriptors(400, 5000)
    d2 = synth_descriptors(350, 5001, base=d1, n_dup=150)
    q1, q2 = quantize(d1), quantize(d2)
    got = O.match(q1, q2, mbm=mbm)
    want = _numpy_match(q1, q2, mbm=mbm)
    assert len(want) > 50
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("distmax,ratiomax,dup", [(0.7, 0.8, 150), (0.9, 1.0, 150),
                                                  (2.0, 1.0, 0), (0.9, 0.5, 300), (2.0, 0.99, 40)])
def test_row_bound_pruning_is_exact(distmax, ratiomax, dup):
    """The pruned column side of the library's plain mutual matcher (k_match_finish /
    k_prune_set), restated with NumPy: tau = the smallest second value s with
    dist[M] >= dist[s] * ratiomax for a passing row maximum M (bisection over the distance
    table), tau_min over the passing rows; the listed columns decided over the rows whose largest
    dot reaches tau_min give the same pairs as over every row (ratiomax <= 1).  The library takes
    the lower bound cos(dist[M] / ratiomax) * 2^18 - 64 (checked one below) instead of the
    bisection; it must not exceed the bisected tau, and lie within 80 of it."""
    d1 = synth_descriptors(400, 7000 + dup)
    d2 = synth_descriptors(350, 7001 + dup, base=d1, n_dup=dup)
    q1, q2 = quantize(d1), quantize(d2)
    q2[:3] = q1[:3]                                 # exact copies: dots above 2^18
    dot = q1.astype(np.int64) @ q2.astype(np.int64).T
    rows = _np_top(dot, distmax, ratiomax, True)
    full = _np_pairs(rows, _np_top(dot.T, distmax, ratiomax), 1)
    table = np.arccos(np.minimum((np.arange(262145).astype(np.float32) * np.float32(2 ** -18))
                                 .astype(np.float64), 1.0)).astype(np.float32)
    rmax = np.maximum(dot.max(axis=1), 0)
    taus = []
    for i in np.nonzero(rows >= 0)[0]:
        dm, lo, hi = table[min(rmax[i], 262144)], 0, 262145
        while lo < hi:
            mid = (lo + hi) // 2
            if dm >= table[mid] * np.float32(ratiomax):
                hi = mid
            else:
                lo = mid + 1
        # the library's bound (k_match_finish): cos estimate less 64, checked one below
        est = int(np.floor(np.float32(np.cos(np.float32(dm / np.float32(ratiomax)))) * np.float32(262144))) - 64
        est = min(max(est, 0), 262144)
        if est > 0 and dm >= table[est - 1] * np.float32(ratiomax):
            est = 0
        assert est <= lo and lo - est <= 80, (est, lo)
        taus.append(est)
    keep = np.nonzero(rmax >= min(taus))[0] if taus else np.zeros(0, np.int64)
    cols = np.full(q2.shape[0], -1)
    if len(keep):
        c = _np_top(dot[keep].T, distmax, ratiomax)
        cols = np.where(c >= 0, keep[np.maximum(c, 0)], -1)
    pruned = _np_pairs(rows, cols, 1)
    np.testing.assert_array_equal(pruned, full)
    assert len(full) > 0
    if (distmax, ratiomax) == (0.7, 0.8):
        assert len(keep) < q1.shape[0] // 2   # planted duplicates among random rows: most pruned


def np_shard_state(q1s, row_begin, q2, distmax=0.7, ratiomax=0.8):
    """What a rank computes for rows [row_begin, row_begin + len(q1s)) of set 1 (restated with
    NumPy): its rows' decisions (RowMatch_Kernel, local) and, per set-2 row, the clamped column
    state (max dot, global set-1 row, second dot) of ColMatch_Kernel over its rows."""
    dot = q1s.astype(np.int64) @ q2.astype(np.int64).T          # [ns][n2]
    rows = _np_top(dot, distmax, ratiomax, True)
    colv = dot.T                                                  # [n2][ns]
    state = np.zeros((q2.shape[0], 3), np.int32)
    state[:, 1] = -1
    if q1s.shape[0]:
        arg = np.argmax(colv, axis=1)                             # first (lowest) row on ties
        mx = colv[np.arange(colv.shape[0]), arg]
        sec = np.sort(colv, axis=1)[:, -2] if q1s.shape[0] > 1 else np.zeros_like(mx)
        pos = mx > 0
        state[:, 0] = np.maximum(mx, 0)
        state[:, 1] = np.where(pos, arg + row_begin, -1)
        state[:, 2] = np.maximum(sec, 0)
    return rows.astype(np.int32), state


@pytest.mark.parametrize("bounds", [[0, 400], [0, 131, 132, 290, 400], [0, 0, 200, 400]])
def test_sharded_match_merge_equals_full(bounds):
    """SURVEY.md §8e sharded matcher: rows of set 1 split over ranks; every rank's local row
    decisions plus the merged column states (sgpu_match_shard_end, host code of libsiftgpu)
    give exactly the single-device pairs -- including exact ties between rows of different
    shards (duplicated rows: equal maxima -> second == max -> rejected)."""
    import sgpu
    d1 = synth_descriptors(400, 5100)
    d2 = synth_descriptors(350, 5101, base=d1, n_dup=150)
    q1, q2 = quantize(d1), quantize(d2)
    q1[300] = q1[20]            # the same row in two shards: a cross-shard tie for its column
    q1[399] = q1[3]
    full = O.match(q1, q2)
    assert len(full) > 50
    shards = list(zip(bounds[:-1], bounds[1:]))
    states = [np_shard_state(q1[a:b], a, q2) for a, b in shards]
    allc = np.stack([st for _, st in states])
    got = np.concatenate([sgpu.match_shard_end(allc, rows, a) for (a, b), (rows, _) in
                          zip(shards, states)])
    np.testing.assert_array_equal(got, full)
    # without the mutual check the column states are not needed
    got0 = np.concatenate([sgpu.match_shard_end(allc, rows, a, mbm=0) for (a, b), (rows, _) in
                           zip(shards, states)])
    np.testing.assert_array_equal(got0, O.match(q1, q2, mbm=0))


def test_matcher_ties_and_wrap():
    # duplicated rows create exact ties (second == max -> rejected); 512*d wraps past 255
    q1 = np.zeros((4, 128), np.uint8)
    q1[:, :3] = [[200, 10, 0], [0, 200, 10], [10, 0, 200], [90, 90, 90]]
    q2 = np.concatenate([q1, q1[:1]])          # row 0 appears twice -> tie for i = 0
    got = O.match(q1, q2)
    want = _numpy_match(q1, q2)
    np.testing.assert_array_equal(got, want)
    assert 0 not in got[:, 0]
    assert quantize(np.array([[0.5]], np.float32))[0, 0] == 0      # int(256.5) -> 256 -> 0


# tied column pairs: within a 32-column group, across threads, same thread (first occurrence)
TIE_COLS = [(5, 34), (40, 66), (3, 99), (31, 32), (7, 39)]


@pytest.mark.parametrize("mbm", [0, 1])
def test_matcher_tie_rules(mbm):
    q1, q2, rows = synth_tie_scene(70, 100, 21, TIE_COLS, [(60, 61)])
    got = O.match(q1, q2, distmax=2.0, ratiomax=1.5, mbm=mbm)
    np.testing.assert_array_equal(got, _numpy_match(q1, q2, 2.0, 1.5, mbm))
    if not mbm:
        pairs = dict(map(tuple, got.tolist()))
        assert [pairs[i] for i in rows] == [tie_winner(a, b) for a, b in TIE_COLS]
        assert [pairs[i] for i in rows] == [34, 66, 3, 32, 7]


def test_golden_fixtures():
    files = sorted(f for f in os.listdir(GOLDEN) if f.startswith("extract_") and f.endswith(".npz"))
    assert files, "golden fixtures missing (tests/make_golden.py)"
    for f in files:
        z = np.load(os.path.join(GOLDEN, f))
        img = z["image"]
        opts = default_options(**{k: int(v) for k, v in zip(z["opt_names"], z["opt_values"])})
        k, d = O.extract(img, opts)
        np.testing.assert_array_equal(k, z["keys"], err_msg=f)
        np.testing.assert_array_equal(d, z["desc"], err_msg=f)
    z = np.load(os.path.join(GOLDEN, "match_small.npz"))
    np.testing.assert_array_equal(O.match(z["q1"], z["q2"]), z["pairs"])


def _round_f32(fr):
    """Round an exact rational to the nearest float32 (ties to even)."""
    from fractions import Fraction
    c = np.float32(float(fr))
    best = None
    for cand in (np.nextafter(c, np.float32(-np.inf)), c, np.nextafter(c, np.float32(np.inf))):
        err = abs(Fraction(float(cand)) - fr)
        key = (err, int(cand.view(np.uint32)) & 1)
        if best is None or key < best[0]:
            best = (key, cand)
    return best[1]


def test_u8_scale_is_exact_division():
    """The Gaussian kernel's u8 ingest computes p/255.0f as q = p*(1/255), q + fma(fma(-q, 255,
    p), 1/255, q) (sift_kernels.hip u8_to_unit); exhaustively equal to the IEEE quotient."""
    from fractions import Fraction
    c = np.float32(1.0) / np.float32(255.0)
    for p in range(256):
        x = np.float32(p)
        q = np.float32(x * c)
        r = _round_f32(-Fraction(float(q)) * 255 + Fraction(float(x)))
        q2 = _round_f32(Fraction(float(r)) * Fraction(float(c)) + Fraction(float(q)))
        assert q2 == np.float32(x / np.float32(255.0)), p


# ---- guided matching (SiftMatchGPU::GetGuidedSiftMatch) ---------------------------------------
def _pass_matrix(l1, l2, H, F, hd, fd):
    return np.array([[O.guided_pass(H, F, float(a[0]), float(a[1]), float(b[0]), float(b[1]), hd, fd)
                      for b in l2] for a in l1], bool)


def _numpy_guided(q1, q2, passm, distmax=0.7, ratiomax=0.8, mbm=1):
    """Dense restatement of MultiplyDescriptorG_Kernel (ProgramCU.cu:1607-1735): a failed pair
    gets -2^18, plus its dot when its 8-row block has a passing row; rows see max(v, 0)."""
    dot = q1.astype(np.int64) @ q2.astype(np.int64).T
    n1 = q1.shape[0]
    nb = (n1 + 7) // 8
    pad = np.zeros((nb * 8, q2.shape[0]), bool)
    pad[:n1] = passm
    good = pad.reshape(nb, 8, -1).any(axis=1)[np.arange(n1) // 8]
    res = np.where(passm, dot, np.where(good, dot - 262144, -262144))
    return _np_pairs(_np_top(np.maximum(res, 0), distmax, ratiomax, True),
                     _np_top(res.T, distmax, ratiomax), mbm)


def test_guided_pass_vs_float64():
    """The geometric test against a float64 evaluation, away from the thresholds."""
    q1, q2, l1, l2, H, F = synth_guided_scene(60, 50, 11)
    H64, F64 = H.astype(np.float64), F.astype(np.float64)
    checked = 0
    for a in l1[:30]:
        for b in l2:
            x1 = np.array([a[0], a[1], 1.0])
            hx = H64 @ x1
            diff = np.abs(hx[:2] / hx[2] - b.astype(np.float64))
            fx1 = F64 @ x1
            ftx2 = F64.T @ np.array([b[0], b[1], 1.0])
            se = (b[0] * fx1[0] + b[1] * fx1[1] + fx1[2]) ** 2 / (fx1[0] ** 2 + fx1[1] ** 2 + ftx2[0] ** 2 + ftx2[1] ** 2)
            for hd, fd in ((32.0, 16.0), (4.0, 0.5), (1e20, 1e20)):
                if np.min(np.abs(diff - hd)) < 1e-2 * hd or abs(se - fd) < 1e-2 * fd:
                    continue
                want = bool(diff.max() < hd and se < fd)
                assert O.guided_pass(H, F, float(a[0]), float(a[1]), float(b[0]), float(b[1]), hd, fd) == want
                checked += 1
    assert checked > 3000


@pytest.mark.parametrize("n1,n2,hd,fd,mbm", [(300, 250, 32.0, 16.0, 1), (301, 257, 8.0, 1.0, 1),
                                             (173, 190, 32.0, 16.0, 0), (9, 7, 64.0, 1e3, 1)])
def test_guided_oracle_vs_numpy(n1, n2, hd, fd, mbm):
    q1, q2, l1, l2, H, F = synth_guided_scene(n1, n2, n1 + n2)
    passm = _pass_matrix(l1, l2, H, F, hd, fd)
    got = O.match_guided(q1, q2, l1, l2, H, F, hdistmax=hd, fdistmax=fd, mbm=mbm)
    want = _numpy_guided(q1, q2, passm, mbm=mbm)
    np.testing.assert_array_equal(got, want)
    if n1 > 100:
        assert len(want) > 10


def test_guided_block_rule_matters():
    """A failed pair whose 8-row block has a passing row keeps max(dot - 2^18, 0).  Plant one:
    set-2 feature j copies row r's descriptor (self dot > 2^18) but sits at H x1 of r's block mate,
    so only the block rule gives row r a positive value at j; with distmax 2, ratiomax 1 and one-way
    matching it is accepted, and a per-pair mask would not accept it."""
    q1, q2, l1, l2, H, F = synth_guided_scene(64, 40, 9, n_dup=0)
    self_dot = (q1.astype(np.int64) ** 2).sum(1)
    r = int(next(i for i in range(1, 64) if self_dot[i] > 262144 and i % 8))
    mate, j = r - r % 8 + (0 if r % 8 else 1), 17
    q2[j] = q1[r]
    x = H.astype(np.float64) @ np.array([l1[mate, 0], l1[mate, 1], 1.0])
    l2[j] = (x[:2] / x[2]).astype(np.float32)
    passm = _pass_matrix(l1, l2, H, F, 32.0, 16.0)
    assert passm[mate, j] and not passm[r, j]
    got = O.match_guided(q1, q2, l1, l2, H, F, distmax=2.0, ratiomax=1.0, mbm=0)
    np.testing.assert_array_equal(got, _numpy_guided(q1, q2, passm, 2.0, 1.0, 0))
    assert [r, j] in got.tolist()
    dot = q1.astype(np.int64) @ q2.astype(np.int64).T
    per_pair = _np_top(np.where(passm, dot, 0), 2.0, 1.0)
    assert per_pair[r] != j


def test_guided_defaults():
    """SiftMatch.cpp:663-677: no matrices = plain matching; an all-accepting geometry (identity,
    thresholds 1e20) gives the plain matches too."""
    q1, q2, l1, l2, H, F = synth_guided_scene(200, 180, 5)
    plain = O.match(q1, q2)
    np.testing.assert_array_equal(O.match_guided(q1, q2, l1, l2, None, None), plain)
    np.testing.assert_array_equal(O.match_guided(q1, q2, l1, l2, np.eye(3), None, hdistmax=1e20), plain)
    np.testing.assert_array_equal(O.match_guided(q1, q2, l1, l2, None, np.eye(3), fdistmax=1e20), plain)
    g = O.match_guided(q1, q2, l1, l2, H, F)
    assert 0 < len(g) < len(plain)


# ---- first octave -fo != 0 ---------------------------------------------------------------------
def test_first_octave_geometry():
    """InitPyramid (PyramidCU.cpp:89-112) + GetRequiredOctaveNum (SiftPyramid.cpp:279-285)."""
    dims = np.zeros(48, np.int32)
    def geo(w, h, fo):
        n = O.lib().oracle_geometry(w, h, -1, dims.ctypes.data, 16, fo)
        return [(int(dims[3 * i]), int(dims[3 * i + 1]), int(dims[3 * i + 2])) for i in range(n)]
    # -fo 1: 800x600 -> 400x300 first, floor(log2(300)) - 3 = 5 octaves
    assert geo(800, 600, 1) == [(400, 300, 400), (200, 150, 200), (100, 75, 100), (50, 37, 52),
                                (25, 18, 28)]
    # -fo -1: 1600x1200, 7 octaves; the width is truncated to a multiple of 4 before scaling
    g = geo(803, 600, -1)
    assert g[0] == (1600, 1200, 1600) and len(g) == 7
    assert geo(1920, 1080, 2)[0] == (480, 270, 480)


def _np_upsample(img_f, s):
    """UpsampleKernel<s> (ProgramCU.cu:225-270) on the flat buffer: independent restatement,
    a*b + c*d as fma(a, b, c*d) (fma in float64 then rounded: a*b is exact in float64)."""
    def fma(a, b, c):
        return (a.astype(np.float64) * np.float64(b) + c.astype(np.float64)).astype(np.float32)
    H, W = img_f.shape
    S = 1 << s
    flat = np.concatenate([img_f.reshape(-1), np.zeros(W + 2, np.float32)])
    out = np.zeros((H * S, W * S), np.float32)
    inv = np.float32(1.0 / S)
    for R in range(H * S):
        row, helper = R >> s, R & (S - 1)
        idx = row * W + np.arange(W)
        if helper:
            w1 = np.float32(inv * np.float32(helper))
            w2 = np.float32(1.0) - w1
            v1 = fma(flat[idx + W], w1, w2 * flat[idx])
            v2 = fma(flat[idx + W + 1], w1, w2 * flat[idx + 1])
        else:
            v1, v2 = flat[idx], flat[idx + 1]
        o = out.reshape(-1)[(W * R) * S:(W * R + W) * S].reshape(W, S)
        o[:, 0] = v1
        for i in range(1, S):
            r2 = np.float32(i) * inv
            o[:, i] = fma(v1, np.float32(1.0) - r2, v2 * r2)
    return out


@pytest.mark.parametrize("fo", [-1, -2, -3, 1, 2])
def test_first_octave_input_vs_numpy(fo):
    img = synth_image(37 * 4 + 3, 29, 5)          # width truncated to a multiple of 4
    got = O.first_octave_input(img, fo)
    f = (img[:, : img.shape[1] & ~3].astype(np.float32) / np.float32(255.0))
    if fo < 0:
        want = _np_upsample(f, -fo)
    else:
        h2, w2 = f.shape[0] >> fo, f.shape[1] >> fo
        wa = (w2 + 3) // 4 * 4
        cols = np.minimum(np.arange(wa) << fo, f.shape[1] - 1)
        want = f[(np.arange(h2) << fo)][:, cols]
    np.testing.assert_array_equal(got, want)


def test_first_octave_minus_two_runs_to_zero_features():
    """-fo -2 makes the reference's initial sigma 0 (SiftGPU.cpp:446-452) and CreateFilterKernel's
    taps NaN (ProgramCU.cu:391-398).  The NaN pyramid passes every ComputeKEY test (all NaN
    comparisons are false), so every interior pixel is listed, and no keypoint gets an
    orientation (no histogram bin exceeds 0.8 * NaN): RunSIFT succeeds with 0 features."""
    k, d = O.extract(synth_image(64, 48, 1), default_options(octave_min=-2))
    assert k.shape == (0, 4) and d.shape == (0, 128)


def test_float_ingest_equals_u8_ingest():
    """u8 p and float p/255.0f are the same input (GLTexImage.cpp:818)."""
    img = synth_image(160, 120, 4)
    k8, d8 = O.extract(img)
    kf, df = O.extract_f32(img.astype(np.float32) / np.float32(255.0))
    np.testing.assert_array_equal(k8, kf)
    np.testing.assert_array_equal(d8, df)


def test_color_formula_kat():
    """(19595 r + 38470 g + 7471 b) / (65535 * 255): the weights sum to 65536, so white is
    65536/65535 (slightly above 1) as in the reference; BGR swaps r and b."""
    px = np.array([[[255, 255, 255, 0], [255, 0, 0, 0], [0, 0, 255, 0], [10, 20, 30, 0]]], np.uint8)
    g = O.gray_from_color(px, "rgba")
    assert g[0, 0] == np.float32(65536 * 255) / np.float32(65535.0 * 255.0) > 1.0
    assert g[0, 1] == np.float32(19595 * 255) / np.float32(65535.0 * 255.0)
    assert O.gray_from_color(px, "bgra")[0, 2] == g[0, 1]


# ---- feature-count limiting (-tc / -tc2 / -tc3) and the first-octave plan ----------------------

def _limit_py(cnt, T, method, list_stage):
    """SiftPyramid::LimitFeatureCount (SiftPyramid.cpp:219-260), with the level skip of
    PyramidCU::GenerateFeatureList (PyramidCU.cpp:829-853) first when list_stage."""
    cnt = list(cnt)
    nl = len(cnt)
    if list_stage and method != 0:
        total = 0
        order = range(nl - 1, -1, -1) if method == 1 else range(nl)
        for l in order:
            if total > T:
                cnt[l] = 0
            else:
                total += cnt[l]
    num = sum(cnt)
    if method == 2:
        i, kept = 0, 0
        while kept < T and i < nl:
            kept += cnt[i]
            i += 1
        for l in range(i, nl):
            cnt[l] = 0
    else:
        i = 0
        while i < nl and num - cnt[i] > T:
            num -= cnt[i]
            cnt[i] = 0
            i += 1
    return cnt


@pytest.mark.parametrize("method", [0, 1, 2])
@pytest.mark.parametrize("T", [30, 200, 600])
def test_feature_limit_keeps_whole_levels(method, T):
    """-tc only removes whole levels: the limited run equals the full run restricted to the
    levels the reference's two LimitFeatureCount passes keep (on the keypoint counts, then on
    the oriented feature counts)."""
    img = synth_image(320, 240, 21)
    d = 3
    full_k, _ = O.extract(img)
    _, lvl = O.features_oct(img)
    ci, _ = O.candidates(img)
    nl = int(max(ci[:, 2].max(), lvl.max())) + 1
    nl = (nl + d - 1) // d * d
    cand = np.bincount(ci[:, 2], minlength=nl)
    feat = np.bincount(lvl, minlength=nl)
    keep1 = _limit_py(cand, T, method, True)
    feat1 = [f if k else 0 for f, k in zip(feat, keep1)]
    keep = _limit_py(feat1, T, method, False)
    want = full_k[np.isin(lvl, [l for l in range(nl) if keep[l]])]
    got, _ = O.extract(img, default_options(feature_count_threshold=T, truncate_method=method))
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    if T < len(full_k):
        assert len(got) < len(full_k)


@pytest.mark.parametrize("w,h,fo,maxd,prep,want", [
    (1920, 1080, 0, 13200, 1, (0, 1920, 1080, 0)),
    (1921, 1080, 1, 13200, 1, (1, 960, 540, 0)),       # -prep: sampled, then octave 0
    (1012, 301, 2, 13200, 1, (2, 252, 75, 0)),         # width truncated after sampling
    (1012, 301, 2, 13200, 0, (0, 1012, 301, 2)),       # -noprep: SampleImageD from the input
    (4096, 4096, 0, 2560, 1, (0, 4096, 4096, 1)),      # -maxd raises octave_min
    (4096, 3000, -1, 4000, 1, (0, 4096, 3000, 1)),     # 8192 > 4000 -> -1 -> 0 -> 1
    (20000, 100, 1, 13200, 0, (1, 10000, 50, 0)),      # beyond _texMaxDim: sampled even -noprep
    (640, 480, -5, 13200, 1, (0, 640, 480, -3)),       # clamped to -3 (PyramidCU.cpp:106-107)
])
def test_first_octave_plan(w, h, fo, maxd, prep, want):
    """sgp::plan_input: GLTexInput::SetImageData (GLTexImage.cpp:928-960) + PyramidCU::
    InitPyramid (PyramidCU.cpp:89-135) as (ds, image w, image h, octave_min)."""
    out = np.zeros(4, np.int32)
    O.lib().oracle_plan(w, h, fo, maxd, prep, out.ctypes.data)
    assert tuple(out) == want


def test_cpu_match_baseline_row_side():
    """bench.py's C5 CPU baseline (oracle_bench_match_rows): exact u8 dots with the reference's
    running top-2 from (0, -1, 0) (ProgramCU.cu:1785-1841), checked through its checksum."""
    d1 = quantize(synth_descriptors(300, 77))
    d2 = quantize(synth_descriptors(500, 78, base=d1, n_dup=100))
    rows = 200
    cs = ctypes.c_longlong(0)
    a = np.ascontiguousarray(d1)
    b = np.ascontiguousarray(d2)
    secs = O.lib().oracle_bench_match_rows(a.ctypes.data, rows, b.ctypes.data, b.shape[0], 2,
                                           ctypes.byref(cs))
    assert secs >= 0.0
    dots = a[:rows].astype(np.int64) @ b.astype(np.int64).T
    want = 0
    for i in range(rows):
        best, second, idx = 0, 0, -1
        for j, v in enumerate(dots[i]):
            if v > best:
                second, best, idx = best, v, j
            elif v > second:
                second = v
        want += idx + (int(second) & 1)
    assert cs.value == want


@pytest.mark.parametrize("n1,n2,dup", [(1, 300, 0), (300, 1, 0), (700, 900, 300), (2000, 1500, 800)])
def test_match_mt_equals_match(n1, n2, dup):
    """The threaded oracle matcher (C5-size tests) makes the single loop's decisions: same folds
    per row and per column, in the same order."""
    d1 = synth_descriptors(n1, 3 * n1 + n2)
    d2 = synth_descriptors(n2, 3 * n2 + n1, base=d1, n_dup=min(dup, n1, n2))
    q1, q2 = quantize(d1), quantize(d2)
    for args in ((0.7, 0.8, 1), (0.7, 0.8, 0), (2.0, 1.5, 1), (2.0, 1.5, 0)):
        assert np.array_equal(O.match_mt(q1, q2, *args, threads=4), O.match(q1, q2, *args))
    q1t, q2t, _ = synth_tie_scene(300, 900, 5, [(200, 129), (130, 2), (40, 33)], [(60, 61)])
    for mbm in (0, 1):
        assert np.array_equal(O.match_mt(q1t, q2t, 2.0, 1.5, mbm, threads=3),
                              O.match(q1t, q2t, 2.0, 1.5, mbm))
