"""ctypes binding of the CPU oracle (oracle/liboracle.so) -- test infrastructure only."""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "modify-sift-gpu_amd", "python"))

from sgpu_types import SgpuOptions, default_options  # noqa: E402

_LIB = None
_PATH = os.path.join(ROOT, "oracle", "liboracle.so")


def use_library(path):
    """Bind a different build of the oracle (e.g. oracle/liboracle_perturb.so, the CUDA-like
    transcendental errors of tests/parity_trust.py) for the calls that follow."""
    global _LIB, _PATH
    _LIB, _PATH = None, path


def lib():
    global _LIB
    if _LIB is None:
        path = _PATH
        if not os.path.exists(path):
            subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(path)
        P = ctypes.POINTER
        L.oracle_extract.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     P(SgpuOptions), ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_int, P(ctypes.c_int)]
        L.oracle_gaussian.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      P(SgpuOptions), ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_int]
        L.oracle_candidates.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        P(SgpuOptions), ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int, P(ctypes.c_int)]
        L.oracle_features_oct.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, P(SgpuOptions), ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_int, P(ctypes.c_int)]
        L.oracle_describe_keys.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, P(SgpuOptions), ctypes.c_void_p,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p]
        L.oracle_match.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                   ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_void_p]
        L.oracle_match_mt.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        L.oracle_match_guided.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
                                          ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.oracle_guided_pass.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_float] * 6
        L.oracle_first_octave_input.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 4 + [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        L.oracle_extract_f32.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_int, ctypes.c_void_p]
        L.oracle_plan.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p]
        L.oracle_save_sift.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_match_distance.argtypes = [ctypes.c_int]
        L.oracle_match_distance.restype = ctypes.c_float
        L.oracle_schedule.argtypes = [ctypes.c_int, P(ctypes.c_float), P(ctypes.c_float),
                                      ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_geometry.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_int, ctypes.c_int]
        L.oracle_hist_widths.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_int]
        L.oracle_exp.argtypes = [ctypes.c_float]
        L.oracle_exp.restype = ctypes.c_float
        L.oracle_log.argtypes = [ctypes.c_float]
        L.oracle_log.restype = ctypes.c_float
        L.oracle_atan2.argtypes = [ctypes.c_float, ctypes.c_float]
        L.oracle_atan2.restype = ctypes.c_float
        L.oracle_sincos.argtypes = [ctypes.c_float, P(ctypes.c_float), P(ctypes.c_float)]
        L.oracle_bench_extract.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, P(SgpuOptions),
                                           ctypes.c_int, P(ctypes.c_longlong)]
        L.oracle_bench_extract.restype = ctypes.c_double
        L.oracle_bench_match_rows.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_int, ctypes.c_int,
                                              ctypes.POINTER(ctypes.c_longlong)]
        L.oracle_bench_match_rows.restype = ctypes.c_double
        _LIB = L
    return _LIB


def _img(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    return img, img.ctypes.data


def extract(img: np.ndarray, opts: SgpuOptions | None = None):
    """Returns (keys [n,4], desc [n,128]) for a gray u8 image [h, w]."""
    opts = opts or default_options()
    img, p = _img(img)
    h, w = img.shape
    n = ctypes.c_int(0)
    lib().oracle_extract(p, w, h, w, ctypes.byref(opts), None, None, 0, ctypes.byref(n))
    keys = np.zeros((max(n.value, 1), 4), np.float32)
    desc = np.zeros((max(n.value, 1), 128), np.float32)
    rc = lib().oracle_extract(p, w, h, w, ctypes.byref(opts), keys.ctypes.data,
                              desc.ctypes.data, n.value, ctypes.byref(n))
    assert rc == 0, rc
    return keys[:n.value], desc[:n.value]


def extract_f32(img: np.ndarray, opts: SgpuOptions | None = None):
    """Float luminance input [h, w] (the GL_FLOAT / converted-RGB ingest path)."""
    opts = opts or default_options()
    img = np.ascontiguousarray(img, np.float32)
    h, w = img.shape
    n = ctypes.c_int(0)
    lib().oracle_extract_f32(img.ctypes.data, w, h, w, ctypes.byref(opts), None, None, 0,
                             ctypes.byref(n))
    keys = np.zeros((max(n.value, 1), 4), np.float32)
    desc = np.zeros((max(n.value, 1), 128), np.float32)
    rc = lib().oracle_extract_f32(img.ctypes.data, w, h, w, ctypes.byref(opts), keys.ctypes.data,
                                  desc.ctypes.data, n.value, ctypes.byref(n))
    assert rc == 0, rc
    return keys[:n.value], desc[:n.value]


def gray_from_color(img: np.ndarray, fmt: str) -> np.ndarray:
    """DownSamplePixelDataI2F<u8> for GL_RGB/RGBA/BGR/BGRA (GLTexImage.cpp:834-858): the exact
    integer numerator over 65535 * 255 as one float division; width truncated to 4."""
    h, w, c = img.shape
    tw = w & ~3
    p = img[:, :tw].astype(np.int64)
    r, g, b = (p[..., 0], p[..., 1], p[..., 2]) if fmt in ("rgb", "rgba") else (p[..., 2], p[..., 1], p[..., 0])
    num = (19595 * r + 38470 * g + 7471 * b).astype(np.float32)
    return num / np.float32(65535.0 * 255.0)


def gaussian(img, octave, level, opts=None):
    opts = opts or default_options()
    img, p = _img(img)
    h, w = img.shape
    cap = (w + 4) * h * (1 << (2 * max(0, -opts.octave_min)))
    out = np.zeros(cap, np.float32)
    n = lib().oracle_gaussian(p, w, h, w, ctypes.byref(opts), octave, level, out.ctypes.data, cap)
    assert n > 0, n
    return out[:n]


def candidates(img, opts=None):
    opts = opts or default_options()
    img, p = _img(img)
    h, w = img.shape
    n = ctypes.c_int(0)
    lib().oracle_candidates(p, w, h, w, ctypes.byref(opts), None, None, 0, ctypes.byref(n))
    ints = np.zeros((max(n.value, 1), 4), np.int32)
    fl = np.zeros((max(n.value, 1), 4), np.float32)
    lib().oracle_candidates(p, w, h, w, ctypes.byref(opts), ints.ctypes.data, fl.ctypes.data,
                            n.value, ctypes.byref(n))
    return ints[:n.value], fl[:n.value]


def features_oct(img, opts=None):
    """Features in octave coordinates [n, 4] (x, y, s, o) and their level ids (octave*d + j)."""
    opts = opts or default_options()
    img, p = _img(img)
    h, w = img.shape
    n = ctypes.c_int(0)
    lib().oracle_features_oct(p, w, h, w, ctypes.byref(opts), None, None, 0, ctypes.byref(n))
    feat = np.zeros((max(n.value, 1), 4), np.float32)
    lvl = np.zeros(max(n.value, 1), np.int32)
    lib().oracle_features_oct(p, w, h, w, ctypes.byref(opts), feat.ctypes.data, lvl.ctypes.data,
                              n.value, ctypes.byref(n))
    return feat[:n.value], lvl[:n.value]


def describe_keys(img, keys, has_orientation=True, opts=None):
    """Reference RunSIFT(num, keys, keys_have_orientation): (keys_out [n,4], desc [n,128])."""
    opts = opts or default_options()
    img, p = _img(img)
    h, w = img.shape
    k = np.ascontiguousarray(keys, np.float32).reshape(-1, 4)
    ko = np.zeros_like(k)
    d = np.zeros((len(k), 128), np.float32)
    ho = -1 if has_orientation == -1 else (1 if has_orientation else 0)
    lib().oracle_describe_keys(p, w, h, w, ctypes.byref(opts), k.ctypes.data, len(k), ho,
                               ko.ctypes.data, d.ctypes.data)
    return ko, d


def match(d1: np.ndarray, d2: np.ndarray, distmax=0.7, ratiomax=0.8, mbm=1, max_match=None):
    d1 = np.ascontiguousarray(d1, np.uint8)
    d2 = np.ascontiguousarray(d2, np.uint8)
    n1, n2 = d1.shape[0], d2.shape[0]
    max_match = n1 if max_match is None else max_match
    out = np.zeros((max(max_match, 1), 2), np.int32)
    m = lib().oracle_match(d1.ctypes.data, n1, d2.ctypes.data, n2, distmax, ratiomax, mbm,
                           max_match, out.ctypes.data)
    return out[:m]


def match_mt(d1: np.ndarray, d2: np.ndarray, distmax=0.7, ratiomax=0.8, mbm=1, max_match=None,
             threads=None):
    """match() with the dot products split over OpenMP threads (the same folds in the same
    order per row and per column): for the benched C5 size."""
    d1 = np.ascontiguousarray(d1, np.uint8)
    d2 = np.ascontiguousarray(d2, np.uint8)
    n1, n2 = d1.shape[0], d2.shape[0]
    max_match = n1 if max_match is None else max_match
    threads = threads or max(1, min(16, os.cpu_count() or 1))
    out = np.zeros((max(max_match, 1), 2), np.int32)
    m = lib().oracle_match_mt(d1.ctypes.data, n1, d2.ctypes.data, n2, distmax, ratiomax, mbm,
                              max_match, out.ctypes.data, threads)
    return out[:m]


def first_octave_input(img, fo):
    """The resampled first-octave input of -fo != 0 (SampleImageD / UpsampleKernel)."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    cap = (w << 3) * (h << 3) + 16
    out = np.zeros(cap, np.float32)
    dims = np.zeros(2, np.int32)
    n = lib().oracle_first_octave_input(img.ctypes.data, w, h, w, fo, out.ctypes.data, cap,
                                        dims.ctypes.data)
    assert n >= 0
    return out[:n].reshape(dims[1], dims[0])


_IDENTITY = np.eye(3, dtype=np.float32)


def match_guided(d1, d2, loc1, loc2, H=None, F=None, distmax=0.7, ratiomax=0.8, hdistmax=32.0,
                 fdistmax=16.0, mbm=1, max_match=None):
    """SiftMatchGPU::GetGuidedSiftMatch (SiftMatch.cpp:663-677) including its NULL-matrix
    defaults; None/None is plain matching."""
    if H is None and F is None:
        return match(d1, d2, distmax, ratiomax, mbm, max_match)
    hdistmax = hdistmax if H is not None else 1.0e20
    fdistmax = fdistmax if F is not None else 1.0e20
    H = np.ascontiguousarray(_IDENTITY if H is None else H, np.float32)
    F = np.ascontiguousarray(_IDENTITY if F is None else F, np.float32)
    d1 = np.ascontiguousarray(d1, np.uint8)
    d2 = np.ascontiguousarray(d2, np.uint8)
    l1 = np.ascontiguousarray(loc1, np.float32)
    l2 = np.ascontiguousarray(loc2, np.float32)
    n1, n2 = d1.shape[0], d2.shape[0]
    max_match = n1 if max_match is None else max_match
    out = np.zeros((max(max_match, 1), 2), np.int32)
    m = lib().oracle_match_guided(d1.ctypes.data, n1, d2.ctypes.data, n2, l1.ctypes.data,
                                  l2.ctypes.data, H.ctypes.data, F.ctypes.data, distmax, ratiomax,
                                  hdistmax, fdistmax, mbm, max_match, out.ctypes.data)
    return out[:m]


def guided_pass(H, F, x1, y1, x2, y2, hdistmax, fdistmax):
    H = np.ascontiguousarray(H, np.float32)
    F = np.ascontiguousarray(F, np.float32)
    return bool(lib().oracle_guided_pass(H.ctypes.data, F.ctypes.data, x1, y1, x2, y2,
                                         hdistmax, fdistmax))


def bench_extract(images: np.ndarray, opts=None, threads=1):
    opts = opts or default_options()
    images = np.ascontiguousarray(images, np.uint8)
    n, h, w = images.shape
    feats = ctypes.c_longlong(0)
    secs = lib().oracle_bench_extract(images.ctypes.data, n, w, h, w, ctypes.byref(opts),
                                      threads, ctypes.byref(feats))
    return secs, feats.value


def bench_match_rows(d1: np.ndarray, rows: int, d2: np.ndarray, threads=1):
    """Wall seconds of the matcher's row side (exact u8 dots + running top-2) for the first
    `rows` rows of d1 against all of d2, row-blocked over `threads` OpenMP threads."""
    d1 = np.ascontiguousarray(d1, np.uint8)
    d2 = np.ascontiguousarray(d2, np.uint8)
    cs = ctypes.c_longlong(0)
    secs = lib().oracle_bench_match_rows(d1.ctypes.data, rows, d2.ctypes.data, d2.shape[0],
                                         threads, ctypes.byref(cs))
    return secs


def save_sift(path, keys, desc, binary=False, normalized=True):
    """SiftPyramid::SaveSIFT's output for (keys [n,4], desc [n,128] or None) -- the
    reference's writer restated in oracle/sift_oracle.cpp (oracle_save_sift)."""
    k = np.ascontiguousarray(keys, np.float32)
    d = None if desc is None else np.ascontiguousarray(desc, np.float32)
    lib().oracle_save_sift(str(path).encode(), k.ctypes.data, None if d is None else d.ctypes.data,
                           len(k), int(binary), int(normalized), int(d is not None))


def read_sift(path, binary=False):
    """Parse a SaveSIFT file (the layout save_sift writes): keys [n, 4] as stored (y, x, scale,
    orientation) and the descriptors -- ASCII: [n, 128] int64 of floor(0.5 + 512 d) (-unn
    files are not parsed here); binary: [n, 128] float32."""
    if binary:
        raw = np.fromfile(path, np.uint8)
        n, dim = np.frombuffer(raw[:8].tobytes(), np.int32)
        rec = np.frombuffer(raw[8:].tobytes(), np.float32).reshape(n, 4 + dim)
        return rec[:, :4].copy(), rec[:, 4:].copy()
    with open(path) as f:
        tok = f.read().split()
    n, dim = int(tok[0]), int(tok[1])
    vals = tok[2:]
    keys = np.array([[float(v) for v in vals[i * (4 + dim):i * (4 + dim) + 4]] for i in range(n)])
    desc = np.array([[int(v) for v in vals[i * (4 + dim) + 4:(i + 1) * (4 + dim)]]
                     for i in range(n)], np.int64).reshape(n, dim)
    return keys, desc
