"""ctypes binding of the C ABI (include/sgpu.h) of lib/libsiftgpu.so.

The binding fails loudly when the library or a usable GPU is missing: there is no CPU path.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import subprocess

import numpy as np

from sgpu_types import SgpuOptions, default_options

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# SGPU_LIB_PATH: an experiment build of the same library (tests/build_variant.sh); default: the
# in-tree product build
LIB_PATH = os.environ.get("SGPU_LIB_PATH") or os.path.join(PKG, "lib", "libsiftgpu.so")

SGPU_OK, SGPU_EINVAL, SGPU_ENODEV, SGPU_ENOMEM, SGPU_ERANGE = 0, -1, -2, -3, -4
SGPU_INPUT_HOST, SGPU_INPUT_DEVICE, SGPU_INPUT_STAGED = 0, 1, 2

# every extern "C" symbol include/sgpu.h declares (tests check the library exports them all)
C_API = [
    "sgpu_default_options", "sgpu_parse_args", "sgpu_ctx_create", "sgpu_ctx_destroy",
    "sgpu_ctx_set_options", "sgpu_last_error", "sgpu_device_count", "sgpu_extract",
    "sgpu_extract_f32", "sgpu_stage_input", "sgpu_feature_count", "sgpu_feature_total", "sgpu_copy_features",
    "sgpu_device_features", "sgpu_match", "sgpu_quantize_descriptors", "sgpu_last_timing",
    "sgpu_debug_geometry", "sgpu_debug_gaussian", "sgpu_debug_candidates",
    "sgpu_debug_set_flags", "sgpu_comm_unique_id", "sgpu_comm_init", "sgpu_comm_allgather_i32",
    "sgpu_comm_allreduce_f64", "sgpu_extract_keypoints", "sgpu_match_guided", "sgpu_extract_color",
    "sgpu_match_shard_begin", "sgpu_match_shard_end", "sgpu_match_sharded",
    "sgpu_extract_stream", "sgpu_host_alloc", "sgpu_host_free", "sgpu_reserve",
    "sgpu_debug_alloc_count", "sgpu_last_pyramid_launches", "sgpu_set_stage_timing",
    "sgpu_set_host_output", "sgpu_debug_set_schedule", "sgpu_debug_set_match_prune",
]

_LIB = None


def build():
    subprocess.check_call(["make", "-C", PKG, "-j8"])


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: build it with `make -C {PKG}`")
        L = ctypes.CDLL(LIB_PATH)
        P, c = ctypes.POINTER, ctypes
        vp = c.c_void_p
        L.sgpu_default_options.argtypes = [P(SgpuOptions)]
        L.sgpu_parse_args.argtypes = [P(SgpuOptions), c.c_int, P(c.c_char_p), P(c.c_int)]
        L.sgpu_ctx_create.argtypes = [c.c_int, P(SgpuOptions), P(vp)]
        L.sgpu_ctx_destroy.argtypes = [vp]
        L.sgpu_ctx_set_options.argtypes = [vp, P(SgpuOptions)]
        L.sgpu_last_error.argtypes = [vp]
        L.sgpu_last_error.restype = c.c_char_p
        L.sgpu_extract.argtypes = [vp, vp, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int]
        L.sgpu_stage_input.argtypes = [vp, vp, c.c_int, c.c_int, c.c_int, c.c_int]
        L.sgpu_reserve.argtypes = [vp, c.c_int, c.c_int, c.c_int, c.c_int]
        L.sgpu_debug_alloc_count.argtypes = []
        L.sgpu_debug_alloc_count.restype = c.c_longlong
        L.sgpu_last_pyramid_launches.argtypes = [vp, P(c.c_int)]
        L.sgpu_set_stage_timing.argtypes = [vp, c.c_int]
        L.sgpu_set_host_output.argtypes = [vp, vp, vp, c.c_int]
        L.sgpu_extract_f32.argtypes = [vp, vp, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int]
        L.sgpu_feature_count.argtypes = [vp, c.c_int]
        L.sgpu_feature_total.argtypes = [vp]
        L.sgpu_feature_total.restype = c.c_int64
        L.sgpu_copy_features.argtypes = [vp, c.c_int, vp, vp]
        L.sgpu_device_features.argtypes = [vp, P(vp), P(vp), P(vp)]
        L.sgpu_match.argtypes = [vp, vp, c.c_int, vp, c.c_int, c.c_float, c.c_float, c.c_int,
                                 c.c_int, vp, c.c_int]
        L.sgpu_match_guided.argtypes = [vp, vp, c.c_int, vp, c.c_int, vp, vp, vp, vp, c.c_float,
                                        c.c_float, c.c_float, c.c_float, c.c_int, c.c_int, vp,
                                        c.c_int]
        L.sgpu_extract_color.argtypes = [vp, vp, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int]
        L.sgpu_quantize_descriptors.argtypes = [vp, c.c_size_t, vp]
        L.sgpu_last_timing.argtypes = [vp, vp, c.c_int]
        L.sgpu_debug_set_flags.argtypes = [vp, c.c_int]
        L.sgpu_debug_set_schedule.argtypes = [vp, c.c_int, c.c_int]
        L.sgpu_debug_set_match_prune.argtypes = [vp, c.c_int]
        L.sgpu_debug_geometry.argtypes = [vp, P(c.c_int), vp, c.c_int]
        L.sgpu_debug_gaussian.argtypes = [vp, c.c_int, c.c_int, c.c_int, vp]
        L.sgpu_debug_candidates.argtypes = [vp, vp, vp, c.c_int, P(c.c_int)]
        L.sgpu_extract_keypoints.argtypes = [vp, c.c_int, vp, c.c_int, c.c_int]
        L.sgpu_comm_unique_id.argtypes = [vp, c.c_int]
        L.sgpu_comm_init.argtypes = [vp, c.c_int, c.c_int, vp, c.c_int]
        L.sgpu_comm_allgather_i32.argtypes = [vp, vp, c.c_int, vp]
        L.sgpu_comm_allreduce_f64.argtypes = [vp, vp, c.c_int, c.c_int]
        L.sgpu_match_shard_begin.argtypes = [vp, vp, c.c_int, c.c_int, vp, c.c_int, c.c_float,
                                             c.c_float, c.c_int, vp, vp, c.c_int]
        L.sgpu_match_shard_end.argtypes = [vp, c.c_int, c.c_int, vp, c.c_int, c.c_int, c.c_float,
                                           c.c_float, c.c_int, c.c_int, vp]
        L.sgpu_match_sharded.argtypes = [vp, vp, c.c_int, c.c_int, vp, c.c_int, c.c_float,
                                         c.c_float, c.c_int, c.c_int, vp, c.c_int]
        L.sgpu_extract_stream.argtypes = [vp, P(vp), c.c_int, c.c_int, c.c_int, c.c_int, c.c_int,
                                          vp, vp, c.c_int64, vp]
        L.sgpu_host_alloc.argtypes = [c.c_size_t]
        L.sgpu_host_alloc.restype = vp
        L.sgpu_host_free.argtypes = [vp]
        _LIB = L
    return _LIB


class PinnedArray:
    """A numpy view of page-locked host memory (sgpu_host_alloc): the form of host buffer whose
    copies overlap the kernels in sgpu_extract_stream.  Freed with .free() or on collection."""

    def __init__(self, shape, dtype):
        dt = np.dtype(dtype)
        n = int(np.prod(shape)) * dt.itemsize
        self._p = lib().sgpu_host_alloc(max(n, 1))
        if not self._p:
            raise MemoryError(f"sgpu_host_alloc({n}) failed")
        buf = (ctypes.c_uint8 * max(n, 1)).from_address(self._p)
        self.array = np.frombuffer(buf, dtype=dt, count=int(np.prod(shape))).reshape(shape)

    def free(self):
        if self._p:
            self.array = None
            lib().sgpu_host_free(self._p)
            self._p = None

    def __del__(self):
        self.free()


def match_shard_end(col_best_all: np.ndarray, row_match: np.ndarray, row_begin: int,
                    distmax=0.7, ratiomax=0.8, mbm=1, max_match=None) -> np.ndarray:
    """Host-side merge of the shards' column states ([nshards][n2][3] int32, rank order) plus
    this shard's row decisions -> this shard's pairs {global i, j} (sgpu_match_shard_end; no
    device involved)."""
    cb = np.ascontiguousarray(col_best_all, np.int32)
    if cb.ndim == 2:
        cb = cb[None]
    rm = np.ascontiguousarray(row_match, np.int32)
    ns, n2 = len(rm), cb.shape[1]
    max_match = ns if max_match is None else max_match
    out = np.zeros((max(max_match, 1), 2), np.int32)
    m = lib().sgpu_match_shard_end(cb.ctypes.data, cb.shape[0], n2, rm.ctypes.data, ns,
                                   row_begin, distmax, ratiomax, mbm, max_match, out.ctypes.data)
    if m < 0:
        raise RuntimeError(f"sgpu_match_shard_end failed ({m})")
    return out[:m].copy()


def comm_unique_id() -> bytes:
    """A fresh RCCL communicator id (rank 0 creates it, the launcher distributes it)."""
    buf = (ctypes.c_uint8 * 128)()
    rc = lib().sgpu_comm_unique_id(buf, 128)
    if rc != SGPU_OK:
        raise RuntimeError(f"sgpu_comm_unique_id failed ({rc})")
    return bytes(buf)


def device_count() -> int:
    return lib().sgpu_device_count()


def quantize(desc: np.ndarray) -> np.ndarray:
    d = np.ascontiguousarray(desc, np.float32)
    out = np.empty(d.shape, np.uint8)
    lib().sgpu_quantize_descriptors(d.ctypes.data, d.size, out.ctypes.data)
    return out


class SiftContext:
    """One HIP device context (sgpu_ctx)."""

    def __init__(self, device: int = 0, opts: SgpuOptions | None = None):
        self.opts = opts or default_options()
        self.device = device
        self._ctx = ctypes.c_void_p()
        rc = lib().sgpu_ctx_create(device, ctypes.byref(self.opts), ctypes.byref(self._ctx))
        if rc != SGPU_OK:
            raise RuntimeError(f"sgpu_ctx_create(device={device}) failed with {rc}: "
                               "no usable gfx950 device")
        self.batch = 0

    def close(self):
        if self._ctx:
            lib().sgpu_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != SGPU_OK:
            raise RuntimeError(f"{what} failed ({rc}): {lib().sgpu_last_error(self._ctx).decode()}")

    def set_options(self, opts: SgpuOptions):
        self.opts = opts
        self._check(lib().sgpu_ctx_set_options(self._ctx, ctypes.byref(opts)), "set_options")

    def reserve(self, n: int, w: int, h: int):
        """Allocate every buffer an extract of n u8 images of w x h needs (sgpu_reserve, the
        SiftGPU::AllocatePyramid entry point); drops the current batch and staged input."""
        self._check(lib().sgpu_reserve(self._ctx, n, w, h, w), "sgpu_reserve")
        self._staged = None
        self.batch = 0
        return self

    def pyramid_launches(self):
        """(kernel launches, level filters) of the last extract's Gaussian pyramid."""
        f = ctypes.c_int(0)
        n = lib().sgpu_last_pyramid_launches(self._ctx, ctypes.byref(f))
        if n < 0:
            raise RuntimeError("sgpu_last_pyramid_launches: no extract")
        return int(n), int(f.value)

    def set_stage_timing(self, on: bool):
        """Per-stage HIP events on/off (sgpu_set_stage_timing; the reference's _timingS)."""
        self._check(lib().sgpu_set_stage_timing(self._ctx, int(bool(on))), "sgpu_set_stage_timing")

    @staticmethod
    def alloc_count() -> int:
        """Device + pinned allocations the library has made so far (sgpu_debug_alloc_count)."""
        return int(lib().sgpu_debug_alloc_count())

    def stage(self, images: np.ndarray):
        """Upload a u8 batch [n, h, w] once; extract_staged() then starts from HBM."""
        a = np.ascontiguousarray(images, np.uint8)
        if a.ndim == 2:
            a = a[None]
        n, h, w = a.shape
        self._check(lib().sgpu_stage_input(self._ctx, a.ctypes.data, n, w, h, w), "stage")
        self._staged = (n, h, w)
        return self

    def extract_staged(self):
        n, h, w = self._staged
        self._check(lib().sgpu_extract(self._ctx, None, n, w, h, w, SGPU_INPUT_STAGED),
                    "sgpu_extract(staged)")
        self.batch = n
        return self

    def extract(self, images: np.ndarray | int, shape=None, device_ptr=False):
        """images: u8 [n, h, w] (or [h, w]) host array, or an int device pointer with
        shape=(n, h, w, stride)."""
        if device_ptr:
            n, h, w, stride = shape
            rc = lib().sgpu_extract(self._ctx, ctypes.c_void_p(images), n, w, h, stride,
                                    SGPU_INPUT_DEVICE)
        else:
            a = np.ascontiguousarray(images)
            if a.ndim == 2:
                a = a[None]
            n, h, w = a.shape
            if a.dtype == np.uint8:
                rc = lib().sgpu_extract(self._ctx, a.ctypes.data, n, w, h, w, SGPU_INPUT_HOST)
            elif a.dtype == np.float32:
                rc = lib().sgpu_extract_f32(self._ctx, a.ctypes.data, n, w, h, w, SGPU_INPUT_HOST)
            else:
                raise TypeError(a.dtype)
        self._check(rc, "sgpu_extract")
        self.batch = n
        return self

    COLOR_FORMATS = {"rgb": 1, "bgr": 2, "rgba": 3, "bgra": 4}

    def extract_color(self, images: np.ndarray, fmt: str = "rgb"):
        """u8 color images [n, h, w, 3|4] (or [h, w, c]): luminance on the device with the
        reference's formula (GLTexImage.cpp:834-858), then the usual pipeline."""
        a = np.ascontiguousarray(images, np.uint8)
        if a.ndim == 3:
            a = a[None]
        n, h, w, c = a.shape
        if c != (3 if fmt in ("rgb", "bgr") else 4):
            raise ValueError("channel count does not match the format")
        self._check(lib().sgpu_extract_color(self._ctx, a.ctypes.data, n, w, h, w * c,
                                             self.COLOR_FORMATS[fmt], SGPU_INPUT_HOST),
                    "extract_color")
        self.batch = n

    def extract_stream(self, batches, keys=None, desc=None, cap=None):
        """Host-in / host-out extraction of a list of u8 batches [n, h, w] (sgpu_extract_stream:
        uploads and downloads overlap the kernels).  keys / desc: optional preallocated [cap, 4] /
        [cap, 128] float32 outputs (PinnedArray(...).array for overlapped copies).  Returns
        (keys, desc, counts[total images]) trimmed to the features written."""
        bl = [np.ascontiguousarray(b) for b in batches]
        if not bl:
            raise ValueError("no batches")
        n, h, w = bl[0].shape
        if any(b.shape != (n, h, w) or b.dtype != np.uint8 for b in bl):
            raise ValueError("batches must be u8 arrays of one shape")
        want_desc = bool(self.opts.descriptors)

        def check_out(a, width, name):
            # the library's copies write cap rows: the array must hold them as C-ordered f32
            if (not isinstance(a, np.ndarray) or a.dtype != np.float32 or a.ndim != 2 or
                    a.shape[1] != width or not a.flags.c_contiguous or not a.flags.writeable):
                raise ValueError(f"{name} must be a writable C-contiguous float32 [cap, {width}]")
        if keys is not None:
            check_out(keys, 4, "keys")
        if desc is not None:
            if not want_desc:
                raise ValueError("descriptors are disabled (-sd): pass desc=None")
            check_out(desc, 128, "desc")
        given = [len(a) for a in (keys, desc) if a is not None]
        if cap is None:
            cap = min(given) if given else 4096 * n * len(bl)
        cap = int(cap)
        if cap < 0 or any(cap > g for g in given):
            raise ValueError(f"cap {cap} exceeds an output array ({given})")
        if keys is None:
            keys = np.zeros((cap, 4), np.float32)
        if desc is None and want_desc:
            desc = np.zeros((cap, 128), np.float32)
        ptrs = (ctypes.c_void_p * len(bl))(*[b.ctypes.data for b in bl])
        counts = np.zeros(n * len(bl), np.int32)
        rc = lib().sgpu_extract_stream(self._ctx, ptrs, len(bl), n, w, h, w, keys.ctypes.data,
                                       desc.ctypes.data if desc is not None else None, cap,
                                       counts.ctypes.data)
        self._check(rc, "sgpu_extract_stream")
        t = int(counts.sum())
        self.batch = 0
        return keys[:t], (desc[:t] if desc is not None else None), counts

    def extract_keypoints(self, keys: np.ndarray, has_orientation=True, image: int = 0):
        """Descriptors of caller-supplied keys [n, 4] (x, y, scale, orientation) on image
        `image` of the last extract (SiftGPU::RunSIFT(num, keys, keys_have_orientation)).
        has_orientation = -1: rectangles (x, y, width, height), the RECT description."""
        k = np.ascontiguousarray(keys, np.float32).reshape(-1, 4)
        ho = -1 if has_orientation == -1 else (1 if has_orientation else 0)
        self._check(lib().sgpu_extract_keypoints(self._ctx, image, k.ctypes.data, len(k), ho),
                    "sgpu_extract_keypoints")
        return self

    def count(self, image: int = 0) -> int:
        return lib().sgpu_feature_count(self._ctx, image)

    def total(self) -> int:
        return lib().sgpu_feature_total(self._ctx)

    def features(self, image: int = 0, descriptors: bool = True):
        n = self.count(image)
        keys = np.zeros((n, 4), np.float32)
        desc = np.zeros((n, 128), np.float32) if descriptors else None
        self._check(lib().sgpu_copy_features(self._ctx, image, keys.ctypes.data if n else None,
                                             desc.ctypes.data if (n and descriptors) else None),
                    "sgpu_copy_features")
        return keys, desc

    def set_host_output(self, keys, descriptors, capacity: int):
        """Register page-locked buffers (PinnedArray .array, [cap, 4] / [cap, 128] float32) that
        the next one-image extract fills from the GPU (sgpu_set_host_output)."""
        self._check(lib().sgpu_set_host_output(
            self._ctx, keys.ctypes.data if keys is not None else None,
            descriptors.ctypes.data if descriptors is not None else None, int(capacity)),
            "sgpu_set_host_output")

    def copy_features_into(self, keys, descriptors, image: int = 0):
        """sgpu_copy_features into caller arrays (e.g. the registered host output)."""
        self._check(lib().sgpu_copy_features(
            self._ctx, image, keys.ctypes.data if keys is not None else None,
            descriptors.ctypes.data if descriptors is not None else None), "sgpu_copy_features")

    def timing(self):
        t = np.zeros(10, np.float32)
        lib().sgpu_last_timing(self._ctx, t.ctypes.data, 10)
        return dict(zip(["upload", "pyramid", "detect", "orientation", "expand", "descriptor",
                         "download", "total", "match", "list"], t.tolist()))

    def match_shard_begin(self, d1_shard: np.ndarray, row_begin: int, d2: np.ndarray,
                          distmax=0.7, ratiomax=0.8, mbm=1):
        """Rows [row_begin, row_begin + len(d1_shard)) of set 1 against all of set 2
        (sgpu_match_shard_begin): (row decisions [ns], column state [n2][3])."""
        d1 = np.ascontiguousarray(d1_shard, np.uint8)
        d2 = np.ascontiguousarray(d2, np.uint8)
        ns, n2 = d1.shape[0], d2.shape[0]
        rows = np.zeros(max(ns, 1), np.int32)
        cols = np.zeros((max(n2, 1), 3), np.int32)
        self._check(lib().sgpu_match_shard_begin(self._ctx, d1.ctypes.data, ns, row_begin,
                                                 d2.ctypes.data, n2, distmax, ratiomax, mbm,
                                                 rows.ctypes.data, cols.ctypes.data,
                                                 SGPU_INPUT_HOST), "sgpu_match_shard_begin")
        return rows[:ns].copy(), cols[:n2].copy()

    def match_sharded(self, d1_shard: np.ndarray, row_begin: int, d2: np.ndarray,
                      distmax=0.7, ratiomax=0.8, mbm=1, max_match=None):
        """This rank's pairs of the sharded matcher; the column states travel by RCCL over the
        context's communicator (comm_init), or stay local without one (sgpu_match_sharded)."""
        d1 = np.ascontiguousarray(d1_shard, np.uint8)
        d2 = np.ascontiguousarray(d2, np.uint8)
        ns = d1.shape[0]
        max_match = ns if max_match is None else max_match
        out = np.zeros((max(max_match, 1), 2), np.int32)
        m = lib().sgpu_match_sharded(self._ctx, d1.ctypes.data, ns, row_begin, d2.ctypes.data,
                                     d2.shape[0], distmax, ratiomax, mbm, max_match,
                                     out.ctypes.data, SGPU_INPUT_HOST)
        if m < 0:
            self._check(m, "sgpu_match_sharded")
        return out[:m].copy()

    def match(self, d1: np.ndarray, d2: np.ndarray, distmax=0.7, ratiomax=0.8, mbm=1,
              max_match=None, device_ptrs=None):
        if device_ptrs is not None:
            p1, n1, p2, n2 = device_ptrs
            flags = SGPU_INPUT_DEVICE
        else:
            d1 = np.ascontiguousarray(d1, np.uint8)
            d2 = np.ascontiguousarray(d2, np.uint8)
            p1, n1, p2, n2 = d1.ctypes.data, d1.shape[0], d2.ctypes.data, d2.shape[0]
            flags = SGPU_INPUT_HOST
        max_match = n1 if max_match is None else max_match
        out = np.zeros((max(max_match, 1), 2), np.int32)
        m = lib().sgpu_match(self._ctx, ctypes.c_void_p(p1), n1, ctypes.c_void_p(p2), n2,
                             distmax, ratiomax, mbm, max_match, out.ctypes.data, flags)
        if m < 0:
            self._check(m, "sgpu_match")
        return out[:m]

    def match_guided(self, d1: np.ndarray, d2: np.ndarray, loc1: np.ndarray, loc2: np.ndarray,
                     H=None, F=None, distmax=0.7, ratiomax=0.8, hdistmax=32.0, fdistmax=16.0,
                     mbm=1, max_match=None):
        """SiftMatchGPU::GetGuidedSiftMatch (SiftMatch.cpp:663-677): loc1/loc2 [n][2] (x, y),
        H/F 3x3 or None (defaults of SiftGPU.h:318-321)."""
        d1 = np.ascontiguousarray(d1, np.uint8)
        d2 = np.ascontiguousarray(d2, np.uint8)
        l1 = np.ascontiguousarray(loc1, np.float32)
        l2 = np.ascontiguousarray(loc2, np.float32)
        n1, n2 = d1.shape[0], d2.shape[0]
        if l1.shape != (n1, 2) or l2.shape != (n2, 2):
            raise ValueError("locations must be [n][2] per descriptor set")
        hm = None if H is None else np.ascontiguousarray(H, np.float32).reshape(9)
        fm = None if F is None else np.ascontiguousarray(F, np.float32).reshape(9)
        max_match = n1 if max_match is None else max_match
        out = np.zeros((max(max_match, 1), 2), np.int32)
        m = lib().sgpu_match_guided(
            self._ctx, d1.ctypes.data, n1, d2.ctypes.data, n2, l1.ctypes.data, l2.ctypes.data,
            None if hm is None else hm.ctypes.data, None if fm is None else fm.ctypes.data,
            distmax, ratiomax, hdistmax, fdistmax, mbm, max_match, out.ctypes.data,
            SGPU_INPUT_HOST)
        if m < 0:
            self._check(m, "sgpu_match_guided")
        return out[:m]

    # ---- multi-GPU (RCCL inside libsiftgpu)
    def comm_init(self, nranks: int, rank: int, uid: bytes):
        buf = (ctypes.c_uint8 * len(uid)).from_buffer_copy(uid)
        self._check(lib().sgpu_comm_init(self._ctx, nranks, rank, buf, len(uid)), "sgpu_comm_init")

    def allgather_i32(self, send: np.ndarray, nranks: int) -> np.ndarray:
        a = np.ascontiguousarray(send, np.int32)
        out = np.zeros(a.size * nranks, np.int32)
        self._check(lib().sgpu_comm_allgather_i32(self._ctx, a.ctypes.data, a.size, out.ctypes.data),
                    "sgpu_comm_allgather_i32")
        return out

    def allreduce_f64(self, v, op_max: bool) -> np.ndarray:
        a = np.ascontiguousarray(np.atleast_1d(v), np.float64).copy()
        self._check(lib().sgpu_comm_allreduce_f64(self._ctx, a.ctypes.data, a.size, 1 if op_max else 0),
                    "sgpu_comm_allreduce_f64")
        return a

    # ---- test hooks
    DEBUG_PARTS2, DEBUG_PARTS4, DEBUG_TINY_CAP, DEBUG_FUSED_MATCH = 1, 2, 4, 8
    DEBUG_EXACT_DESCRIPTOR = 16
    DEBUG_GAUSS_BLOCK = 32    # workgroup strip Gaussian (k_gauss_pk2)
    DEBUG_BAND_SHIFT = 20     # (rows << 20), rows < 2048: the wave kernels' forced band height (0: automatic)
    DEBUG_KEYED_MATCH = 64    # keyed matcher epilogue even when ratiomax <= 1
    DEBUG_FULL_COLUMNS = 128  # mutual matching decides every column, not only the matched ones
    DEBUG_DESC_DUAL = 256     # descriptors through the round-4 dual-cell kernel
    DEBUG_ORIENT_WAVE = 512   # orientation one wave per candidate for any candidate count
    DEBUG_GAUSS_TILE_ALWAYS = 1024  # every level (k_gauss_tile) and the extrema (k_extrema_tile) in tiles
    DEBUG_MATCH_REGSTAGE = 2048  # keyless matcher with register staging (k_match_rows<RAW>)
    DEBUG_PYR_SERIAL = 4096    # all pyramid octaves on one stream
    DEBUG_GAUSS_LONG_BANDS = 8192  # Gaussian bands of >= 4 chunks on every level
    DEBUG_DUO_ALWAYS = 16384   # paired-level Gaussian launches whatever the level size
    DEBUG_DUO_OFF = 32768      # no paired-level launches (one level per launch)
    DEBUG_GAUSS_TILE_OFF = 65536       # no tile launches (the wave-streaming level kernels)
    DEBUG_DESC_WIDE_OFF = 131072       # descriptors one wave per feature for every count
    DEBUG_DESC_WIDE_ALWAYS = 262144    # descriptors one workgroup per feature for every count
    DEBUG_EXTREMA_TILE_OFF = 524288    # extremum detection always through k_extrema_wave2

    def set_debug_flags(self, flags: int):
        """Per-context debug flags (sgpu_debug_set_flags; 0 = shipped configuration)."""
        self._check(lib().sgpu_debug_set_flags(self._ctx, flags), "sgpu_debug_set_flags")

    TRIO_OFF, TRIO_ON, TRIO_ALWAYS = 0, 1, 2
    PAIRS_FRONT, PAIRS_END = 0, 1

    def set_schedule(self, trio: int = 0, pairs: int = 1):
        """The batch pyramid's launch plan (sgpu_debug_set_schedule): three-level launches
        (TRIO_OFF, shipped; TRIO_ON: the size rule; TRIO_ALWAYS: wherever the widths and the
        decimation allow) and the octave's level pairs from its end (PAIRS_END, shipped) or its
        front (PAIRS_FRONT)."""
        self._check(lib().sgpu_debug_set_schedule(self._ctx, trio, pairs), "sgpu_debug_set_schedule")

    def set_match_prune(self, on: bool = True):
        """Plain mutual matching's column side over the rows of set 1 that can change a listed
        column's decision (sgpu_debug_set_match_prune; on = shipped): the same pairs."""
        self._check(lib().sgpu_debug_set_match_prune(self._ctx, int(bool(on))),
                    "sgpu_debug_set_match_prune")

    @contextlib.contextmanager
    def exact_descriptors(self):
        """Within the block the descriptors come from the bit-exact kernel (the reference's fma
        order, the oracle's transcendentals) instead of the shipped relaxed-order one."""
        self.set_debug_flags(self.DEBUG_EXACT_DESCRIPTOR)
        try:
            yield self
        finally:
            self.set_debug_flags(0)

    def geometry(self):
        n = ctypes.c_int(0)
        dims = np.zeros(48, np.int32)
        lib().sgpu_debug_geometry(self._ctx, ctypes.byref(n), dims.ctypes.data, 16)
        return [tuple(dims[3 * i:3 * i + 3]) for i in range(n.value)]

    def gaussian(self, image, octave, level):
        w, h, wa = self.geometry()[octave]
        out = np.zeros(wa * h, np.float32)
        self._check(lib().sgpu_debug_gaussian(self._ctx, image, octave, level, out.ctypes.data),
                    "sgpu_debug_gaussian")
        return out

    def candidates(self):
        n = ctypes.c_int(0)
        lib().sgpu_debug_candidates(self._ctx, None, None, 0, ctypes.byref(n))
        ints = np.zeros((max(n.value, 1), 4), np.int32)
        fl = np.zeros((max(n.value, 1), 4), np.float32)
        self._check(lib().sgpu_debug_candidates(self._ctx, ints.ctypes.data, fl.ctypes.data,
                                                n.value, ctypes.byref(n)), "sgpu_debug_candidates")
        return ints[:n.value], fl[:n.value]
