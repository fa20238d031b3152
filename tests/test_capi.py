"""CPU tests of the drop-in boundary: the C ABI library loads and exports every symbol
include/sgpu.h declares, host-side semantics (options, CLI parsing, quantisation), no CPU
fallback, and the C++ API's binary layout against the reference header."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import sgpu
from sgpu_types import SgpuOptions, default_options
from sift_synth import quantize

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


def _exported(path):
    out = subprocess.check_output(["nm", "-D", "--defined-only", path], text=True)
    return {ln.split()[-1] for ln in out.splitlines() if len(ln.split()) >= 3}


def test_library_exports_header_symbols():
    hdr = open(os.path.join(ROOT, "include", "sgpu.h")).read()
    declared = set(re.findall(r"^\s*(?:int|void\*?|int64_t|long long|const char\*)\s+(sgpu_\w+)\s*\(", hdr, re.M))
    assert declared == set(sgpu.C_API), declared ^ set(sgpu.C_API)
    syms = _exported(sgpu.LIB_PATH)
    missing = [s for s in declared if s not in syms]
    assert not missing, missing
    for f in ["CreateNewSiftGPU", "CreateNewSiftMatchGPU", "CreateComboSiftGPU",
              "CreateRemoteSiftGPU"]:
        assert f in syms, f
    sgpu.lib()   # loads with every argtype bound


def test_test_hooks_live_outside_the_product_library():
    """The candidate dump's kernel (k_debug_candidates) is not in libsiftgpu.so: it lives in
    lib/libsiftgpu_debug.so beside it, which sgpu_debug_candidates loads on first use."""
    lib = sgpu.LIB_PATH
    dbg = os.path.join(os.path.dirname(lib), "libsiftgpu_debug.so")
    with open(lib, "rb") as f:
        assert b"k_debug_candidates" not in f.read()
    assert "sgpu_testhook_candidates" in _exported(dbg)
    with open(dbg, "rb") as f:
        assert b"k_debug_candidates" in f.read()


def test_default_options_match_reference_defaults():
    o = SgpuOptions()
    sgpu.lib().sgpu_default_options(ctypes.byref(o))
    d = default_options()
    for name, _ in SgpuOptions._fields_:
        assert getattr(o, name) == getattr(d, name), name


def _parse(args, opts=None, device=-1):
    o = opts or default_options()
    arr = (ctypes.c_char_p * len(args))(*[a.encode() for a in args])
    dev = ctypes.c_int(device)
    assert sgpu.lib().sgpu_parse_args(ctypes.byref(o), len(args), arr, ctypes.byref(dev)) == 0
    return o, dev.value


def test_parse_simplesift_argv():
    # TestWin/SimpleSIFT.cpp:145: {"-cuda"," -fo", "-1", "-v", "1"}: " -fo" is skipped,
    # "-1" is an unknown option, so only -cuda and -v 1 take effect
    o, dev = _parse(["-cuda", " -fo", "-1", "-v", "1"])
    d = default_options()
    assert o.octave_min == 0 and o.verbose == 1 and dev == -1
    for name in ["max_orientation", "subpixel", "descriptors", "normalized", "octave_num"]:
        assert getattr(o, name) == getattr(d, name)


def test_parse_options():
    o, dev = _parse(["-fo", "0", "-no", "4", "-d", "4", "-m", "1", "-s", "0", "-t", "0.01",
                     "-e", "5", "-sd", "-unn", "-loweo", "-CUDA", "3", "-w", "3", "-dw", "2.5"])
    assert (o.octave_min, o.octave_num, o.dog_level_num, o.max_orientation, o.subpixel) == (0, 4, 4, 1, 0)
    assert abs(o.dog_threshold - 0.01) < 1e-9 and o.edge_threshold == 5.0
    assert (o.descriptors, o.normalized, o.lowe_origin, dev) == (0, 0, 1, 3)
    assert o.orientation_window_factor == 3.0 and o.descriptor_window_factor == 2.5
    o, _ = _parse(["-t", "0.7", "-no", "0", "-m"])          # out-of-range values are ignored
    assert o.dog_threshold == 0.0 and o.octave_num == -1 and o.max_orientation == 2
    o, _ = _parse(["-ofix"])
    assert o.fixed_orientation == 1
    o, _ = _parse(["-ofix-not"])
    assert o.fixed_orientation == 0


def test_parse_feature_limit_and_first_octave_options():
    # SiftGPU.cpp:1185-1203: -tc / -tc1 -> method 0, -tc2 -> 1, -tc3 -> 2, count > 0 consumed;
    # :1213-1222: -maxd > 0; :921-926: -prep / -noprep
    d = default_options()
    assert (d.feature_count_threshold, d.truncate_method, d.max_dimension, d.preprocess_on_cpu) == (-1, 0, 13200, 1)
    for flag, method in [("-tc", 0), ("-tc1", 0), ("-tc2", 1), ("-TC3", 2)]:
        o, _ = _parse([flag, "500"])
        assert (o.feature_count_threshold, o.truncate_method) == (500, method), flag
    o, _ = _parse(["-tc2", "0", "-d", "4"])          # count not > 0: method set, "0" not consumed
    assert (o.feature_count_threshold, o.truncate_method, o.dog_level_num) == (-1, 1, 4)
    o, _ = _parse(["-maxd", "2560", "-noprep"])
    assert (o.max_dimension, o.preprocess_on_cpu) == (2560, 0)
    o, _ = _parse(["-maxd", "-5", "-noprep", "-prep"])
    assert (o.max_dimension, o.preprocess_on_cpu) == (13200, 1)


def test_quantize_matches_reference_semantics():
    rng = np.random.default_rng(3)
    d = np.concatenate([rng.uniform(0, 0.6, 4000), [0.0, 0.4990234, 0.5, 0.75, 1.0]]).astype(np.float32)
    np.testing.assert_array_equal(sgpu.quantize(d), quantize(d))


def test_no_cpu_fallback():
    if sgpu.device_count() > 0:
        pytest.skip("a GPU is visible; the no-device path is exercised on CPU runners")
    ctx = ctypes.c_void_p()
    rc = sgpu.lib().sgpu_ctx_create(0, None, ctypes.byref(ctx))
    assert rc == sgpu.SGPU_ENODEV and not ctx.value
    with pytest.raises(RuntimeError):
        sgpu.SiftContext(0)


def _compile(src, out, include):
    subprocess.check_call(["g++", "-std=c++11", "-O1", "-I", include, "-o", out, src, "-ldl"])


@pytest.mark.parametrize("header", ["ours", "reference"])
def test_cpp_abi_layout(tmp_path, header):
    inc = os.path.join(ROOT, "include")
    if header == "reference":
        inc = os.path.join(REF, "SiftGPU")
        if not os.path.exists(os.path.join(inc, "SiftGPU.h")):
            pytest.skip("reference checkout not present (GPU box)")
    exe = str(tmp_path / "abi_check")
    _compile(os.path.join(ROOT, "tests", "abi", "abi_check.cpp"), exe, inc)
    r = subprocess.run([exe, sgpu.LIB_PATH], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "abi ok" in r.stdout, (r.returncode, r.stdout, r.stderr)


def test_reference_simplesift_compiles_against_our_header(tmp_path):
    src = os.path.join(REF, "TestWin", "SimpleSIFT.cpp")
    if not os.path.exists(src):
        pytest.skip("reference checkout not present (GPU box)")
    # SimpleSIFT.cpp includes "../SiftGPU/SiftGPU.h": give it a tree whose SiftGPU/ is ours
    (tmp_path / "SiftGPU").mkdir()
    (tmp_path / "TestWin").mkdir()
    os.symlink(os.path.join(ROOT, "include", "SiftGPU.h"), tmp_path / "SiftGPU" / "SiftGPU.h")
    os.symlink(src, tmp_path / "TestWin" / "SimpleSIFT.cpp")
    # compile-only check (-fsyntax-only): the file is never copied into the repository
    r = subprocess.run(["g++", "-std=c++11", "-fsyntax-only", "-fpermissive", "-w",
                        "-DSIFTGPU_DLL_RUNTIME", str(tmp_path / "TestWin" / "SimpleSIFT.cpp")],
                       capture_output=True, text=True, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
