"""The drop-in C++ API (include/SiftGPU.h) driven by compiled replicas of the reference's own
call sequences:
  * SiftGPU::SaveSIFT, byte for byte against the reference's writer restated on the oracle side
    (SiftPyramid.cpp:311-387): ASCII and -b binary, normalised and -unn, with and without
    descriptors (-sd), plus option paths that change the feature list (-fo, -tc2, -maxd through
    SetMaxDimension);
  * SiftMatchGPU::SetDescriptors' id cache (SiftMatchCU.cpp:71-101);
  * TestWin/MultiThreadSIFT.cpp: one SiftGPU per thread on one device, initialisation
    serialised, the runs concurrent."""
import os
import subprocess

import numpy as np
import pytest

import oracle_py as O
from sgpu_types import default_options
from sift_synth import quantize, synth_descriptors, synth_image

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "modify-sift-gpu_amd", "lib")


def _compile(tmp_path, name):
    exe = tmp_path / name
    r = subprocess.run(["g++", "-std=c++11", "-O1", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "abi", name + ".cpp"), "-o", str(exe),
                        "-L" + LIBDIR, "-lsiftgpu", "-Wl,-rpath," + LIBDIR, "-lpthread"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return str(exe)


def _write_pgm(path, img):
    h, w = img.shape
    with open(path, "wb") as f:
        f.write(f"P5\n{w} {h}\n255\n".encode())
        f.write(np.ascontiguousarray(img, np.uint8).tobytes())


# (replica command-line options, oracle options, binary, normalised, descriptors)
SAVE_CASES = [
    ([], {}, False, True, True),
    (["-b"], {}, True, True, True),
    (["-unn"], {"normalized": 0}, False, False, True),
    (["-b", "-unn"], {"normalized": 0}, True, False, True),
    (["-sd"], {"descriptors": 0}, False, True, False),
    (["-sd", "-b"], {"descriptors": 0}, True, True, False),
    (["-fo", "1"], {"octave_min": 1}, False, True, True),
    (["-tc2", "200"], {"feature_count_threshold": 200, "truncate_method": 1}, False, True, True),
    (["=maxd", "300"], {"max_dimension": 300}, False, True, True),
    (["-maxd", "200", "-noprep", "-fo", "1"], {"max_dimension": 200, "octave_min": 1,
                                                "preprocess_on_cpu": 0}, False, True, True),
]


@pytest.mark.parametrize("args,over,binary,normalized,desc", SAVE_CASES,
                         ids=lambda v: " ".join(v) if isinstance(v, list) else None)
def test_save_sift_bytes_vs_reference_writer(tmp_path, args, over, binary, normalized, desc):
    """Byte for byte, with the bit-exact descriptor kernel (SGPU_EXACT_DESCRIPTOR=1)."""
    exe = _compile(tmp_path, "save_sift_replica")
    img = synth_image(480, 352, 91)
    pgm = tmp_path / "in.pgm"
    _write_pgm(pgm, img)
    out = tmp_path / "gpu.sift"
    r = subprocess.run([exe, str(pgm), str(out)] + args, capture_output=True, text=True,
                       timeout=120, env=dict(os.environ, SGPU_EXACT_DESCRIPTOR="1"))
    assert r.returncode == 0, r.stdout + r.stderr
    num = int([l for l in r.stdout.split("\n") if l.startswith("NUM ")][0].split()[1])
    rk, rd = O.extract(img, default_options(**over))
    assert num == len(rk) > 0
    ref = tmp_path / "oracle.sift"
    O.save_sift(ref, rk, rd if desc else None, binary=binary, normalized=normalized)
    a, b = out.read_bytes(), ref.read_bytes()
    assert a == b, f"{len(a)} vs {len(b)} bytes; first difference at {next((i for i in range(min(len(a), len(b))) if a[i] != b[i]), None)}"


@pytest.mark.parametrize("binary", [False, True])
def test_save_sift_shipped_descriptors(tmp_path, binary):
    """The shipped (relaxed-order) descriptors through SaveSIFT: the key columns are the
    oracle's, and every descriptor entry floor(0.5 + 512 d) is within 1 of the oracle's."""
    exe = _compile(tmp_path, "save_sift_replica")
    img = synth_image(480, 352, 91)
    pgm = tmp_path / "in.pgm"
    _write_pgm(pgm, img)
    out = tmp_path / "gpu.sift"
    env = {k: v for k, v in os.environ.items() if k != "SGPU_EXACT_DESCRIPTOR"}
    r = subprocess.run([exe, str(pgm), str(out)] + (["-b"] if binary else []),
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    rk, rd = O.extract(img, default_options())
    ref = tmp_path / "oracle.sift"
    O.save_sift(ref, rk, rd, binary=binary, normalized=True)
    ka, da = O.read_sift(out, binary=binary)
    kb, db = O.read_sift(ref, binary=binary)
    assert np.array_equal(ka, kb)
    assert da.shape == db.shape and len(da) > 0
    if binary:
        assert np.linalg.norm(da.astype(np.float64) - db, axis=1).max() < 1e-4
    else:
        assert np.abs(da - db).max() <= 1 and (da != db).mean() < 1e-3


def test_match_id_cache(tmp_path):
    exe = _compile(tmp_path, "match_id_replica")
    a = synth_descriptors(900, 11)
    b = synth_descriptors(1000, 12, base=a, n_dup=600)
    c = synth_descriptors(800, 13, base=b, n_dup=300)
    paths = []
    for name, d in (("a", a), ("b", b), ("c", c)):
        p = tmp_path / f"{name}.f32"
        np.ascontiguousarray(d, np.float32).tofile(p)
        paths += [str(p), str(len(d))]
    r = subprocess.run([exe] + paths, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = {l.split()[1]: int(l.split()[2]) for l in r.stdout.splitlines() if l.startswith("COUNT")}
    ab = len(O.match(quantize(a), quantize(b)))
    cb = len(O.match(quantize(c), quantize(b)))
    assert ab != cb and ab > 100
    assert got == {"ab": ab, "cached": ab, "cb": cb, "cb_again": cb}


def test_multithread_contexts_one_device(tmp_path):
    exe = _compile(tmp_path, "multithread_replica")
    imgs = [synth_image(640, 480, 300 + i) for i in range(2)]
    args = ["0", "10"]
    for i, img in enumerate(imgs):
        _write_pgm(tmp_path / f"{i}.pgm", img)
        args += [str(tmp_path / f"{i}.pgm"), str(tmp_path / f"{i}.bin")]
    r = subprocess.run([exe] + args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [l.split() for l in r.stdout.splitlines() if l.startswith("THREAD")]
    assert len(lines) == 2
    opts = default_options(octave_min=-1)   # MultiThreadSIFT.cpp:148: -fo -1
    for i, (_, _, num, equal) in enumerate(lines):
        assert int(equal) == 1, f"thread {i}: a repeated run differed"
        rk, rd = O.extract(imgs[i], opts)
        assert int(num) == len(rk) > 0
        raw = np.fromfile(tmp_path / f"{i}.bin", np.float32)
        k = raw[:4 * len(rk)].reshape(-1, 4)
        d = raw[4 * len(rk):].reshape(-1, 128)
        assert np.array_equal(k.view(np.uint32), rk.view(np.uint32))
        assert np.linalg.norm(d.astype(np.float64) - rd, axis=1).max() < 1e-4


def test_speed_replica_timing_slots(tmp_path):
    """TestWin/speed.cpp's protocol (speed.cpp:60-155) through bin/speed_replica: the feature count
    is stable over the runs and equals the oracle's, and the reference's _timing slots
    (SiftGPU.cpp:368, printed by speed.cpp:136-153) are filled: every stage slot is a finite
    non-negative time, the pyramid and descriptor slots are positive, and the slots add up to no
    more than the wall time per RunSIFT of that second (stage-timed, SetVerbose(-2)) loop, plus a
    small allowance for event rounding.  The first loop runs with the stage timing off
    (SetVerbose(0) -> _timingS 0, SiftGPU.cpp:426-427).  Wall-clock ratios between the two loops
    and the relative sizes of the slots go to bench.py's report, not here (one C2 run once read
    0.53 ms against 0.38-0.41 for its neighbours)."""
    exe = os.path.join(ROOT, "modify-sift-gpu_amd", "bin", "speed_replica")
    img = synth_image(1920, 1080, 2000)      # the C2 image of bench.py
    pgm = tmp_path / "c2.pgm"
    _write_pgm(pgm, img)
    r = subprocess.run([exe, "20", "--", "-i", str(pgm), "-fo", "0", "-no", "4", "-d", "3"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    import json
    sp = json.loads(r.stdout.strip().splitlines()[-1])
    assert sp["stable"] and sp["features"] == len(O.extract(img, default_options(octave_num=4))[0])
    t = sp["timing_ms"]
    slots = ["build_pyramid", "detection", "feature_list", "orientation", "mo_feature_list",
             "download_keys", "descriptor"]
    assert all(np.isfinite(t[s]) and t[s] >= 0 for s in slots), t
    assert t["descriptor"] > 0 and t["build_pyramid"] > 0, t
    total = sum(t[s] for s in slots)
    # the stage events lie inside each RunSIFT of the timed loop, so their sum is bounded by its
    # wall time per call (plus event rounding), and the slots are not lost or zeroed: they cover
    # at least half of it (the rest is host work between the events)
    assert 0.5 * sp["timed_avg_ms"] <= total <= 1.10 * sp["timed_avg_ms"] + 0.02, \
        (total, sp["timed_avg_ms"], t)


def test_allocate_pyramid_then_runsift_allocates_nothing(tmp_path):
    """SiftGPU::AllocatePyramid (SiftGPU.cpp:1435-1460) sizes the pyramid and every other
    buffer for a w x h image: the first RunSIFT of that size after it allocates nothing
    (the library's allocation counter, sgpu_debug_alloc_count), and its features equal the
    oracle's."""
    exe = _compile(tmp_path, "allocate_replica")
    img = synth_image(1280, 720, 2024)
    pgm = tmp_path / "a.pgm"
    _write_pgm(pgm, img)
    r = subprocess.run([exe, str(pgm), "1280", "720"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    f = dict(kv.split("=") for kv in r.stdout.split("ALLOC", 1)[1].split())
    assert f["reserve"] == "1" and int(f["during_reserve"]) > 0, f
    assert int(f["during_run"]) == 0 and int(f["again"]) == 0, f
    assert int(f["features"]) == len(O.extract(img, default_options())[0]) > 0


def test_reserve_then_extract_allocates_nothing(gpu_ctx):
    """sgpu_reserve through the C ABI: a batch of 8 HD images extracts without a new allocation
    after it, and the results equal those of an unreserved context (same bits)."""
    from sift_synth import synth_batch_fast
    imgs = synth_batch_fast(8, 1280, 720, 2025)
    gpu_ctx.set_options(default_options())
    gpu_ctx.extract(imgs)
    ref = [gpu_ctx.features(i) for i in range(8)]
    gpu_ctx.reserve(8, 1280, 720)
    assert gpu_ctx.total() == 0   # the reservation replaced the batch
    c0 = gpu_ctx.alloc_count()
    gpu_ctx.stage(imgs)
    gpu_ctx.extract_staged()
    assert gpu_ctx.alloc_count() == c0
    for i in range(8):
        k, d = gpu_ctx.features(i)
        assert np.array_equal(k.view(np.uint32), ref[i][0].view(np.uint32))
        assert np.array_equal(d, ref[i][1])


@pytest.mark.parametrize("cap", [4096, 16])
@pytest.mark.parametrize("wide", [True, False])
def test_host_output_equals_copy_features(gpu_ctx, cap, wide):
    """sgpu_set_host_output: the next one-image extract writes image 0's keys and descriptors
    from the GPU into the registered page-locked buffers (k_copy_out, in the extract's stream);
    they equal sgpu_copy_features' copies bit for bit, sgpu_copy_features on those pointers copies
    nothing more, and with a capacity below the count (16) the GPU writes exactly the first 16
    keys and descriptors and nothing past them, and sgpu_copy_features into buffers of the image's
    size does the work.  Both writers: the workgroup-per-feature descriptor kernel itself (wide,
    the single-image default) and k_copy_out after the one-wave kernel.  The registration serves
    one extract: the one after it writes nothing there."""
    import sgpu
    img = synth_image(640, 480, 77)
    gpu_ctx.set_options(default_options())
    gpu_ctx.set_debug_flags(gpu_ctx.DEBUG_DESC_WIDE_ALWAYS if wide else gpu_ctx.DEBUG_DESC_WIDE_OFF)
    hk = sgpu.PinnedArray((cap, 4), np.float32)
    hd = sgpu.PinnedArray((cap, 128), np.float32)
    try:
        hk.array[:] = -1.0
        hd.array[:] = -1.0
        gpu_ctx.set_host_output(hk.array, hd.array, cap)
        gpu_ctx.extract(img)
        k, d = gpu_ctx.features(0)
        n = len(k)
        assert n > 16
        if n <= cap:
            assert np.array_equal(hk.array[:n].view(np.uint32), k.view(np.uint32))
            assert np.array_equal(hd.array[:n].view(np.uint32), d.view(np.uint32))
            assert np.all(hk.array[n:] == -1.0)
        else:
            assert np.array_equal(hk.array.view(np.uint32), k[:cap].view(np.uint32))
            assert np.array_equal(hd.array.view(np.uint32), d[:cap].view(np.uint32))
        # through the registered pointers (when they hold the image): the fast path
        if n <= cap:
            gpu_ctx.copy_features_into(hk.array, hd.array)
            assert np.array_equal(hd.array[:n].view(np.uint32), d.view(np.uint32))
        # consumed: a second extract leaves the buffers alone
        hk.array[:] = -2.0
        gpu_ctx.extract(img)
        assert np.all(hk.array == -2.0)
        k2, _ = gpu_ctx.features(0)
        assert np.array_equal(k2.view(np.uint32), k.view(np.uint32))
    finally:
        gpu_ctx.set_debug_flags(0)
        hk.free()
        hd.free()


def test_rejected_extract_consumes_host_output(gpu_ctx):
    """an extract rejected for its arguments still consumes a registered host output
    (sgpu_set_host_output), so a later good extract does not write into buffers the caller may
    have freed since: the buffers keep their sentinel values."""
    import ctypes
    import sgpu
    img = synth_image(320, 240, 6)
    gpu_ctx.set_options(default_options())
    hk = sgpu.PinnedArray((4096, 4), np.float32)
    hd = sgpu.PinnedArray((4096, 128), np.float32)
    try:
        hk.array[:] = -3.0
        hd.array[:] = -3.0
        gpu_ctx.set_host_output(hk.array, hd.array, 4096)
        buf = np.zeros((8, 8), np.uint8)
        rc = sgpu.lib().sgpu_extract(gpu_ctx._ctx, buf.ctypes.data_as(ctypes.c_void_p), 1, 8, 8, 4, 0)
        assert rc != 0   # stride < width: rejected
        gpu_ctx.extract(img)
        assert gpu_ctx.total() > 0
        assert np.all(hk.array == -3.0) and np.all(hd.array == -3.0)
    finally:
        hk.free()
        hd.free()


def test_rejected_extract_keeps_previous_results(gpu_ctx):
    """An sgpu_extract call rejected for its arguments queues nothing and leaves the previous
    extract's features readable (the C ABI's argument checks run before the batch is replaced)."""
    import ctypes
    import sgpu
    img = synth_image(320, 240, 5)
    gpu_ctx.set_options(default_options())
    gpu_ctx.extract(img)
    k0, d0 = gpu_ctx.features(0)
    n0 = gpu_ctx.total()
    buf = np.zeros((8, 8), np.uint8)
    rc = sgpu.lib().sgpu_extract(gpu_ctx._ctx, buf.ctypes.data_as(ctypes.c_void_p), 1, 8, 8, 4, 0)
    assert rc != 0   # stride < width
    assert gpu_ctx.total() == n0 > 0
    k1, d1 = gpu_ctx.features(0)
    assert np.array_equal(k0.view(np.uint32), k1.view(np.uint32)) and np.array_equal(d0, d1)
