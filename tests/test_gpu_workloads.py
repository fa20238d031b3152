"""The BASELINE.json configurations on the HIP path:
  * C4 -- one 4096 x 4096 tile with 6 octaves, every keypoint and descriptor against the oracle;
  * C3 -- the per-GPU shard the bench times (128 distinct 1920 x 1080 images, -fo 0 -no 4 -d 3):
    every image of the batch equals its single-image run, two of them equal the oracle;
  * C5 -- the benched 50,000 x 50,000 mutual match (seeds 5000/5001, 20,000 planted
    near-duplicates, bench.py bench_match) against the oracle's pairs, plus the keyed path
    (ratiomax 1.5) and the one-sided match (mbm 0) at 20,000 x 20,000;
  * the keypoint-capacity overflow path of a batch (grow the buffers, re-run the part)."""
import numpy as np
import pytest

import oracle_py as O
from sgpu_types import default_options
from sift_synth import quantize, synth_batch_fast, synth_descriptors, synth_image

pytestmark = pytest.mark.gpu

DESC_L2_TOL = 1e-4


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _equal(a, b):
    return a[0].shape == b[0].shape and np.array_equal(_bits(a[0]), _bits(b[0])) and \
        np.array_equal(_bits(a[1]), _bits(b[1]))


def test_c4_4096_six_octaves_vs_oracle(gpu_ctx):
    img = synth_batch_fast(1, 4096, 4096, 4000)[0]
    opts = default_options(octave_num=6)
    gpu_ctx.set_options(opts)
    gpu_ctx.extract(img)
    assert len(gpu_ctx.geometry()) == 6 and gpu_ctx.geometry()[5][:2] == (128, 128)
    k, d = gpu_ctx.features(0)
    rk, rd = O.extract(img, opts)
    assert k.shape == rk.shape and len(k) > 2000, (k.shape, rk.shape)
    assert np.array_equal(_bits(k), _bits(rk))
    assert np.linalg.norm(d.astype(np.float64) - rd, axis=1).max() < DESC_L2_TOL
    with gpu_ctx.exact_descriptors():
        gpu_ctx.extract(img)
        k, d = gpu_ctx.features(0)
    assert np.array_equal(_bits(k), _bits(rk))
    assert np.array_equal(_bits(d), _bits(rd))
    gpu_ctx.set_options(default_options())


def _c5_sets(n, n_dup):
    # bench.py bench_match: the same seeds and planted duplicates
    d1 = synth_descriptors(n, 5000)
    d2 = synth_descriptors(n, 5001, base=d1, n_dup=n_dup)
    return quantize(d1), quantize(d2)


def test_c5_50k_mutual_match_vs_oracle(gpu_ctx):
    """BASELINE configs[4] at its benched size: the shipped path (keyless fold, matched-columns
    list, device-sized grids; ProgramCU.cu:1466-1564, 1785-1900, SiftMatchCU.cpp:149-179) gives
    exactly the oracle's pairs."""
    q1, q2 = _c5_sets(50000, 20000)
    got = gpu_ctx.match(q1, q2)
    ref = O.match_mt(q1, q2)
    assert len(ref) >= 20000
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("ratiomax,mbm", [(1.5, 1), (1.5, 0), (0.8, 0)])
def test_c5_20k_keyed_and_one_sided_vs_oracle(gpu_ctx, ratiomax, mbm):
    """ratiomax > 1 runs the keyed epilogue (exact ties are accepted, so the tie order shows);
    mbm = 0 skips the column side."""
    q1, q2 = _c5_sets(20000, 8000)
    got = gpu_ctx.match(q1, q2, 0.7, ratiomax, mbm)
    ref = O.match_mt(q1, q2, 0.7, ratiomax, mbm)
    assert len(ref) >= 8000
    assert np.array_equal(got, ref)


def test_c3_shard_128_full_hd(gpu_ctx):
    n = 128
    imgs = synth_batch_fast(n, 1920, 1080, 3000)
    opts = default_options(octave_num=4)
    gpu_ctx.set_options(opts)
    gpu_ctx.extract(imgs)
    batch = [gpu_ctx.features(i) for i in range(n)]
    total = gpu_ctx.total()
    assert total == sum(len(b[0]) for b in batch) and total > n * 500
    for i in range(n):
        gpu_ctx.extract(imgs[i])
        assert _equal(gpu_ctx.features(0), batch[i]), f"image {i}: batch != single"
    for i in (0, n - 1):
        rk, rd = O.extract(imgs[i], opts)
        assert np.array_equal(_bits(batch[i][0]), _bits(rk)), i
        assert np.linalg.norm(batch[i][1].astype(np.float64) - rd, axis=1).max() < DESC_L2_TOL
    gpu_ctx.set_options(default_options())


def test_capacity_overflow_rerun(gpu_ctx):
    """SGPU_DEBUG_TINY_CAP starts the keypoint capacity at 64: the first pass overflows, the
    part is re-run with grown buffers and the results equal the normal run's."""
    import sgpu
    imgs = np.stack([synth_image(480, 360, 200 + i) for i in range(3)])
    ctx = sgpu.SiftContext(0)
    try:
        ctx.extract(imgs)
        ref = [ctx.features(i) for i in range(3)]
        assert ctx.total() > 64
        ctx2 = sgpu.SiftContext(0)
        try:
            ctx2.set_debug_flags(ctx2.DEBUG_TINY_CAP)
            ctx2.extract(imgs)
            for i in range(3):
                assert _equal(ctx2.features(i), ref[i]), i
            ctx2.extract(imgs[:1])   # grown buffers persist: no overflow the second time
            assert _equal(ctx2.features(0), ref[0])
        finally:
            ctx2.close()
    finally:
        ctx.close()


def _stream_reference(ctx, batches):
    keys, desc, counts = [], [], []
    for b in batches:
        ctx.extract(b)
        for i in range(len(b)):
            k, d = ctx.features(i)
            keys.append(k)
            desc.append(d)
            counts.append(len(k))
    return np.concatenate(keys), np.concatenate(desc), np.array(counts, np.int32)


@pytest.mark.parametrize("pinned", [True, False])
def test_extract_stream_equals_batches(gpu_ctx, pinned):
    """sgpu_extract_stream (two slots, uploads and downloads on the copy engines beside the
    kernels) gives exactly the batch-by-batch results, for 5 batches (every slot reused twice)."""
    import sgpu
    gpu_ctx.set_options(default_options())
    batches = [synth_batch_fast(6, 480, 360, 700 + 10 * k) for k in range(5)]
    rk, rd, rc = _stream_reference(gpu_ctx, batches)
    cap = len(rk) + 100
    bufs = []
    if pinned:
        pin_in = [sgpu.PinnedArray(b.shape, np.uint8) for b in batches]
        for p, b in zip(pin_in, batches):
            p.array[...] = b
        kb, db = sgpu.PinnedArray((cap, 4), np.float32), sgpu.PinnedArray((cap, 128), np.float32)
        bufs = pin_in + [kb, db]
        k, d, c = gpu_ctx.extract_stream([p.array for p in pin_in], kb.array, db.array)
    else:
        k, d, c = gpu_ctx.extract_stream(batches, cap=cap)
    assert np.array_equal(c, rc)
    assert np.array_equal(_bits(k), _bits(rk)) and np.array_equal(_bits(d), _bits(rd))
    for p in bufs:
        p.free()


def test_extract_stream_capacity_and_first_octave(gpu_ctx):
    """Output capacity: SGPU_ERANGE with complete counts; -fo 1 (sampled input, the serial
    path) equals the batch-by-batch results too."""
    import sgpu
    batches = [synth_batch_fast(3, 320, 240, 900 + k) for k in range(3)]
    gpu_ctx.set_options(default_options())
    rk, rd, rc = _stream_reference(gpu_ctx, batches)
    with pytest.raises(RuntimeError):
        gpu_ctx.extract_stream(batches, cap=int(rc[:5].sum()))
    gpu_ctx.set_options(default_options(octave_min=1))
    fk, fd, fc = _stream_reference(gpu_ctx, batches)
    k, d, c = gpu_ctx.extract_stream(batches, cap=len(fk))
    assert np.array_equal(c, fc) and np.array_equal(_bits(k), _bits(fk))
    assert np.array_equal(_bits(d), _bits(fd))
    gpu_ctx.set_options(default_options())


def test_failed_stream_leaves_no_batch(gpu_ctx):
    """After a failed extract the per-image queries see no batch (not the previous batch's
    offsets under the new geometry), and the context keeps working."""
    gpu_ctx.set_options(default_options())
    batches = [synth_batch_fast(2, 320, 240, 950 + k) for k in range(2)]
    gpu_ctx.extract(batches[0])
    assert gpu_ctx.count(0) > 0
    with pytest.raises(RuntimeError):
        gpu_ctx.extract_stream(batches, cap=1)
    assert gpu_ctx.count(0) == 0 and gpu_ctx.total() == 0
    gpu_ctx.extract(batches[0])
    assert gpu_ctx.count(0) > 0


def test_extract_stream_without_descriptors(gpu_ctx):
    """-sd: the stream returns keys only (no descriptor buffer is passed)."""
    batches = [synth_batch_fast(2, 320, 240, 960 + k) for k in range(3)]
    gpu_ctx.set_options(default_options(descriptors=0))
    try:
        keys = []
        for b in batches:
            gpu_ctx.extract(b)
            keys += [gpu_ctx.features(i, descriptors=False)[0] for i in range(len(b))]
        rk = np.concatenate(keys)
        k, d, c = gpu_ctx.extract_stream(batches, cap=len(rk) + 10)
        assert d is None and np.array_equal(_bits(k), _bits(rk))
        with pytest.raises(ValueError):
            gpu_ctx.extract_stream(batches, desc=np.zeros((10, 128), np.float32))
    finally:
        gpu_ctx.set_options(default_options())


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2])
def test_one_stream_small_batch_equals_stream_layout(n):
    """A small batch (C2: one image through RunSIFT) runs every stage on one stream; the batch
    layout (octaves >= 1 and the feature stages on their own streams, SGPU_STREAMS=multi) gives the
    same keys and descriptors bit for bit."""
    import os
    import sgpu
    imgs = np.stack([synth_image(1920, 1080, 2000 + i) for i in range(n)])
    out = {}
    for mode in ("", "multi"):
        os.environ["SGPU_STREAMS"] = mode   # read at context creation
        try:
            ctx = sgpu.SiftContext(0)
        finally:
            del os.environ["SGPU_STREAMS"]
        try:
            ctx.extract(imgs)
            out[mode] = [ctx.features(i) for i in range(n)]
        finally:
            ctx.close()
    for i in range(n):
        assert out[""][i][0].shape[0] > 100
        assert _equal(out[""][i], out["multi"][i]), i
