"""Gaussian pyramid kernels on the GPU: the shipped wave-streaming level kernel (k_gauss_lean) and
the workgroup strip kernel (k_gauss_pk2, test hook SGPU_DEBUG_GAUSS_BLOCK) against each other and
the oracle, bit for bit.

Both kernels restate FilterH / FilterV (ProgramCU.cu:115-222) with the taps summed i = 0..FW-1
and the 2x decimation of DownsampleKernel<1> (ProgramCU.cu:287-298) fused into the level that
feeds the next octave; the band walk (rows per wave), the lag between H and V passes and the
ring wrap must not change a single bit, so every level of every octave is compared."""
import numpy as np
import pytest

import oracle_py as O
import sgpu
from sgpu_types import default_options
from sift_synth import synth_batch, synth_image

pytestmark = pytest.mark.gpu

BLOCK = sgpu.SiftContext.DEBUG_GAUSS_BLOCK


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _levels(ctx, image, opts):
    geo = ctx.geometry()
    return [[ctx.gaussian(image, o, lvl).copy() for lvl in range(opts.dog_level_num + 3)]
            for o in range(len(geo))]


@pytest.mark.parametrize("w,h,seed", [(16, 16, 3), (203, 97, 2), (640, 480, 1000)])
def test_wave_levels_vs_oracle(gpu_ctx, w, h, seed):
    """The shipped kernel (k_gauss_lean) against the oracle, every level of every octave."""
    img = synth_image(w, h, seed)
    opts = default_options()
    gpu_ctx.set_options(opts)
    gpu_ctx.set_debug_flags(0)
    try:
        gpu_ctx.extract(img)
        for o in range(len(gpu_ctx.geometry())):
            for lvl in range(opts.dog_level_num + 3):
                g = gpu_ctx.gaussian(0, o, lvl)
                r = O.gaussian(img, o, lvl, opts)
                assert np.array_equal(_bits(g), _bits(r)), (o, lvl)
    finally:
        gpu_ctx.set_debug_flags(0)


# band heights: auto, one chunk, bands not a multiple of the lag span, a band taller than the
# image; sizes: tiny, ragged (width not a multiple of 64, odd height), 1080p
@pytest.mark.parametrize("rows", [0, 8, 24, 40, 2040])
@pytest.mark.parametrize("n,w,h", [(2, 16, 16), (3, 203, 97), (2, 1920, 1080), (5, 300, 1203)])
def test_wave_levels_equal_block_kernel(gpu_ctx, rows, n, w, h):
    imgs = synth_batch(n, w, h, 40 + w % 7)
    opts = default_options()
    gpu_ctx.set_options(opts)
    gpu_ctx.set_debug_flags(BLOCK)
    gpu_ctx.extract(imgs)
    ref = [_levels(gpu_ctx, i, opts) for i in (0, n - 1)]
    k_ref = [gpu_ctx.features(i)[0].copy() for i in range(n)]
    try:
        # the shipped k_gauss_lean with the forced band height
        for kernel in (0,):
            gpu_ctx.set_debug_flags((rows << sgpu.SiftContext.DEBUG_BAND_SHIFT) | kernel)
            gpu_ctx.extract(imgs)
            got = [_levels(gpu_ctx, i, opts) for i in (0, n - 1)]
            for a, b in zip(ref, got):
                for o, (la, lb) in enumerate(zip(a, b)):
                    for lvl, (x, y) in enumerate(zip(la, lb)):
                        assert np.array_equal(_bits(x), _bits(y)), (kernel, o, lvl)
            for i in range(n):
                assert np.array_equal(_bits(gpu_ctx.features(i)[0]), _bits(k_ref[i])), kernel
    finally:
        gpu_ctx.set_debug_flags(0)


# every filter width of the lean kernel: -d changes the level sigmas (FW 5 .. 25 at the default
# -f 4, the 32-row ring), -f 5.5 reaches FW 27 .. 33 (the 64-row ring of 8 chunk slots); first
# octaves -1 / 0 / 1 (float and u8 first levels)
@pytest.mark.parametrize("over", [dict(dog_level_num=1), dict(dog_level_num=2),
                                  dict(dog_level_num=5), dict(filter_width_factor=5.5),
                                  dict(filter_width_factor=2.0), dict(octave_min=-1),
                                  dict(octave_min=1)])
def test_lean_levels_all_widths(gpu_ctx, over):
    imgs = synth_batch(2, 517, 389, 77)
    opts = default_options(**over)
    gpu_ctx.set_options(opts)
    try:
        gpu_ctx.set_debug_flags(BLOCK)
        gpu_ctx.extract(imgs)
        ref = [_levels(gpu_ctx, i, opts) for i in (0, 1)]
        gpu_ctx.set_debug_flags(0)
        gpu_ctx.extract(imgs)
        got = [_levels(gpu_ctx, i, opts) for i in (0, 1)]
        for a, b in zip(ref, got):
            for o, (la, lb) in enumerate(zip(a, b)):
                for lvl, (x, y) in enumerate(zip(la, lb)):
                    assert np.array_equal(_bits(x), _bits(y)), (o, lvl)
        r = O.gaussian(imgs[1], len(got[1]) - 1, opts.dog_level_num + 2, opts)
        assert np.array_equal(_bits(got[1][-1][-1]), _bits(r))
    finally:
        gpu_ctx.set_debug_flags(0)
        gpu_ctx.set_options(default_options())


@pytest.mark.parametrize("fo", [1, -1])
def test_block_first_octave_float_path(gpu_ctx, fo):
    """-fo != 0 feeds the first level from an f32 buffer (the resampled input); the block kernel
    (the wave kernel runs this case in test_gpu_parity.py::test_first_octave_levels_bitwise)."""
    img = synth_image(321, 241, 17 + fo)
    opts = default_options(octave_min=fo)
    gpu_ctx.set_options(opts)
    gpu_ctx.set_debug_flags(BLOCK)
    try:
        gpu_ctx.extract(img)
        for o in range(min(len(gpu_ctx.geometry()), 2)):
            for lvl in range(opts.dog_level_num + 3):
                g = gpu_ctx.gaussian(0, o, lvl)
                r = O.gaussian(img, o, lvl, opts)
                assert np.array_equal(_bits(g), _bits(r)), (o, lvl)
    finally:
        gpu_ctx.set_debug_flags(0)
        gpu_ctx.set_options(default_options())


@pytest.mark.parametrize("n,w,h,no", [(3, 1920, 1080, 4), (2, 517, 389, -1), (1, 4096, 4096, 6)])
def test_octave_streams_equal_serial(gpu_ctx, n, w, h, no):
    """The shipped one-stream schedule (flags 0: the diagonal schedule, octave o+1's first
    levels sharing k_gauss_diag launches with octave o's last ones, and the paired-level kernels
    where they apply) against the serial one-level-per-launch order (SGPU_DEBUG_PYR_SERIAL): the
    same levels and keypoints, bit for bit -- the schedules only reorder or fuse launches whose
    inputs are complete."""
    imgs = synth_batch(n, w, h, 90 + n)
    opts = default_options(octave_num=no) if no > 0 else default_options()
    gpu_ctx.set_options(opts)
    try:
        gpu_ctx.set_debug_flags(gpu_ctx.DEBUG_PYR_SERIAL)
        gpu_ctx.extract(imgs)
        ref = _levels(gpu_ctx, n - 1, opts)
        k_ref = [gpu_ctx.features(i)[0].copy() for i in range(n)]
        for flags in (0, gpu_ctx.DEBUG_DUO_ALWAYS):
            gpu_ctx.set_debug_flags(flags)
            gpu_ctx.extract(imgs)
            got = _levels(gpu_ctx, n - 1, opts)
            for o, (la, lb) in enumerate(zip(ref, got)):
                for lvl, (x, y) in enumerate(zip(la, lb)):
                    assert np.array_equal(_bits(x), _bits(y)), (flags, o, lvl)
            for i in range(n):
                assert np.array_equal(_bits(gpu_ctx.features(i)[0]), _bits(k_ref[i])), flags
    finally:
        gpu_ctx.set_debug_flags(0)
        gpu_ctx.set_options(default_options())


DUO = sgpu.SiftContext.DEBUG_DUO_ALWAYS
DUO_OFF = sgpu.SiftContext.DEBUG_DUO_OFF


# band heights: auto, one chunk (each band re-walks 2 (RA + RB) halo rows), not a multiple of
# 8, taller than the image; sizes: tiny (one strip with both edges), ragged widths (not a
# multiple of the 104- / 116-column strips), odd heights (the (H-1, H-1) bottom pair), 1080p
@pytest.mark.parametrize("pairs", [sgpu.SiftContext.PAIRS_END, sgpu.SiftContext.PAIRS_FRONT])
@pytest.mark.parametrize("rows", [0, 8, 36, 2040])
@pytest.mark.parametrize("n,w,h", [(2, 16, 16), (3, 203, 97), (2, 1920, 1080), (2, 300, 1203),
                                   (1, 104, 33)])
def test_duo_levels_equal_single_level(gpu_ctx, pairs, rows, n, w, h):
    """The paired-level kernel (k_gauss_duo: levels k+1, k+2 from level k in one pass, both
    vertical passes pushed into register accumulators) against one level per launch
    (SGPU_DEBUG_DUO_OFF): every level of every octave and every keypoint, bit for bit.  The pairs
    from the octave's end take the u8 ingest pair (13, 11), (13, 17) with the second level
    decimated and (21, 25); from its front (11, 13) and (17, 21) with the first decimated."""
    imgs = synth_batch(n, w, h, 140 + w % 11)
    opts = default_options()
    gpu_ctx.set_options(opts)
    try:
        gpu_ctx.set_debug_flags(DUO_OFF)
        gpu_ctx.extract(imgs)
        ref = [_levels(gpu_ctx, i, opts) for i in (0, n - 1)]
        k_ref = [gpu_ctx.features(i)[0].copy() for i in range(n)]
        gpu_ctx.set_schedule(gpu_ctx.TRIO_OFF, pairs)
        gpu_ctx.set_debug_flags((rows << sgpu.SiftContext.DEBUG_BAND_SHIFT) | DUO)
        gpu_ctx.extract(imgs)
        got = [_levels(gpu_ctx, i, opts) for i in (0, n - 1)]
        for a, b in zip(ref, got):
            for o, (la, lb) in enumerate(zip(a, b)):
                for lvl, (x, y) in enumerate(zip(la, lb)):
                    assert np.array_equal(_bits(x), _bits(y)), (o, lvl)
        for i in range(n):
            assert np.array_equal(_bits(gpu_ctx.features(i)[0]), _bits(k_ref[i]))
    finally:
        gpu_ctx.set_schedule()
        gpu_ctx.set_debug_flags(0)


@pytest.mark.parametrize("w,h,seed", [(640, 480, 1000), (1921, 1081, 5)])
def test_duo_levels_vs_oracle(gpu_ctx, w, h, seed):
    """k_gauss_duo's levels against the oracle (FilterH / FilterV, ProgramCU.cu:115-222), every
    level of every octave."""
    img = synth_image(w, h, seed)
    opts = default_options()
    gpu_ctx.set_options(opts)
    gpu_ctx.set_debug_flags(DUO)
    try:
        gpu_ctx.extract(img)
        for o in range(len(gpu_ctx.geometry())):
            for lvl in range(opts.dog_level_num + 3):
                g = gpu_ctx.gaussian(0, o, lvl)
                r = O.gaussian(img, o, lvl, opts)
                assert np.array_equal(_bits(g), _bits(r)), (o, lvl)
    finally:
        gpu_ctx.set_debug_flags(0)


# sizes: ragged (odd heights: the (H-1, H-1) bottom pairs and a last row that decimates into
# no row; octave 1's padded width takes no trio), 1080p (the shipped case: two bands), a tall
# ragged batch (three strips), a narrow one (one strip with both edges, 2 octaves), a small
# square; band heights as the duo's
@pytest.mark.parametrize("rows", [0, 8, 36, 2040])
@pytest.mark.parametrize("n,w,h", [(3, 203, 97), (2, 1920, 1080), (2, 296, 1203), (1, 104, 33),
                                   (2, 64, 64)])
def test_trio_levels_equal_single_level(gpu_ctx, rows, n, w, h):
    """The three-level kernel (k_gauss_trio: levels k+1 .. k+3 and the decimation from level k in
    one pass, three vertical passes pushed into register accumulators, sgpu_debug_set_schedule
    ALWAYS) against one level per launch (SGPU_DEBUG_DUO_OFF): every level of every octave and
    every keypoint, bit for bit; and it ran (fewer launches than one level per launch)."""
    imgs = synth_batch(n, w, h, 170 + w % 13)
    opts = default_options()
    gpu_ctx.set_options(opts)
    try:
        gpu_ctx.set_debug_flags(DUO_OFF)
        gpu_ctx.extract(imgs)
        ref = [_levels(gpu_ctx, i, opts) for i in (0, n - 1)]
        k_ref = [gpu_ctx.features(i)[0].copy() for i in range(n)]
        band = rows << sgpu.SiftContext.DEBUG_BAND_SHIFT
        gpu_ctx.set_schedule(gpu_ctx.TRIO_OFF)
        gpu_ctx.set_debug_flags(band)
        gpu_ctx.extract(imgs)
        single_launches = gpu_ctx.pyramid_launches()[0]
        # the trio alone (levels too small for pairs), then beside the paired levels
        for flags in (band, band | DUO):
            gpu_ctx.set_schedule(gpu_ctx.TRIO_ALWAYS)
            gpu_ctx.set_debug_flags(flags)
            gpu_ctx.extract(imgs)
            if flags == band:
                assert gpu_ctx.pyramid_launches()[0] < single_launches
            got = [_levels(gpu_ctx, i, opts) for i in (0, n - 1)]
            for a, b in zip(ref, got):
                for o, (la, lb) in enumerate(zip(a, b)):
                    for lvl, (x, y) in enumerate(zip(la, lb)):
                        assert np.array_equal(_bits(x), _bits(y)), (flags, o, lvl)
            for i in range(n):
                assert np.array_equal(_bits(gpu_ctx.features(i)[0]), _bits(k_ref[i]))
    finally:
        gpu_ctx.set_schedule()
        gpu_ctx.set_debug_flags(0)


@pytest.mark.parametrize("w,h,seed", [(640, 480, 1000), (1921, 1081, 5)])
def test_trio_levels_vs_oracle(gpu_ctx, w, h, seed):
    """k_gauss_trio's levels (and the decimated next-octave bases) against the oracle
    (FilterH / FilterV, ProgramCU.cu:115-222; DownsampleKernel, :287-298), every level of every
    octave."""
    img = synth_image(w, h, seed)
    opts = default_options()
    gpu_ctx.set_options(opts)
    gpu_ctx.set_schedule(gpu_ctx.TRIO_ALWAYS)
    try:
        gpu_ctx.extract(img)
        for o in range(len(gpu_ctx.geometry())):
            for lvl in range(opts.dog_level_num + 3):
                g = gpu_ctx.gaussian(0, o, lvl)
                r = O.gaussian(img, o, lvl, opts)
                assert np.array_equal(_bits(g), _bits(r)), (o, lvl)
    finally:
        gpu_ctx.set_schedule()


TILE = sgpu.SiftContext.DEBUG_GAUSS_TILE_ALWAYS
TILE_OFF = sgpu.SiftContext.DEBUG_GAUSS_TILE_OFF


# sizes: tiny (one tile with every edge), ragged (width not a multiple of 64, height not of 32),
# 1080p (C2's image: every level tiled by default), a tall ragged batch, C4's 4096^2 x 6 octaves
@pytest.mark.parametrize("n,w,h,no", [(2, 16, 16, -1), (3, 203, 97, -1), (1, 1920, 1080, 4),
                                      (2, 300, 1203, -1), (1, 4096, 4096, 6)])
def test_tile_levels_equal_wave_kernel(gpu_ctx, n, w, h, no):
    """The 2-D tile kernel (k_gauss_tile / k_gauss_tile_diag, sift_gauss_tile.hip: a workgroup's
    whole input window loaded at once, H pass into LDS, V pass from LDS) for every level against
    the wave-streaming kernels (SGPU_DEBUG_GAUSS_TILE_OFF): every level of every octave and every
    keypoint, bit for bit -- including the u8 ingest level and the decimating levels."""
    imgs = synth_batch(n, w, h, 170 + w % 13)
    opts = default_options(octave_num=no) if no > 0 else default_options()
    gpu_ctx.set_options(opts)
    try:
        gpu_ctx.set_debug_flags(TILE_OFF)
        gpu_ctx.extract(imgs)
        ref = [_levels(gpu_ctx, i, opts) for i in (0, n - 1)]
        k_ref = [gpu_ctx.features(i)[0].copy() for i in range(n)]
        # TILE | DUO: the tile-duo schedule (two levels per tile launch, SGPU_TILE_DUO)
        for flags in (TILE, TILE | DUO, TILE | gpu_ctx.DEBUG_PYR_SERIAL, 0):
            gpu_ctx.set_debug_flags(flags)
            gpu_ctx.extract(imgs)
            got = [_levels(gpu_ctx, i, opts) for i in (0, n - 1)]
            for a, b in zip(ref, got):
                for o, (la, lb) in enumerate(zip(a, b)):
                    for lvl, (x, y) in enumerate(zip(la, lb)):
                        assert np.array_equal(_bits(x), _bits(y)), (flags, o, lvl)
            for i in range(n):
                assert np.array_equal(_bits(gpu_ctx.features(i)[0]), _bits(k_ref[i])), flags
    finally:
        gpu_ctx.set_debug_flags(0)
        gpu_ctx.set_options(default_options())


# every filter width 5 .. 33 (as test_lean_levels_all_widths), first octaves -1 / 0 / 1 (the
# float first level after the resampling), float input
@pytest.mark.parametrize("over", [dict(dog_level_num=1), dict(dog_level_num=2),
                                  dict(dog_level_num=5), dict(filter_width_factor=5.5),
                                  dict(filter_width_factor=2.0), dict(octave_min=-1),
                                  dict(octave_min=1)])
def test_tile_levels_all_widths(gpu_ctx, over):
    imgs = synth_batch(2, 517, 389, 77)
    opts = default_options(**over)
    gpu_ctx.set_options(opts)
    try:
        gpu_ctx.set_debug_flags(TILE_OFF)
        gpu_ctx.extract(imgs)
        ref = [_levels(gpu_ctx, i, opts) for i in (0, 1)]
        for flags in (TILE, TILE | DUO):
            gpu_ctx.set_debug_flags(flags)
            gpu_ctx.extract(imgs)
            got = [_levels(gpu_ctx, i, opts) for i in (0, 1)]
            for a, b in zip(ref, got):
                for o, (la, lb) in enumerate(zip(a, b)):
                    for lvl, (x, y) in enumerate(zip(la, lb)):
                        assert np.array_equal(_bits(x), _bits(y)), (flags, o, lvl)
        gpu_ctx.set_debug_flags(TILE)
        fimgs = (imgs.astype(np.float32) / np.float32(255.0)).astype(np.float32)
        gpu_ctx.extract(fimgs[1])
        got_f = [[gpu_ctx.gaussian(0, o, lvl).copy() for lvl in range(opts.dog_level_num + 3)]
                 for o in range(len(gpu_ctx.geometry()))]
        gpu_ctx.set_debug_flags(TILE_OFF)
        gpu_ctx.extract(fimgs[1])
        for o in range(len(got_f)):
            for lvl in range(opts.dog_level_num + 3):
                assert np.array_equal(_bits(gpu_ctx.gaussian(0, o, lvl)), _bits(got_f[o][lvl])), (o, lvl)
    finally:
        gpu_ctx.set_debug_flags(0)
        gpu_ctx.set_options(default_options())


@pytest.mark.parametrize("w,h,seed", [(640, 480, 1000), (1921, 1081, 5)])
def test_tile_levels_vs_oracle(gpu_ctx, w, h, seed):
    """k_gauss_tile's levels (the shipped single-image path) against the oracle (FilterH /
    FilterV, ProgramCU.cu:115-222), every level of every octave."""
    img = synth_image(w, h, seed)
    opts = default_options()
    gpu_ctx.set_options(opts)
    gpu_ctx.set_debug_flags(TILE)
    try:
        gpu_ctx.extract(img)
        for o in range(len(gpu_ctx.geometry())):
            for lvl in range(opts.dog_level_num + 3):
                g = gpu_ctx.gaussian(0, o, lvl)
                r = O.gaussian(img, o, lvl, opts)
                assert np.array_equal(_bits(g), _bits(r)), (o, lvl)
    finally:
        gpu_ctx.set_debug_flags(0)


def test_debug_flags_do_not_alias_band_field(gpu_ctx):
    """the descriptor-kernel flag used to share bit 16 with the band-height field.
    Every flag bit now lies below SGPU_DEBUG_BAND_SHIFT, and a forced band height leaves the
    descriptor kernel alone: same descriptors with and without (8 << shift)."""
    C = sgpu.SiftContext
    flags = [v for k, v in vars(C).items() if k.startswith("DEBUG_") and k != "DEBUG_BAND_SHIFT"]
    assert all(0 < f < (1 << C.DEBUG_BAND_SHIFT) for f in flags)
    assert len(set(flags)) == len(flags)
    img = synth_image(640, 480, 31)
    gpu_ctx.set_options(default_options())
    try:
        gpu_ctx.set_debug_flags(0)
        gpu_ctx.extract(img)
        k0, d0 = gpu_ctx.features(0)
        gpu_ctx.set_debug_flags(8 << C.DEBUG_BAND_SHIFT)
        gpu_ctx.extract(img)
        k1, d1 = gpu_ctx.features(0)
        assert np.array_equal(_bits(k0), _bits(k1)) and np.array_equal(_bits(d0), _bits(d1))
    finally:
        gpu_ctx.set_debug_flags(0)
