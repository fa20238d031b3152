"""GPU parity for the first-octave and feature-count options (SURVEY.md §8 rows A3 and the
RunSIFT stage sequence): -maxd / SetMaxDimension octave skipping (PyramidCU.cpp:129-135), the
-prep / -noprep input sampling of -fo > 0 (GLTexImage.cpp:928-1009) and -tc / -tc2 / -tc3
feature-count limiting (SiftPyramid.cpp:219-260, PyramidCU.cpp:829-853).  The HIP path is
compared with the oracle bit for bit (keys) and to L2 < 1e-4 (descriptors; bitwise in practice)."""
import numpy as np
import pytest

import oracle_py as O
from sgpu_types import default_options
from sift_synth import synth_image

pytestmark = pytest.mark.gpu

DESC_L2_TOL = 1e-4


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _check(gpu_ctx, img, opts, what):
    gpu_ctx.set_options(opts)
    gpu_ctx.extract(img)
    k, d = gpu_ctx.features(0)
    rk, rd = O.extract(img, opts)
    assert k.shape == rk.shape, f"{what}: {k.shape} vs oracle {rk.shape}"
    assert np.array_equal(_bits(k), _bits(rk)), what
    if len(k):
        assert np.linalg.norm(d.astype(np.float64) - rd, axis=1).max() < DESC_L2_TOL, what
    return k


@pytest.mark.parametrize("method", [0, 1, 2])
@pytest.mark.parametrize("threshold", [40, 300, 100000])
def test_feature_count_limit_vs_oracle(gpu_ctx, method, threshold):
    img = synth_image(400, 300, 31)
    k = _check(gpu_ctx, img, default_options(feature_count_threshold=threshold,
                                             truncate_method=method), f"tc{method} {threshold}")
    full = O.extract(img)[0]
    if threshold >= len(full):
        assert len(k) == len(full)          # nothing to drop
    else:
        assert len(k) < len(full)


@pytest.mark.parametrize("over", [{"max_orientation": 1}, {"fixed_orientation": 1},
                                  {"dog_level_num": 4}, {"octave_min": -1}])
def test_feature_count_limit_options(gpu_ctx, over):
    """Without multi-orientation the oriented stage is skipped (SiftPyramid.cpp:152)."""
    img = synth_image(360, 280, 44)
    for method in (0, 1, 2):
        _check(gpu_ctx, img, default_options(feature_count_threshold=150, truncate_method=method,
                                             **over), f"{over} tc{method}")


def test_feature_count_limit_per_image_of_a_batch(gpu_ctx):
    """The limit applies per image (one RunSIFT each), also inside a batch."""
    imgs = np.stack([synth_image(320, 240, 70 + i) for i in range(4)])
    opts = default_options(feature_count_threshold=120, truncate_method=1)
    gpu_ctx.set_options(opts)
    gpu_ctx.extract(imgs)
    for i in range(4):
        k, d = gpu_ctx.features(i)
        rk, rd = O.extract(imgs[i], opts)
        assert np.array_equal(_bits(k), _bits(rk)), i
    gpu_ctx.set_options(default_options())


@pytest.mark.parametrize("maxd,fo,expect_first", [(256, 0, 1), (150, 0, 2), (500, -1, 0),
                                                  (1000, -1, -1), (100, 1, 2)])
def test_max_dimension_vs_oracle(gpu_ctx, maxd, fo, expect_first):
    """-maxd raises the first octave while it is wider or taller than the limit."""
    img = synth_image(401, 301, 9)
    opts = default_options(max_dimension=maxd, octave_min=fo)
    _check(gpu_ctx, img, opts, f"maxd {maxd} fo {fo}")
    geo = gpu_ctx.geometry()
    w0 = (401 & ~3) if fo <= 0 else ((401 >> fo) & ~3)
    want = w0 >> expect_first if expect_first >= 0 else w0 << -expect_first
    if fo > 0:   # -prep: sampled by 2^fo first, then raised relative to that image
        want = w0 >> (expect_first - fo)
    assert geo[0][0] == want, (geo[0], want)
    gpu_ctx.set_options(default_options())


@pytest.mark.parametrize("fo", [1, 2])
@pytest.mark.parametrize("prep", [1, 0])
@pytest.mark.parametrize("w,h", [(1012, 301), (203, 97), (400, 300)])
def test_prep_first_octave_vs_oracle(gpu_ctx, fo, prep, w, h):
    """-fo > 0: with -prep (the default) the input is sampled by 2^fo and its width truncated to
    a multiple of 4 before the pyramid; with -noprep the first octave is SampleImageD of the
    full input with the padded width."""
    img = synth_image(w, h, 13 + fo)
    _check(gpu_ctx, img, default_options(octave_min=fo, preprocess_on_cpu=prep),
           f"fo {fo} prep {prep}")
    geo = gpu_ctx.geometry()
    if prep:
        assert geo[0][0] == ((w >> fo) & ~3)
    else:
        assert geo[0][0] == ((w & ~3) >> fo)
    gpu_ctx.set_options(default_options())


def test_prep_first_octave_float_input(gpu_ctx):
    img = synth_image(322, 241, 3).astype(np.float32) / np.float32(255.0)
    opts = default_options(octave_min=1)
    gpu_ctx.set_options(opts)
    gpu_ctx.extract(img)
    k, d = gpu_ctx.features(0)
    rk, rd = O.extract_f32(img, opts)
    assert np.array_equal(_bits(k), _bits(rk))
    gpu_ctx.set_options(default_options())
