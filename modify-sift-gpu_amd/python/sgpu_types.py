"""ctypes mirror of `sgpu_options` (include/sgpu.h) and the reference defaults
(SiftGPU/GlobalUtil.cpp:50-135)."""
from __future__ import annotations

import ctypes


class SgpuOptions(ctypes.Structure):
    _fields_ = [
        ("filter_width_factor", ctypes.c_float),
        ("descriptor_window_factor", ctypes.c_float),
        ("orientation_window_factor", ctypes.c_float),
        ("orientation_gaussian_factor", ctypes.c_float),
        ("dog_threshold", ctypes.c_float),
        ("edge_threshold", ctypes.c_float),
        ("subpixel", ctypes.c_int),
        ("max_orientation", ctypes.c_int),
        ("fixed_orientation", ctypes.c_int),
        ("octave_min", ctypes.c_int),
        ("octave_num", ctypes.c_int),
        ("dog_level_num", ctypes.c_int),
        ("lowe_origin", ctypes.c_int),
        ("normalized", ctypes.c_int),
        ("descriptors", ctypes.c_int),
        ("keep_extremum_sign", ctypes.c_int),
        ("circular_window", ctypes.c_int),
        ("verbose", ctypes.c_int),
        ("max_dimension", ctypes.c_int),
        ("preprocess_on_cpu", ctypes.c_int),
        ("feature_count_threshold", ctypes.c_int),
        ("truncate_method", ctypes.c_int),
    ]


def default_options(**kw) -> SgpuOptions:
    o = SgpuOptions(filter_width_factor=4.0, descriptor_window_factor=3.0,
                    orientation_window_factor=2.0, orientation_gaussian_factor=1.5,
                    dog_threshold=0.0, edge_threshold=0.0, subpixel=1, max_orientation=2,
                    fixed_orientation=0, octave_min=0, octave_num=-1, dog_level_num=3,
                    lowe_origin=0, normalized=1, descriptors=1, keep_extremum_sign=0,
                    circular_window=0, verbose=0, max_dimension=13200, preprocess_on_cpu=1,
                    feature_count_threshold=-1, truncate_method=0)
    for k, v in kw.items():
        setattr(o, k, v)
    return o
