"""ctypes mirror of include/sfmfeat.h (constants and the POD parameter struct).

Pure Python: importing this module loads no native code.  `params_from_dict` maps the
reference's `extractor_params` dict (read with `.get(key, default)` at
FeatureExtractor.py:11, NaiveSIFT.py:35-39, ScaleRotInvSIFT.py:12-13) onto `SfmParams`.
"""
from __future__ import annotations

import ctypes

import numpy as np

SFM_OK = 0
SFM_EINVAL = 1
SFM_ESTATE = 2
SFM_EDEVICE = 3
SFM_ERANGE = 4
SFM_EINDEX = 5

SFM_MODE_SCALEROT = 0
SFM_MODE_NAIVE = 1

SFM_DESC_DIM = 128
SFM_MAX_GAUSS = 15
SFM_MAX_KSIZE = 31
SFM_MAX_FW = 64
SFM_MAX_LEVELS = 12


class SfmParams(ctypes.Structure):
    _fields_ = [
        ("mode", ctypes.c_int32),
        ("num_interest_points", ctypes.c_int32),
        ("ksize", ctypes.c_int32),
        ("gaussian_size", ctypes.c_int32),
        ("feature_width", ctypes.c_int32),
        ("pyramid_level", ctypes.c_int32),
        ("sigma", ctypes.c_double),
        ("alpha", ctypes.c_double),
        ("pyramid_scale_factor", ctypes.c_double),
        ("gauss_kernel_set", ctypes.c_int32),
        ("reserved0", ctypes.c_int32),
        ("gauss_kernel", ctypes.c_float * (SFM_MAX_GAUSS * SFM_MAX_GAUSS)),
    ]


def generate_gaussian_kernel(ksize: int, sigma: float) -> np.ndarray:
    """Same expression as NaiveSIFT._generate_gaussian_kernel (NaiveSIFT.py:175-199),
    evaluated by numpy so the float32 taps handed to the device are the reference's."""
    mean = ksize // 2
    axis = np.linspace(-mean, mean, ksize)
    x_square = axis[:, np.newaxis] ** 2
    y_square = axis[np.newaxis, :] ** 2
    kernel = (1 / (2 * np.pi * sigma ** 2)) * np.exp(-(x_square + y_square) / (2 * sigma ** 2))
    kernel = kernel / np.sum(kernel)
    return kernel


def params_from_dict(extractor_params: dict | None, mode: int) -> SfmParams:
    ep = {} if extractor_params is None else extractor_params
    p = SfmParams()
    p.mode = mode
    p.num_interest_points = int(ep.get("num_interest_points", 2500))
    p.ksize = int(ep.get("ksize", 7))
    p.gaussian_size = int(ep.get("gaussian_size", 7))
    p.sigma = float(ep.get("sigma", 5))
    p.alpha = float(ep.get("alpha", 0.05))
    p.feature_width = int(ep.get("feature_width", 16))
    p.pyramid_level = int(ep.get("pyramid_level", 4)) if mode == SFM_MODE_SCALEROT else 1
    p.pyramid_scale_factor = float(ep.get("pyramid_scale_factor", 2))
    gs = p.gaussian_size
    if 1 <= gs <= SFM_MAX_GAUSS:
        k = generate_gaussian_kernel(gs, ep.get("sigma", 5)).astype(np.float32).ravel()
        for i, v in enumerate(k):
            p.gauss_kernel[i] = float(v)
        p.gauss_kernel_set = 1
    return p


def keypoint_capacity(p: SfmParams) -> int:
    if p.mode == SFM_MODE_NAIVE:
        return max(int(p.num_interest_points), 0)
    L = int(p.pyramid_level)
    return max(L * int(p.num_interest_points / L), 0)
