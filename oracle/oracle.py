"""TEST INFRASTRUCTURE ONLY — ctypes front-end of the C oracle (oracle/sfm_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module; the product package never does.  Every function mirrors one reference
function (see the citations in sfm_oracle.c).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from sfmfromscratch_amd._abi import SfmParams, params_from_dict, keypoint_capacity, SFM_MODE_SCALEROT

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

_fp = ctypes.POINTER(ctypes.c_float)
_dp = ctypes.POINTER(ctypes.c_double)
_i64p = ctypes.POINTER(ctypes.c_int64)
_i32p = ctypes.POINTER(ctypes.c_int32)


def build(force: bool = False) -> str:
    src = os.path.join(_HERE, "sfm_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_gaussian_kernel.argtypes = [ctypes.c_int, ctypes.c_double, _fp]
        L.orc_filter2d.argtypes = [_fp, ctypes.c_int, ctypes.c_int, _fp, ctypes.c_int, ctypes.c_int, _fp]
        L.orc_resize.argtypes = [_fp, ctypes.c_int, ctypes.c_int, _fp, ctypes.c_int, ctypes.c_int]
        L.orc_pyramid_dims.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, _i32p]
        L.orc_harris_response.argtypes = [_fp, ctypes.c_int, ctypes.c_int, _fp, ctypes.c_int, ctypes.c_double, _fp]
        L.orc_median.argtypes = [_fp, ctypes.c_long]
        L.orc_median.restype = ctypes.c_float
        L.orc_detect.argtypes = [_fp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 _fp, ctypes.c_int, ctypes.c_double, _i64p, _i64p, _fp, _dp]
        L.orc_detect.restype = ctypes.c_long
        L.orc_atan2f_vec.argtypes = [_fp, _fp, _fp, ctypes.c_long]
        L.orc_histogram.argtypes = [_dp, _fp, ctypes.c_int, _dp, ctypes.c_int, _fp]
        L.orc_descriptors.argtypes = [_fp, ctypes.c_int, ctypes.c_int, _i64p, _i64p, ctypes.c_long,
                                      ctypes.c_int, ctypes.c_int, _fp]
        L.orc_extract.argtypes = [_fp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(SfmParams), _i64p, _i64p,
                                  _fp, _fp, ctypes.c_long, _i32p]
        L.orc_extract.restype = ctypes.c_long
        L.orc_match.argtypes = [_fp, ctypes.c_long, _fp, ctypes.c_long, ctypes.c_float, _i64p, _fp]
        L.orc_match.restype = ctypes.c_long
        L.orc_sqdist128.argtypes = [_fp, _fp]
        L.orc_sqdist128.restype = ctypes.c_float
        _lib = L
    return _lib


def _f(a):
    return a.ctypes.data_as(_fp)


def _c32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def gaussian_kernel(ks: int, sigma: float) -> np.ndarray:
    out = np.zeros(ks * ks, np.float32)
    rc = lib().orc_gaussian_kernel(ks, float(sigma), _f(out))
    assert rc == 0
    return out.reshape(ks, ks)


def filter2d(img, ker):
    img, ker = _c32(img), _c32(ker)
    out = np.empty_like(img)
    lib().orc_filter2d(_f(img), img.shape[0], img.shape[1], _f(ker), ker.shape[0], ker.shape[1], _f(out))
    return out


def resize(img, dh: int, dw: int):
    img = _c32(img)
    out = np.empty((dh, dw), np.float32)
    rc = lib().orc_resize(_f(img), img.shape[0], img.shape[1], _f(out), dh, dw)
    assert rc == 0
    return out


def pyramid_dims(H, W, L, s):
    d = np.zeros(2 * L, np.int32)
    rc = lib().orc_pyramid_dims(H, W, L, float(s), d.ctypes.data_as(_i32p))
    if rc != 0:
        raise ValueError("bad pyramid")
    return [(int(d[2 * i]), int(d[2 * i + 1])) for i in range(L)]


def harris_response(img, params: dict | None = None):
    p = params_from_dict(params, SFM_MODE_SCALEROT)
    img = _c32(img)
    gk = np.array(p.gauss_kernel[: p.gaussian_size ** 2], np.float32)
    R = np.empty_like(img)
    lib().orc_harris_response(_f(img), img.shape[0], img.shape[1], _f(gk), p.gaussian_size, p.alpha, _f(R))
    return R


def median(R) -> np.float32:
    R = _c32(R)
    return np.float32(lib().orc_median(_f(R), R.size))


def detect(img, k: int, fw: int, params: dict | None = None, debug: bool = False):
    """NaiveSIFT._find_harris_interest_points (NaiveSIFT.py:54-120) -> x, y, c."""
    p = params_from_dict(params, SFM_MODE_SCALEROT)
    img = _c32(img)
    gk = np.array(p.gauss_kernel[: p.gaussian_size ** 2], np.float32)
    kk = max(int(k), 0)
    x = np.zeros(max(kk, 1), np.int64)
    y = np.zeros(max(kk, 1), np.int64)
    c = np.zeros(max(kk, 1), np.float32)
    dbg = np.zeros(3, np.float64)
    m = lib().orc_detect(_f(img), img.shape[0], img.shape[1], kk, int(fw), p.ksize, _f(gk), p.gaussian_size,
                         p.alpha, x.ctypes.data_as(_i64p), y.ctypes.data_as(_i64p), _f(c), dbg.ctypes.data_as(_dp))
    out = (x[:m], y[:m], c[:m])
    if debug:
        return out + ({"median": np.float32(dbg[0]), "n_candidates": int(dbg[1]), "n_top": int(dbg[2])},)
    return out


def atan2(y, x):
    y, x = _c32(y), _c32(x)
    out = np.empty_like(y)
    lib().orc_atan2f_vec(_f(y), _f(x), _f(out), y.size)
    return out


def histogram(values, weights, edges):
    v = np.ascontiguousarray(values, dtype=np.float64).ravel()
    w = _c32(weights).ravel()
    e = np.ascontiguousarray(edges, dtype=np.float64)
    out = np.zeros(len(e) - 1, np.float32)
    lib().orc_histogram(v.ctypes.data_as(_dp), _f(w), v.size, e.ctypes.data_as(_dp), len(e) - 1, _f(out))
    return out


def descriptors(img, X, Y, fw: int, rotate: bool):
    img = _c32(img)
    X = np.ascontiguousarray(X, dtype=np.int64)
    Y = np.ascontiguousarray(Y, dtype=np.int64)
    out = np.zeros((max(len(X), 1), 128), np.float32)
    lib().orc_descriptors(_f(img), img.shape[0], img.shape[1], X.ctypes.data_as(_i64p), Y.ctypes.data_as(_i64p),
                          len(X), int(fw), 1 if rotate else 0, _f(out))
    return out[: len(X)]


def extract(img, params: dict | None = None, mode: int = SFM_MODE_SCALEROT, with_conf: bool = False):
    """Whole extractor: returns X, Y (int64), desc (N,128) float32, level_counts
    (+ per-keypoint Harris confidences when with_conf)."""
    p = params_from_dict(params, mode)
    img = _c32(img)
    cap = max(keypoint_capacity(p), 1)
    X = np.zeros(cap, np.int64)
    Y = np.zeros(cap, np.int64)
    D = np.zeros((cap, 128), np.float32)
    lc = np.zeros(max(p.pyramid_level, 1), np.int32)
    C = np.zeros(cap, np.float32)
    n = lib().orc_extract(_f(img), img.shape[0], img.shape[1], ctypes.byref(p), X.ctypes.data_as(_i64p),
                          Y.ctypes.data_as(_i64p), _f(D), _f(C), cap, lc.ctypes.data_as(_i32p))
    if n < 0:
        raise ValueError(f"oracle extract failed: {-n}")
    if with_conf:
        return X[:n], Y[:n], D[:n], lc, C[:n]
    return X[:n], Y[:n], D[:n], lc


def match(f1, f2, ratio: float = 0.8):
    """NNRatioFeatureMatcher.match_features_ratio_test -> matches (k,2) int64, conf (k,) f32."""
    f1, f2 = _c32(f1), _c32(f2)
    n1, n2 = f1.shape[0], f2.shape[0]
    m = np.zeros((max(n1, 1), 2), np.int64)
    c = np.zeros(max(n1, 1), np.float32)
    k = lib().orc_match(_f(f1), n1, _f(f2), n2, ctypes.c_float(np.float32(ratio)), m.ctypes.data_as(_i64p), _f(c))
    if k < 0:
        raise IndexError("index 1 is out of bounds")
    return m[:k], c[:k]


def sqdist128(a, b) -> np.float32:
    a, b = _c32(a), _c32(b)
    return np.float32(lib().orc_sqdist128(_f(a), _f(b)))
