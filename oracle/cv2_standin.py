"""TEST INFRASTRUCTURE ONLY — numpy restatement of the two OpenCV calls on the hot path.

opencv-python 4.10.0.84 (reference requirements.txt:25) is not installed in this image
and cannot be installed offline.  tools/gen_golden.py injects this module as `cv2`
before importing the reference, so the reference's own numpy code (Harris, max-pool,
median, top-k, histograms, descriptors, matcher) runs unmodified and produces the
golden vectors.  The rules below are the ones oracle/sfm_oracle.c and the HIP kernels
implement; parity with real OpenCV is UNPINNED for these two calls.

filter2D  (NaiveSIFT.py:67-69, 212-213): correlation, anchor at the kernel centre,
          BORDER_CONSTANT zeros, float32 kernel; acc = +0, then acc = fma(k, p, acc) for
          every non-zero tap in row-major kernel order (OpenCV's FilterVec_32f v_muladd
          chain).  numpy has no fused multiply-add, so this delegates to the C oracle's
          orc_filter2d (fmaf), the same restatement the oracle and the HIP kernels use.
resize    (ScaleRotInvSIFT.py:114), INTER_LINEAR on float32: exact 2x downscale uses
          OpenCV's INTER_AREA-fast switch ((a00+a01)+(a10+a11))*0.25; otherwise
          half-pixel bilinear with OpenCV's coefficient rule (see _coeffs).
"""
from __future__ import annotations

import numpy as np

BORDER_CONSTANT = 0
INTER_LINEAR = 1


def filter2D(src, ddepth, kernel, dst=None, anchor=None, delta=0, borderType=BORDER_CONSTANT):
    src = np.asarray(src)
    if src.dtype != np.float32 or src.ndim != 2:
        raise TypeError("cv2 stand-in: filter2D supports 2-D float32 only")
    if ddepth != -1 or borderType != BORDER_CONSTANT or delta != 0:
        raise TypeError("cv2 stand-in: only ddepth=-1, BORDER_CONSTANT, delta=0")
    from oracle import oracle as _orc  # C restatement with fmaf
    k = np.asarray(kernel).astype(np.float32)
    return _orc.filter2d(np.ascontiguousarray(src), k)


def _coeffs(dn: int, sn: int):
    inv = dn / sn
    scale = 1.0 / inv
    d = np.arange(dn, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = f - s.astype(np.float32)
    neg = s < 0
    s[neg] = 0
    f[neg] = 0
    single = s + 1 >= sn
    clamp = s >= sn - 1
    s[clamp] = sn - 1
    f[clamp] = 0
    return s, (np.float32(1) - f).astype(np.float32), f.astype(np.float32), single


def resize(src, dsize, dst=None, fx=None, fy=None, interpolation=INTER_LINEAR):
    src = np.asarray(src)
    if src.dtype != np.float32 or src.ndim != 2:
        raise TypeError("cv2 stand-in: resize supports 2-D float32 only")
    if interpolation != INTER_LINEAR:
        raise TypeError("cv2 stand-in: INTER_LINEAR only")
    dw, dh = int(dsize[0]), int(dsize[1])
    H, W = src.shape
    if dw <= 0 or dh <= 0:
        raise ValueError("cv2 stand-in: empty dsize")
    if H == 2 * dh and W == 2 * dw:
        t0 = src[0:2 * dh:2, 0:2 * dw:2] + src[0:2 * dh:2, 1:2 * dw:2]
        t1 = src[1:2 * dh:2, 0:2 * dw:2] + src[1:2 * dh:2, 1:2 * dw:2]
        return ((t0 + t1) * np.float32(0.25)).astype(np.float32)
    xo, xa0, xa1, xs = _coeffs(dw, W)
    yo, ya0, ya1, _ = _coeffs(dh, H)
    xo1 = np.minimum(xo + 1, W - 1)
    yo1 = np.minimum(yo + 1, H - 1)

    def hrow(S):
        two = S[:, xo] * xa0 + S[:, xo1] * xa1
        return np.where(xs[None, :], S[:, xo], two).astype(np.float32)

    h0 = hrow(src[yo])
    h1 = hrow(src[yo1])
    return (h0 * ya0[:, None] + h1 * ya1[:, None]).astype(np.float32)
