"""Certified-mode NMS kernels against a numpy restatement of the predicate.

NaiveSIFT.py:77-95: a pixel is a candidate when R equals the max of R over the ksize x
ksize window clipped to the image; the certified path keeps those whose
order key fkey(R) reaches the plane's threshold tnms.  The streaming kernel (k_nms_stream,
the default for 3x3 and W % 4 == 0) and the tiled kernel (k_nms_tile) must both produce
exactly the numpy candidate key set, on ragged shapes (strips cut by the bottom edge,
column groups wrapping across wavefronts), plateaus and negative values.
"""
from __future__ import annotations

import numpy as np
import pytest

from sfmfromscratch_amd import _native

pytestmark = pytest.mark.gpu


def fkey(a: np.ndarray) -> np.ndarray:
    b = a.astype(np.float32).view(np.uint32).copy()
    b[b == 0x80000000] = 0
    return np.where(b & 0x80000000, ~b, b | 0x80000000).astype(np.uint32)


def numpy_candidates(R: np.ndarray, tnms: int, ksize: int) -> np.ndarray:
    H, W = R.shape
    h = ksize // 2
    P = np.full((H + 2 * h, W + 2 * h), -np.inf, np.float32)
    P[h:h + H, h:h + W] = R
    m = np.full((H, W), -np.inf, np.float32)
    for dy in range(ksize):
        for dx in range(ksize):
            m = np.maximum(m, P[dy:dy + H, dx:dx + W])
    k = fkey(R)
    ok = (k >= np.uint32(tnms)) & (R == m)
    idx = np.flatnonzero(ok.ravel()).astype(np.uint64)
    keys = ((~k.ravel()[idx]).astype(np.uint64) << np.uint64(32)) | idx
    return np.sort(keys)


def planes(B, H, W, seed):
    rng = np.random.default_rng(seed)
    R = rng.standard_normal((B, H, W)).astype(np.float32)
    R[0] = np.round(R[0] * 2) / 2           # plateaus: many equal neighbours
    if B > 1:
        R[1] = np.abs(R[1]) * 1e3           # positive, large
    if B > 2:
        R[2, :, : W // 2] = 0.0             # a flat half (R == 0 plateaus)
    return R


@pytest.mark.parametrize("B,H,W", [(3, 37, 100), (2, 64, 256), (3, 270, 480), (2, 9, 4), (1, 540, 960),
                                   (2, 33, 102)])
@pytest.mark.parametrize("quantile", [0.0, 0.5, 0.97])
def test_certified_nms_stream_and_tile_vs_numpy(B, H, W, quantile):
    R = planes(B, H, W, seed=H * 1000 + W)
    tnms = np.array([np.quantile(fkey(R[b]).astype(np.float64), quantile) for b in range(B)]).astype(np.uint32)
    want = [numpy_candidates(R[b], int(tnms[b]), 3) for b in range(B)]
    for tile in (False, True):
        got = _native.debug_nms(R, tnms, ksize=3, tile=tile)
        for b in range(B):
            assert got[b].size == want[b].size, (tile, b, got[b].size, want[b].size)
            assert np.array_equal(got[b], want[b]), (tile, b)


@pytest.mark.parametrize("ksize", [1, 5, 7])
def test_certified_nms_other_window_sizes_vs_numpy(ksize):
    R = planes(2, 45, 120, seed=ksize)
    tnms = np.array([np.quantile(fkey(R[b]).astype(np.float64), 0.8) for b in range(2)]).astype(np.uint32)
    got = _native.debug_nms(R, tnms, ksize=ksize)
    for b in range(2):
        assert np.array_equal(got[b], numpy_candidates(R[b], int(tnms[b]), ksize)), b
