"""NNRatioFeatureMatcher on the MI355X HIP path — mirror of
FeatureMatcher/NNRatioFeatureMatcher.py:4-60 (same constructor, method, return types,
IndexError for fewer than two target descriptors, (0,) empty results)."""
from __future__ import annotations

from typing import Tuple

import numpy as np

from . import _abi
from ._native import context_for


def ratio_as_float32(r) -> np.float32:
    """The float32 threshold T such that `nndr <= T` (float32 compare) equals the
    reference's `nndr <= ratio_threshold` (:49) for every float32 nndr.
    Python scalars are NEP 50 'weak' and are cast to float32; a numpy float64 is strong,
    the compare happens in float64, which equals comparing against the largest float32
    <= r."""
    if isinstance(r, np.float32):
        return r
    if isinstance(r, np.floating):
        r64 = np.float64(r)
        r32 = np.float32(r64)
        if np.float64(r32) > r64:
            r32 = np.nextafter(r32, np.float32(-np.inf))
        return r32
    return np.float32(r)


class NNRatioFeatureMatcher:
    def __init__(self, ratio_threshold=0.8):
        self.ratio_threshold = ratio_threshold

    def match_features_ratio_test(self, features1: np.ndarray,
                                  features2: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """Nearest-neighbour distance ratio matching.

        Returns matches (k, 2) int64 [index in features1, index in features2] and
        confidences (k,) float32 sorted ascending; both are empty float64 (0,) arrays when
        nothing matches, like the reference."""
        f1 = np.asarray(features1)
        f2 = np.asarray(features2)
        n1 = 0 if f1.size == 0 else f1.shape[0]
        n2 = 0 if f2.size == 0 else f2.shape[0]
        if n1 > 0 and (f1.ndim != 2 or f1.shape[1] != 128):
            raise ValueError("features1 must be (n, 128)")
        if n2 > 0 and (f2.ndim != 2 or f2.shape[1] != 128):
            raise ValueError("features2 must be (n, 128)")
        if n1 >= 1 and n2 < 2:
            raise IndexError("index 1 is out of bounds for axis 0 with size %d" % n2)
        if n1 == 0:
            return np.array([]), np.array([])
        from .sift import current_device
        params = _abi.params_from_dict({}, _abi.SFM_MODE_NAIVE)
        m, c = context_for(params, current_device()).match(f1.reshape(n1, 128), f2.reshape(n2, 128),
                                                  ratio_as_float32(self.ratio_threshold))
        if len(c) == 0:
            return np.array([]), np.array([])
        return m.astype(np.int64), c.astype(np.float32)
