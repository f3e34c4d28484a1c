"""Drop-in extractor plugins: NaiveSIFT and ScaleRotInvSIFT on the MI355X HIP path.

Same constructor signature, method names, return types and error behaviour as the
reference classes (FeatureExtractor/SIFT/NaiveSIFT.py, FeatureExtractor/SIFT/
ScaleRotInvSIFT.py); the arithmetic runs in libsfmfeat (include/sfmfeat.h).  There is
no CPU fallback: without the library or a GPU, construction / detection raises.
"""
from __future__ import annotations

import os
import threading
from typing import Tuple

import numpy as np

from . import _abi
from ._native import context_for
from .feature_extractor import FeatureExtractor

_DEFAULT_DEVICE = int(os.environ.get("SFMFEAT_DEVICE", "0"))
_tls = threading.local()


def set_device(device: int) -> None:
    """HIP device used by the drop-in classes (extractors and matcher) for this thread's
    future calls; other threads keep theirs (the reference drives the classes from 8 threads,
    Runner.py:183-191).  A thread that never calls it uses SFMFEAT_DEVICE (default 0)."""
    _tls.device = int(device)


def current_device() -> int:
    """This thread's device for the drop-in classes (set_device, else SFMFEAT_DEVICE)."""
    return getattr(_tls, "device", _DEFAULT_DEVICE)


def _reference_fvs(desc: np.ndarray) -> np.ndarray:
    """np.squeeze(np.array(fvs)) of NaiveSIFT.py:173 / ScaleRotInvSIFT.py:87:
    (n,128) for n >= 2, (128,) for n == 1, float64 (0,) for n == 0."""
    if desc.shape[0] == 0:
        return np.squeeze(np.array([]))
    return np.squeeze(desc.reshape(desc.shape[0], 128, 1))


class NaiveSIFT(FeatureExtractor):
    """Harris detector + un-rotated 4x4x8 RootSIFT descriptors (NaiveSIFT.py:9-213)."""

    def __init__(self, image_bw: np.ndarray, extractor_params: dict = {}):  # noqa: B006 (reference signature)
        self.SOBEL_X_KERNEL = np.array([[-1, 0, 1], [-2, 0, 2], [-1, 0, 1]]).astype(np.float32)
        self.SOBEL_Y_KERNEL = np.array([[-1, -2, -1], [0, 0, 0], [1, 2, 1]]).astype(np.float32)
        super().__init__(image_bw, extractor_params)
        self._ksize = extractor_params.get("ksize", 7)
        self._gaussian_size = extractor_params.get("gaussian_size", 7)
        self._sigma = extractor_params.get("sigma", 5)
        self._alpha = extractor_params.get("alpha", 0.05)
        self._feature_width = extractor_params.get("feature_width", 16)
        self._extractor_params = extractor_params

    def _run(self, mode: int):
        img = np.asarray(self.image)
        assert img.ndim == 2, "Image must be grayscale"
        params = _abi.params_from_dict(self._extractor_params, mode)
        return context_for(params, current_device()).extract(img)

    def detect_keypoints(self) -> Tuple[np.ndarray, np.ndarray]:
        """Detect interest points using Harris corner detection (NaiveSIFT.py:42-45)."""
        X, Y, D, C, _ = self._run(_abi.SFM_MODE_NAIVE)
        self._X, self._Y, self.confidences = X, Y, C
        self._descriptors_dev = D
        return self._X, self._Y

    def extract_descriptors(self) -> np.ndarray:
        """Extract SIFT descriptors at detected keypoints (NaiveSIFT.py:47-52)."""
        if not hasattr(self, "_X") or not hasattr(self, "_Y"):
            raise RuntimeError("Keypoints not detected. Call detect_keypoints() before extract_descriptors().")
        self.descriptors = _reference_fvs(self._descriptors_dev)
        return self.descriptors


class ScaleRotInvSIFT(NaiveSIFT):
    """Resize pyramid + per-level Harris + dominant-orientation descriptors; all work is
    done eagerly in the constructor like ScaleRotInvSIFT.py:9-16."""

    def __init__(self, image_bw: np.ndarray, extractor_params: dict = {}):  # noqa: B006
        super().__init__(image_bw, extractor_params)
        self._pyramid_level = extractor_params.get("pyramid_level", 4)
        self._pyramid_scale_factor = extractor_params.get("pyramid_scale_factor", 2)
        self.compute(self.num_interest_points)

    def detect_keypoints(self):
        return self._X, self._Y

    def extract_descriptors(self):
        return self._feature_vec

    def compute(self, k: int):
        """ScaleRotInvSIFT.compute (ScaleRotInvSIFT.py:89-107): level-ordered concatenation
        with the reference's list semantics (a level with exactly one keypoint is extended
        element-wise, :103)."""
        params = dict(self._extractor_params)
        params["num_interest_points"] = k
        X, Y, D, C, lc = self._run_params(params)
        xs, ys, fv = [], [], []
        off = 0
        for n in lc.tolist():
            xs.extend(X[off:off + n])
            ys.extend(Y[off:off + n])
            fv.extend(_reference_fvs(D[off:off + n]))
            off += n
        self._X = np.array(xs)
        self._Y = np.array(ys)
        self._feature_vec = np.array(fv)
        self.confidences = C

    def _run_params(self, params: dict):
        img = np.asarray(self.image)
        assert img.ndim == 2, "Image must be grayscale"
        p = _abi.params_from_dict(params, _abi.SFM_MODE_SCALEROT)
        return context_for(p, current_device()).extract(img)
