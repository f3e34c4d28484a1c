"""FeatureRunner on the HIP path — the reference harness's stage 1 (Runner.py:22-73) with
its image ingest on the device.

The reference decodes each JPEG with PIL (_load_image, Runner.py:551-563), halves it
with PIL's BICUBIC resize (_PIL_resize, :37-42 / :481-493), converts it to gray
(_rgb2gray, :467-478), runs the injected extractor class on both frames and matches them
with NNRatioFeatureMatcher (:49-63).  Here the JPEG decode stays on the host (PIL), the
resize + gray conversion run in libsfmfeat (sfm_ingest_rgb: Pillow's fixed-point
resampler, bit-exact), and the matcher is the HIP one.  The extractor class is the
caller's, exactly as in the reference (any FeatureExtractor plugin: this package's
ScaleRotInvSIFT / NaiveSIFT, or the reference's own).

Plotting (print_img / print_features / print_matches) belongs to the Visualizer side of
the reference and is out of scope: asking for it raises.
"""
from __future__ import annotations

import numpy as np

from . import _abi
from ._native import context_for
from .matcher import NNRatioFeatureMatcher


def load_image_u8(path: str) -> np.ndarray:
    """The decoded frame _load_image reads (Runner.py:561-562), as uint8 (its float32
    /255 copy is exactly reconstructible, tests/test_ingest_cpu.py)."""
    from PIL import Image
    with Image.open(path) as img:
        a = np.asarray(img)
    if a.dtype != np.uint8:
        raise ValueError(f"{path}: expected an 8-bit image, got {a.dtype}")
    return a


def drop_opaque_alpha(a: np.ndarray, what: str = "frame") -> np.ndarray:
    """[H, W, 3] RGB view of a decoded RGB or RGBA frame.  The reference reads channels
    0-2 after `_PIL_resize` (Runner.py:478), and PIL resizes RGBA in premultiplied alpha,
    so only a fully opaque RGBA frame resizes to the same RGB as its RGB channels alone
    (checked against PIL in tests/test_ingest_cpu.py).  Translucent RGBA is rejected
    (ValueError): the device ingest has no premultiplied path (a documented divergence)."""
    if a.ndim != 3 or a.shape[2] not in (3, 4):
        raise ValueError(f"{what}: the reference's _rgb2gray needs an [H, W, 3] RGB (or RGBA) frame")
    if a.shape[2] == 4:
        if not np.all(a[..., 3] == 255):
            raise ValueError(f"{what}: translucent RGBA frames are not supported (PIL resizes them premultiplied)")
        a = a[..., :3]
    return np.ascontiguousarray(a)


def ingest_frame(rgb: np.ndarray, scale_factor: float = 0.5, device: int = 0) -> np.ndarray:
    """Runner.py:33-46 for one decoded frame: resize to (int(W*s), int(H*s)) with PIL's
    BICUBIC filter, then _rgb2gray; float32 [H2, W2].  A 2-D gray frame fails in the
    reference's _rgb2gray (:478) and here (ValueError); RGBA frames go through
    `drop_opaque_alpha`."""
    rgb = drop_opaque_alpha(rgb)
    ctx = context_for(_abi.params_from_dict({}, _abi.SFM_MODE_NAIVE), device)
    return ctx.ingest_rgb(rgb, scale_factor)


def convert_matches_to_coords(sift_matches, X1, Y1, X2, Y2, num_matches=2500):
    """_convert_matches_to_coords (Runner.py:423-434): the first num_matches matches as
    (x, y) pixel pairs; empty input gives two empty float64 arrays."""
    sift_matches = np.asarray(sift_matches)
    if sift_matches.shape[0] == 0:
        return np.array([]), np.array([])
    m = sift_matches[:num_matches]
    pts1 = np.column_stack((X1[m[:, 0]], Y1[m[:, 0]]))
    pts2 = np.column_stack((X2[m[:, 1]], Y2[m[:, 1]]))
    return pts1, pts2


class FeatureRunner:
    """Mirror of Runner.FeatureRunner (Runner.py:22-73): same constructor, attributes
    (_image1_bw, X1, Y1, descriptors1, ..., matches, confidences) and console lines."""

    def __init__(self, im1_path: str, im2_path: str, scale_factor: float = 0.5,
                 feature_extractor_class=None, extractor_params: dict = {},
                 print_img: bool = False, print_features: bool = False,
                 print_matches: bool = False, output_suffix="", match_threshold=0.8, device: int = 0):
        self.feature_extractor = feature_extractor_class
        if self.feature_extractor is None:
            raise ValueError("Please provide a feature extractor class")
        if print_img or print_features or print_matches:
            raise NotImplementedError("plotting is the Visualizer's job (out of scope, DESIGN.md §10)")
        self.outputSuffix = output_suffix
        self._image1_bw = ingest_frame(load_image_u8(im1_path), scale_factor, device)
        self._image2_bw = ingest_frame(load_image_u8(im2_path), scale_factor, device)

        self.extractor1 = self.feature_extractor(self._image1_bw, extractor_params)
        self.extractor2 = self.feature_extractor(self._image2_bw, extractor_params)
        self.X1, self.Y1 = self.extractor1.detect_keypoints()
        self.descriptors1 = self.extractor1.extract_descriptors()
        self.X2, self.Y2 = self.extractor2.detect_keypoints()
        self.descriptors2 = self.extractor2.extract_descriptors()
        print(f'{len(self.X1)} corners in image 1, {len(self.X2)} corners in image 2')
        print(f'{len(self.descriptors1)} descriptors in image 1, {len(self.descriptors2)} descriptors in image 2')

        self.matcher = NNRatioFeatureMatcher(ratio_threshold=match_threshold)
        self.matches, self.confidences = self.matcher.match_features_ratio_test(self.descriptors1,
                                                                                self.descriptors2)
        print(f'{len(self.matches)} matches found')
