"""sfmfromscratch_amd — MI355X-native detect + describe + match stage of reesque/SfmFromScratch.

Drop-in classes (same names and behaviour as the reference's plugin API):
    NaiveSIFT, ScaleRotInvSIFT      FeatureExtractor/SIFT/*.py
    NNRatioFeatureMatcher           FeatureMatcher/NNRatioFeatureMatcher.py
Throughput API on device-resident frames: pipeline.BatchExtractor / BatchMatcher.
The arithmetic runs in lib/libsfmfeat.so (hand-written HIP for gfx950, C-ABI in
include/sfmfeat.h); there is no CPU fallback.
"""
from .feature_extractor import FeatureExtractor
from .matcher import NNRatioFeatureMatcher
from .sift import NaiveSIFT, ScaleRotInvSIFT, set_device

__all__ = ["FeatureExtractor", "NaiveSIFT", "ScaleRotInvSIFT", "NNRatioFeatureMatcher", "set_device"]
