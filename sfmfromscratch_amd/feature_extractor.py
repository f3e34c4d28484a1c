"""FeatureExtractor plugin interface — mirror of FeatureExtractor/FeatureExtractor.py:4-21."""
from __future__ import annotations

from abc import ABC, abstractmethod

import numpy as np


class FeatureExtractor(ABC):
    """Interface for feature extractor classes (on images)."""

    def __init__(self, image: np.ndarray, extractor_params=None):
        if extractor_params is None:
            extractor_params = {}
        self.image = image
        self.num_interest_points = extractor_params.get("num_interest_points", 2500)

    @abstractmethod
    def detect_keypoints(self) -> np.ndarray:
        """Detects keypoints in the image and returns their coordinates."""

    @abstractmethod
    def extract_descriptors(self) -> np.ndarray:
        """Extracts descriptors for the detected keypoints."""
