"""CPU: pair schedules and the .npz feature / match formats of sequence.py (SURVEY §8f
rows 3-4); no device calls."""
from __future__ import annotations

import numpy as np

from sfmfromscratch_amd import sequence as S


def test_pair_schedules():
    assert S.pair_schedule(5).tolist() == [[0, 1], [1, 2], [2, 3], [3, 4]]  # Runner.py:183
    assert len(S.pair_schedule(6, "all")) == 15
    w2 = S.pair_schedule(5, 2).tolist()
    assert w2 == [[0, 1], [0, 2], [1, 2], [1, 3], [2, 3], [2, 4], [3, 4]]


def test_feature_npz_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    X = [rng.integers(0, 100, n) for n in (5, 0, 3)]
    Y = [rng.integers(0, 100, n) for n in (5, 0, 3)]
    D = [rng.random((n, 128), dtype=np.float32) for n in (5, 0, 3)]
    p = str(tmp_path / "f.npz")
    S.save_features(p, X, Y, D)
    X2, Y2, D2 = S.load_features(p)
    for a, b in zip(X + Y, X2 + Y2):
        assert np.array_equal(a, b) and b.dtype == np.int64
    for a, b in zip(D, D2):
        assert np.array_equal(a.reshape(-1, 128), b) and b.dtype == np.float32


def test_match_npz_roundtrip_keeps_empty_quirk(tmp_path):
    pairs = np.array([[0, 1], [1, 2]], np.int32)
    res = [(np.array([[3, 4], [1, 0]], np.int64), np.array([0.1, 0.5], np.float32)), (np.array([]), np.array([]))]
    p = str(tmp_path / "m.npz")
    S.save_matches(p, pairs, res)
    pp, r2 = S.load_matches(p)
    assert np.array_equal(pp, pairs)
    assert np.array_equal(r2[0][0], res[0][0]) and np.array_equal(r2[0][1], res[0][1])
    assert r2[1][0].shape == (0,) and r2[1][0].dtype == np.float64  # NNRatioFeatureMatcher's empty result
