"""GPU: SFMRunner stage 1 on the device (sequence.py) against the oracle — frames
decoded once, ingested + extracted once into the resident descriptor table, pairs matched
from it."""
from __future__ import annotations

import numpy as np
import pytest

from oracle import ingest as I
from oracle import oracle as O
from sfmfromscratch_amd import synth
from tests.golden_util import P_OCT, assert_matches_equal

pytestmark = pytest.mark.gpu


def test_stage1_consecutive_pairs_vs_oracle(tmp_path):
    Image = pytest.importorskip("PIL.Image")
    from sfmfromscratch_amd import sequence as S
    n = 4
    for i in range(n):
        Image.fromarray(synth.make_frame_rgb_u8(360, 640, 31, i)).save(str(tmp_path / f"{i + 1}.jpg"), quality=95)
    pp = dict(P_OCT, num_interest_points=600)
    all_m, cache = S.stage1(str(tmp_path), n, pp, match_threshold=0.85, single_K=np.eye(3))
    feats = []
    for i in range(n):
        rgb = np.asarray(Image.open(str(tmp_path / f"{i + 1}.jpg")))
        X, Y, D, _ = O.extract(I.ingest(rgb, 0.5), pp)
        cx, cy = cache.keypoints(i)
        assert np.array_equal(cx, X) and np.array_equal(cy, Y)
        feats.append((X, Y, D))
    for i1 in range(1, n):
        i2 = i1 + 1
        m = all_m[i1][i2]
        om, oc = O.match(feats[i1 - 1][2], feats[i2 - 1][2], 0.85)
        assert_matches_equal(om, oc, m.matches, m.confidence)
        r = all_m[i2][i1]
        assert np.array_equal(r.p1, m.p2) and np.array_equal(r.p2, m.p1) and r.K1 is m.K2
        assert np.array_equal(m.p1[:, 0], feats[i1 - 1][0][m.matches[:2500, 0]])
    assert all_m[1][3] is None


def test_cache_all_pairs_and_mixed_sizes_vs_dropin(tmp_path):
    from sfmfromscratch_amd import NNRatioFeatureMatcher
    from sfmfromscratch_amd import sequence as S
    frames = [synth.make_frame_rgb_u8(270, 480, 41, i) for i in range(3)] + \
             [synth.make_frame(180, 300, 42, i) for i in range(2)]  # RGB + float gray, two sizes
    pp = dict(P_OCT, num_interest_points=400)
    cache = S.FeatureCache(frames, pp, batch=2)
    pairs = S.pair_schedule(5, "all")
    res = S.match_schedule(cache, pairs, 0.8)
    mt = NNRatioFeatureMatcher(0.8)
    for (i, j), (mm, cc) in zip(pairs, res):
        rm, rc = mt.match_features_ratio_test(cache.descriptors(i), cache.descriptors(j))
        assert np.array_equal(mm, rm) and np.array_equal(cc, rc)
    g = I.ingest(frames[0], 0.5)
    X, Y, D, _ = O.extract(g, pp)
    assert np.array_equal(cache.keypoints(0)[0], X)
    X, Y, D, _ = O.extract(frames[4], pp)
    assert np.array_equal(cache.keypoints(4)[1], Y)
    p = str(tmp_path / "f.npz")
    cache.save(p)
    X2, Y2, D2 = S.load_features(p)
    assert np.array_equal(D2[4], cache.descriptors(4))


def test_stage1_with_ransac_vs_oracle(tmp_path):
    """Runner.py:349-351: every pair but (1, 2) filtered by find_inliers (reference
    iteration count), batched on the device == the oracle's find_inliers per pair."""
    Image = pytest.importorskip("PIL.Image")
    from oracle import ransac as R
    from sfmfromscratch_amd import sequence as S
    n = 4
    for i in range(n):
        Image.fromarray(synth.make_frame_rgb_u8(360, 640, 51, i)).save(str(tmp_path / f"{i + 1}.jpg"), quality=95)
    pp = dict(P_OCT, num_interest_points=600)
    raw, _ = S.stage1(str(tmp_path), n, pp)
    filt, _ = S.stage1(str(tmp_path), n, pp, ransac=True, ransac_max_it=400)
    assert np.array_equal(filt[1][2].p1, raw[1][2].p1)  # the initial pair is not filtered
    for i1 in (2, 3):
        o = R.find_inliers(raw[i1][i1 + 1].p1, raw[i1][i1 + 1].p2, 1.0, 400)
        assert np.array_equal(filt[i1][i1 + 1].p1, o[0]) and np.array_equal(filt[i1][i1 + 1].p2, o[1])
        assert np.array_equal(filt[i1 + 1][i1].p1, o[1])
