"""GPU: the certified keypoint select (median bounded from the Harris histogram) against the
exact-median path (SFMFEAT_SELECT=exact) and the C oracle — bit-identical keypoints and
descriptors — on batches that mix planes which certify with planes that must fall back
(flat regions full of R == 0, constant frames), all decided per plane inside one launch."""
from __future__ import annotations

import os

import numpy as np
import pytest

from oracle import oracle as O
from sfmfromscratch_amd import synth
from tests.golden_util import P_MAIN, P_OCT

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def mixed_batch(H, W):
    rng = np.random.default_rng(5)
    textured = synth.make_frame(H, W, 1234, 0)
    blobs = np.zeros((H, W), np.float32)  # mostly flat: R == 0 almost everywhere
    yy, xx = np.mgrid[0:H, 0:W]
    for _ in range(6):
        cy, cx = rng.integers(10, H - 10), rng.integers(10, W - 10)
        blobs += np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / 30.0).astype(np.float32)
    blobs = np.clip(blobs, 0, 1).astype(np.float32)
    const = np.full((H, W), 0.5, np.float32)
    noise = (rng.integers(0, 256, (H, W)) / 255.0).astype(np.float32)
    return np.stack([textured, blobs, const, noise])


def run(imgs, pp, exact, serial=False):
    import torch
    from sfmfromscratch_amd.pipeline import BatchExtractor
    # both switches are read when the context is created
    old = {k: os.environ.pop(k, None) for k in ("SFMFEAT_SELECT", "SFMFEAT_SERIAL")}
    try:
        if exact:
            os.environ["SFMFEAT_SELECT"] = "exact"
        if serial:
            os.environ["SFMFEAT_SERIAL"] = "1"
        ex = BatchExtractor(pp)
    finally:
        for k, v in old.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v
    s = ex.extract(torch.from_numpy(imgs).cuda())
    torch.cuda.synchronize()
    stats = ex.ctx.select_stats()
    return s.xy.cpu().numpy(), s.desc.cpu().numpy(), s.count.cpu().numpy(), stats


@pytest.mark.parametrize("H,W,pp", [(270, 480, dict(P_OCT, num_interest_points=600)),
                                    (240, 320, dict(P_MAIN, num_interest_points=300)),
                                    (300, 400, dict(P_OCT, num_interest_points=40, ksize=7))])
def test_certified_select_equals_exact_and_oracle(H, W, pp):
    imgs = mixed_batch(H, W)
    xy, desc, cnt, (fb, tot) = run(imgs, pp, exact=False)
    xe, de, ce, (fbe, tote) = run(imgs, pp, exact=True)
    assert fbe == tote == tot
    assert 0 < fb < tot, (fb, tot)  # both paths exercised in one batch
    assert np.array_equal(cnt, ce)
    for b in range(len(imgs)):
        n = cnt[b]
        assert np.array_equal(xy[b, :n], xe[b, :n])
        assert np.array_equal(bits(desc[b, :n]), bits(de[b, :n]))
        X, Y, D, _ = O.extract(imgs[b], pp)
        assert n == len(X)
        assert np.array_equal(xy[b, :n, 0], X) and np.array_equal(xy[b, :n, 1], Y)
        assert np.array_equal(bits(desc[b, :n]), bits(D))


def test_1080p_planes_certify():
    """At the metric's configuration every plane of textured frames certifies, except the
    levels too small to hold ~k window maxima (h*w < 64 k), which go straight to the exact
    path by design (sfmfeat_api.hip, extract_impl)."""
    pp = P_OCT
    imgs = np.stack([synth.make_frame(1080, 1920, 1234, i) for i in range(2)])
    xy, desc, cnt, (fb, tot) = run(imgs, pp, exact=False)
    xe, de, ce, _ = run(imgs, pp, exact=True)
    L = pp["pyramid_level"]
    kcap = pp["num_interest_points"] // L
    small = sum(1 for l in range(L) if (1080 >> l) * (1920 >> l) < 64 * kcap)
    assert tot == 2 * L and fb == 2 * small
    assert np.array_equal(cnt, ce)
    for b in range(2):
        n = cnt[b]
        assert np.array_equal(xy[b, :n], xe[b, :n])
        assert np.array_equal(bits(desc[b, :n]), bits(de[b, :n]))


@pytest.mark.parametrize("exact,serial", [(False, False), (True, False), (True, True)])
def test_scale_1_1_four_levels_selection_regions_vs_oracle(exact, serial):
    """pyramid_scale_factor 1.1 (the reference's main.py:19-28 parameters) keeps every level large, so the caller stream's merged selection
    regions (one per level, packed after the aux stream's) and the serial layout (every
    level from 0) cover far more than 2 x B x A0 slots.  Noise planes give C > 2048
    candidates, so the tie lists are written; the exact path writes the median lists.
    Every plane must still equal the oracle (sfmfeat_api.hip reserve_impl sizes both)."""
    pp = dict(P_MAIN, num_interest_points=2000, pyramid_level=4, pyramid_scale_factor=1.1)
    H, W = 360, 640
    rng = np.random.default_rng(11)
    imgs = np.stack([synth.make_frame(H, W, 1234, 0), (rng.integers(0, 256, (H, W)) / 255.0).astype(np.float32),
                     synth.make_frame(H, W, 1234, 1), (rng.integers(0, 256, (H, W)) / 255.0).astype(np.float32)])
    xy, desc, cnt, _ = run(imgs, pp, exact=exact, serial=serial)
    for b in range(len(imgs)):
        n = cnt[b]
        X, Y, D, _ = O.extract(imgs[b], pp)
        assert n == len(X)
        assert np.array_equal(xy[b, :n, 0], X) and np.array_equal(xy[b, :n, 1], Y)
        assert np.array_equal(bits(desc[b, :n]), bits(D))
