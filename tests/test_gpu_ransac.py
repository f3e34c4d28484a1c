"""GPU: the RANSAC consumer (ransac.hip, pose.find_inliers) against the reference's own
CameraPose.find_inliers outputs (tests/golden/ransac.npz) and the oracle restatement.
Bar: identical inlier arrays (float64 differences between LAPACK's SVD and the device's
elimination could only move a point within ~1e-12 of the threshold)."""
from __future__ import annotations

import numpy as np
import pytest

from oracle import ransac as R
from sfmfromscratch_amd import _abi, _native, pose
from tests.golden_util import load

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("i", range(5))
def test_find_inliers_vs_reference_golden(i):
    z = load("ransac.npz")
    p1, p2 = z[f"c{i}_p1"], z[f"c{i}_p2"]
    r = pose.find_inliers(p1, p2, threshold=float(z[f"c{i}_thr"]), max_iterations=int(z[f"c{i}_meta"][0]))
    if f"c{i}_none" in z:
        assert r == (None, None, None, None)
    else:
        assert np.array_equal(r[0], z[f"c{i}_in1"]) and np.array_equal(r[1], z[f"c{i}_in2"])
        assert r[0].dtype == z[f"c{i}_in1"].dtype


@pytest.mark.parametrize("seed,n,frac", [(1, 40, 0.8), (2, 500, 0.5), (3, 2500, 0.6)])
def test_find_inliers_planted_vs_oracle(seed, n, frac):
    rng = np.random.default_rng(seed)
    p1 = rng.integers(0, 1900, (n, 2)).astype(np.int64)
    p2 = p1 + np.array([5, -3])
    out = rng.random(n) > frac
    p2[out] = rng.integers(0, 1900, (int(out.sum()), 2))
    r = pose.find_inliers(p1, p2, max_iterations=300)
    o = R.find_inliers(p1, p2, 1.0, 300)
    assert np.array_equal(r[0], o[0]) and np.array_equal(r[1], o[1])


def test_batch_dev_api_matches_host_api():
    torch = pytest.importorskip("torch")
    import ctypes
    z = load("ransac.npz")
    cases = [(z[f"c{i}_p1"], z[f"c{i}_p2"]) for i in range(4)]
    nmax = max(len(a) for a, _ in cases)
    P = len(cases)
    pts = np.zeros((P, nmax, 4), np.int32)
    npts = np.array([len(a) for a, _ in cases], np.int32)
    for p, (a, b) in enumerate(cases):
        pts[p, :len(a), :2] = a
        pts[p, :len(a), 2:] = b
    ctx = _native.context_for(_abi.params_from_dict({}, _abi.SFM_MODE_NAIVE))
    d_pts = torch.from_numpy(pts).cuda()
    d_n = torch.from_numpy(npts).cuda()
    o_pts = torch.zeros_like(d_pts)
    o_n = torch.zeros(P, dtype=torch.int32, device="cuda")
    o_it = torch.zeros(P, dtype=torch.int32, device="cuda")
    rc = ctx.lib.sfm_ransac_find_inliers_dev(ctx.handle, d_pts.data_ptr(), d_n.data_ptr(),
                                             npts.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), P, nmax, 700,
                                             ctypes.c_double(1.0), o_pts.data_ptr(), o_n.data_ptr(),
                                             o_it.data_ptr(), None)
    _native.check(rc, ctx.handle)
    torch.cuda.synchronize()
    on = o_n.cpu().numpy()
    op = o_pts.cpu().numpy()
    for p, (a, b) in enumerate(cases):
        r = pose.find_inliers(a, b, max_iterations=700)
        k = int(on[p])
        assert k == len(r[0])
        assert np.array_equal(op[p, :k, :2], r[0]) and np.array_equal(op[p, :k, 2:], r[1])


def test_zero_iterations_after_a_call_with_inliers():
    """max_iterations=0: the reference's loop never runs and it returns two empty arrays;
    the result must not be the previous call's (stale device counters)."""
    z = load("ransac.npz")
    p1, p2 = z["c0_p1"], z["c0_p2"]
    r = pose.find_inliers(p1, p2, max_iterations=200)
    assert len(r[0]) > 0
    r0 = pose.find_inliers(p1, p2, max_iterations=0)
    assert len(r0) == 2 and r0[0].shape == (0,) and r0[1].shape == (0,)
    rb = pose.find_inliers_batch([(p1, p2), (p1[:7], p2[:7]), (p1, p2)], max_iterations=0)
    assert rb[1] == (None, None, None, None)
    for k in (0, 2):
        assert rb[k][0].shape == (0,) and rb[k][1].shape == (0,)
    o = R.find_inliers(p1, p2, 1.0, 0)
    assert len(o[0]) == 0


def test_more_points_than_one_lds_chunk_vs_oracle():
    """n = 4000 > the 2560-point LDS chunk of k_ransac_count (the reference has no limit)."""
    rng = np.random.default_rng(7)
    n = 4000
    p1 = rng.integers(0, 1900, (n, 2)).astype(np.int64)
    p2 = p1 + np.array([4, 2])
    out = rng.random(n) > 0.55
    p2[out] = rng.integers(0, 1900, (int(out.sum()), 2))
    r = pose.find_inliers(p1, p2, max_iterations=150)
    o = R.find_inliers(p1, p2, 1.0, 150)
    assert np.array_equal(r[0], o[0]) and np.array_equal(r[1], o[1])
    rb = pose.find_inliers_batch([(p1, p2), (p1[:900], p2[:900])], max_iterations=150)
    assert np.array_equal(rb[0][0], o[0]) and np.array_equal(rb[0][1], o[1])
    o2 = R.find_inliers(p1[:900], p2[:900], 1.0, 150)
    assert np.array_equal(rb[1][0], o2[0]) and np.array_equal(rb[1][1], o2[1])


def test_batch_rejects_float_coordinates():
    p = np.arange(40, dtype=np.float64).reshape(20, 2)
    with pytest.raises(ValueError):
        pose.find_inliers_batch([(p + 0.5, p)], max_iterations=10)
