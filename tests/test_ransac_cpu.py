"""CPU: the RANSAC consumer's pieces that need no device — the native replay of numpy's
legacy sampling stream, and the oracle restatement of CameraPose.find_inliers (SFM.py:
126-160) against the reference's own outputs (tests/golden/ransac.npz)."""
from __future__ import annotations

import numpy as np
import pytest

from oracle import ransac as R
from sfmfromscratch_amd import pose
from tests.golden_util import load


@pytest.mark.parametrize("n,iters", [(8, 60), (9, 60), (50, 100), (300, 80), (691, 40), (2500, 12)])
def test_native_sample_stream_equals_numpy(n, iters):
    rs = np.random.RandomState(5)  # np.random.seed(5) (SFM.py:133)
    ref = np.stack([rs.choice(n, 8, replace=False) for _ in range(iters)])
    assert np.array_equal(pose.sample_indices(n, iters, 5), ref)


def test_ransac_iterations_like_runner():
    assert pose.calculate_num_ransac_iterations(0.98, 8, 0.4) == 5967  # Runner.py:170


@pytest.mark.parametrize("i", range(5))
def test_oracle_find_inliers_vs_reference_golden(i):
    z = load("ransac.npz")
    p1, p2 = z[f"c{i}_p1"], z[f"c{i}_p2"]
    r = R.find_inliers(p1, p2, float(z[f"c{i}_thr"]), int(z[f"c{i}_meta"][0]))
    if f"c{i}_none" in z:
        assert r == (None, None, None, None)
    else:
        assert np.array_equal(r[0], z[f"c{i}_in1"]) and np.array_equal(r[1], z[f"c{i}_in2"])
