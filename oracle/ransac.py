"""TEST INFRASTRUCTURE ONLY — numpy restatement of CameraPose.find_inliers (SFM.py:126-160)
and _compute_fundamental_matrix (SFM.py:190-236), the reference's algorithm with numpy's
own RNG and LAPACK SVD, vectorised over the iterations (np.linalg.svd on a stack runs the
same LAPACK routine per matrix).  Pinned to tests/golden/ransac.npz, which
tools/gen_golden.py makes by calling the reference's CameraPose.find_inliers.
Only tests/ import this module."""
from __future__ import annotations

import numpy as np


def samples(n: int, iters: int, seed: int = 5) -> np.ndarray:
    rs = np.random.RandomState(seed)  # np.random.seed(5) + np.random.choice (SFM.py:133-137)
    return np.stack([rs.choice(n, 8, replace=False) for _ in range(iters)]) if iters else np.zeros((0, 8), int)


def _normalise(pts):  # CameraPose.normalize_points (SFM.py:164-178), pts [..., 8, 3]
    mean = pts[..., :2].mean(axis=-2)
    cu, cv = mean[..., 0], mean[..., 1]
    d = np.sqrt((pts[..., 0] - cu[..., None]) ** 2 + (pts[..., 1] - cv[..., None]) ** 2).mean(axis=-1)
    s = np.sqrt(2) / d
    T = np.zeros(pts.shape[:-2] + (3, 3))
    T[..., 0, 0] = s
    T[..., 0, 2] = -s * cu
    T[..., 1, 1] = s
    T[..., 1, 2] = -s * cv
    T[..., 2, 2] = 1
    return pts @ np.swapaxes(T, -1, -2), T


def fundamental(s1, s2):
    """_compute_fundamental_matrix for a stack of 8-point samples [..., 8, 2]."""
    one = np.ones(s1.shape[:-1] + (1,))
    a, T1 = _normalise(np.concatenate([s1, one], -1))
    b, T2 = _normalise(np.concatenate([s2, one], -1))
    x1, y1, x2, y2 = a[..., 0], a[..., 1], b[..., 0], b[..., 1]
    A = np.stack([x1 * x2, y1 * x2, x2, x1 * y2, y1 * y2, y2, x1, y1, np.ones_like(x1)], -1)
    _, _, VT = np.linalg.svd(A)
    F = VT[..., -1, :].reshape(s1.shape[:-2] + (3, 3))
    U, D, Vt = np.linalg.svd(F)
    D[..., 2] = 0
    F2 = U @ (D[..., :, None] * Vt)
    return np.swapaxes(T2, -1, -2) @ F2 @ T1


def find_inliers(p1, p2, threshold=1.0, max_iterations=1000):
    p1 = np.asarray(p1)
    p2 = np.asarray(p2)
    if len(p1) < 8:
        return None, None, None, None
    idx = samples(len(p1), max_iterations)
    best_n, best_mask = 0, None
    a_h = np.column_stack((p1, np.ones(len(p1))))
    b_h = np.column_stack((p2, np.ones(len(p2))))
    for c0 in range(0, max_iterations, 512):
        sl = idx[c0:c0 + 512]
        F = fundamental(p1[sl].astype(np.float64), p2[sl].astype(np.float64))
        lb = np.einsum("kij,nj->kni", F, a_h)
        d = np.abs(np.sum(lb * b_h[None], axis=2)) / np.sqrt(lb[..., 0] ** 2 + lb[..., 1] ** 2)
        masks = d < threshold
        cnt = masks.sum(axis=1)
        for k in range(len(sl)):  # strict > keeps the first best (SFM.py:156)
            if cnt[k] > best_n:
                best_n, best_mask = int(cnt[k]), masks[k]
    if best_mask is None:
        return np.array([]), np.array([])
    return p1[best_mask], p2[best_mask]
