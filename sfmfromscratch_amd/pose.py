"""The match consumer on the HIP path: CameraPose.find_inliers (SFM.py:126-160), the
8-point RANSAC SFMRunner applies to every stage-1 pair but (1, 2) (Runner.py:349-351)
— SURVEY.md §8f row 2.  Same signature, sampling stream, selection rule and return
values as the reference (ransac.hip has the numerics):

* samples: numpy's legacy RandomState after np.random.seed(5), one
  np.random.choice(n, 8, replace=False) per iteration (replayed natively, bit-exact);
* per sample the normalised 8-point fundamental matrix with rank 2 enforced, and the
  count of correspondences whose epipolar distance is below `threshold` (float64);
* the first sample with the most inliers wins; its inliers are returned in input order
  as p1[mask], p2[mask]; no inliers at all gives the reference's empty float64 arrays;
  fewer than 8 correspondences gives its (None, None, None, None).
"""
from __future__ import annotations

import numpy as np

from . import _abi
from ._native import check, context_for, load_library


def calculate_num_ransac_iterations(prob_success: float, sample_size: int, ind_prob_correct: float) -> int:
    """CameraPose.calculate_num_ransac_iterations (SFM.py:184-187)."""
    num_samples = np.log(1 - prob_success) / np.log(1 - (ind_prob_correct ** sample_size))
    return int(num_samples)


def sample_indices(n: int, iters: int, seed: int = 5) -> np.ndarray:
    """[iters, 8] int32: np.random.seed(seed); [np.random.choice(n, 8, replace=False) ...]
    (numpy's legacy MT19937 + Fisher-Yates, replayed natively; host only)."""
    import ctypes
    out = np.empty((max(iters, 0), 8), np.int32)
    rc = load_library().sfm_ransac_sample_indices(int(n), int(iters), ctypes.c_uint32(seed),
                                                  out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    check(rc)
    return out


def find_inliers(p1, p2, threshold=1.0, max_iterations=1000, device: int = 0):
    """Drop-in for CameraPose.find_inliers (SFM.py:126-160).

    Deliberate divergence: the reference also accepts non-integer coordinates; the device
    path stores points as int32 (what Runner._convert_matches_to_coords, Runner.py:423-434,
    produces from the int64 keypoints), so non-integer input raises ValueError instead of
    being silently truncated."""
    p1 = np.asarray(p1)
    p2 = np.asarray(p2)
    if len(p1) < 8:
        return None, None, None, None  # the reference's 4-tuple (SFM.py:130-131)
    if not (np.array_equal(p1, np.round(p1)) and np.array_equal(p2, np.round(p2))):
        raise ValueError("find_inliers takes integer pixel coordinates (Runner.py:423-434)")
    ctx = context_for(_abi.params_from_dict({}, _abi.SFM_MODE_NAIVE), device)
    res = ctx.ransac_find_inliers(p1, p2, float(threshold), int(max_iterations))
    in1, in2, _ = res
    if len(in1) == 0:
        return np.array([]), np.array([])
    return in1.astype(p1.dtype, copy=False), in2.astype(p2.dtype, copy=False)


def find_inliers_batch(pairs, threshold=1.0, max_iterations=1000, device: int = 0):
    """find_inliers over many correspondence sets in one device pass (one launch set for
    all pairs; sample streams shared by sets of equal size).  Integer coordinates only, as
    `find_inliers` (a documented divergence).  pairs: [(p1, p2), ...];
    returns the per-pair results of find_inliers."""
    import ctypes

    import torch
    res = [None] * len(pairs)
    todo = []
    for k, (a, b) in enumerate(pairs):
        a, b = np.asarray(a), np.asarray(b)
        if len(a) < 8:
            res[k] = (None, None, None, None)
            continue
        if not (np.array_equal(a, np.round(a)) and np.array_equal(b, np.round(b))):
            raise ValueError(f"pair {k}: find_inliers takes integer pixel coordinates (Runner.py:423-434)")
        if a.shape != b.shape or a.ndim != 2 or a.shape[1] != 2:
            raise ValueError(f"pair {k}: p1 and p2 must both be [n, 2]")
        todo.append((k, a, b))
    if not todo:
        return res
    nmax = max(len(a) for _, a, _ in todo)
    P = len(todo)
    pts = np.zeros((P, nmax, 4), np.int32)
    npts = np.array([len(a) for _, a, _ in todo], np.int32)
    for p, (_, a, b) in enumerate(todo):
        pts[p, :len(a), :2] = a
        pts[p, :len(a), 2:] = b
    ctx = context_for(_abi.params_from_dict({}, _abi.SFM_MODE_NAIVE), device)
    dev = torch.device("cuda", device)
    d_pts = torch.from_numpy(pts).to(dev)
    d_n = torch.from_numpy(npts).to(dev)
    o_pts = torch.zeros_like(d_pts)
    o_n = torch.zeros(P, dtype=torch.int32, device=dev)
    o_it = torch.zeros(P, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    check(ctx.lib.sfm_ransac_find_inliers_dev(ctx.handle, d_pts.data_ptr(), d_n.data_ptr(),
                                              npts.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), P, nmax,
                                              int(max_iterations), ctypes.c_double(threshold), o_pts.data_ptr(),
                                              o_n.data_ptr(), o_it.data_ptr(), stream or None), ctx.handle)
    on = o_n.cpu().numpy()
    op = o_pts.cpu().numpy()
    for p, (k, a, b) in enumerate(todo):
        n = int(on[p])
        if n <= 0:
            res[k] = (np.array([]), np.array([]))
        else:
            res[k] = (op[p, :n, :2].astype(a.dtype), op[p, :n, 2:].astype(b.dtype))
    return res
