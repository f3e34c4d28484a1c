"""RANSAC consumer timing (diagnostic): `pairs` correspondence sets
shaped like SFMRunner's stage-1 output (first <= 2,500 matches of consecutive 1080p pairs,
~50 % inliers of a planted epipolar motion), max_iterations = 5,967 as Runner.py:170, all
through one sfm_ransac_find_inliers_dev call.  Reports the cold call (host replay of the
sampling streams included), warm calls (streams cached), the device kernels alone (HIP
events on the call's stream), and optionally the oracle's numpy time for one pair."""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_sets(P, nlo, nhi, seed=0):
    import numpy as np
    rng = np.random.default_rng(seed)
    out = []
    for p in range(P):
        n = int(rng.integers(nlo, nhi + 1))
        p1 = rng.integers(0, 1900, (n, 2)).astype(np.int64)
        p2 = p1 + np.array([int(rng.integers(-9, 10)), int(rng.integers(-9, 10))])
        bad = rng.random(n) < 0.5
        p2[bad] = rng.integers(0, 1900, (int(bad.sum()), 2))
        out.append((p1, p2))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=31)
    ap.add_argument("--nlo", type=int, default=900)
    ap.add_argument("--nhi", type=int, default=1300)
    ap.add_argument("--iters", type=int, default=5967)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--oracle", action="store_true", help="also time the numpy oracle on one pair")
    args = ap.parse_args()
    import numpy as np
    import torch
    from sfmfromscratch_amd import _abi, _native
    sets = make_sets(args.pairs, args.nlo, args.nhi)
    P = len(sets)
    nmax = max(len(a) for a, _ in sets)
    pts = np.zeros((P, nmax, 4), np.int32)
    npts = np.array([len(a) for a, _ in sets], np.int32)
    for p, (a, b) in enumerate(sets):
        pts[p, :len(a), :2] = a
        pts[p, :len(a), 2:] = b
    ctx = _native.context_for(_abi.params_from_dict({}, _abi.SFM_MODE_NAIVE))
    d_pts = torch.from_numpy(pts).cuda()
    d_n = torch.from_numpy(npts).cuda()
    o_pts = torch.zeros_like(d_pts)
    o_n = torch.zeros(P, dtype=torch.int32, device="cuda")
    o_it = torch.zeros(P, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def call():
        _native.check(ctx.lib.sfm_ransac_find_inliers_dev(
            ctx.handle, d_pts.data_ptr(), d_n.data_ptr(), npts.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), P,
            nmax, args.iters, ctypes.c_double(1.0), o_pts.data_ptr(), o_n.data_ptr(), o_it.data_ptr(), st or None),
            ctx.handle)

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    call()
    cold = time.perf_counter() - t0
    warm = []
    dev = []
    for _ in range(args.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        call()
        e1.record()
        torch.cuda.synchronize()
        warm.append(time.perf_counter() - t0)
        dev.append(e0.elapsed_time(e1))
    on = o_n.cpu().numpy()
    evals = float(npts.astype(np.int64).sum()) * args.iters
    msg = (f"ransac {P} pairs, n {npts.min()}..{npts.max()} ({len(set(npts.tolist()))} distinct), iters {args.iters}: "
           f"cold {cold * 1e3:.1f} ms, warm {np.median(warm) * 1e3:.2f} ms, events {np.median(dev):.3f} ms "
           f"({evals / (np.median(dev) * 1e-3) / 1e9:.1f} G point-tests/s), inliers mean {on.mean():.0f}")
    print(msg, flush=True)
    if args.oracle:
        from oracle import ransac as R
        a, b = sets[0]
        t0 = time.perf_counter()
        R.find_inliers(a, b, 1.0, args.iters)
        print(f"oracle (numpy, vectorised) one pair n={len(a)}: {time.perf_counter() - t0:.2f} s", flush=True)


if __name__ == "__main__":
    main()
