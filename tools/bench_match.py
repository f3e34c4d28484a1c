"""Matcher-only timing (diagnostic): extract one batch of synthetic 1080p frames once, then
time `iters` launches of the pair matcher over its consecutive pairs (HIP events)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--allpairs", action="store_true", help="all B(B-1)/2 pairs instead of consecutive")
    ap.add_argument("--4k", dest="k4", action="store_true", help="BASELINE configs[4]: 4K, 5 octaves, k 8000, 8 frames")
    args = ap.parse_args()
    import numpy as np
    import torch
    from sfmfromscratch_amd import synth
    from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, all_pairs, consecutive_pairs
    P_OCT = {"num_interest_points": 2500, "ksize": 3, "gaussian_size": 7, "sigma": 6, "alpha": 0.05,
             "feature_width": 18, "pyramid_level": 4, "pyramid_scale_factor": 2}
    H, W = 1080, 1920
    if args.k4:
        H, W = 2160, 3840
        P_OCT.update(num_interest_points=8000, pyramid_level=5)
        if args.batch == 32:
            args.batch = 8
    B = args.batch
    ex = BatchExtractor(P_OCT)
    u8 = np.stack([synth.make_frame_u8(H, W, 1234, i) for i in range(B)])
    slots = ex.extract(torch.from_numpy(u8).cuda())
    pairs = torch.from_numpy(all_pairs(B) if args.allpairs else consecutive_pairs(B)).cuda()
    m = BatchMatcher(0.85, ctx=ex.ctx)
    out = m.match(slots, pairs)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        m.match(slots, pairs, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    print(f"match {pairs.shape[0]} pairs: {ms * 1e3 / pairs.shape[0]:.2f} us/pair, {ms:.3f} ms per call, keypoints mean {slots.count.float().mean().item():.0f}, "
          f"matches mean {out[2].float().mean().item():.0f}")


if __name__ == "__main__":
    main()
