import os, sys
sys.path.insert(0, "/root/repo")
import numpy as np
import pytest

def test_dbg():
    import torch
    from sfmfromscratch_amd import synth
    from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, BatchPipeline, consecutive_pairs
    pp = {'num_interest_points': 600, 'ksize': 3, 'gaussian_size': 7, 'sigma': 6, 'alpha': 0.05, 'feature_width': 18, 'pyramid_level': 4, 'pyramid_scale_factor': 2}
    B, H, W = 4, 270, 480
    batches = [torch.from_numpy(synth.make_batch_u8(B, H, W, seed=300 + i)).cuda() for i in range(3)]
    pairs = torch.from_numpy(consecutive_pairs(B)).cuda()
    pipe = BatchPipeline(pp, 0.85, B, H, W, pairs, inflight=2, extra_slots=0)
    lanes = [pipe.submit(f) for f in batches]
    pipe.join()
    torch.cuda.synchronize()
    ex = BatchExtractor(pp)
    m = BatchMatcher(0.85, ctx=ex.ctx)
    nbad = 0
    for i in (1, 2):
        s = ex.extract(batches[i])
        torch.cuda.synchronize()
        xy0 = s.xy.clone()
        mm, mc, nm = m.match(s, pairs)
        torch.cuda.synchronize()
        print("matcher changed slots:", int((xy0 != s.xy).sum()), int((xy0 != s.xy).any(2).sum()))
        ln = lanes[i]
        for b, n in enumerate(s.count.tolist()):
            a = s.xy[b, :n].cpu().numpy(); c = ln["slots"].xy[b, :n].cpu().numpy(); a0 = xy0[b, :n].cpu().numpy()
            bad = np.nonzero((a != c).any(1))[0]
            bad0 = np.nonzero((a0 != c).any(1))[0]
            nbad += len(bad)
            print(i, b, n, "bad", len(bad), "bad-before-match", len(bad0), bad[:6], a[bad[:2]].tolist() if len(bad) else "", c[bad[:2]].tolist() if len(bad) else "")
    assert nbad == 0
