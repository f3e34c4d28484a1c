"""Diagnostic: BatchPipeline lanes vs serial extraction, per batch / frame / field."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from sfmfromscratch_amd import synth
from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, BatchPipeline, consecutive_pairs

P_OCT = {"num_interest_points": 600, "ksize": 3, "gaussian_size": 7, "sigma": 6, "alpha": 0.05,
         "feature_width": 18, "pyramid_level": 4, "pyramid_scale_factor": 2}
B, H, W = 4, 270, 480
batches = [torch.from_numpy(synth.make_batch_u8(B, H, W, seed=300 + i)).cuda() for i in range(3)]
pairs = torch.from_numpy(consecutive_pairs(B)).cuda()
nomatch = len(sys.argv) > 1 and sys.argv[1] == "nomatch"
pipe = BatchPipeline(P_OCT, 0.85, B, H, W, pairs if not nomatch else pairs[:0], inflight=2, extra_slots=0)
lanes = [pipe.submit(f) for f in batches]
pipe.join()
torch.cuda.synchronize()
ex = BatchExtractor(P_OCT)
m = BatchMatcher(0.85, ctx=ex.ctx)
for i in (1, 2):
    s = ex.extract(batches[i])
    torch.cuda.synchronize()
    xy0 = s.xy.clone()
    mm, mc, nm = m.match(s, pairs)
    torch.cuda.synchronize()
    print("slot xy changed by the matcher:", int((xy0 != s.xy).sum()), "desc finite:", bool(torch.isfinite(s.desc).all()))
    ln = lanes[i]
    print("nmatch serial", nm.tolist(), "lane", ln["mout"][2].tolist())
    for b, n in enumerate(s.count.tolist()):
        a = s.xy[b, :n].cpu().numpy()
        c = ln["slots"].xy[b, :n].cpu().numpy()
        bad = np.nonzero((a != c).any(1))[0]
        print(f"batch {i} frame {b}: n={n} lane n={int(ln['slots'].count[b])} bad rows {len(bad)} first {bad[:5]}"
              + (f" serial {a[bad[0]]} lane {c[bad[0]]}" if len(bad) else ""))
