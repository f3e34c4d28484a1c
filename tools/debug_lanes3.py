"""Diagnostic stress: BatchPipeline lanes vs serial extraction over many seeds; on a
mismatch print the conflicting rows and the R values (debug_harris) at their pixels."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from sfmfromscratch_amd import _abi, _native, synth
from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, BatchPipeline, consecutive_pairs

pp = {"num_interest_points": 600, "ksize": 3, "gaussian_size": 7, "sigma": 6, "alpha": 0.05,
      "feature_width": 18, "pyramid_level": 4, "pyramid_scale_factor": 2}
B, H, W = 4, 270, 480
pairs = torch.from_numpy(consecutive_pairs(B)).cuda()
ex = BatchExtractor(pp)
m = BatchMatcher(0.85, ctx=ex.ctx)
pipe = BatchPipeline(pp, 0.85, B, H, W, pairs, inflight=2, extra_slots=0)
bad_total = 0
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    batches = [torch.from_numpy(synth.make_batch_u8(B, H, W, seed=300 + 3 * it + i)).cuda() for i in range(3)]
    lanes = [pipe.submit(f) for f in batches]
    pipe.join()
    torch.cuda.synchronize()
    for i in range(3):
        ln = lanes[i]
        if i == 0:
            continue  # lane 0 reused by batch 2
        s = ex.extract(batches[i])
        m.match(s, pairs)
        torch.cuda.synchronize()
        for b, n in enumerate(s.count.tolist()):
            a = s.xy[b, :n].cpu().numpy()
            c = ln["slots"].xy[b, :n].cpu().numpy()
            bad = np.nonzero((a != c).any(1))[0]
            if len(bad):
                bad_total += 1
                img = batches[i][b].cpu().numpy().astype(np.float32) / np.float32(255)
                R, med, _ = _native.debug_harris(img, _abi.params_from_dict(pp, _abi.SFM_MODE_SCALEROT))
                pts = [tuple(v) for v in a[bad[:4]].tolist()] + [tuple(v) for v in c[bad[:4]].tolist()]
                print(f"it {it} batch {i} frame {b} n {n} bad rows {bad[:8].tolist()}")
                for (x, y) in dict.fromkeys(pts):
                    print(f"   ({x},{y}) R={R[y, x]!r} bits={np.float32(R[y, x]).view(np.uint32):08x}")
print("mismatching frames:", bad_total)
