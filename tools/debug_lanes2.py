import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
import tests.test_gpu_parity as t
import torch
from sfmfromscratch_amd import synth
from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, BatchPipeline, consecutive_pairs
P_OCT = t.P_OCT
B, H, W = 4, 270, 480
pp = dict(P_OCT, num_interest_points=600)
print(pp)
batches = [torch.from_numpy(synth.make_batch_u8(B, H, W, seed=300 + i)).cuda() for i in range(3)]
pairs = torch.from_numpy(consecutive_pairs(B)).cuda()
pipe = BatchPipeline(pp, 0.85, B, H, W, pairs, inflight=2, extra_slots=0)
lanes = [pipe.submit(f) for f in batches]
pipe.join()
torch.cuda.synchronize()
ex = BatchExtractor(pp)
m = BatchMatcher(0.85, ctx=ex.ctx)
for i in (1, 2):
    s = ex.extract(batches[i])
    mm, mc, nm = m.match(s, pairs)
    torch.cuda.synchronize()
    ln = lanes[i]
    for b, n in enumerate(s.count.tolist()):
        a = s.xy[b, :n].cpu().numpy(); c = ln["slots"].xy[b, :n].cpu().numpy()
        bad = np.nonzero((a != c).any(1))[0]
        print(i, b, n, len(bad), bad[:8], a[bad[:3]].tolist() if len(bad) else "", c[bad[:3]].tolist() if len(bad) else "")
