"""Diagnostic: compare BatchPipeline lanes with serial extraction (where do they differ?)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from sfmfromscratch_amd import synth
from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, BatchPipeline, consecutive_pairs
from tests.golden_util import P_OCT
B, H, W = 4, 270, 480
pp = dict(P_OCT, num_interest_points=600)
batches = [torch.from_numpy(synth.make_batch_u8(B, H, W, seed=300 + i)).cuda() for i in range(3)]
pairs = torch.from_numpy(consecutive_pairs(B)).cuda()
ex = BatchExtractor(pp)
ref = []
for f in batches:
    s = ex.extract(f)
    torch.cuda.synchronize()
    ref.append({k: getattr(s, k).clone() for k in ("xy", "desc", "count")})
for mode in ("sync", "async"):
    for infl in (1, 2):
        pipe = BatchPipeline(pp, 0.85, B, H, W, pairs, inflight=infl, extra_slots=0)
        for i, f in enumerate(batches):
            ln = pipe.submit(f)
            if mode == "sync" or i == len(batches) - 1:
                pipe.join(); torch.cuda.synchronize()
            if mode == "sync" or i >= len(batches) - infl:
                pass
        pipe.join(); torch.cuda.synchronize()
        for i in range(len(batches) - infl, len(batches)):
            ln = pipe.lanes[i % infl]
            for k in ("xy", "desc", "count"):
                a, b = ref[i][k], ln["slots"].__dict__[k] if k in ln["slots"].__dict__ else getattr(ln["slots"], k)
                if not torch.equal(a, b):
                    d = (a != b).nonzero()
                    print(mode, infl, "batch", i, k, "differs at", d[:5].tolist(), "n", d.shape[0],
                          "counts", ref[i]["count"].tolist(), ln["slots"].count.tolist())
                else:
                    print(mode, infl, "batch", i, k, "ok")
