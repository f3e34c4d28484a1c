"""Diagnostic: the headline pipeline (pipeline.BatchPipeline, 2 lanes, 32 x 1080p batches)
against B = 1 extractions: every lane's slots after every batch must equal the clean ones."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from sfmfromscratch_amd import distributed as D
from sfmfromscratch_amd import synth
from sfmfromscratch_amd.pipeline import BatchExtractor, BatchPipeline, consecutive_pairs

P_OCT = {"num_interest_points": 2500, "ksize": 3, "gaussian_size": 7, "sigma": 6, "alpha": 0.05,
         "feature_width": 18, "pyramid_level": 4, "pyramid_scale_factor": 2}
H, W, B = 1080, 1920, 32
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda", 0)
u8 = np.stack([synth.make_frame_u8(H, W, 1234, i) for i in range(B)])
frames = torch.from_numpy(synth.u8_to_gray(u8)).to(dev)
ex1 = BatchExtractor(P_OCT)
ref = torch.cat([D.slot_checksums(torch, ex1.extract(frames[b:b + 1].contiguous())) for b in range(B)])
pairs = torch.from_numpy(consecutive_pairs(B)).to(dev)
pipe = BatchPipeline(P_OCT, 0.85, B, H, W, pairs, inflight=2, extra_slots=1)
cks = []
for s in range(steps):
    ln = pipe.submit(frames)
    with torch.cuda.stream(ln["stream"]):
        cks.append(D.slot_checksums(torch, ln["view"]))
pipe.join()
torch.cuda.synchronize()
for s, ck in enumerate(cks):
    bad = (ck != ref).any(1).nonzero().flatten().tolist()
    print(f"batch {s}: {len(bad)} of {B} frames differ {bad[:12]}", flush=True)
