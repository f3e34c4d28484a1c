"""Diagnostic: run the configs[3] world-1 job (distributed.ChunkedGatherJob) and compare every
gathered slot with a fresh extraction of its frame (B = 1 and the same 32-frame chunk).
Prints the frames that differ and how (set-equal keypoints in another order, or not)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from sfmfromscratch_amd import distributed as D
from sfmfromscratch_amd import synth
from sfmfromscratch_amd.pipeline import BatchExtractor

P_OCT = {"num_interest_points": 2500, "ksize": 3, "gaussian_size": 7, "sigma": 6, "alpha": 0.05,
         "feature_width": 18, "pyramid_level": 4, "pyramid_scale_factor": 2}
H, W = 1080, 1920
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
inflight = int(sys.argv[3]) if len(sys.argv) > 3 else 2
U = min(n, 64)
dev = torch.device("cuda", 0)
uq = torch.from_numpy(np.stack([synth.make_frame_u8(H, W, 1234, i) for i in range(U)])).to(dev)
frames = uq[torch.arange(n, device=dev) % U].contiguous()
plan = D.GatherPlan(n, 1, 32, "consecutive")
job = D.ChunkedGatherJob(P_OCT, 0.85, plan, 0, H, W, inflight=inflight)
what = sys.argv[4] if len(sys.argv) > 4 else "all"
if what in ("none", "prep"):
    job.matcher.match = lambda *a, **k: None
if what == "none":
    job.matcher.prep = lambda *a, **k: None
print("matcher:", what, "inflight", inflight, flush=True)
ex = BatchExtractor(P_OCT)
ref = {}
for u in range(U):
    s = ex.extract(uq[u:u + 1])
    c = int(s.count[0])
    ref[u] = (c, s.xy[0, :c].cpu().numpy().copy(), s.desc[0, :c].cpu().numpy().copy())
for r in range(runs):
    job.run(frames)
    torch.cuda.synchronize()
    xy = job.table.xy.cpu().numpy()
    cnt = job.table.count.cpu().numpy()
    bad = []
    for g in range(n):
        t = int(plan.slot_of(g))
        c, rxy, _ = ref[g % U]
        if cnt[t] != c or not np.array_equal(xy[t, :c], rxy):
            same_set = cnt[t] == c and set(map(tuple, xy[t, :c].tolist())) == set(map(tuple, rxy.tolist()))
            first = int(np.argmax((xy[t, :c] != rxy).any(1))) if cnt[t] == c else -1
            bad.append((g, int(cnt[t]), c, bool(same_set), first))
    print(f"run {r}: {len(bad)} of {n} frames differ: {bad[:12]}", flush=True)
