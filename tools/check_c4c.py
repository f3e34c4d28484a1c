"""Diagnostic: which extraction stage goes wrong when the matcher runs concurrently?  Like
check_c4b (lane stream extracts 32-frame chunks into the table, a second stream preps and
matches the ready pairs), but after each chunk the lane context's level images and R maps
are snapshotted on the lane stream and compared with a clean B = 1 extraction's."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from sfmfromscratch_amd import distributed as D
from sfmfromscratch_amd import synth
from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, SlotTable

P_OCT = {"num_interest_points": 2500, "ksize": 3, "gaussian_size": 7, "sigma": 6, "alpha": 0.05,
         "feature_width": 18, "pyramid_level": 4, "pyramid_scale_factor": 2}
H, W = 1080, 1920
n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
U = min(n, 64)
L = 4
dims = [(H >> l, W >> l) for l in range(L)]
dev = torch.device("cuda", 0)
uq = torch.from_numpy(np.stack([synth.make_frame_u8(H, W, 1234, i) for i in range(U)])).to(dev)
frames = uq[torch.arange(n, device=dev) % U].contiguous()
ex1 = BatchExtractor(P_OCT)
refR = [torch.empty((U, h, w), device=dev) for h, w in dims]
refI = [torch.empty((U, h, w), device=dev) for h, w in dims]
refck = []
cur = torch.cuda.current_stream()
for u in range(U):
    refck.append(D.slot_checksums(torch, ex1.extract(uq[u:u + 1])))
    for l in range(L):
        ex1.ctx.copy_level(l, 0, refR[l][u].data_ptr(), cur.cuda_stream)
        ex1.ctx.copy_level(l, 1, refI[l][u].data_ptr(), cur.cuda_stream)
refck = torch.cat(refck)
torch.cuda.synchronize()
plan = D.GatherPlan(n, 1, 32, "consecutive")
ex = BatchExtractor(P_OCT)
ex.reserve(32, H, W)
table = SlotTable(torch, n, ex.cap, dev)
m = BatchMatcher(0.85)
sched = [torch.from_numpy(np.ascontiguousarray(p, np.int32)).to(dev) for p in plan.schedule(plan.rank_pairs(0))]
outs = [m.match(table, s) for s in sched]
torch.cuda.synchronize()
ls, ms = torch.cuda.Stream(), torch.cuda.Stream()
snapR = [torch.empty((n, h, w), device=dev) for h, w in dims]
snapI = [torch.empty((n, h, w), device=dev) for h, w in dims]


def view(lo, k):
    v = SlotTable.__new__(SlotTable)
    v.B, v.cap = k, table.cap
    v.xy, v.desc, v.count = table.xy[lo:lo + k], table.desc[lo:lo + k], table.count[lo:lo + k]
    return v


for run in range(2):
    ck = torch.zeros((n, 3), dtype=torch.int64, device=dev)
    ls.wait_stream(cur)
    ms.wait_stream(cur)
    for c in range(plan.C):
        l0 = c * 32
        with torch.cuda.stream(ls):
            ex.extract(frames[l0:l0 + 32], out=view(l0, 32))
            ck[l0:l0 + 32] = D.slot_checksums(torch, view(l0, 32))
            for l in range(L):
                ex.ctx.copy_level(l, 0, snapR[l][l0].data_ptr(), ls.cuda_stream)
                ex.ctx.copy_level(l, 1, snapI[l][l0].data_ptr(), ls.cuda_stream)
        with torch.cuda.stream(ms):
            ms.wait_stream(ls)
            m.prep(table, l0, 32)
            if len(sched[c]):
                m.match(table, sched[c], out=outs[c], prepped=True)
    cur.wait_stream(ls)
    cur.wait_stream(ms)
    torch.cuda.synchronize()
    idx = torch.arange(n, device=dev) % U
    bad = (ck != refck[idx]).any(1).nonzero().flatten().tolist()
    print(f"run {run}: {len(bad)} frames wrong: {bad[:16]}", flush=True)
    for g in bad[:6]:
        u = g % U
        msg = []
        for l in range(L):
            dI = (snapI[l][g] != refI[l][u])
            dR = (snapR[l][g].view(torch.int32) != refR[l][u].view(torch.int32))
            nI, nR = int(dI.sum()), int(dR.sum())
            box = ""
            if nR:
                ys, xs = dR.nonzero(as_tuple=True)
                box = f"[{int(ys.min())}:{int(ys.max())}, {int(xs.min())}:{int(xs.max())}]"
            msg.append(f"L{l}: img {nI} R {nR} {box}")
        print(f"  frame {g}: " + "; ".join(msg), flush=True)
