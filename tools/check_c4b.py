"""Diagnostic for the configs[3] world-1 job: extraction into the chunk-major table on a lane
stream, prep + prepped matching of each chunk's pairs on a second stream.  Per chunk the
slots' checksums are taken on the lane stream right after extraction; after the job they
are compared with the table (modified later?) and with B = 1 reference extractions
(computed wrong?).  argv: n_frames, mode (two = lane + match stream, one = one stream)."""
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
n = int(sys.argv[1])
mode = sys.argv[2]
noise = sys.argv[3] if len(sys.argv) > 3 else "match"  # what the second stream runs
U = min(n, 64)
dev = torch.device("cuda", 0)
uq = torch.from_numpy(np.stack([synth.make_frame_u8(H, W, 1234, i) for i in range(U)])).to(dev)
frames = uq[torch.arange(n, device=dev) % U].contiguous()
if os.environ.get("C4B_F32") == "1":  # f32 frames (u8 / 255): level 0 is read from the caller's tensor
    frames = torch.from_numpy(synth.u8_to_gray(frames.cpu().numpy())).to(dev)
    uq = torch.from_numpy(synth.u8_to_gray(uq.cpu().numpy())).to(dev)
ex1 = BatchExtractor(P_OCT)
refck = []
for u in range(U):
    refck.append(D.slot_checksums(torch, ex1.extract(uq[u:u + 1])))
refck = torch.cat(refck)
plan = D.GatherPlan(n, 1, 32, "consecutive")
ex = BatchExtractor(P_OCT)
ex.reserve(32, H, W)
table = SlotTable(torch, n, ex.cap, dev)
m = BatchMatcher(0.85)
sched = [torch.from_numpy(np.ascontiguousarray(p, np.int32)).to(dev) for p in plan.schedule(plan.rank_pairs(0))]
outs = [m.match(table, s) for s in sched]  # allocate outputs (and the matcher's buffers)
torch.cuda.synchronize()
ls, ms = torch.cuda.Stream(), torch.cuda.Stream()
junk = torch.empty(256 << 20, dtype=torch.float32, device=dev)
ma = torch.randn(4096, 4096, device=dev)
mo = torch.empty_like(ma)


def view(lo, k):
    v = SlotTable.__new__(SlotTable)
    v.B, v.cap = k, table.cap
    v.xy, v.desc, v.count = table.xy[lo:lo + k], table.desc[lo:lo + k], table.count[lo:lo + k]
    return v


for run in range(3):
    ck = torch.zeros((n, 3), dtype=torch.int64, device=dev)
    cur = torch.cuda.current_stream()
    ls.wait_stream(cur)
    ms.wait_stream(cur)
    for c in range(plan.C):
        l0 = c * 32
        st = ls if mode == "two" else ms
        with torch.cuda.stream(st):
            ex.extract(frames[l0:l0 + 32], out=view(l0, 32))
            ck[l0:l0 + 32] = D.slot_checksums(torch, view(l0, 32))
        with torch.cuda.stream(ms):
            if mode == "two":
                ms.wait_stream(ls)
            if noise == "match":
                m.prep(table, l0, 32)
                if len(sched[c]):
                    m.match(table, sched[c], out=outs[c], prepped=True)
            elif noise == "fill":
                for _ in range(20):
                    junk.fill_(float(c))
            elif noise == "mm":
                for _ in range(4):
                    torch.mm(ma, ma, out=mo)
    cur.wait_stream(ls)
    cur.wait_stream(ms)
    torch.cuda.synchronize()
    final = D.slot_checksums(torch, table)
    ref = refck[torch.arange(n, device=dev) % U]
    at_extract = (ck != ref).any(1).nonzero().flatten().tolist()
    later = (final != ck).any(1).nonzero().flatten().tolist()
    print(f"{mode}/{noise} run {run}: wrong at extraction {len(at_extract)} {at_extract[:10]}; "
          f"changed after extraction {len(later)} {later[:10]}", flush=True)
