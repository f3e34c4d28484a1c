"""Diagnostic: extract the same 32-frame 1080p chunk repeatedly with one BatchExtractor and
compare every repetition's slots with a B = 1 extraction of each frame.  Modes (argv[1]):
u8 | f32 input; env SFMFEAT_SERIAL / SFMFEAT_SELECT switch the library's schedule."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from sfmfromscratch_amd import synth
from sfmfromscratch_amd.pipeline import BatchExtractor

P_OCT = {"num_interest_points": 2500, "ksize": 3, "gaussian_size": 7, "sigma": 6, "alpha": 0.05,
         "feature_width": 18, "pyramid_level": 4, "pyramid_scale_factor": 2}
H, W = 1080, 1920
mode = sys.argv[1] if len(sys.argv) > 1 else "u8"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
B = int(sys.argv[3]) if len(sys.argv) > 3 else 32
dev = torch.device("cuda", 0)
u8 = torch.from_numpy(np.stack([synth.make_frame_u8(H, W, 1234, i) for i in range(B)])).to(dev)
src = u8 if mode == "u8" else (u8.float() / 255.0).contiguous()
if mode != "u8":  # the exact u8 / 255 float32 frames
    src = torch.from_numpy(synth.u8_to_gray(u8.cpu().numpy())).to(dev)
ex1 = BatchExtractor(P_OCT)
ref = []
for b in range(B):
    s = ex1.extract(src[b:b + 1].contiguous())
    c = int(s.count[0])
    ref.append((c, s.xy[0, :c].cpu().numpy().copy(), s.desc[0, :c].cpu().numpy().copy()))
ex = BatchExtractor(P_OCT)
ex.reserve(B, H, W)
out = ex.new_slots(B)
for r in range(reps):
    ex.extract(src, out=out)
    torch.cuda.synchronize()
    xy, cnt = out.xy.cpu().numpy(), out.count.cpu().numpy()
    desc = out.desc.cpu().numpy()
    bad = []
    for b in range(B):
        c, rxy, rd = ref[b]
        if cnt[b] != c or not np.array_equal(xy[b, :c], rxy) or not np.array_equal(desc[b, :c], rd):
            first = int(np.argmax((xy[b, :c] != rxy).any(1))) if cnt[b] == c else -1
            bad.append((b, int(cnt[b]), c, first))
    print(f"{mode} rep {r}: {len(bad)} of {B} differ {bad[:10]}", flush=True)
