"""Diagnostic: how many planes of a 1080p P-oct batch take the exact path (select stats),
per build; SFMFEAT_SELECT=exact for comparison."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from sfmfromscratch_amd import synth
from sfmfromscratch_amd.pipeline import BatchExtractor

P_OCT = {"num_interest_points": 2500, "ksize": 3, "gaussian_size": 7, "sigma": 6, "alpha": 0.05,
         "feature_width": 18, "pyramid_level": 4, "pyramid_scale_factor": 2}
B = 32
u8 = np.stack([synth.make_frame_u8(1080, 1920, 1234, i) for i in range(B)])
frames = torch.from_numpy(synth.u8_to_gray(u8)).cuda()
ex = BatchExtractor(P_OCT)
ex.extract(frames)
torch.cuda.synchronize()
print("fallback planes / total:", ex.ctx.select_stats(), flush=True)
# level-3 R maps: how many 3x3 window maxima lie above the median's digit-1 bucket?
L, l = 4, 3
h, w = 1080 >> l, 1920 >> l
Rm = torch.empty((B, h, w), device="cuda")
ex.ctx.copy_level(l, 0, Rm.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
R = Rm.cpu().numpy()


def fkey(a):
    b = a.astype(np.float32).view(np.uint32).copy()
    b[b == 0x80000000] = 0
    return np.where(b & 0x80000000, ~b, b | 0x80000000).astype(np.uint32)


for b in range(3):
    r = R[b]
    pad = np.pad(r, 1, constant_values=-np.inf)
    m = np.max(np.stack([pad[dy:dy + h, dx:dx + w] for dy in range(3) for dx in range(3)]), 0)
    med = np.median(r)
    keys = fkey(r)
    b1 = fkey(np.array([np.sort(r.ravel())[r.size // 2 - 1]]))[0] >> 21
    b2 = fkey(np.array([np.sort(r.ravel())[r.size // 2]]))[0] >> 21
    maxima = np.sort(r[(r == m)])[::-1]
    above = maxima[fkey(maxima) >= (b1 << 21)]
    kth = above[624] if len(above) > 624 else None
    print(f"plane {b}: median {med:.3e}, maxima {len(maxima)}, at/above median bucket {len(above)}, "
          f"625th {kth}, tcert key {(b2 + 1) << 21:#x}, 625th key {fkey(np.array([kth]))[0] if kth is not None else None:#x}", flush=True)
