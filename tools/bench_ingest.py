"""Ingest-only timing (diagnostic): B decoded 4K RGB frames -> 1080p gray on the device."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from sfmfromscratch_amd import _abi, _native, synth
from sfmfromscratch_amd.pipeline import ingest_rgb
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
uniq = [synth.make_frame_rgb_u8(2160, 3840, 1234, i) for i in range(4)]
rgb = torch.from_numpy(np.stack([uniq[i % 4] for i in range(B)])).cuda()
ctx = _native.Context(_abi.params_from_dict({}, _abi.SFM_MODE_NAIVE))
out = ingest_rgb(ctx, rgb)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    ingest_rgb(ctx, rgb, out=out)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 10
gb = B * (2160 * 3840 * 3 + 1080 * 1920 * 4) / 1e9
print(f"ingest {B} x 4K RGB -> 1080p gray: {ms:.3f} ms, {gb / ms * 1e3:.0f} GB/s algorithmic")
