"""Harris alone, per pyramid level of the configs[1] step: the mean duration of one k_harris<7>
launch over 32 planes of each P-oct level size (sfm_debug_time_harris, abl 0: the product kernel
on synthetic planes, no other work on the GPU), and their sum = Harris per step alone.
usage: python tools/harris_alone.py [iters] [lib.so] [abl]  (abl != 0: the diagnostic build's timing
ablations, e.g. 1 = no digit histogram)"""
import os
import sys

import ctypes  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sfmfromscratch_amd import _native  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
_native._preload_torch_hip_runtime()
L = ctypes.CDLL(sys.argv[2] if len(sys.argv) > 2 else _native.LIB_PATH)  # any build (A/B): one symbol bound
f = L.sfm_debug_time_harris
f.restype = ctypes.c_float
f.argtypes = [ctypes.c_int32] * 6
abl = int(sys.argv[3]) if len(sys.argv) > 3 else 0
f(0, abl, 32, 1080, 1920, 3)  # warm-up
tot, px = 0.0, 0
for lvl in range(4):
    H, W = 1080 >> lvl, 1920 >> lvl
    ms = f(0, abl, 32, H, W, iters)
    tot += ms
    px += 32 * H * W
    print(f"L{lvl} {H}x{W} x32: {ms * 1e3:8.1f} us", flush=True)
tf = 328 * px / (tot / 1e3) / 1e12
print(f"sum {tot:.4f} ms per step alone: {tf:.1f} TFLOP/s = {tf / 157.3:.3f} of the FP32 peak")
