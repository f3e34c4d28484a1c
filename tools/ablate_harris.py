"""Time k_harris<7> ablation variants on the GPU (diagnostic)."""
import ctypes, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sfmfromscratch_amd import _native
L = _native.load_library()
f = L.sfm_debug_time_harris
f.restype = ctypes.c_float
f.argtypes = [ctypes.c_int32] * 6
for B, H, W in [(32, 1080, 1920)]:
    for abl, name in [(0, "full"), (1, "no-hist"), (2, "window-1row"), (4, "no-barriers"), (0, "full")]:
        print(f"B={B} {H}x{W} {name:10s} {f(0, abl, B, H, W, 20):8.3f} ms", flush=True)
