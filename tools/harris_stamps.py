"""Per-workgroup timeline of one k_harris<7> launch (ABL = 3 timestamps; diagnostic):
start / end spread over the workgroups, per-tile times, the tail."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sfmfromscratch_amd import _native
L = _native.load_library()
B, H, W = 32, 1080, 1920
cap = 1024 * B * 48
buf = np.zeros(cap, np.uint64)
ms = L.sfm_debug_harris_stamps(0, 3, B, H, W, 5, buf.ctypes.data, cap)
print(f"mean launch {ms:.3f} ms")
st = buf.reshape(-1, 48)
st = st[st[:, 0] > 0]
t0 = st[:, 0].min()
s = (st[:, 0] - t0) / 100.0  # us
e = (st[:, 1] - t0) / 100.0
nt = st[:, 3].astype(int)
print(f"workgroups {len(st)}, kernel span {e.max():.1f} us")
print("start us: min %.1f p50 %.1f p90 %.1f max %.1f" % (s.min(), *np.percentile(s, [50, 90]), s.max()))
print("end   us: min %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f" % (e.min(), *np.percentile(e, [10, 50, 90]), e.max()))
life = e - s
print("life  us: min %.1f p50 %.1f max %.1f; mean life / span %.3f" % (life.min(), np.median(life), life.max(), life.mean() / e.max()))
tt = []
for r in st:
    n = min(int(r[3]), 44)
    ts = np.concatenate([[r[0]], r[4:4 + n]]).astype(np.float64)
    tt.append(np.diff(ts) / 100.0)
tt = np.concatenate(tt)
print("tile us: min %.2f p10 %.2f p50 %.2f p90 %.2f max %.2f" % (tt.min(), *np.percentile(tt, [10, 50, 90]), tt.max()))
cus = st[:, 2].astype(int)
print("distinct CU ids", len(np.unique(cus)), "tiles per wg", np.bincount(nt).nonzero()[0].tolist())
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/harris_stamps.npy", st)
# per CU: the two workgroups' end times; by wall-clock slot of tiles
order = np.argsort(cus)
pairs = {}
for r, c in zip(st, cus):
    pairs.setdefault(int(c), []).append(((r[0] - t0) / 100.0, (r[1] - t0) / 100.0))
spread = [abs(v[0][1] - v[1][1]) for v in pairs.values() if len(v) == 2]
print("per-CU |end difference| us: p50 %.1f p90 %.1f; CUs with 2 WGs %d" % (np.median(spread), np.percentile(spread, 90), len(spread)))
ends = np.array([max(a[1] for a in v) for c, v in sorted(pairs.items())])
print("per-CU last end, by CU id blocks of 32:", [round(float(ends[i:i + 32].mean()), 1) for i in range(0, len(ends), 32)])
