"""Timeline of the matcher sweep from in-kernel clock stamps (diagnostic build; results of the
stamped launch are not checked).  Runs tools/bench_match.py's workload (one batch of 32
synthetic 1080p frames, 31 consecutive pairs) with the diagnostic library and
SFMFEAT_MATCH_ABL=32, then prints, per stage (averaged over the stamped workgroups' waves), the
shader-clock cycles of: the stage barrier (end of the previous stage's DMA issue -> after the
barrier), sub-tile region 0, sub-tile region 1, and the DMA issue; and the clock rate.
usage: python tools/match_stamps.py [--4k]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("SFMFEAT_LIB", os.path.join(ROOT, "sfmfromscratch_amd", "lib_diag", "libsfmfeat.so"))
os.environ["SFMFEAT_MATCH_ABL"] = "32"


def main():
    import numpy as np
    import torch
    from sfmfromscratch_amd import _native, synth
    from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, consecutive_pairs
    P_OCT = {"num_interest_points": 2500, "ksize": 3, "gaussian_size": 7, "sigma": 6, "alpha": 0.05,
             "feature_width": 18, "pyramid_level": 4, "pyramid_scale_factor": 2}
    H, W, B = 1080, 1920, 32
    if "--4k" in sys.argv:
        H, W, B = 2160, 3840, 8
        P_OCT.update(num_interest_points=8000, pyramid_level=5)
    ex = BatchExtractor(P_OCT)
    u8 = np.stack([synth.make_frame_u8(H, W, 1234, i) for i in range(B)])
    slots = ex.extract(torch.from_numpy(u8).cuda())
    pairs = torch.from_numpy(consecutive_pairs(B)).cuda()
    m = BatchMatcher(0.85, ctx=ex.ctx)
    out = m.match(slots, pairs)
    for _ in range(3):
        m.match(slots, pairs, out=out)
    torch.cuda.synchronize()
    L = _native.load_library()
    n = 16 * 8 * 41 * 4 + 1024 * 4
    buf = np.zeros(n, np.uint64)
    got = L.sfm_debug_match_stamps(buf.ctypes.data, n)
    if got != n:
        raise SystemExit(f"sfm_debug_match_stamps returned {got}: not the diagnostic library?")
    st = buf[:16 * 8 * 41 * 4].reshape(16, 8, 41, 4).astype(np.int64)
    wg = buf[16 * 8 * 41 * 4:].reshape(1024, 4).astype(np.int64)
    live = wg[:, 1] > 0
    t0 = wg[live, 0].min()
    real = live & (wg[:, 3] != 0) | (live & (np.arange(1024) < 8))
    ends = (wg[:, 1] - t0) / 100.0
    starts = (wg[:, 0] - t0) / 100.0
    print(f"workgroups stamped {live.sum()}; start us: min {starts[live].min():.1f} max {starts[live].max():.1f}; "
          f"end us max {ends[live].max():.1f}")
    hist = np.histogram(starts[live], bins=[0, 1, 5, 20, 40, 60, 80, 100, 150, 400])
    print("start-time histogram (us bins -> workgroups):", list(zip(hist[1][:-1].tolist(), hist[0].tolist())))
    np.save(os.path.join(ROOT, "gpurun_out", "match_wg.npy"), wg)
    meta = st[:, :, 40, :]
    nst = int(meta[0, 0, 3] >> 32)
    S = min(nst, 40)
    t = st[:, :, :S, :]
    bar = t[:, :, 1:, 0] - t[:, :, :-1, 3]
    r0 = t[:, :, :, 1] - t[:, :, :, 0]
    r1 = t[:, :, :, 2] - t[:, :, :, 1]
    dma = t[:, :, :, 3] - t[:, :, :, 2]
    first = t[:, :, 0, 0] - meta[:, :, 0]
    cyc = (t[:, :, S - 1, 3] - meta[:, :, 0]).astype(np.float64)
    rt = (meta[:, :, 2] - meta[:, :, 1]).astype(np.float64) * 10.0  # 100 MHz -> ns (end: after the loop)
    print(f"stages {nst} (stamped {S}); clock ~{np.median(cyc / rt) * 1e3:.0f} MHz (loop cycles / wall, median over waves)")
    print(f"prologue (start -> after stage 0 barrier): {np.median(first):.0f} cycles")
    print(f"{'stage':>5s} {'barrier':>8s} {'region0':>8s} {'region1':>8s} {'dma':>6s} {'total':>7s}   (median over 16 WGs x 8 waves, cycles)")
    tot = np.zeros(4)
    for s in range(S):
        b = np.median(bar[:, :, s - 1]) if s > 0 else 0.0
        row = [b, np.median(r0[:, :, s]), np.median(r1[:, :, s]), np.median(dma[:, :, s])]
        if s >= 2:
            tot += row
        if s < 6 or s % 8 == 0 or s == S - 1:
            print(f"{s:5d} {row[0]:8.0f} {row[1]:8.0f} {row[2]:8.0f} {row[3]:6.0f} {sum(row):7.0f}")
    k = max(S - 2, 1)
    print(f"mean over stages 2..{S - 1}: barrier {tot[0] / k:.0f}, region0 {tot[1] / k:.0f}, region1 {tot[2] / k:.0f}, "
          f"dma {tot[3] / k:.0f}, total {tot.sum() / k:.0f} cycles per stage")
    # spread of waves: how long the first wave of a workgroup waits for the last at each barrier
    arr = t[:, :, 1:, 0] - t[:, :, :-1, 3]
    print(f"barrier wait, per wave, stages 2+: min {np.median(arr[:, :, 1:].min(axis=1)):.0f} / max "
          f"{np.median(arr[:, :, 1:].max(axis=1)):.0f} cycles (median over WGs and stages)")
    np.save(os.path.join(ROOT, "gpurun_out", "match_stamps.npy"), st)


if __name__ == "__main__":
    main()
