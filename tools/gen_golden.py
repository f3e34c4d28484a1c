#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE's own code.

Runs only in the build container (it imports /root/reference, which never travels to
the GPU box).  The reference's extractor imports cv2 (OpenCV 4.10, absent from the
image); oracle/cv2_standin.py is injected as `cv2`, so the reference's numpy code —
Harris, max-pool, median, top-k, edge filter, histograms, descriptors, matcher — runs
unmodified.  Fixtures hold inputs (generator arguments + SHA-256 of each frame, or the
explicit small arrays) and the reference's outputs.

    PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py [--skip-1080p]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden")

sys.dont_write_bytecode = True
sys.path.insert(0, ROOT)
from oracle import cv2_standin  # noqa: E402
from sfmfromscratch_amd import synth  # noqa: E402

sys.modules["cv2"] = cv2_standin
sys.path.insert(0, REF)
from FeatureExtractor.SIFT.NaiveSIFT import NaiveSIFT  # noqa: E402
from FeatureExtractor.SIFT.ScaleRotInvSIFT import ScaleRotInvSIFT  # noqa: E402
from FeatureMatcher.NNRatioFeatureMatcher import NNRatioFeatureMatcher  # noqa: E402

P_MAIN = {"num_interest_points": 2500, "ksize": 3, "gaussian_size": 7, "sigma": 6, "alpha": 0.05,
          "feature_width": 18, "pyramid_level": 3, "pyramid_scale_factor": 1.1}  # main.py:19-28
P_OCT = dict(P_MAIN, pyramid_level=4, pyramid_scale_factor=2)  # BASELINE.json configs[1]


def save(name, **arrays):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **arrays)
    print(f"  wrote {name} ({os.path.getsize(path) / 1024:.0f} KiB)")


def frame(H, W, seed, idx):
    u8 = synth.make_frame_u8(H, W, seed, idx)
    return synth.u8_to_gray(u8), synth.frame_sha256(u8)


def gen_atan2():
    rng = np.random.default_rng(20241223)
    ys, xs = [], []
    y = rng.standard_normal(20000).astype(np.float32); x = rng.standard_normal(20000).astype(np.float32)
    ys.append(y); xs.append(x)
    # Sobel-like values of /255-quantised images: small integer combinations / 255
    y = (rng.integers(-1020, 1021, 20000) / 255).astype(np.float32)
    x = (rng.integers(-1020, 1021, 20000) / 255).astype(np.float32)
    ys.append(y); xs.append(x)
    # diagonals and axis-near values (bin-edge critical: multiples of pi/4)
    v = rng.standard_normal(6000).astype(np.float32)
    for a, b in [(1, 1), (1, -1), (-1, 1), (-1, -1), (2, 1), (1, 2)]:
        ys.append((v * a).astype(np.float32)); xs.append((v * b).astype(np.float32))
    z = np.array([0.0, -0.0, 1.0, -1.0, 1e-30, -1e-30, 3.0], np.float32)
    yy, xx = np.meshgrid(z, z)
    ys.append(yy.ravel()); xs.append(xx.ravel())
    y = np.concatenate(ys); x = np.concatenate(xs)
    save("atan2.npz", y=y, x=x, out=np.arctan2(y, x))


def gen_histograms():
    rng = np.random.default_rng(7)
    e9 = np.linspace(-np.pi, np.pi, 9)
    e37 = np.linspace(-np.pi, np.pi, 37)
    vals, wts, edges_id, outs, lens = [], [], [], [], []
    pi32 = np.float32(np.pi)
    for case in range(400):
        n = [0, 1, 2, 4, 9, 16, 64, 81, 324][case % 9]
        kind = case % 4
        if kind == 0:
            v = rng.uniform(-np.pi, np.pi, n).astype(np.float32).astype(np.float64)
        elif kind == 1:  # float64 relative angles, some out of [-pi, pi]
            v = rng.uniform(-4.5, 4.5, n)
        elif kind == 2:  # exact edges, +-f32(pi), ties
            pool = np.concatenate([e9, e37, [pi32, -pi32, 0.0, np.float32(np.pi / 4)]]).astype(np.float64)
            v = rng.choice(pool, n)
        else:
            v = np.round(rng.uniform(-3.2, 3.2, n), 1)  # many ties
        w = rng.uniform(0, 2, n).astype(np.float32)
        eid = case % 2
        e = e9 if eid == 0 else e37
        h = np.histogram(v, bins=e, weights=w)[0]
        vals.append(v); wts.append(w); edges_id.append(eid); outs.append(h.astype(np.float32)); lens.append(n)
    save("histogram.npz", values=np.concatenate(vals), weights=np.concatenate(wts), lens=np.array(lens),
         edges_id=np.array(edges_id), out_flat=np.concatenate(outs), e9=e9, e37=e37)


def gen_gauss():
    cases = [(7, 5), (7, 6), (3, 1), (5, 2.5), (9, 3), (15, 7), (7, 0.7), (1, 1.0), (11, 2)]
    ns = NaiveSIFT(np.zeros((8, 8), np.float32), {})
    ks = np.array([c[0] for c in cases]); sg = np.array([c[1] for c in cases], np.float64)
    flat = np.concatenate([ns._generate_gaussian_kernel(k, s).astype(np.float32).ravel() for k, s in cases])
    save("gauss.npz", ksize=ks, sigma=sg, taps=flat)


DETECT_CASES = [
    # (H, W, seed, idx, k, fw, params)
    (120, 160, 7, 0, 300, 18, P_MAIN),
    (120, 160, 7, 0, 300, 16, {}),            # reference defaults: ksize 7, sigma 5
    (97, 131, 3, 2, 200, 9, P_MAIN),          # odd sizes (odd H*W -> median is the middle element)
    (96, 128, 4, 0, 1000, 4, dict(P_MAIN, ksize=5, alpha=0.04)),
    (64, 64, 5, 0, 50, 3, dict(P_MAIN, gaussian_size=5, sigma=2.5)),
    (30, 41, 6, 0, 100, 18, P_MAIN),          # tiny
]


def gen_detect():
    out = {}
    for i, (H, W, seed, idx, k, fw, pp) in enumerate(DETECT_CASES):
        img, sha = frame(H, W, seed, idx)
        ns = NaiveSIFT(img, pp)
        x, y, c = ns._find_harris_interest_points(img, k, fw)
        out[f"c{i}_x"] = x; out[f"c{i}_y"] = y; out[f"c{i}_c"] = c
        out[f"c{i}_sha"] = np.array(sha)
        print(f"  detect case {i}: {len(x)} keypoints")
    save("detect.npz", **out)


def gen_descriptors():
    out = {}
    cases = []
    for fw in (3, 4, 9, 14, 16, 18):
        for rotate in (0, 1):
            cases.append((100, 140, 9, 1, fw, rotate))
    for i, (H, W, seed, idx, fw, rotate) in enumerate(cases):
        img, sha = frame(H, W, seed, idx)
        cls = ScaleRotInvSIFT if rotate else NaiveSIFT
        obj = NaiveSIFT(img, P_MAIN)
        x, y, _ = obj._find_harris_interest_points(img, 120, fw)
        if rotate:
            # call the ScaleRot method without running its eager constructor
            inst = ScaleRotInvSIFT.__new__(ScaleRotInvSIFT)
            NaiveSIFT.__init__(inst, img, P_MAIN)
            d = inst._get_SIFT_descriptors(img, x, y, fw)
        else:
            d = obj._get_SIFT_descriptors(img, x, y, fw)
        d = np.asarray(d, np.float32).reshape(len(x), 128) if len(x) else np.zeros((0, 128), np.float32)
        out[f"c{i}_meta"] = np.array([H, W, seed, idx, fw, rotate])
        out[f"c{i}_x"] = x; out[f"c{i}_y"] = y; out[f"c{i}_d"] = d; out[f"c{i}_sha"] = np.array(sha)
        print(f"  descriptor case {i}: fw={fw} rotate={rotate} n={len(x)} ({cls.__name__})")
    save("descriptors.npz", ncases=np.array(len(cases)), **out)


def run_extract(img, pp, mode):
    if mode == "scalerot":
        obj = ScaleRotInvSIFT(img, pp)
    else:
        obj = NaiveSIFT(img, pp)
    X, Y = obj.detect_keypoints()
    D = obj.extract_descriptors()
    return np.asarray(X), np.asarray(Y), np.asarray(D, np.float32)


def gen_extract(name, H, W, seed, pp, mode, nframes=2, desc_stride=1, ratio=0.85):
    out = {"meta": np.array([H, W, seed, nframes, desc_stride]), "mode": np.array(mode),
           "params_keys": np.array(list(pp.keys())), "params_vals": np.array([float(v) for v in pp.values()])}
    descs = []
    for f in range(nframes):
        img, sha = frame(H, W, seed, f)
        t = time.time()
        X, Y, D = run_extract(img, pp, mode)
        dt = time.time() - t
        out[f"f{f}_sha"] = np.array(sha)
        out[f"f{f}_X"] = X; out[f"f{f}_Y"] = Y
        out[f"f{f}_D"] = D[::desc_stride]
        out[f"f{f}_Drowsum"] = D.astype(np.float64).sum(axis=1)
        out[f"f{f}_time_s"] = np.array(dt)
        descs.append(D)
        print(f"  {name} frame {f}: {len(X)} keypoints, reference {dt:.1f} s")
    if nframes >= 2:
        m, c = NNRatioFeatureMatcher(ratio_threshold=ratio).match_features_ratio_test(descs[0], descs[1])
        out["matches"] = np.asarray(m).reshape(-1, 2).astype(np.int64)
        out["conf"] = np.asarray(c, np.float32)
        out["ratio"] = np.array(ratio)
        print(f"  {name} matches: {len(c)}")
    save(name, **out)


class _StableSortNumpy:
    """numpy with a stable argsort, for numpy's histogram module only."""

    def __getattr__(self, name):
        return getattr(np, name)

    @staticmethod
    def argsort(a, *args, **kw):
        kw.pop("kind", None)
        return np.argsort(a, *args, kind="stable", **kw)


def gen_extract_stable_hist(name, H, W, seed, pp, mode, nframes=2):
    """The reference's extraction with np.histogram's weighted path sorting STABLY (ties of
    equal orientations summed in window raster order).  numpy's default argsort is unstable,
    so which order a tie's weights are summed in is CPU-specific and a near-empty bin (a
    difference of two float32 prefix sums) can move by a few ulp of the running total; with a
    stable sort the reference's descriptors are fully determined, and tests compare them
    without the near-empty-bin escape (tests/golden_util.desc_close max_escapes=0).  Only
    the histogram module's numpy is replaced; keypoint selection is untouched."""
    import numpy.lib._histograms_impl as hist_impl
    saved = hist_impl.np
    hist_impl.np = _StableSortNumpy()
    try:
        gen_extract(name, H, W, seed, pp, mode, nframes=nframes)
    finally:
        hist_impl.np = saved


def gen_match():
    out = {}
    cases = []
    cases.append(("rand_dup", 300, 1, 400, 2, 3, 0.8))
    cases.append(("small", 50, 3, 2, 4, 1, 0.85))
    cases.append(("ratio1", 60, 5, 70, 6, 0, 1.0))
    for i, (nm, n1, s1, n2, s2, jit, ratio) in enumerate(cases):
        a, ha = synth.make_descriptor_table(n1, s1)
        b, _ = synth.make_descriptor_table(n2, s2, dup_of=ha, jitter=jit)
        m, c = NNRatioFeatureMatcher(ratio_threshold=ratio).match_features_ratio_test(a, b)
        out[f"c{i}_meta"] = np.array([n1, s1, n2, s2, jit])
        out[f"c{i}_ratio"] = np.array(ratio)
        out[f"c{i}_m"] = np.asarray(m).reshape(-1, 2).astype(np.int64)
        out[f"c{i}_c"] = np.asarray(c, np.float32)
        print(f"  match case {nm}: {len(c)} matches")
    save("match.npz", ncases=np.array(len(cases)), **out)


def gen_ingest():
    """FeatureRunner's ingest (Runner.py:33-46) run by the reference's own helpers on
    synthetic decoded RGB frames: _load_image's u8 -> float32 / 255 (:551-563),
    _PIL_resize to (int(W*s), int(H*s)) (:37-42, :481-493), _rgb2gray (:467-478).
    Small cases keep the whole gray output; the 4K -> 1080p case keeps its SHA-256."""
    import Runner  # the reference harness (imports PIL, matplotlib and the cv2 stand-in)
    cases = [(240, 320, 11, 0, 0.5), (241, 479, 12, 1, 0.5), (64, 97, 13, 2, 0.5), (90, 60, 14, 0, 0.75),
             (2160, 3840, 15, 0, 0.5)]
    out = {"ncases": np.int64(len(cases))}
    for i, (H, W, seed, idx, s) in enumerate(cases):
        rgb = synth.make_frame_rgb_u8(H, W, seed, idx)
        img = rgb.astype(np.float64).astype(np.float32) / 255           # _load_image / _im2single
        size = (int(img.shape[1] * s), int(img.shape[0] * s))
        g = Runner._rgb2gray(Runner._PIL_resize(img, size))
        assert g.dtype == np.float32
        out[f"c{i}_meta"] = np.array([H, W, seed, idx], np.int64)
        out[f"c{i}_scale"] = np.float64(s)
        out[f"c{i}_sha_in"] = np.array(synth.frame_sha256(rgb))
        out[f"c{i}_sha_out"] = np.array(synth.frame_sha256(g))
        out[f"c{i}_shape"] = np.array(g.shape, np.int64)
        if H * W <= 240 * 480:
            out[f"c{i}_gray"] = g
    save("ingest.npz", **out)


def ransac_cases():
    """Correspondence sets for the RANSAC consumer (SFM.py:126-160): matched keypoints of
    synthetic frame pairs through the oracle's extract + match and the reference's own
    _convert_matches_to_coords rule (first 2,500 matches, Runner.py:423-434), a planted
    translation with outliers, and a set below 8 points."""
    from oracle import oracle as O
    cases = []
    for (H, W, seed, iters, thr) in [(540, 960, 77, 5967, 1.0), (720, 1280, 78, 1500, 1.0), (540, 960, 79, 800, 0.5)]:
        f = [synth.make_frame(H, W, seed, i) for i in range(2)]
        E = [O.extract(x, P_OCT) for x in f]
        m, _ = O.match(E[0][2], E[1][2], 0.85)
        mm = m[:2500]
        p1 = np.column_stack((E[0][0][mm[:, 0]], E[0][1][mm[:, 0]]))
        p2 = np.column_stack((E[1][0][mm[:, 1]], E[1][1][mm[:, 1]]))
        cases.append((p1, p2, iters, thr))
    rng = np.random.default_rng(5)
    p1 = rng.integers(0, 900, (300, 2)).astype(np.int64)
    p2 = p1 + np.array([3, 2])
    out = rng.random(300) < 0.3
    p2[out] = rng.integers(0, 900, (int(out.sum()), 2))
    cases.append((p1, p2, 500, 1.0))
    cases.append((p1[:7], p2[:7], 100, 1.0))
    return cases


def gen_ransac():
    """The reference's CameraPose.find_inliers itself on ransac_cases() (its cv2 import is
    the stand-in; find_inliers uses numpy only)."""
    from SFM import CameraPose
    out = {}
    cases = ransac_cases()
    out["ncases"] = np.int64(len(cases))
    for i, (p1, p2, iters, thr) in enumerate(cases):
        t0 = time.time()
        r = CameraPose.find_inliers(p1, p2, threshold=thr, max_iterations=iters)
        out[f"c{i}_p1"], out[f"c{i}_p2"] = p1, p2
        out[f"c{i}_meta"] = np.array([iters], np.int64)
        out[f"c{i}_thr"] = np.float64(thr)
        if len(r) == 4:  # fewer than 8 points: (None, None, None, None)
            out[f"c{i}_none"] = np.int64(1)
        else:
            out[f"c{i}_in1"], out[f"c{i}_in2"] = np.asarray(r[0]), np.asarray(r[1])
        print(f"  case {i}: n={len(p1)} iters={iters} -> {'None' if len(r) == 4 else len(r[0])} "
              f"({time.time() - t0:.1f} s)")
    save("ransac.npz", **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-1080p", action="store_true")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    os.makedirs(OUT, exist_ok=True)
    steps = {
        "atan2": gen_atan2,
        "histogram": gen_histograms,
        "gauss": gen_gauss,
        "detect": gen_detect,
        "descriptors": gen_descriptors,
        "match": gen_match,
        "ingest": gen_ingest,
        "ransac": gen_ransac,
        "small": lambda: (gen_extract("extract_small_scalerot.npz", 150, 200, 21, P_OCT, "scalerot"),
                          gen_extract("extract_small_pmain.npz", 151, 203, 22, P_MAIN, "scalerot"),
                          gen_extract("extract_small_naive.npz", 150, 200, 23, {"num_interest_points": 500},
                                      "naive", ratio=0.8),
                          gen_extract("extract_small_defaults.npz", 128, 160, 24, {}, "scalerot")),
        "stable": lambda: (gen_extract_stable_hist("extract_small_pmain_stablehist.npz", 151, 203, 22, P_MAIN,
                                                   "scalerot"),
                           gen_extract_stable_hist("extract_small_scalerot_stablehist.npz", 150, 200, 21, P_OCT,
                                                   "scalerot")),
        "c1": lambda: gen_extract("extract_c1_640x480_pmain.npz", 480, 640, 1234, P_MAIN, "scalerot",
                                  desc_stride=4),
        "c2": lambda: gen_extract("extract_c2_1080p_poct.npz", 1080, 1920, 1234, P_OCT, "scalerot",
                                  desc_stride=8),
    }
    for name, fn in steps.items():
        if a.only and name not in a.only.split(","):
            continue
        if name == "c2" and a.skip_1080p:
            continue
        print(f"[{name}]")
        fn()


if __name__ == "__main__":
    main()
