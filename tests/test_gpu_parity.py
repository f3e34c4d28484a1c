"""GPU parity: the HIP path (through the C-ABI) against the golden fixtures generated from
the reference and against the C oracle on the same seeded inputs.

Bars: keypoint X/Y and match pairs bit-identical (ties as sets);
descriptors within 1e-4 relative of the reference (tests/golden_util.desc_close) and
BIT-identical to the oracle, which shares the restated norm order.
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle as O
from sfmfromscratch_amd import NaiveSIFT, NNRatioFeatureMatcher, ScaleRotInvSIFT, _abi, _native, synth
from tests.golden_util import (P_MAIN, P_OCT, assert_keypoints_equal, assert_matches_equal, desc_close, frame,
                               load, params_of, tie_permutation)

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def test_device_atan2_bitexact():
    z = load("atan2.npz")
    out = _native.debug_atan2(z["y"], z["x"])
    assert np.array_equal(bits(out), bits(z["out"]))


@pytest.mark.parametrize("H,W,pp", [(120, 160, P_MAIN), (97, 131, P_MAIN), (120, 160, {}),
                                    (64, 64, dict(P_MAIN, gaussian_size=5, sigma=2.5)),
                                    (33, 70, dict(P_MAIN, gaussian_size=3, ksize=5))])
def test_harris_R_median_bitexact_vs_oracle(H, W, pp):
    img = synth.make_frame(H, W, 17, 1)
    p = _abi.params_from_dict(pp, _abi.SFM_MODE_SCALEROT)
    R, med, ncand = _native.debug_harris(img, p)
    Ro = O.harris_response(img, pp)
    assert np.array_equal(bits(R), bits(Ro))
    assert np.float32(med) == O.median(Ro)
    _, _, _, dbg = O.detect(img, 10 ** 7, 0, pp, debug=True)
    assert ncand == dbg["n_candidates"]


DETECT_CASES = [
    (120, 160, 7, 0, 300, 18, P_MAIN),
    (120, 160, 7, 0, 300, 16, {}),
    (97, 131, 3, 2, 200, 9, P_MAIN),
    (96, 128, 4, 0, 1000, 4, dict(P_MAIN, ksize=5, alpha=0.04)),
    (64, 64, 5, 0, 50, 3, dict(P_MAIN, gaussian_size=5, sigma=2.5)),
    (30, 41, 6, 0, 100, 18, P_MAIN),
]


@pytest.mark.parametrize("i", range(len(DETECT_CASES)))
def test_naive_detect_vs_golden(i):
    z = load("detect.npz")
    H, W, seed, idx, k, fw, pp = DETECT_CASES[i]
    img = frame(H, W, seed, idx, z[f"c{i}_sha"])
    ns = NaiveSIFT(img, dict(pp, num_interest_points=k, feature_width=fw))
    x, y = ns.detect_keypoints()
    assert x.dtype == np.int64 and y.dtype == np.int64
    assert_keypoints_equal(z[f"c{i}_x"], z[f"c{i}_y"], x, y, z[f"c{i}_c"], ns.confidences)


def test_descriptors_vs_golden_all_widths():
    z = load("descriptors.npz")
    for i in range(int(z["ncases"])):
        H, W, seed, idx, fw, rotate = (int(v) for v in z[f"c{i}_meta"])
        img = frame(H, W, seed, idx, z[f"c{i}_sha"])
        pp = dict(P_MAIN, num_interest_points=120, feature_width=fw)
        if rotate:
            obj = ScaleRotInvSIFT(img, dict(pp, pyramid_level=1))
            x, y = obj.detect_keypoints()
            d = obj.extract_descriptors()
        else:
            obj = NaiveSIFT(img, pp)
            x, y = obj.detect_keypoints()
            d = obj.extract_descriptors()
        assert np.array_equal(x, z[f"c{i}_x"]) and np.array_equal(y, z[f"c{i}_y"]), (fw, rotate)
        assert desc_close(z[f"c{i}_d"], d), (fw, rotate)
        od = O.descriptors(img, x, y, fw, bool(rotate))
        assert np.array_equal(bits(d), bits(od)), (fw, rotate)


@pytest.mark.parametrize("fw", [24, 32, 48])
@pytest.mark.parametrize("rotate", [True, False])
def test_wide_feature_width_describe_fallback_vs_oracle(fw, rotate):
    """Feature widths above the quad kernel's limit (22) run k_describe, one wavefront per
    keypoint (describe.hip): its descriptors are bit-identical to the oracle's
    (ScaleRotInvSIFT.py:33-87 / NaiveSIFT.py:122-173 at windows of 24-48 px, where the 4 x 4
    cells cover only the window's top-left 16 x 16)."""
    img = synth.make_frame(160, 224, 31, fw)
    pp = dict(P_MAIN, num_interest_points=150, feature_width=fw)
    if rotate:
        obj = ScaleRotInvSIFT(img, dict(pp, pyramid_level=1))
    else:
        obj = NaiveSIFT(img, pp)
    x, y = obj.detect_keypoints()
    d = obj.extract_descriptors()
    assert len(x) > 20
    od = O.descriptors(img, x, y, fw, rotate)
    assert np.array_equal(bits(d), bits(od)), (fw, rotate)


EXTRACT_FIXTURES = ["extract_small_scalerot.npz", "extract_small_pmain.npz", "extract_small_naive.npz",
                    "extract_small_defaults.npz", "extract_c1_640x480_pmain.npz", "extract_c2_1080p_poct.npz"]


@pytest.mark.parametrize("name", EXTRACT_FIXTURES)
def test_extract_and_match_vs_golden_and_oracle(name):
    z = load(name)
    H, W, seed, nframes, stride = (int(v) for v in z["meta"])
    pp = params_of(z)
    naive = str(z["mode"]) == "naive"
    descs = []
    for f in range(nframes):
        img = frame(H, W, seed, f, z[f"f{f}_sha"])
        if naive:
            obj = NaiveSIFT(img, pp)
            X, Y = obj.detect_keypoints()
            D = obj.extract_descriptors()
        else:
            obj = ScaleRotInvSIFT(img, pp)
            X, Y = obj.detect_keypoints()
            D = obj.extract_descriptors()
        assert D.dtype == np.float32 and D.shape == (len(X), 128)
        perm = tie_permutation(z[f"f{f}_X"], z[f"f{f}_Y"], X, Y, obj.confidences)
        assert desc_close(z[f"f{f}_D"], D[perm][::stride])
        OX, OY, OD, _, OC = O.extract(img, pp, mode=1 if naive else 0, with_conf=True)
        assert np.array_equal(X, OX) and np.array_equal(Y, OY)
        assert np.array_equal(bits(obj.confidences), bits(OC))
        assert np.array_equal(bits(D), bits(OD))
        descs.append(D)
    if "matches" in z.files:
        ratio = float(z["ratio"])
        m, c = NNRatioFeatureMatcher(ratio).match_features_ratio_test(descs[0], descs[1])
        om, oc = O.match(descs[0], descs[1], ratio)
        assert_matches_equal(om, oc, m, c)
        a = set(map(tuple, z["matches"].tolist()))
        b = set(map(tuple, m.tolist()))
        assert a == b, (len(a), len(b), len(a ^ b))  # bit-identical pairs (north_star)


@pytest.mark.parametrize("name", ["extract_small_pmain_stablehist.npz", "extract_small_scalerot_stablehist.npz"])
def test_descriptors_vs_reference_stable_histogram_no_escape(name):
    """Against the reference run with a stable np.histogram sort (its tie order = ours): every
    descriptor element within 5e-7 absolute, no near-empty-bin escape."""
    z = load(name)
    H, W, seed, nframes, stride = (int(v) for v in z["meta"])
    pp = params_of(z)
    for f in range(nframes):
        img = frame(H, W, seed, f, z[f"f{f}_sha"])
        obj = ScaleRotInvSIFT(img, pp)
        X, Y = obj.detect_keypoints()
        D = obj.extract_descriptors()
        perm = tie_permutation(z[f"f{f}_X"], z[f"f{f}_Y"], X, Y, obj.confidences)
        ref = z[f"f{f}_D"]
        assert desc_close(ref, D[perm][::stride], rtol=0.0, atol=5e-7, max_escapes=0), \
            float(np.abs(ref - D[perm][::stride]).max())


def test_matcher_vs_golden_tables():
    z = load("match.npz")
    for i in range(int(z["ncases"])):
        n1, s1, n2, s2, jit = (int(v) for v in z[f"c{i}_meta"])
        a, ha = synth.make_descriptor_table(n1, s1)
        b, _ = synth.make_descriptor_table(n2, s2, dup_of=ha, jitter=jit)
        m, c = NNRatioFeatureMatcher(float(z[f"c{i}_ratio"])).match_features_ratio_test(a, b)
        if len(z[f"c{i}_c"]) == 0:
            assert m.shape == (0,)
        else:
            assert_matches_equal(z[f"c{i}_m"], z[f"c{i}_c"], m, c)


@pytest.mark.parametrize("n1,n2,ratio", [(1, 2, 0.8), (5, 700, 0.9), (333, 65, 0.7), (2500, 2400, 0.85),
                                         (64, 64, 1.0)])
def test_matcher_vs_oracle_sizes(n1, n2, ratio):
    a, ha = synth.make_descriptor_table(n1, 100 + n1)
    b, _ = synth.make_descriptor_table(n2, 200 + n2, dup_of=ha, jitter=2)
    m, c = NNRatioFeatureMatcher(ratio).match_features_ratio_test(a, b)
    om, oc = O.match(a, b, ratio)
    if len(oc) == 0:
        assert m.shape == (0,)
    else:
        assert_matches_equal(om, oc, m, c)


@pytest.mark.parametrize("n1,n2,jit,ratio", [(10, 700, 0, 0.9), (10, 700, 1, 0.9), (40, 900, 0, 1.0),
                                             (300, 300, 0, 0.8), (4, 1500, 0, 0.9), (4, 1500, 1, 1.0),
                                             (200, 3000, 0, 0.9)])
def test_matcher_duplicate_targets_overflow_path(n1, n2, jit, ratio):
    """Runs of identical / near-identical targets widen the prefilter window past the
    per-row candidate list (128) and exercise the exact full-row overflow kernel (n2 / n1
    duplicates of each source row: 375 at (4, 1500))."""
    a, ha = synth.make_descriptor_table(n1, 7 + n1)
    b, _ = synth.make_descriptor_table(n2, 9 + n2, dup_of=ha, jitter=jit)
    q, _ = synth.make_descriptor_table(n1, 11 + n1, dup_of=ha, jitter=2)
    for qq in (a, q):
        m, c = NNRatioFeatureMatcher(ratio).match_features_ratio_test(qq, b)
        om, oc = O.match(qq, b, ratio)
        if len(oc) == 0:
            assert m.shape == (0,)
        else:
            assert_matches_equal(om, oc, m, c)


def test_matcher_index_error_and_empty():
    a, _ = synth.make_descriptor_table(4, 1)
    with pytest.raises(IndexError):
        NNRatioFeatureMatcher().match_features_ratio_test(a, a[:1])
    # identical sets: every nearest distance is 0 with a non-zero second -> nndr 0
    m, c = NNRatioFeatureMatcher(0.5).match_features_ratio_test(a, a)
    assert np.array_equal(np.sort(m[:, 0]), np.arange(4)) and np.all(c == 0)


def test_ragged_single_keypoint_level_mirrors_reference():
    # a level that yields exactly one keypoint is extended element-wise by the reference
    # (ScaleRotInvSIFT.py:103); numpy 2 then refuses the inhomogeneous list
    img = synth.make_frame(64, 64, 3, 0)
    pp = dict(P_OCT, num_interest_points=8, pyramid_level=2)
    X, Y, D, lc = O.extract(img, pp)
    if 1 in lc.tolist() and lc.sum() > 1:
        with pytest.raises(ValueError):
            ScaleRotInvSIFT(img, pp)
    else:
        obj = ScaleRotInvSIFT(img, pp)
        assert np.array_equal(obj.detect_keypoints()[0], X)


def test_empty_outputs_like_reference():
    img = np.full((40, 40), 0.5, np.float32)  # flat: only R == 0 candidates
    obj = ScaleRotInvSIFT(img, dict(P_OCT, num_interest_points=0))
    X, Y = obj.detect_keypoints()
    assert X.shape == (0,) and X.dtype == np.float64
    assert obj.extract_descriptors().shape == (0,)


def test_flat_image_ties_match_oracle():
    img = np.full((48, 50), 0.25, np.float32)
    pp = dict(P_MAIN, num_interest_points=40, feature_width=4)
    ns = NaiveSIFT(img, pp)
    x, y = ns.detect_keypoints()
    ox, oy, oc = O.detect(img, 40, 4, pp)
    assert np.array_equal(x, ox) and np.array_equal(y, oy)


def test_batch_api_u8_and_f32_agree_with_oracle():
    torch = pytest.importorskip("torch")
    from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, consecutive_pairs
    B, H, W = 4, 135, 240
    u8 = synth.make_batch_u8(B, H, W, seed=77)
    pp = dict(P_OCT, num_interest_points=400)
    ex = BatchExtractor(pp)
    t_u8 = torch.from_numpy(u8).cuda()
    t_f32 = torch.from_numpy(synth.u8_to_gray(u8)).cuda()
    s1 = ex.extract(t_u8)
    s2 = ex.extract(t_f32)
    torch.cuda.synchronize()
    for k in ("xy", "desc", "count"):
        assert torch.equal(getattr(s1, k), getattr(s2, k))
    pairs = torch.from_numpy(consecutive_pairs(B)).cuda()
    mm, mc, nm = BatchMatcher(0.85).match(s1, pairs)
    torch.cuda.synchronize()
    counts = s1.count.cpu().numpy()
    xy = s1.xy.cpu().numpy()
    desc = s1.desc.cpu().numpy()
    for b in range(B):
        X, Y, D, _ = O.extract(synth.u8_to_gray(u8[b]), pp)
        n = counts[b]
        assert n == len(X)
        assert np.array_equal(xy[b, :n, 0], X) and np.array_equal(xy[b, :n, 1], Y)
        assert np.array_equal(bits(desc[b, :n]), bits(D))
    for p in range(B - 1):
        i, j = p, p + 1
        om, oc = O.match(desc[i, :counts[i]], desc[j, :counts[j]], 0.85)
        k = int(nm[p])
        assert_matches_equal(om, oc, mm[p, :k].cpu().numpy(), mc[p, :k].cpu().numpy())


def test_1080p_batch_consistency_and_golden():
    """Full BASELINE size: every copy of the golden 1080p frames in one batch gives the
    golden keypoints (batch independence + parity at the metric's configuration)."""
    torch = pytest.importorskip("torch")
    from sfmfromscratch_amd.pipeline import BatchExtractor
    z = load("extract_c2_1080p_poct.npz")
    H, W, seed = (int(v) for v in z["meta"][:3])
    pp = params_of(z)
    frames = np.stack([synth.make_frame_u8(H, W, seed, f % 2) for f in range(6)])
    ex = BatchExtractor(pp)
    s = ex.extract(torch.from_numpy(frames).cuda())
    torch.cuda.synchronize()
    counts = s.count.cpu().numpy()
    xy = s.xy.cpu().numpy()
    desc = s.desc.cpu().numpy()
    for b in range(6):
        f = b % 2
        n = counts[b]
        if b < 2:
            OX, OY, OD, _, OC = O.extract(synth.u8_to_gray(frames[b]), pp, with_conf=True)
            assert n == len(OX)
            assert np.array_equal(xy[b, :n, 0], OX) and np.array_equal(xy[b, :n, 1], OY)
            assert np.array_equal(bits(desc[b, :n]), bits(OD))
            perm = tie_permutation(z[f"f{f}_X"], z[f"f{f}_Y"], OX, OY, OC)
            assert desc_close(z[f"f{f}_D"], desc[b, :n][perm][::8])
        assert np.array_equal(xy[b, :n], xy[f, :n])
        assert np.array_equal(bits(desc[b, :n]), bits(desc[f, :n]))


@pytest.mark.parametrize("gate,lane_streams,serial_lanes", [(False, "torch", []), (True, "torch", []),
                                                            (False, "context", [0]), (True, "context", [0, 1])])
def test_pipeline_batches_in_flight_match_serial(gate, lane_streams, serial_lanes):
    """pipeline.BatchPipeline (2 batches in flight on separate contexts/streams; with and
    without the lane gate, on torch pool streams or the contexts' own streams, lanes with
    and without the aux-stream overlap) gives the same slots and matches as one
    BatchExtractor/BatchMatcher run per batch."""
    torch = pytest.importorskip("torch")
    from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, BatchPipeline, consecutive_pairs
    B, H, W = 4, 270, 480
    pp = dict(P_OCT, num_interest_points=600)
    batches = [torch.from_numpy(synth.make_batch_u8(B, H, W, seed=300 + i)).cuda() for i in range(3)]
    pairs = torch.from_numpy(consecutive_pairs(B)).cuda()
    pipe = BatchPipeline(pp, 0.85, B, H, W, pairs, inflight=2, extra_slots=0, gate=gate, lane_streams=lane_streams,
                         serial_lanes=serial_lanes)
    assert (pipe.gate is not None) == gate
    lanes = [pipe.submit(f) for f in batches]
    pipe.join()
    torch.cuda.synchronize()
    ex = BatchExtractor(pp)
    m = BatchMatcher(0.85, ctx=ex.ctx)
    for i in (1, 2):  # lane 0 was reused by batch 2
        s = ex.extract(batches[i])
        mm, mc, nm = m.match(s, pairs)
        torch.cuda.synchronize()
        ln = lanes[i]
        assert ln is pipe.lanes[i % 2]
        assert torch.equal(s.count, ln["slots"].count)
        for b, n in enumerate(s.count.tolist()):  # rows past the count are stale in a reused lane
            assert torch.equal(s.xy[b, :n], ln["slots"].xy[b, :n])
            assert torch.equal(s.desc[b, :n], ln["slots"].desc[b, :n])
        assert torch.equal(nm, ln["mout"][2])
        for p in range(B - 1):
            k = int(nm[p])
            assert torch.equal(mm[p, :k], ln["mout"][0][p, :k]) and torch.equal(mc[p, :k], ln["mout"][1][p, :k])


def test_pipeline_fused_matcher_operands_1080p_with_halo_vs_oracle():
    """BatchPipeline's lanes extract with fused matcher operands (sfm_ctx_set_fused_prep: the
    descriptor kernel writes the split-f16 operands, norms and block maxima of every row, and
    the last level's launch the padding rows), so the match preps only the halo slot the hook
    filled.  At 1080p P-oct with the halo pair (B-1, B): keypoints, descriptors and every pair's
    matches equal the oracle's."""
    torch = pytest.importorskip("torch")
    from sfmfromscratch_amd import distributed as D
    from sfmfromscratch_amd.pipeline import BatchPipeline
    B, H, W = 4, 1080, 1920
    frames = [synth.make_frame(H, W, 77, i) for i in range(B)]
    pairs_np = D.local_consecutive_pairs(B, 0, 2)  # (0,1) .. (B-2,B-1), (B-1, B)
    pipe = BatchPipeline(P_OCT, 0.85, B, H, W, torch.from_numpy(pairs_np).cuda(), inflight=2, extra_slots=1)
    assert pipe.fused_prep and not pipe.batch_only_pairs

    def halo(slots, n):  # slot B := slot 0 (what a neighbour rank's first frame would be)
        slots.xy[n].copy_(slots.xy[0])
        slots.desc[n].copy_(slots.desc[0])
        slots.count[n:n + 1].copy_(slots.count[0:1])

    batch = torch.from_numpy(np.stack(frames)).cuda()
    for _ in range(2):  # both lanes
        ln = pipe.submit(batch, hook=halo)
    pipe.join()
    torch.cuda.synchronize()
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(B) as pool:
        ext = list(pool.map(lambda f: O.extract(f, P_OCT), frames))
    descs = [e[2] for e in ext] + [ext[0][2]]
    counts = ln["slots"].count.cpu().numpy()
    for i, (OX, OY, OD, _) in enumerate(ext):
        n = int(counts[i])
        assert n == len(OX)
        assert np.array_equal(bits(ln["slots"].desc[i, :n].cpu().numpy()), bits(OD))
    mm, mc, nm = (t.cpu().numpy() for t in ln["mout"])
    for p, (i, j) in enumerate(pairs_np):
        om, oc = O.match(descs[i], descs[j], 0.85)
        k = int(nm[p])
        assert k == len(oc), (i, j)
        assert_matches_equal(om, oc, mm[p, :k], mc[p, :k])


P_4K = dict(P_MAIN, num_interest_points=8000, pyramid_level=5, pyramid_scale_factor=2)


def test_4k_five_octaves_k8000_vs_oracle():
    """BASELINE configs[4] at full size: 4K frames, 5-level x2 pyramid, k = 8000
    (1600 per level).  Keypoints + descriptors bit-identical to the oracle, and the
    ~7-8k x 7-8k pair matched identically."""
    torch = pytest.importorskip("torch")
    from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, consecutive_pairs
    H, W = 2160, 3840
    u8 = synth.make_batch_u8(2, H, W, seed=4321)
    ex = BatchExtractor(P_4K)
    s = ex.extract(torch.from_numpy(u8).cuda())
    pairs = torch.from_numpy(consecutive_pairs(2)).cuda()
    mm, mc, nm = BatchMatcher(0.85, ctx=ex.ctx).match(s, pairs)
    torch.cuda.synchronize()
    counts = s.count.cpu().numpy()
    xy = s.xy.cpu().numpy()
    desc = s.desc.cpu().numpy()
    assert counts.min() > 5000, counts
    OX, OY, OD, _ = O.extract(synth.u8_to_gray(u8[0]), P_4K)
    n = counts[0]
    assert n == len(OX)
    assert np.array_equal(xy[0, :n, 0], OX) and np.array_equal(xy[0, :n, 1], OY)
    assert np.array_equal(bits(desc[0, :n]), bits(OD))
    om, oc = O.match(desc[0, :counts[0]], desc[1, :counts[1]], 0.85)
    k = int(nm[0])
    assert k > 1000
    assert_matches_equal(om, oc, mm[0, :k].cpu().numpy(), mc[0, :k].cpu().numpy())


def test_all_pairs_schedule_vs_oracle():
    """All-pairs matching (BASELINE configs[2] schedule) over one slot table: every
    upper-triangle pair equals the oracle's matcher on the same descriptors."""
    torch = pytest.importorskip("torch")
    from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, all_pairs
    B, H, W = 6, 270, 480
    pp = dict(P_OCT, num_interest_points=800)
    ex = BatchExtractor(pp)
    s = ex.extract(torch.from_numpy(synth.make_batch_u8(B, H, W, seed=91)).cuda())
    pairs_np = all_pairs(B)
    mm, mc, nm = BatchMatcher(0.85, ctx=ex.ctx).match(s, torch.from_numpy(pairs_np).cuda())
    torch.cuda.synchronize()
    counts = s.count.cpu().numpy()
    desc = s.desc.cpu().numpy()
    assert len(pairs_np) == B * (B - 1) // 2
    for p, (i, j) in enumerate(pairs_np):
        om, oc = O.match(desc[i, :counts[i]], desc[j, :counts[j]], 0.85)
        k = int(nm[p])
        assert_matches_equal(om, oc, mm[p, :k].cpu().numpy(), mc[p, :k].cpu().numpy())


def test_configs2_workload_1080p_all_pairs_vs_oracle():
    """BASELINE configs[2] at its own frame size and parameters: 10 x 1080p frames, the
    4-level octave pyramid with k = 2500, every one of the 45 pairs matched.  Keypoints and
    descriptors bit-equal to the oracle's, every pair's matches equal to the oracle's
    matcher on those descriptors (the C oracle runs on host threads)."""
    torch = pytest.importorskip("torch")
    from concurrent.futures import ThreadPoolExecutor

    from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, all_pairs
    B, H, W = 10, 1080, 1920
    u8 = synth.make_batch_u8(B, H, W, seed=1234)
    ex = BatchExtractor(P_OCT)
    s = ex.extract(torch.from_numpy(synth.u8_to_gray(u8)).cuda())
    pairs_np = all_pairs(B)
    mm, mc, nm = BatchMatcher(0.85, ctx=ex.ctx).match(s, torch.from_numpy(pairs_np).cuda())
    torch.cuda.synchronize()
    counts, xy, desc = s.count.cpu().numpy(), s.xy.cpu().numpy(), s.desc.cpu().numpy()
    mm, mc, nm = mm.cpu().numpy(), mc.cpu().numpy(), nm.cpu().numpy()
    gray = synth.u8_to_gray(u8)
    with ThreadPoolExecutor(16) as pool:
        ext = list(pool.map(lambda i: O.extract(gray[i], P_OCT), range(B)))
        for i, (OX, OY, OD, _) in enumerate(ext):
            n = int(counts[i])
            assert n == len(OX) and n > 1500
            assert np.array_equal(xy[i, :n, 0], OX) and np.array_equal(xy[i, :n, 1], OY)
            assert np.array_equal(bits(desc[i, :n]), bits(OD))
        om = list(pool.map(lambda p: O.match(desc[p[0], :counts[p[0]]], desc[p[1], :counts[p[1]]], 0.85),
                           [tuple(p) for p in pairs_np]))
    for p in range(len(pairs_np)):
        k = int(nm[p])
        assert_matches_equal(om[p][0], om[p][1], mm[p, :k], mc[p, :k])


RAGGED_NS = [0, 1, 2, 127, 128, 129, 255, 256, 257, 300, 511, 513, 700, 64, 400, 5, 260, 768]


def ragged_match_case():
    """The ragged work-unit case of test_matcher_work_units_ragged_counts_many_pairs: its
    slot table (host copy), counts, pairs and the GPU matcher's outputs."""
    import torch
    from sfmfromscratch_amd.pipeline import BatchMatcher, SlotTable, all_pairs
    S, cap = 48, 768
    counts = [RAGGED_NS[i % len(RAGGED_NS)] for i in range(S)]
    base, hb = synth.make_descriptor_table(cap, 4242)
    slots = SlotTable(torch, S, cap, "cuda")
    host = np.zeros((S, cap, 128), np.float32)
    for i, n in enumerate(counts):
        if n:
            t, _ = synth.make_descriptor_table(n, 5000 + i, dup_of=hb[:n] if i % 3 else None, jitter=2)
            host[i, :n] = t
    slots.desc.copy_(torch.from_numpy(host))
    slots.count.copy_(torch.tensor(counts, dtype=torch.int32))
    pairs_np = all_pairs(S)
    mm, mc, nm = BatchMatcher(0.85).match(slots, torch.from_numpy(pairs_np).cuda())
    torch.cuda.synchronize()
    return host, counts, pairs_np, mm.cpu().numpy(), mc.cpu().numpy(), nm.cpu().numpy()


@pytest.mark.parametrize("stage", ["3", "1"])
def test_matcher_work_units_ragged_counts_many_pairs(stage, tmp_path):
    """The sweep's work units (k_match_units): ragged per-image counts around the query blocks
    of both sweep forms — 128 rows (the default half-CU form, SFMFEAT_MATCH_STAGE 3: 0-6 blocks
    per pair) and 256 rows (the one-CU form, SFMFEAT_MATCH_STAGE=1, run in a child process since
    the library reads the switch once): counts 0, 1, 127, 128, 129, 255, 256, 257, 511, 513, ...,
    so some pairs have no block, and 1,128 pairs (the unit scan's second 1,024-pair chunk); every
    pair equals the oracle (n2 < 2: the reference's IndexError, nmatch -1)."""
    pytest.importorskip("torch")
    if stage == "3":
        host, counts, pairs_np, mm, mc, nm = ragged_match_case()
    else:
        import os
        import subprocess
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        path = str(tmp_path / "ragged.npz")
        code = ("import sys, numpy as np; sys.path.insert(0, %r); from tests import test_gpu_parity as t; "
                "h, c, p, mm, mc, nm = t.ragged_match_case(); np.savez(%r, host=h, counts=np.array(c), pairs=p, "
                "mm=mm, mc=mc, nm=nm)" % (root, path))
        r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, SFMFEAT_MATCH_STAGE=stage), cwd=root,
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        z = np.load(path)
        host, counts, pairs_np, mm, mc, nm = (z["host"], [int(v) for v in z["counts"]], z["pairs"], z["mm"],
                                              z["mc"], z["nm"])
    assert len(pairs_np) > 1024

    def ref(pq):
        i, j = pq
        try:
            return O.match(host[i, :counts[i]], host[j, :counts[j]], 0.85)
        except IndexError:
            return None

    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(16) as pool:
        refs = list(pool.map(ref, [tuple(p) for p in pairs_np]))
    for p, (i, j) in enumerate(pairs_np):
        if refs[p] is None:
            assert nm[p] == -1, (i, j, counts[i], counts[j], nm[p])
            continue
        om, oc = refs[p]
        k = int(nm[p])
        assert k == len(oc), (i, j, counts[i], counts[j], k, len(oc))
        if k:
            assert_matches_equal(om, oc, mm[p, :k], mc[p, :k])


def test_prep_ranges_then_prepped_match_equal_full_match():
    """sfm_match_prep_dev over slot ranges + sfm_match_pairs_prepped_dev (the configs[3]
    chunked path) give exactly sfm_match_pairs_dev's results; prepped matching on a fresh
    context is refused (SFM_ESTATE -> RuntimeError)."""
    torch = pytest.importorskip("torch")
    from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, all_pairs
    B, H, W = 6, 270, 480
    ex = BatchExtractor(dict(P_OCT, num_interest_points=800))
    s = ex.extract(torch.from_numpy(synth.make_batch_u8(B, H, W, seed=93)).cuda())
    pairs = torch.from_numpy(all_pairs(B)).cuda()
    ref = BatchMatcher(0.85).match(s, pairs)
    m = BatchMatcher(0.85)
    with pytest.raises(RuntimeError):
        m.match(s, pairs, prepped=True)
    m.prep(s, 0, 2)
    m.prep(s, 2, 4)
    got = m.match(s, pairs, prepped=True)
    torch.cuda.synchronize()
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
    # a table other than the one last prepped on this context is refused too
    s2 = ex.extract(torch.from_numpy(synth.make_batch_u8(B, H, W, seed=94)).cuda())
    with pytest.raises(RuntimeError):
        m.match(s2, pairs, prepped=True)


def test_match_workspace_budget_sub_launches_equal_one_launch(monkeypatch):
    """A call with more pairs than the per-pair workspace budget runs as consecutive
    sub-launches (bounded allocation); the results equal one launch's."""
    torch = pytest.importorskip("torch")
    from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, all_pairs
    B, H, W = 6, 270, 480
    ex = BatchExtractor(dict(P_OCT, num_interest_points=800))
    s = ex.extract(torch.from_numpy(synth.make_batch_u8(B, H, W, seed=95)).cuda())
    pairs = torch.from_numpy(all_pairs(B)).cuda()
    ref = BatchMatcher(0.85).match(s, pairs)
    monkeypatch.setenv("SFMFEAT_MATCH_BUDGET_MB", "1")  # ~2 pairs per sub-launch at cap 800
    small = BatchMatcher(0.85)
    got = small.match(s, pairs)
    small.prep(s)
    got2 = small.match(s, pairs, prepped=True)
    torch.cuda.synchronize()
    for a, b, c in zip(ref, got, got2):
        assert torch.equal(a, b) and torch.equal(a, c)



def test_seven_levels_fused_pyramid_then_down2x3_vs_oracle():
    """L = 7 at a size that is a multiple of 64: levels 1-3 come from the level-0 Harris launch
    and levels 4-6 from a k_down2x3 pass after it.  That pass must not zero the histograms and
    counters level 0's Harris has already written (the fill launches did).  Keypoints and
    descriptors of both frames bit-identical to the oracle."""
    torch = pytest.importorskip("torch")
    from sfmfromscratch_amd.pipeline import BatchExtractor
    H, W = 512, 1024
    pp = dict(P_OCT, num_interest_points=1400, pyramid_level=7)
    u8 = synth.make_batch_u8(2, H, W, seed=77)
    s = BatchExtractor(pp).extract(torch.from_numpy(u8).cuda())
    torch.cuda.synchronize()
    counts, xy, desc = s.count.cpu().numpy(), s.xy.cpu().numpy(), s.desc.cpu().numpy()
    for i in range(2):
        OX, OY, OD, _ = O.extract(synth.u8_to_gray(u8[i]), pp)
        n = counts[i]
        assert n == len(OX) and n > 500
        assert np.array_equal(xy[i, :n, 0], OX) and np.array_equal(xy[i, :n, 1], OY)
        assert np.array_equal(bits(desc[i, :n]), bits(OD))
