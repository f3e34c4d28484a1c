"""GPU: device ingest (sfm_ingest_rgb*, ingest.hip) against the golden vectors made by the
reference's own _load_image / _PIL_resize / _rgb2gray (Runner.py:33-46), against PIL and
the oracle restatement on other sizes, and FeatureRunner end to end against the oracle.
Bar: bit-identical float32 gray frames."""
from __future__ import annotations

import numpy as np
import pytest

from oracle import ingest as I
from oracle import oracle as O
from sfmfromscratch_amd import _abi, _native, synth
from tests.golden_util import P_OCT, assert_matches_equal, load

pytestmark = pytest.mark.gpu


def ctx():
    return _native.context_for(_abi.params_from_dict({}, _abi.SFM_MODE_NAIVE))


@pytest.mark.parametrize("i", range(5))
def test_ingest_vs_reference_golden(i):
    z = load("ingest.npz")
    H, W, seed, idx = (int(v) for v in z[f"c{i}_meta"])
    rgb = synth.make_frame_rgb_u8(H, W, seed, idx)
    g = ctx().ingest_rgb(rgb, float(z[f"c{i}_scale"]))
    assert tuple(g.shape) == tuple(z[f"c{i}_shape"])
    if f"c{i}_gray" in z:
        assert np.array_equal(g.view(np.uint32), z[f"c{i}_gray"].view(np.uint32))
    assert synth.frame_sha256(g) == str(z[f"c{i}_sha_out"])


@pytest.mark.parametrize("H,W,s", [(37, 53, 0.5), (120, 91, 0.5), (64, 64, 0.25), (45, 77, 0.6), (30, 41, 1.7),
                                   (1080, 1920, 0.5)])
def test_ingest_vs_pil_and_oracle(H, W, s):
    Image = pytest.importorskip("PIL.Image")
    rgb = np.random.default_rng(H + W).integers(0, 256, (H, W, 3), dtype=np.uint8)
    H2, W2 = I.resize_dims(H, W, s)
    ref = I.rgb_to_gray(np.asarray(Image.fromarray(rgb).resize((W2, H2))))
    g = ctx().ingest_rgb(rgb, s)
    assert np.array_equal(g.view(np.uint32), ref.view(np.uint32))
    if H * W < 100000:
        assert np.array_equal(g.view(np.uint32), I.ingest(rgb, s).view(np.uint32))


def test_ingest_batch_dev_equals_host():
    torch = pytest.importorskip("torch")
    from sfmfromscratch_amd.pipeline import ingest_rgb
    frames = np.stack([synth.make_frame_rgb_u8(270, 481, 5, i) for i in range(3)])
    g = ingest_rgb(ctx(), torch.from_numpy(frames).cuda(), 0.5)
    torch.cuda.synchronize()
    got = g.cpu().numpy()
    for b in range(3):
        assert np.array_equal(got[b].view(np.uint32), I.ingest(frames[b], 0.5).view(np.uint32))


def test_feature_runner_end_to_end(tmp_path):
    """runner.FeatureRunner (Runner.py:22-73 mirror) on two PNG-encoded synthetic RGB
    frames == oracle ingest + extract + match."""
    Image = pytest.importorskip("PIL.Image")
    from sfmfromscratch_amd import ScaleRotInvSIFT
    from sfmfromscratch_amd.runner import FeatureRunner, convert_matches_to_coords
    paths = []
    frames = [synth.make_frame_rgb_u8(540, 960, 7, i) for i in range(2)]
    for i, f in enumerate(frames):
        p = str(tmp_path / f"{i + 1}.png")
        Image.fromarray(f).save(p)
        paths.append(p)
    pp = dict(P_OCT, num_interest_points=800)
    r = FeatureRunner(paths[0], paths[1], feature_extractor_class=ScaleRotInvSIFT, extractor_params=pp,
                      match_threshold=0.85)
    g = [I.ingest(f, 0.5) for f in frames]
    assert np.array_equal(r._image1_bw, g[0]) and np.array_equal(r._image2_bw, g[1])
    X1, Y1, D1, _ = O.extract(g[0], pp)
    X2, Y2, D2, _ = O.extract(g[1], pp)
    assert np.array_equal(r.X1, X1) and np.array_equal(r.Y2, Y2)
    om, oc = O.match(D1, D2, 0.85)
    assert_matches_equal(om, oc, r.matches, r.confidences)
    p1, p2 = convert_matches_to_coords(r.matches, r.X1, r.Y1, r.X2, r.Y2)
    assert p1.shape == (len(r.matches), 2) and np.array_equal(p1[:, 0], r.X1[r.matches[:, 0]])
