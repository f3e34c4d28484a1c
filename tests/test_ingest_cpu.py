"""CPU: the ingest restatement (oracle/ingest.py) against the golden vectors made by the
reference's own _load_image / _PIL_resize / _rgb2gray (Runner.py:33-46, 467-563) and
against PIL itself (the reference's resize is PIL's BICUBIC, Pillow pinned 11.0.0)."""
from __future__ import annotations

import numpy as np
import pytest

from oracle import ingest as I
from sfmfromscratch_amd import synth
from tests.golden_util import load


def golden_cases():
    z = load("ingest.npz")
    for i in range(int(z["ncases"])):
        H, W, seed, idx = (int(v) for v in z[f"c{i}_meta"])
        yield i, z, H, W, seed, idx, float(z[f"c{i}_scale"])


@pytest.mark.parametrize("i", range(5))
def test_ingest_restatement_vs_reference_golden(i):
    z = load("ingest.npz")
    H, W, seed, idx = (int(v) for v in z[f"c{i}_meta"])
    rgb = synth.make_frame_rgb_u8(H, W, seed, idx)
    assert synth.frame_sha256(rgb) == str(z[f"c{i}_sha_in"])
    g = I.ingest(rgb, float(z[f"c{i}_scale"]))
    assert g.dtype == np.float32 and tuple(g.shape) == tuple(z[f"c{i}_shape"])
    if f"c{i}_gray" in z:
        assert np.array_equal(g.view(np.uint32), z[f"c{i}_gray"].view(np.uint32))
    assert synth.frame_sha256(g) == str(z[f"c{i}_sha_out"])


@pytest.mark.parametrize("H,W,s", [(37, 53, 0.5), (120, 91, 0.5), (64, 64, 0.25), (45, 77, 0.6), (30, 41, 1.7)])
def test_bicubic_restatement_vs_pil(H, W, s):
    Image = pytest.importorskip("PIL.Image")
    rgb = np.random.default_rng(H * W).integers(0, 256, (H, W, 3), dtype=np.uint8)
    H2, W2 = I.resize_dims(H, W, s)
    ref = np.asarray(Image.fromarray(rgb).resize((W2, H2)))
    assert np.array_equal(I.pil_bicubic_resize(rgb, H2, W2), ref)


def test_u8_float_roundtrip_is_exact():
    """_PIL_resize multiplies _load_image's u8/255 float32 by 255 and truncates to u8
    (Runner.py:541-545): exact for every value, so ingest may start from the u8 frame."""
    u = np.arange(256, dtype=np.uint8)
    f = u.astype(np.float64).astype(np.float32) / 255
    f *= 255
    assert np.array_equal(np.uint8(f), u)


def test_opaque_rgba_drops_alpha_translucent_rejected():
    """PIL resizes RGBA premultiplied: an opaque RGBA frame resizes to the same RGB as its
    RGB channels (so runner.drop_opaque_alpha is exact), a translucent one does not and is
    rejected (ValueError, the documented divergence)."""
    from PIL import Image

    from sfmfromscratch_amd.runner import drop_opaque_alpha
    rng = np.random.default_rng(7)
    a = rng.integers(0, 256, (37, 53, 4), dtype=np.uint8)
    a[..., 3] = 255
    via_rgba = np.asarray(Image.fromarray(a).resize((26, 18)))[..., :3]
    rgb = drop_opaque_alpha(a)
    assert rgb.shape == (37, 53, 3) and rgb.flags.c_contiguous
    assert np.array_equal(via_rgba, np.asarray(Image.fromarray(rgb).resize((26, 18))))
    a[0, 0, 3] = 254
    with pytest.raises(ValueError):
        drop_opaque_alpha(a)
    with pytest.raises(ValueError):
        drop_opaque_alpha(a[..., 0])
