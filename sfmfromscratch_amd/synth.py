"""Deterministic synthetic textured frames (SURVEY.md §8d 'Synthetic inputs').

Frames are built with integer arithmetic only (numpy PCG64 integer draws, int32/uint32
ops), so the same (seed, index, size) gives bit-identical uint8 frames on every host —
the golden fixtures store only the generator arguments plus a SHA-256 of each frame.

Scene: ~200 integer cone blobs and ~100 rectangles per 1080p-sized area over a gentle
integer ramp, plus uniform noise of +-3 levels from a per-frame integer hash, folded (not clipped)
into [0, 255] so that no flat saturated regions appear.  Frame i
shows the scene translated by (+3*i, +2*i) pixels with a fresh noise seed, so
consecutive frames have true correspondences (the reference's consecutive-pair
schedule, Runner.py:183).  The float image is value/255 in float32, mirroring
Runner.py:507-509,521.
"""
from __future__ import annotations

import hashlib

import numpy as np

SHIFT_X = 3
SHIFT_Y = 2


def _hash_noise(H: int, W: int, seed: int) -> np.ndarray:
    """Uniform integers in [-3, 3] from a 32-bit integer hash of (x, y, seed)."""
    y = np.arange(H, dtype=np.uint32)[:, None]
    x = np.arange(W, dtype=np.uint32)[None, :]
    with np.errstate(over="ignore"):
        h = x * np.uint32(0x9E3779B1) + y * np.uint32(0x85EBCA77) + np.uint32(seed * 0x27D4EB2F & 0xFFFFFFFF)
        h ^= h >> np.uint32(15)
        h *= np.uint32(0x2C1B3C6D)
        h ^= h >> np.uint32(12)
        h *= np.uint32(0x297A2D39)
        h ^= h >> np.uint32(15)
    return (h % np.uint32(7)).astype(np.int32) - 3


def make_frame_u8(H: int, W: int, seed: int = 1234, index: int = 0) -> np.ndarray:
    """Frame `index` of the synthetic sequence `seed`, as an H x W uint8 array."""
    rng = np.random.default_rng(seed)
    tx, ty = SHIFT_X * index, SHIFT_Y * index
    area = (W + 64) * (H + 64)
    nb = max(24, int(200 * area // (1920 * 1080)))
    nr = max(12, int(100 * area // (1920 * 1080)))
    span_w, span_h = W + 64 + SHIFT_X * 64, H + 64 + SHIFT_Y * 64
    yy = np.arange(H, dtype=np.int32)[:, None] + ty
    xx = np.arange(W, dtype=np.int32)[None, :] + tx
    img = 90 + ((xx * 3 + yy * 5) // 97) % 37  # gentle ramp, int32
    img = np.broadcast_to(img, (H, W)).astype(np.int32)
    cx = rng.integers(-32, span_w, nb)
    cy = rng.integers(-32, span_h, nb)
    rad = rng.integers(6, 60, nb)
    amp = rng.integers(-90, 91, nb)
    for i in range(nb):
        r = int(rad[i])
        x0, x1 = max(int(cx[i]) - r - tx, 0), min(int(cx[i]) + r + 1 - tx, W)
        y0, y1 = max(int(cy[i]) - r - ty, 0), min(int(cy[i]) + r + 1 - ty, H)
        if x0 >= x1 or y0 >= y1:
            continue
        dx = np.arange(x0, x1, dtype=np.int32)[None, :] + tx - int(cx[i])
        dy = np.arange(y0, y1, dtype=np.int32)[:, None] + ty - int(cy[i])
        w = np.maximum(0, r * r - (dx * dx + dy * dy))
        img[y0:y1, x0:x1] += (int(amp[i]) * w) // (r * r)
    rx = rng.integers(-32, span_w, nr)
    ry = rng.integers(-32, span_h, nr)
    rw = rng.integers(8, 120, nr)
    rh = rng.integers(8, 120, nr)
    rl = rng.integers(-60, 61, nr)
    for i in range(nr):
        x0, x1 = max(int(rx[i]) - tx, 0), min(int(rx[i] + rw[i]) - tx, W)
        y0, y1 = max(int(ry[i]) - ty, 0), min(int(ry[i] + rh[i]) - ty, H)
        if x0 < x1 and y0 < y1:
            img[y0:y1, x0:x1] += int(rl[i])
    img += _hash_noise(H, W, seed * 1000 + index)
    # fold (triangle wave) into [0, 255] instead of clipping: clipping would create flat
    # saturated regions whose R == 0 ties the reference orders arbitrarily
    img = np.mod(img, 510)
    img = np.where(img > 255, 510 - img, img)
    return img.astype(np.uint8)


def make_frame_rgb_u8(H: int, W: int, seed: int = 1234, index: int = 0) -> np.ndarray:
    """Frame `index` as an H x W x 3 uint8 RGB array (the decoded JPEG the reference's
    _load_image reads, Runner.py:551-563): one scene per channel (seeds seed, seed+1,
    seed+2), so the channels are correlated in motion but differ in content."""
    return np.stack([make_frame_u8(H, W, seed + c, index) for c in range(3)], axis=-1)


def u8_to_gray(u8: np.ndarray) -> np.ndarray:
    """value / 255 in float32 (Runner.py:521 `_im2single`-style conversion)."""
    return u8.astype(np.float32) / np.float32(255.0)


def make_frame(H: int, W: int, seed: int = 1234, index: int = 0) -> np.ndarray:
    return u8_to_gray(make_frame_u8(H, W, seed, index))


def make_batch_u8(B: int, H: int, W: int, seed: int = 1234) -> np.ndarray:
    return np.stack([make_frame_u8(H, W, seed, i) for i in range(B)])


def frame_sha256(u8: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(u8).tobytes()).hexdigest()


def make_descriptor_table(n: int, seed: int, dup_of: np.ndarray | None = None,
                          jitter: int = 0) -> np.ndarray:
    """Deterministic RootSIFT-like (n, 128) float32 table from integer histograms.

    Every float op is exactly rounded (int->f32, division, sqrt), so tables are
    bit-identical on every host.  With `dup_of` (an integer histogram table) rows are
    perturbed copies of it (near duplicates -> interesting ratio-test cases).
    """
    rng = np.random.default_rng(seed)
    if dup_of is None:
        h = rng.integers(0, 40, (n, 128)) * (rng.integers(0, 4, (n, 128)) == 0)
        h = h.astype(np.int64)
    else:
        src = rng.integers(0, dup_of.shape[0], n)
        h = dup_of[src].copy() + rng.integers(-jitter, jitter + 1, (n, 128))
        h = np.maximum(h, 0)
    h[h.sum(axis=1) == 0, 0] = 1
    s = h.sum(axis=1, keepdims=True).astype(np.float32)
    return np.sqrt(h.astype(np.float32) / s), h
