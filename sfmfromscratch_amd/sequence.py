"""Stage 1 of SFMRunner (Runner.py:176-191) on the device: every frame extracted once into a
resident descriptor table, then the pair schedule matched from it.

The reference runs `corner_detect_and_matching_process(i1, i1 + 1)` for every
consecutive pair on an 8-thread pool (Runner.py:183-191, 336-355); each task builds a
FeatureRunner, so every interior frame is decoded, resized and extracted twice, and the
ThreadPool's Python work serialises on the GIL.  Here:

* `FeatureCache` decodes each frame once on the host, ingests it on the device
  (PIL BICUBIC x scale + _rgb2gray, ingest.hip) and extracts it once, in batches, into
  one slot table (xy, desc, count) that stays resident — the descriptor-table cache;
* `match_schedule` matches any pair schedule (the reference's consecutive pairs, all
  pairs, or a sliding window) from that table in large batched launches;
* `stage1` mirrors what SFMRunner.perform leaves in `all_matches` after its thread pool:
  `all_matches[i1][i2] = Matches(matches, confidences, p1, p2, K1, K2)` and the swapped
  entry `[i2][i1]` (Runner.py:354-355), with p1 / p2 from _convert_matches_to_coords
  (Runner.py:423-434, first 2,500 matches).  With `ransac=True` the RANSAC inlier
  filter the reference applies to every pair but (1, 2) (Runner.py:349-351) runs on the
  device for all pairs at once (pose.find_inliers_batch); otherwise p1 /
  p2 are the pre-RANSAC correspondences.  EXIF intrinsics (CameraPose.construct_K) are
  out of scope: K is the caller's `single_K` (or None).

Feature tables and matches are saved / loaded as .npz (the
reference's own output format is np.savez, Runner.py:357-359).

Semantics are the batch path's: a pyramid level that yields exactly one keypoint is
stored as one keypoint (the drop-in ScaleRotInvSIFT reproduces the reference's ragged
`extend` of such a level instead, ScaleRotInvSIFT.py:103).
"""
from __future__ import annotations

import numpy as np

from .runner import convert_matches_to_coords, drop_opaque_alpha, load_image_u8


class Matches:
    """Runner.Matches (Runner.py:118-125)."""

    def __init__(self, matches, confidence, p1, p2, K1, K2):
        self.matches = matches
        self.confidence = confidence
        self.p1 = p1
        self.p2 = p2
        self.K1 = K1
        self.K2 = K2


def pair_schedule(n: int, schedule="consecutive") -> np.ndarray:
    """Frame-index pairs (i, j), i < j: "consecutive" (Runner.py:183), "all", or an int w
    for every pair with j - i <= w."""
    if schedule == "consecutive":
        schedule = 1
    if schedule == "all":
        i, j = np.triu_indices(n, k=1)
    else:
        w = int(schedule)
        if w < 1:
            raise ValueError("window must be >= 1")
        i, j = np.triu_indices(n, k=1)
        keep = (j - i) <= w
        i, j = i[keep], j[keep]
    return np.stack([i, j], axis=1).astype(np.int32)


class FeatureCache:
    """Descriptor-table cache: frames extracted once, resident on the device.

    `frames` are decoded frames — [H, W, 3] uint8 RGB (ingested on the device with the
    reference's resize + gray conversion, Runner.py:33-46) or [H, W] float32 gray images
    (used as given) — or image paths (decoded with PIL on the host)."""

    def __init__(self, frames, extractor_params: dict | None = None, scale_factor: float = 0.5,
                 batch: int = 32, device: int = 0):
        import torch
        from .pipeline import BatchExtractor, SlotTable, ingest_rgb
        self.torch = torch
        dev = torch.device("cuda", device)
        self.extractor = BatchExtractor(extractor_params, device=device)
        self.cap = self.extractor.cap
        n = len(frames)
        self.n = n
        self.slots = SlotTable(torch, max(n, 1), self.cap, dev)
        self.shapes = [None] * n
        loaded = []
        for f in frames:
            if isinstance(f, str):
                # a 2-D gray file fails in the reference's _rgb2gray (Runner.py:478), so it
                # fails here instead of being extracted at the wrong scale; opaque RGBA
                # files work there and here
                a = drop_opaque_alpha(load_image_u8(f), f)
            else:
                a = np.asarray(f)
                if a.ndim == 3:
                    a = drop_opaque_alpha(a)
                if a.ndim == 2 and a.dtype != np.float32:
                    raise ValueError("gray frames must be float32 [H, W] in [0, 1] (the extractor's input)")
            loaded.append(a)
        # group frames of one kind and size into batches (one launch sequence per batch)
        groups: dict = {}
        for i, a in enumerate(loaded):
            key = (a.dtype.str, a.shape)
            groups.setdefault(key, []).append(i)
        for (_, shape), idx in groups.items():
            for b0 in range(0, len(idx), batch):
                chunk = idx[b0:b0 + batch]
                arr = np.stack([loaded[i] for i in chunk])
                t = torch.from_numpy(arr).to(dev)
                if t.dim() == 4:  # decoded RGB -> device ingest
                    if t.dtype != torch.uint8 or t.shape[3] != 3:
                        raise ValueError("RGB frames must be [H, W, 3] uint8")
                    gray = ingest_rgb(self.extractor.ctx, t, scale_factor)
                elif t.dim() == 3:
                    gray = t
                else:
                    raise ValueError("frames must be [H, W, 3] uint8 RGB or [H, W] gray")
                sel = torch.tensor(chunk, device=dev)
                tmp = self.extractor.extract(gray.contiguous())
                self.slots.xy.index_copy_(0, sel, tmp.xy)
                self.slots.desc.index_copy_(0, sel, tmp.desc)
                self.slots.count.index_copy_(0, sel, tmp.count)
                for i in chunk:
                    self.shapes[i] = tuple(gray.shape[1:])
        torch.cuda.synchronize(dev)

    # host views of one frame's features (the reference's X, Y, descriptors)
    def keypoints(self, i: int):
        n = int(self.slots.count[i].item())
        xy = self.slots.xy[i, :n].cpu().numpy().astype(np.int64)
        return xy[:, 0], xy[:, 1]

    def descriptors(self, i: int) -> np.ndarray:
        n = int(self.slots.count[i].item())
        return self.slots.desc[i, :n].cpu().numpy()

    def save(self, path: str) -> None:
        """Features of every frame as .npz: counts, offsets, X, Y (int64), desc (float32)."""
        counts = self.slots.count.cpu().numpy().astype(np.int64)[: self.n]
        xy = self.slots.xy.cpu().numpy()
        desc = self.slots.desc.cpu().numpy()
        save_features(path, [xy[i, :counts[i], 0] for i in range(self.n)],
                      [xy[i, :counts[i], 1] for i in range(self.n)],
                      [desc[i, :counts[i]] for i in range(self.n)])


def save_features(path: str, X: list, Y: list, D: list) -> None:
    """Per-frame keypoints + descriptors as one .npz (concatenated, with offsets)."""
    counts = np.array([len(x) for x in X], np.int64)
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    np.savez(path, format=np.array("sfmfeat-features-v1"), counts=counts, offsets=off,
             X=np.concatenate([np.asarray(x, np.int64) for x in X]) if len(X) else np.zeros(0, np.int64),
             Y=np.concatenate([np.asarray(y, np.int64) for y in Y]) if len(Y) else np.zeros(0, np.int64),
             desc=np.concatenate([np.asarray(d, np.float32).reshape(-1, 128) for d in D]) if len(D)
             else np.zeros((0, 128), np.float32))


def load_features(path: str):
    """-> (X list, Y list, desc list) as written by save_features."""
    with np.load(path, allow_pickle=False) as z:
        if str(z["format"]) != "sfmfeat-features-v1":
            raise ValueError(f"{path}: not an sfmfeat feature file")
        off = z["offsets"]
        X, Y, D = z["X"], z["Y"], z["desc"]
        return ([X[off[i]:off[i + 1]] for i in range(len(off) - 1)],
                [Y[off[i]:off[i + 1]] for i in range(len(off) - 1)],
                [D[off[i]:off[i + 1]] for i in range(len(off) - 1)])


def save_matches(path: str, pairs: np.ndarray, results: list) -> None:
    """Per-pair (matches (k,2) int64, confidences (k,) float32) as one .npz."""
    counts = np.array([len(c) for _, c in results], np.int64)
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    m = [np.asarray(mm, np.int64).reshape(-1, 2) for mm, _ in results]
    c = [np.asarray(cc, np.float32).reshape(-1) for _, cc in results]
    np.savez(path, format=np.array("sfmfeat-matches-v1"), pairs=np.asarray(pairs, np.int32), offsets=off,
             matches=np.concatenate(m) if m else np.zeros((0, 2), np.int64),
             conf=np.concatenate(c) if c else np.zeros(0, np.float32))


def load_matches(path: str):
    """-> (pairs, [(matches, conf), ...]); empty pairs come back as the reference's
    float64 (0,) arrays (NNRatioFeatureMatcher.py:53-60)."""
    with np.load(path, allow_pickle=False) as z:
        if str(z["format"]) != "sfmfeat-matches-v1":
            raise ValueError(f"{path}: not an sfmfeat match file")
        off, m, c = z["offsets"], z["matches"], z["conf"]
        res = []
        for p in range(len(off) - 1):
            if off[p + 1] == off[p]:
                res.append((np.array([]), np.array([])))
            else:
                res.append((m[off[p]:off[p + 1]], c[off[p]:off[p + 1]]))
        return z["pairs"], res


def match_schedule(cache: FeatureCache, pairs: np.ndarray, ratio_threshold: float = 0.85, chunk: int = 4096):
    """Match every (i, j) of `pairs` from the resident table; returns per pair
    (matches (k,2) int64, confidences (k,) float32) exactly as
    NNRatioFeatureMatcher.match_features_ratio_test on the two frames' descriptors,
    including its float64 (0,) empty results.  Raises IndexError like the reference
    when a pair's second frame has fewer than 2 keypoints."""
    torch = cache.torch
    from .pipeline import BatchMatcher
    pairs = np.asarray(pairs, np.int32).reshape(-1, 2)
    dev = cache.slots.desc.device
    m = BatchMatcher(ratio_threshold, device=dev.index, ctx=cache.extractor.ctx)
    out = []
    for a in range(0, len(pairs), chunk):
        pt = torch.from_numpy(pairs[a:a + chunk]).to(dev)
        mm, cc, nm = m.match(cache.slots, pt)
        nm = nm.cpu().numpy()
        mm = mm.cpu().numpy()
        cc = cc.cpu().numpy()
        for p in range(len(pt)):
            k = int(nm[p])
            if k < 0:
                raise IndexError("index 1 is out of bounds (fewer than 2 target descriptors)")
            if k == 0:
                out.append((np.array([]), np.array([])))
            else:
                out.append((mm[p, :k].astype(np.int64), cc[p, :k].astype(np.float32)))
    return out


def stage1(img_path: str, max_img: int, extractor_params: dict, match_threshold: float = 0.85,
           single_K=None, scale_factor: float = 0.5, num_matches: int = 2500, device: int = 0,
           ransac: bool = False, ransac_max_it: int | None = None):
    """SFMRunner.perform's stage 1 (Runner.py:183-191): frames "{img_path}/{i}.jpg" for
    i = 1..max_img, consecutive pairs; returns all_matches[(max_img+1) x (max_img+1)] of
    Matches as the reference fills it (Runner.py:174-175, 354-355).  With ransac=True the
    pairs other than (1, 2) get the reference's inlier filter (Runner.py:349-351,
    pose.find_inliers with max_iterations = ransac_max_it, default
    calculate_num_ransac_iterations(0.98, 8, 0.4) as Runner.py:170), all pairs in one
    device pass; a pair with fewer than 8 correspondences raises ValueError, as the
    reference's tuple unpacking of find_inliers' four Nones does."""
    paths = ["{}/{}.jpg".format(img_path, i) for i in range(1, max_img + 1)]
    cache = FeatureCache(paths, extractor_params, scale_factor=scale_factor, device=device)
    pairs = pair_schedule(max_img, "consecutive")
    res = match_schedule(cache, pairs, match_threshold)
    all_matches = [[None for _ in range(max_img + 1)] for _ in range(max_img + 1)]
    coords = []
    for (a, b), (mm, cc) in zip(pairs, res):
        X1, Y1 = cache.keypoints(int(a))
        X2, Y2 = cache.keypoints(int(b))
        coords.append(convert_matches_to_coords(mm, X1, Y1, X2, Y2, num_matches))
    if ransac:
        from . import pose
        iters = ransac_max_it if ransac_max_it is not None else pose.calculate_num_ransac_iterations(0.98, 8, 0.4)
        sel = [k for k, (a, b) in enumerate(pairs) if (int(a) + 1, int(b) + 1) != (1, 2)]
        filt = pose.find_inliers_batch([coords[k] for k in sel], max_iterations=iters, device=device)
        for k, r in zip(sel, filt):
            if len(r) != 2:
                raise ValueError("too many values to unpack (expected 2)")  # Runner.py:351 on four Nones
            coords[k] = r
    for k, ((a, b), (mm, cc)) in enumerate(zip(pairs, res)):
        i1, i2 = int(a) + 1, int(b) + 1
        p1, p2 = coords[k]
        all_matches[i1][i2] = Matches(mm, cc, p1, p2, single_K, single_K)
        all_matches[i2][i1] = Matches(mm, cc, p2, p1, single_K, single_K)
    return all_matches, cache
