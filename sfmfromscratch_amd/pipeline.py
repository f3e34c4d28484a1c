"""Device-resident batch API over the C-ABI (the throughput path).

torch is used only as device-memory / stream plumbing: tensors hand their data pointers
to libsfmfeat, and the library enqueues on torch's current HIP stream so its kernels are
ordered with any torch work around them.

Slot table: xy [B, cap, 2] int32, desc [B, cap, 128] float32,
count [B] int32, cap = L * int(k / L).
"""
from __future__ import annotations

import numpy as np

from . import _abi
from ._native import Context
from .matcher import ratio_as_float32


def consecutive_pairs(n: int, offset: int = 0) -> np.ndarray:
    """(i, i+1) pairs of the reference's schedule (Runner.py:183)."""
    i = np.arange(max(n - 1, 0), dtype=np.int32) + offset
    return np.stack([i, i + 1], axis=1).astype(np.int32)


def all_pairs(n: int) -> np.ndarray:
    i, j = np.triu_indices(n, k=1)
    return np.stack([i, j], axis=1).astype(np.int32)


class SlotTable:
    def __init__(self, torch, B: int, cap: int, device):
        self.B, self.cap = B, cap
        self.xy = torch.zeros((B, max(cap, 1), 2), dtype=torch.int32, device=device)
        self.desc = torch.zeros((B, max(cap, 1), 128), dtype=torch.float32, device=device)
        self.count = torch.zeros((B,), dtype=torch.int32, device=device)


def ingest_rgb(ctx: Context, rgb, scale: float = 0.5, out=None):
    """Device ingest of a batch of decoded RGB frames (FeatureRunner, Runner.py:33-46):
    rgb [B, H, W, 3] uint8 cuda tensor -> [B, int(H*scale), int(W*scale)] float32 gray
    (PIL BICUBIC resize, /255, _rgb2gray), enqueued on torch's current stream."""
    import torch
    from ._native import resize_dims
    assert rgb.is_cuda and rgb.dtype == torch.uint8 and rgb.dim() == 4 and rgb.shape[3] == 3
    rgb = rgb.contiguous()
    B, H, W, _ = rgb.shape
    H2, W2 = resize_dims(H, W, scale)
    if out is None:
        out = torch.empty((B, H2, W2), dtype=torch.float32, device=rgb.device)
    assert out.shape == (B, H2, W2) and out.dtype == torch.float32 and out.is_contiguous()
    stream = torch.cuda.current_stream(rgb.device).cuda_stream
    ctx.ingest_rgb_dev(rgb.data_ptr(), B, H, W, H2, W2, out.data_ptr(), stream)
    return out


class BatchExtractor:
    """Batched ScaleRotInvSIFT / NaiveSIFT extraction on device-resident frames."""

    def __init__(self, extractor_params: dict | None = None, mode: str = "scalerot", device: int = 0):
        import torch
        self.torch = torch
        self.mode = _abi.SFM_MODE_NAIVE if mode == "naive" else _abi.SFM_MODE_SCALEROT
        self.params = _abi.params_from_dict(extractor_params, self.mode)
        self.device = device
        self.ctx = Context(self.params, device)
        self.cap = self.ctx.capacity

    def reserve(self, B: int, H: int, W: int):
        self.ctx.reserve(B, H, W)

    def new_slots(self, B: int) -> SlotTable:
        return SlotTable(self.torch, B, self.cap, f"cuda:{self.device}")

    def extract(self, imgs, out: SlotTable | None = None) -> SlotTable:
        torch = self.torch
        assert imgs.is_cuda and imgs.dim() == 3 and imgs.is_contiguous()
        B, H, W = imgs.shape
        if out is None:
            out = self.new_slots(B)
        stream = torch.cuda.current_stream(imgs.device).cuda_stream
        self.ctx.extract_batch_dev(imgs.data_ptr(), B, H, W, out.xy.data_ptr(), out.desc.data_ptr(),
                                   out.count.data_ptr(), max(self.cap, 1), stream,
                                   u8=(imgs.dtype == torch.uint8))
        return out


class BatchMatcher:
    """NNRatioFeatureMatcher over image pairs of a slot table."""

    def __init__(self, ratio_threshold=0.8, device: int = 0, ctx: Context | None = None):
        import torch
        self.torch = torch
        self.ratio32 = float(ratio_as_float32(ratio_threshold))
        self.ctx = ctx or Context(_abi.params_from_dict({}, _abi.SFM_MODE_NAIVE), device)
        self.device = device

    def prep(self, slots: SlotTable, lo: int = 0, n: int | None = None):
        """Build the matcher's operands for slots [lo, lo + n) of `slots` (default: all) on
        torch's current stream; later `match(..., prepped=True)` calls on pairs of prepped
        slots skip the per-call prep of the whole table (large resident tables)."""
        torch = self.torch
        S, cap = slots.desc.shape[0], slots.desc.shape[1]
        n = S - lo if n is None else n
        stream = torch.cuda.current_stream(slots.desc.device).cuda_stream
        self.ctx.match_prep_dev(slots.desc.data_ptr(), slots.count.data_ptr(), S, cap, lo, n, stream)

    def match(self, slots: SlotTable, pairs, out=None, prepped: bool = False):
        """pairs: (P, 2) int32 tensor on the device.  Returns (matches [P,cap,2] int32,
        conf [P,cap] f32, nmatch [P] int32 (-1 = the reference's IndexError)).  With
        `prepped`, every slot the pairs touch must have been prepped by `prep` since its
        descriptors last changed."""
        torch = self.torch
        P = int(pairs.shape[0])
        cap = slots.desc.shape[1]
        dev = slots.desc.device
        if out is None:
            out = (torch.zeros((max(P, 1), cap, 2), dtype=torch.int32, device=dev),
                   torch.zeros((max(P, 1), cap), dtype=torch.float32, device=dev),
                   torch.zeros((max(P, 1),), dtype=torch.int32, device=dev))
        if P == 0:
            return out
        stream = torch.cuda.current_stream(dev).cuda_stream
        self.ctx.match_pairs_dev(slots.desc.data_ptr(), slots.count.data_ptr(), slots.desc.shape[0], cap,
                                 pairs.data_ptr(), P, self.ratio32, out[0].data_ptr(), out[1].data_ptr(),
                                 out[2].data_ptr(), stream, prepped=prepped)
        return out


class BatchPipeline:
    """Detect + describe + match over a stream of frame batches, `inflight` batches at a
    time (the throughput path of SURVEY.md §8d; Runner.py:183-191 does the same work one
    pair at a time on 8 host threads).

    Each in-flight lane owns a context (device workspace + its aux HIP stream), a torch
    stream, a slot table and match outputs, so batch i+1's pyramid / Harris fill the
    GPU while batch i's small levels, descriptors and matcher drain.  Batch i runs on
    lane i % inflight; lanes are reused in order, so a lane's outputs stay valid until
    `inflight` further batches are submitted (`join()` orders the caller's stream after
    every lane).

    `hook(slots, B)` runs on the lane's stream between extraction and matching (the halo
    exchange of a sharded run, distributed.halo_exchange).

    `gate` (default: SFMFEAT_LANE_GATE, off unless "1"): the lanes' contexts share one
    sfm_gate, so batch i+1's pyramid and level-0 Harris start when batch i's level-0 Harris
    has ended and overlap batch i's level-0 NMS, selection and descriptors by construction,
    instead of by whatever order the HIP runtime's shared hardware queues happen to give."""

    def __init__(self, extractor_params: dict | None, ratio_threshold: float, batch: int, H: int, W: int,
                 pairs, inflight: int = 2, device: int = 0, extra_slots: int = 1, gate: bool | None = None,
                 lane_streams: str | None = None, serial_lanes=None):
        import os

        import torch
        self.torch = torch
        if gate is None:
            gate = os.environ.get("SFMFEAT_LANE_GATE", "0") == "1"
        # lane_streams: "context" (default: the lane context's own stream, wrapped as a torch
        # ExternalStream: no torch stream pool, so the process's streams are exactly the lanes'
        # host and aux streams — four with two lanes, one per hardware queue at the runtime's
        # default of four) or "torch" (a stream from torch's pool per lane, which shares
        # hardware queues with the contexts' aux streams by creation order: 35.05k vs 36.03k
        # img/s over five interleaved driver-command runs each, DESIGN_LOG.md §B).  serial_lanes: lane indices whose
        # extraction runs on one stream (sfm_ctx_set_serial), e.g. "0" in SFMFEAT_SERIAL_LANES
        if lane_streams is None:
            lane_streams = os.environ.get("SFMFEAT_LANE_STREAMS", "context")
        # SFMFEAT_LANE_PRIO=1 (A/B): the first lane's streams (host and aux) at the higher HIP
        # stream priority.  With torch's lane streams a high-priority first lane gained 4 %
        # (35.1k -> 36.5k img/s); with the contexts' own streams (the default) it measured
        # 37.36k vs 37.45k at configs[1] and 8.91k vs 9.05k at configs[4], so it stays off
        lane_prio = os.environ.get("SFMFEAT_LANE_PRIO", "0") == "1"
        if serial_lanes is None:
            env = os.environ.get("SFMFEAT_SERIAL_LANES", "")
            serial_lanes = [int(v) for v in env.replace("+", ",").split(",") if v.strip()]
        self.lane_streams = lane_streams
        self.serial_lanes = sorted(set(int(v) for v in serial_lanes))
        # fused matcher operands (sfm_ctx_set_fused_prep): each lane's extraction writes the
        # matcher's operands of its batch, so the match launches no operand prep for them (its
        # table is the lane's own; the halo hook writes only the extra slots, which the match
        # preps).  SFMFEAT_FUSED_PREP=0: the separate prep launch (A/B)
        fused_prep = os.environ.get("SFMFEAT_FUSED_PREP", "1") != "0"
        self.fused_prep = fused_prep
        self.B, self.H, self.W = batch, H, W
        self.inflight = max(1, int(inflight))
        self.pairs = pairs
        dev = torch.device("cuda", device)
        P = int(pairs.shape[0])
        self.lanes = []
        for li in range(self.inflight):
            ex = BatchExtractor(extractor_params, device=device)
            ex.reserve(batch, H, W)
            if li in self.serial_lanes:
                ex.ctx.set_serial(True)
            if fused_prep:
                ex.ctx.set_fused_prep(True)
            if lane_streams == "context":
                if li == 0 and lane_prio:
                    ex.ctx.set_priority(-1)
                stream = torch.cuda.ExternalStream(ex.ctx.stream(), device=dev)
            elif lane_streams == "torch-prio":  # A/B: lane 0 on a high-priority stream
                stream = torch.cuda.Stream(device=dev, priority=-1 if li == 0 else 0)
            else:
                stream = torch.cuda.Stream(device=dev)
            m = BatchMatcher(ratio_threshold, device=device, ctx=ex.ctx)
            slots = SlotTable(torch, batch + extra_slots, ex.cap, dev)
            view = SlotTable.__new__(SlotTable)
            view.B, view.cap = batch, ex.cap
            view.xy, view.desc, view.count = slots.xy[:batch], slots.desc[:batch], slots.count[:batch]
            mout = (torch.zeros((max(P, 1), max(ex.cap, 1), 2), dtype=torch.int32, device=dev),
                    torch.zeros((max(P, 1), max(ex.cap, 1)), dtype=torch.float32, device=dev),
                    torch.zeros((max(P, 1),), dtype=torch.int32, device=dev))
            self.lanes.append({"ex": ex, "m": m, "slots": slots, "view": view, "mout": mout, "stream": stream})
        self.cap = self.lanes[0]["ex"].cap
        # pairs within the batch only (no halo pair): the match reads the batch's slots alone
        self.batch_only_pairs = P == 0 or int(pairs.max().item()) < batch
        self.n = 0
        self.gate = None
        if gate and self.inflight > 1:
            from ._native import Gate
            self.gate = Gate(device)
            for ln in self.lanes:
                self.gate.attach(ln["ex"].ctx)

    @property
    def contexts(self):
        return [ln["ex"].ctx for ln in self.lanes]

    def submit(self, frames, hook=None):
        """Enqueue one batch (device [B, H, W] f32 or u8 frames); returns its lane."""
        torch = self.torch
        ln = self.lanes[self.n % self.inflight]
        self.n += 1
        cur = torch.cuda.current_stream(frames.device)
        ln["stream"].wait_stream(cur)
        # the lane reads `frames` after the caller may have dropped it: keep its memory
        # out of the caching allocator until the lane's work is done.  A context-owned lane
        # stream (lane_streams "context") is destroyed with its context, possibly before the
        # allocator would query an event recorded by record_stream on it: such lanes hold the
        # frames instead, released once the caller's stream has waited for the extraction.
        if self.lane_streams == "context":
            if ln.get("hold_ev") is not None:
                cur.wait_event(ln["hold_ev"])
            ln["hold"] = frames
        else:
            frames.record_stream(ln["stream"])
        with torch.cuda.stream(ln["stream"]):
            ln["ex"].extract(frames, out=ln["view"])
            if self.lane_streams == "context":
                ln["hold_ev"] = torch.cuda.Event()
                ln["hold_ev"].record(ln["stream"])
            if hook is not None:
                hook(ln["slots"], self.B)
            ln["m"].match(ln["view"] if self.batch_only_pairs else ln["slots"], self.pairs, out=ln["mout"])
        return ln

    def join(self):
        """Make the caller's current stream wait for every lane (no host sync)."""
        cur = self.torch.cuda.current_stream()
        for ln in self.lanes:
            cur.wait_stream(ln["stream"])

    def start(self):
        """Make every lane wait for the caller's current stream (e.g. after an event)."""
        cur = self.torch.cuda.current_stream()
        for ln in self.lanes:
            ln["stream"].wait_stream(cur)
