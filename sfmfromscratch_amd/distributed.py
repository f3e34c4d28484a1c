"""Multi-GPU image sharding: one process per GPU, torch.distributed over
RCCL ("nccl" on ROCm) — or gloo on CPU for the tests.

Extraction is independent per image, so rank r owns the contiguous block of frames
[lo, hi) of the global sequence (`shard_range`) and nothing is exchanged for it.  The
only data-path exchange is what the match schedule needs:

* consecutive pairs (the reference's schedule, Runner.py:183-191): rank r additionally
  matches (its last frame, rank r+1's first frame).  `halo_exchange` moves exactly that
  one slot (xy, desc, count) from rank r+1 to rank r with a point-to-point send/recv —
  1.3 MB per rank at k = 2500, independent of the world size;
* all pairs (BASELINE configs[2]/[3]): `allgather_slots` builds the global slot table on
  every rank (one all_gather_into_tensor per field, fixed-capacity slots), and
  `all_pairs_for_rank` deals the upper-triangle pairs round-robin over ranks.

The slot-table layout is pipeline.SlotTable: xy [S, cap, 2] int32, desc [S, cap, 128]
float32, count [S] int32.  Works for any backend whose tensors live on the slot table's
device (RCCL: cuda tensors; gloo: CPU tensors).
"""
from __future__ import annotations

import numpy as np

from .pipeline import all_pairs, consecutive_pairs


def shard_range(n_global: int, world: int, rank: int) -> tuple[int, int]:
    """[lo, hi) of the frames owned by `rank`: contiguous blocks, the first
    n_global % world ranks get one extra frame."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    base, extra = divmod(n_global, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def local_consecutive_pairs(n_local: int, rank: int, world: int, n_next: int = 1) -> np.ndarray:
    """Slot-index pairs rank `rank` matches for the global consecutive schedule: its own
    (i, i+1) pairs plus (n_local-1, n_local) — slot n_local holds the next rank's first
    frame after `halo_exchange` — unless it is the last rank (or either side is empty)."""
    pairs = consecutive_pairs(n_local)
    if rank < world - 1 and n_local > 0 and n_next > 0:
        pairs = np.concatenate([pairs, np.array([[n_local - 1, n_local]], np.int32)])
    return pairs.astype(np.int32)


def halo_exchange(dist, slots, n_local: int, rank: int, world: int, group=None) -> None:
    """Copy rank r+1's slot 0 into this rank's slot `n_local` (needs S >= n_local + 1).
    Point-to-point: rank r sends its slot 0 to r-1 and receives r+1's slot 0."""
    if world == 1:
        return
    ops = []
    fields = (slots.xy, slots.desc, slots.count)
    if rank > 0:
        for f in fields:
            src = f[0:1] if f.dim() == 1 else f[0]
            ops.append(dist.P2POp(dist.isend, src.contiguous(), rank - 1, group))
    if rank < world - 1:
        for f in fields:
            dst = f[n_local:n_local + 1] if f.dim() == 1 else f[n_local]
            ops.append(dist.P2POp(dist.irecv, dst, rank + 1, group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()


def allgather_slots(dist, slots, n_local: int, world: int, out=None, group=None):
    """Gather every rank's first n_local slots into a global table [world * n_local, ...]
    (equal shard sizes; pad shards to the largest one before calling)."""
    torch = _torch()
    if out is None:
        out = type(slots).__new__(type(slots))
        out.B, out.cap = world * n_local, slots.cap
        out.xy = torch.empty((world * n_local,) + tuple(slots.xy.shape[1:]), dtype=slots.xy.dtype,
                             device=slots.xy.device)
        out.desc = torch.empty((world * n_local,) + tuple(slots.desc.shape[1:]), dtype=slots.desc.dtype,
                               device=slots.desc.device)
        out.count = torch.empty((world * n_local,), dtype=slots.count.dtype, device=slots.count.device)
    for f_out, f_in in ((out.xy, slots.xy), (out.desc, slots.desc), (out.count, slots.count)):
        dist.all_gather_into_tensor(f_out, f_in[:n_local].contiguous(), group=group)
    return out


def all_pairs_for_rank(n_global: int, rank: int, world: int) -> np.ndarray:
    """Upper-triangle pairs (i < j) of the global table dealt round-robin: pair p goes to
    rank p % world.  The union over ranks is every pair exactly once."""
    return all_pairs(n_global)[rank::world].astype(np.int32)


def _torch():
    import torch
    return torch
