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

import heapq

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


def weighted_deal(pairs: np.ndarray, counts: np.ndarray, world: int) -> list[np.ndarray]:
    """Deal pairs over ranks by matcher cost n_i * n_j (longest-processing-time greedy:
    heaviest pair first, to the least-loaded rank; ties to the lower rank).  Deterministic,
    so every rank computes the same deal from the same gathered counts.  Each rank's list
    keeps the global pair order."""
    pairs = np.asarray(pairs, np.int32).reshape(-1, 2)
    counts = np.asarray(counts, np.int64)
    cost = counts[pairs[:, 0]] * counts[pairs[:, 1]] + 1  # +1: empty pairs still cost a launch slot
    order = np.argsort(-cost, kind="stable")
    owner = np.empty(len(pairs), np.int64)
    heap = [(0, r) for r in range(world)]
    for p in order:
        load, r = heapq.heappop(heap)
        owner[p] = r
        heapq.heappush(heap, (load + int(cost[p]), r))
    return [pairs[owner == r] for r in range(world)]


class GatherPlan:
    """BASELINE configs[3] schedule: `n_global` frames in contiguous shards
    of S = n_global / world per rank, each shard extracted in chunks of `chunk` frames, and
    every chunk all-gathered over RCCL as soon as it is extracted, so chunk c's gather
    overlaps chunk c+1's extraction.

    Global table layout (chunk-major, so one chunk's gather writes one contiguous region):
    chunk c occupies slots [c * world * chunk, c * world * chunk + world * bc_c) with
    bc_c = min(chunk, S - c * chunk), and rank r's part of it starts at r * bc_c.  Frame g
    (owned by rank g // S at local index g % S) therefore lives at `slot_of(g)`.

    Pairs (global frame indices) come from `global_pairs`: 'consecutive' is the
    reference's (i, i+1) schedule (Runner.py:183-191); 'window:w' adds every (i, i+d),
    d <= w (a sequential-SfM neighbourhood); 'all' is every i < j.  For consecutive and
    window schedules a pair belongs to the owner of its first frame (equal shards give
    equal pair counts, +-w); it is matched after the gather of the later of its two chunks
    (`ready_chunk`), so matching also overlaps later chunks' extraction.  'all' pairs are
    dealt by cost with `weighted_deal` once the counts are gathered."""

    def __init__(self, n_global: int, world: int, chunk: int, pairs: str = "consecutive"):
        if world < 1 or n_global < 1 or n_global % world:
            raise ValueError(f"{n_global} frames do not split evenly over {world} ranks")
        if chunk < 1:
            raise ValueError("chunk must be >= 1")
        self.n, self.world = n_global, world
        self.S = n_global // world
        self.chunk = min(chunk, self.S)
        self.C = -(-self.S // self.chunk)
        self.pairs_mode = pairs
        self.window = 0
        if pairs == "consecutive":
            self.window = 1
        elif pairs.startswith("window:"):
            self.window = int(pairs.split(":", 1)[1])
            if self.window < 1:
                raise ValueError("window must be >= 1")
        elif pairs != "all":
            raise ValueError(f"unknown pair schedule {pairs!r}")

    def chunk_size(self, c: int) -> int:
        return min(self.chunk, self.S - c * self.chunk)

    def chunk_base(self, c: int) -> int:
        """First table slot of chunk c."""
        return c * self.world * self.chunk

    def local_frames(self, rank: int, c: int) -> tuple[int, int]:
        """[lo, hi) of the global frames rank `rank` extracts in chunk c."""
        lo = rank * self.S + c * self.chunk
        return lo, lo + self.chunk_size(c)

    def slot_of(self, g):
        g = np.asarray(g, np.int64)
        r, l = np.divmod(g, self.S)
        c, b = np.divmod(l, self.chunk)
        bc = np.minimum(self.chunk, self.S - c * self.chunk)
        return (c * self.world * self.chunk + r * bc + b).astype(np.int32)

    def chunk_of(self, g):
        return (np.asarray(g, np.int64) % self.S) // self.chunk

    def global_pairs(self) -> np.ndarray:
        if self.pairs_mode == "all":
            return all_pairs(self.n)
        out = []
        for d in range(1, self.window + 1):
            i = np.arange(max(self.n - d, 0), dtype=np.int32)
            out.append(np.stack([i, i + d], axis=1))
        p = np.concatenate(out) if out else np.zeros((0, 2), np.int32)
        return p[np.lexsort((p[:, 1], p[:, 0]))].astype(np.int32)

    def rank_pairs(self, rank: int) -> np.ndarray:
        """Global-frame pairs rank `rank` matches (consecutive / window schedules)."""
        if self.pairs_mode == "all":
            raise ValueError("'all' pairs are dealt by cost: use weighted_deal on the gathered counts")
        p = self.global_pairs()
        return p[p[:, 0] // self.S == rank]

    def ready_chunk(self, pairs: np.ndarray) -> np.ndarray:
        pairs = np.asarray(pairs).reshape(-1, 2)
        return np.maximum(self.chunk_of(pairs[:, 0]), self.chunk_of(pairs[:, 1]))

    def schedule(self, pairs: np.ndarray) -> list[np.ndarray]:
        """Per chunk c: the given global pairs ready after chunk c's gather, as table-slot
        pairs (int32 [P_c, 2])."""
        pairs = np.asarray(pairs, np.int64).reshape(-1, 2)
        rc = self.ready_chunk(pairs)
        return [self.slot_of(pairs[rc == c]).reshape(-1, 2) for c in range(self.C)]

    def frame_of_slot(self) -> np.ndarray:
        """Inverse of slot_of over the whole table."""
        inv = np.empty(self.n, np.int64)
        inv[self.slot_of(np.arange(self.n))] = np.arange(self.n)
        return inv


def allgather_chunk(dist, table, plan: GatherPlan, c: int, src, async_op: bool = False, group=None):
    """All-gather chunk c: every rank's `src` slots [0, bc) (its freshly extracted chunk)
    land in the chunk's table region, rank-major.  One collective per field (xy, desc,
    count).  With async_op the work handles are returned; `w.wait()` under a stream
    makes that stream wait for the collective without blocking the host (RCCL)."""
    bc = plan.chunk_size(c)
    base = plan.chunk_base(c)
    n = plan.world * bc
    works = []
    for f_out, f_in in ((table.xy, src.xy), (table.desc, src.desc), (table.count, src.count)):
        w = dist.all_gather_into_tensor(f_out[base:base + n], f_in[:bc], group=group, async_op=async_op)
        if async_op:
            works.append(w)
    return works


def _torch():
    import torch
    return torch
