"""Multi-process (gloo, CPU) tests of the image-sharding path:
shard ranges, the point-to-point halo exchange for consecutive pairs, the all-gather of
slot tables and the round-robin all-pairs deal.  The same functions run over RCCL in
bench.py; here every rank is a CPU process with fake slot contents keyed by the global
frame index, so each received slot can be checked exactly."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sfmfromscratch_amd import distributed as D
from sfmfromscratch_amd.pipeline import SlotTable

CAP = 16


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fill_slot(slots, s: int, g: int):
    """Slot s holds global frame g: count 3 + g % 7, xy / desc derived from g."""
    slots.count[s] = 3 + g % 7
    slots.xy[s] = torch.arange(CAP * 2, dtype=torch.int32).view(CAP, 2) + 1000 * g
    slots.desc[s] = torch.arange(CAP * 128, dtype=torch.float32).view(CAP, 128) * 1e-3 + g


def _worker(rank, world, port, n_global, mode, errq):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        lo, hi = D.shard_range(n_global, world, rank)
        n_local = hi - lo
        if mode == "halo":
            slots = SlotTable(torch, n_local + 1, CAP, "cpu")
            for s in range(n_local):
                _fill_slot(slots, s, lo + s)
            D.halo_exchange(dist, slots, n_local, rank, world)
            pairs = D.local_consecutive_pairs(n_local, rank, world)
            if rank < world - 1:
                ref = SlotTable(torch, 1, CAP, "cpu")
                _fill_slot(ref, 0, hi)
                assert torch.equal(slots.desc[n_local], ref.desc[0])
                assert torch.equal(slots.xy[n_local], ref.xy[0])
                assert int(slots.count[n_local]) == int(ref.count[0])
            else:
                assert int(slots.count[n_local]) == 0  # untouched
            glob = [(lo + int(i), lo + int(j)) for i, j in pairs]
        elif mode.startswith("compact"):  # the count-compacted chunk gather (counts, then M rows)
            plan = D.GatherPlan(n_global, world, 3, "consecutive")
            table = SlotTable(torch, n_global, CAP, "cpu")
            src = SlotTable(torch, plan.chunk, CAP, "cpu")
            stage = D.CompactStage(torch, world, plan.chunk, CAP, "cpu")
            moved = 0
            for c in range(plan.C):
                lo, hi = plan.local_frames(rank, c)
                for b, g in enumerate(range(lo, hi)):
                    _fill_slot(src, b, g)
                    src.desc[b, int(src.count[b]):] = -7.0 - rank  # rows past the count: not live
                    src.xy[b, int(src.count[b]):] = -7 - rank
                for w in D.allgather_chunk_counts(dist, table, plan, c, src, async_op=True):
                    w.wait()
                bc, base = plan.chunk_size(c), plan.chunk_base(c)
                M = int(table.count[base:base + world * bc].max())
                assert M == max(3 + g % 7 for r in range(world) for g in range(*plan.local_frames(r, c)))
                _, nb = D.allgather_chunk_rows(dist, table, plan, c, src, stage, M)
                moved += nb
            for g in range(n_global):  # every frame's live rows at slot_of(g), bit-equal
                ref = SlotTable(torch, 1, CAP, "cpu")
                _fill_slot(ref, 0, g)
                s, n = int(plan.slot_of(g)), int(ref.count[0])
                assert int(table.count[s]) == n
                assert torch.equal(table.desc[s, :n], ref.desc[0, :n]) and torch.equal(table.xy[s, :n], ref.xy[0, :n])
                Mg = max(3 + h % 7 for h in range(n_global) if plan.chunk_of(h) == plan.chunk_of(g))
                assert not table.desc[s, Mg:].any()  # rows past the chunk's M are never sent
            ck = D.slot_checksums(torch, table, torch.from_numpy(plan.slot_of(np.arange(n_global)).astype(np.int64)))
            for g in range(n_global):  # checksums see only the live rows
                ref = SlotTable(torch, 1, CAP, "cpu")
                _fill_slot(ref, 0, g)
                ref.desc[0, int(ref.count[0]):] = 123.0
                assert torch.equal(ck[g], D.slot_checksums(torch, ref)[0])
            assert 0 < moved < (world - 1) * plan.S * CAP * (128 * 4 + 8)
            glob = []  # no pairs in this mode
        elif mode.startswith("plan"):  # configs[3]: chunked all-gather (distributed.GatherPlan)
            sched_name = mode.split("/", 1)[1]
            plan = D.GatherPlan(n_global, world, 3, sched_name)
            table = SlotTable(torch, n_global, CAP, "cpu")
            src = SlotTable(torch, plan.chunk, CAP, "cpu")
            for c in range(plan.C):
                lo, hi = plan.local_frames(rank, c)
                for b, g in enumerate(range(lo, hi)):
                    _fill_slot(src, b, g)
                for w in D.allgather_chunk(dist, table, plan, c, src, async_op=True):
                    w.wait()
            for g in range(n_global):  # every frame at slot_of(g), bit-equal
                ref = SlotTable(torch, 1, CAP, "cpu")
                _fill_slot(ref, 0, g)
                s = int(plan.slot_of(g))
                assert torch.equal(table.desc[s], ref.desc[0]) and torch.equal(table.xy[s], ref.xy[0])
                assert int(table.count[s]) == int(ref.count[0])
            assert sorted(plan.frame_of_slot().tolist()) == list(range(n_global))
            if sched_name == "all":
                counts = table.count.numpy()[plan.slot_of(np.arange(n_global))]
                mine = D.weighted_deal(plan.global_pairs(), counts, world)[rank]
            else:
                mine = plan.rank_pairs(rank)
            glob = []
            inv = plan.frame_of_slot()
            for c, sp in enumerate(plan.schedule(mine)):
                for a, b in sp.tolist():
                    i, j = int(inv[a]), int(inv[b])
                    # ready: both frames' chunks gathered by chunk c
                    assert plan.chunk_of(i) <= c and plan.chunk_of(j) <= c
                    glob.append((i, j))
        else:  # allgather
            per = -(-n_global // world)
            slots = SlotTable(torch, per, CAP, "cpu")
            for s in range(n_local):
                _fill_slot(slots, s, lo + s)
            table = D.allgather_slots(dist, slots, per, world)
            for r in range(world):
                rlo, rhi = D.shard_range(n_global, world, r)
                for s in range(rhi - rlo):
                    ref = SlotTable(torch, 1, CAP, "cpu")
                    _fill_slot(ref, 0, rlo + s)
                    assert torch.equal(table.desc[r * per + s], ref.desc[0])
                    assert int(table.count[r * per + s]) == int(ref.count[0])
            glob = [tuple(map(int, p)) for p in D.all_pairs_for_rank(n_global, rank, world)]
        gathered = [None] * world
        dist.all_gather_object(gathered, glob)
        if rank == 0 and not mode.startswith("compact"):
            allp = sorted(p for g in gathered for p in g)
            if mode in ("halo", "plan/consecutive"):
                expect = [(i, i + 1) for i in range(n_global - 1)]
            elif mode.startswith("plan/window:"):
                w = int(mode.split(":")[1])
                expect = sorted((i, i + d) for d in range(1, w + 1) for i in range(n_global - d))
            else:
                expect = [(i, j) for i in range(n_global) for j in range(i + 1, n_global)]
            assert allp == expect, (allp, expect)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001 — report to the parent
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


def _run(world, n_global, mode):
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_global, mode, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not alive, "a rank hung"
    assert not errs and all(p.exitcode == 0 for p in procs), errs


@pytest.mark.parametrize("world,n_global", [(2, 8), (2, 7), (3, 10)])
def test_halo_exchange_consecutive_pairs(world, n_global):
    _run(world, n_global, "halo")


@pytest.mark.parametrize("world,n_global", [(2, 6), (3, 7)])
def test_allgather_all_pairs(world, n_global):
    _run(world, n_global, "allgather")


@pytest.mark.parametrize("world,n_global,sched", [(2, 16, "consecutive"), (2, 14, "window:4"), (3, 21, "all"),
                                                  (3, 9, "consecutive")])
def test_chunked_allgather_plan(world, n_global, sched):
    """configs[3]'s schedule: chunked all-gather lands every frame bit-equal at its table
    slot on every rank; the ranks' pairs cover the global schedule exactly once, each in a
    chunk at which both of its frames are gathered."""
    _run(world, n_global, "plan/" + sched)


@pytest.mark.parametrize("world,n_global", [(2, 16), (3, 21)])
def test_count_compacted_chunk_gather(world, n_global):
    """The count-compacted gather (counts first, then each chunk's first M rows, M = its
    largest count over the ranks): every frame's live rows land bit-equal at its slot, rows
    past a count are never sent, checksums cover the live rows only, and fewer bytes move
    than with full-capacity slots."""
    _run(world, n_global, "compact")


def test_gather_plan_layout_and_weighted_deal():
    plan = D.GatherPlan(64, 4, 5)  # S = 16 per rank: chunks of 5, 5, 5, 1
    assert plan.C == 4 and [plan.chunk_size(c) for c in range(4)] == [5, 5, 5, 1]
    slots = plan.slot_of(np.arange(64))
    assert sorted(slots.tolist()) == list(range(64))
    for c in range(plan.C):  # one chunk's region is contiguous and rank-major
        region = [int(plan.slot_of(g)) for r in range(4) for g in range(*plan.local_frames(r, c))]
        assert region == list(range(plan.chunk_base(c), plan.chunk_base(c) + 4 * plan.chunk_size(c)))
    with pytest.raises(ValueError):
        D.GatherPlan(10, 4, 2)
    with pytest.raises(ValueError):
        D.GatherPlan(8, 2, 2, "bogus")
    counts = np.array([10, 1, 1, 1, 10, 1], np.int64)
    deal = D.weighted_deal(D.all_pairs(6), counts, 2)
    cost = [sum(int(counts[i] * counts[j] + 1) for i, j in d) for d in deal]
    assert sum(len(d) for d in deal) == 15 and abs(cost[0] - cost[1]) <= 101
    assert {tuple(p) for d in deal for p in d.tolist()} == {tuple(p) for p in D.all_pairs(6).tolist()}


def test_shard_range_partitions():
    for n in range(0, 40):
        for world in range(1, 9):
            spans = [D.shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        D.shard_range(4, 2, 2)


def test_local_pairs_edge_cases():
    assert D.local_consecutive_pairs(0, 0, 2).shape == (0, 2)
    assert D.local_consecutive_pairs(1, 0, 2).tolist() == [[0, 1]]
    assert D.local_consecutive_pairs(3, 1, 2).tolist() == [[0, 1], [1, 2]]
    assert D.local_consecutive_pairs(3, 0, 1).tolist() == [[0, 1], [1, 2]]
    a = np.concatenate([D.all_pairs_for_rank(9, r, 4) for r in range(4)])
    assert len(a) == 36 and len({tuple(p) for p in a.tolist()}) == 36


def test_nccl_options_high_priority_stream(monkeypatch):
    """The exchange's RCCL group runs on a high-priority stream unless SFM_NCCL_HIPRIO=0."""
    import torch.distributed as dist

    from sfmfromscratch_amd.distributed import nccl_options
    monkeypatch.delenv("SFM_NCCL_HIPRIO", raising=False)
    assert nccl_options(dist).is_high_priority_stream
    monkeypatch.setenv("SFM_NCCL_HIPRIO", "0")
    assert not nccl_options(dist).is_high_priority_stream
