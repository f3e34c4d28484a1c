"""GPU parity of BASELINE configs[3]'s data path: distributed.ChunkedGatherJob
— chunked extraction into the chunk-major gathered table (GatherPlan), per-chunk matcher
prep and ready-chunk matching of prepped slots — against the C oracle.

Every gathered slot must equal O.extract of its frame bit for bit, and every pair the rank
matched must equal O.match on the gathered descriptors (NNRatioFeatureMatcher.py:8-60).
Runs at world 1 (>= 4 chunks) and with 2 ranks spawned over gloo sharing the one GPU
(RCCL needs a GPU per rank; the data path is the same code)."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from oracle import oracle as O
from sfmfromscratch_amd import synth
from tests.golden_util import P_OCT, assert_matches_equal

pytestmark = pytest.mark.gpu

H, W = 270, 480
PP = dict(P_OCT, num_interest_points=600)
RATIO = 0.85
SEED = 4242


def _frames(torch, plan, rank):
    lo = rank * plan.S
    u8 = np.stack([synth.make_frame_u8(H, W, SEED, g) for g in range(lo, lo + plan.S)])
    return torch.from_numpy(u8).cuda()


def _check_job_vs_oracle(torch, job):
    """Every gathered slot == O.extract(frame); every matched pair == O.match."""
    plan = job.plan
    torch.cuda.synchronize()
    xy = job.table.xy.cpu().numpy()
    desc = job.table.desc.cpu().numpy()
    count = job.table.count.cpu().numpy()
    od = {}
    for g in range(plan.n):
        t = int(plan.slot_of(g))
        OX, OY, OD, _ = O.extract(synth.u8_to_gray(synth.make_frame_u8(H, W, SEED, g)), PP)
        n = int(count[t])
        assert n == len(OX), (g, n, len(OX))
        assert np.array_equal(xy[t, :n, 0], OX) and np.array_equal(xy[t, :n, 1], OY), g
        assert np.array_equal(desc[t, :n].view(np.uint32), OD.view(np.uint32)), g
        od[t] = OD
    checked = 0
    if job.sched is None:  # 'all' pairs: the dealt pairs and their kept results
        groups = [(job.last_all_pairs.cpu().numpy(), job.out_all)]
    else:
        groups = list(zip(job.sched, job.outs))
    for sp, outs in groups:
        mm, mc, nm = (o.cpu().numpy() for o in outs)
        for k, (a, b) in enumerate(np.asarray(sp).tolist()):
            om, oc = O.match(od[a], od[b], RATIO)
            kk = int(nm[k])
            if len(oc) == 0:
                assert kk == 0
            else:
                assert_matches_equal(om, oc, mm[k, :kk].astype(np.int64), mc[k, :kk])
            checked += 1
    return checked


@pytest.mark.parametrize("pairs", ["consecutive", "window:2"])
def test_chunked_gather_job_world1_vs_oracle(pairs):
    """World 1, 16 frames in 4 chunks of 4, two chunks in flight: the chunk-major table, the
    per-chunk prep and the ready-chunk prepped matching equal the oracle."""
    torch = pytest.importorskip("torch")
    from sfmfromscratch_amd import distributed as D
    plan = D.GatherPlan(16, 1, 4, pairs)
    assert plan.C == 4
    job = D.ChunkedGatherJob(PP, RATIO, plan, 0, H, W, inflight=2)
    frames = _frames(torch, plan, 0)
    job.run(frames)
    job.run(frames)  # a second job on the same buffers (lanes / prepped operands reused)
    checked = _check_job_vs_oracle(torch, job)
    assert checked == len(plan.global_pairs())


def test_chunked_gather_job_all_pairs_keeps_every_result():
    """'all' pairs with keep_all_results: 10 frames (45 pairs, more than one 4,096-pair
    sub-batch would need at CH = 16) keep every pair's result, each equal to O.match."""
    torch = pytest.importorskip("torch")
    from sfmfromscratch_amd import distributed as D
    plan = D.GatherPlan(10, 1, 4, "all")
    job = D.ChunkedGatherJob(PP, RATIO, plan, 0, H, W, inflight=2, keep_all_results=True)
    job.CH = 16  # several sub-batches
    frames = _frames(torch, plan, 0)
    job.run(frames)
    assert _check_job_vs_oracle(torch, job) == 45


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_worker(rank, world, port, pairs, errq):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import torch
        import torch.distributed as dist

        from sfmfromscratch_amd import distributed as D
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        plan = D.GatherPlan(16, world, 3, pairs)  # S = 8 per rank: chunks of 3, 3, 2
        job = D.ChunkedGatherJob(PP, RATIO, plan, rank, H, W, dist=dist, inflight=2)
        assert not job.coalesce  # gloo: one collective per field
        # the count-compacted gather stages each lane's rows in that lane's own buffers (the
        # lanes' streams are not ordered against each other)
        assert job.compact and len({id(ln["stage"]) for ln in job.lanes}) == len(job.lanes) == 2
        frames = _frames(torch, plan, rank)
        job.run(frames, record_sent=True)
        torch.cuda.synchronize()
        assert job.verify_exchange() == 0
        checked = _check_job_vs_oracle(torch, job)
        assert checked == len(plan.rank_pairs(rank))
        n = torch.tensor([checked], dtype=torch.int64)
        dist.all_reduce(n)
        assert int(n) == len(plan.global_pairs())
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001 — report to the parent
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


@pytest.mark.parametrize("pairs", ["consecutive", "window:3"])
def test_chunked_gather_job_two_ranks_gloo_vs_oracle(pairs):
    """Two ranks (gloo, sharing the GPU): each rank's gathered table holds every frame of
    both shards bit-equal to the oracle, the exchange check passes, and the ranks' matched
    pairs cover the global schedule, each equal to O.match."""
    pytest.importorskip("torch")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, pairs, errq)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not alive, "a rank hung"
    assert not errs and all(p.exitcode == 0 for p in procs), errs


P_1080 = dict(P_OCT)  # BASELINE configs[1] parameters, k = 2500


def _clean_checksums(torch, frames_u8):
    """Per-frame slot checksums of a B = 1 extraction of each frame (nothing else on the GPU)."""
    from sfmfromscratch_amd import distributed as D
    from sfmfromscratch_amd.pipeline import BatchExtractor
    ex = BatchExtractor(P_1080)
    return torch.cat([D.slot_checksums(torch, ex.extract(frames_u8[i:i + 1])) for i in range(frames_u8.shape[0])])


def test_chunked_job_1080p_concurrent_matching_equals_clean_extraction():
    """configs[3]'s job at full size: 1080p chunks extracted on two lanes while the ready pairs
    are matched on a third stream.  Every gathered slot must equal a clean single-frame
    extraction of its frame bit for bit (this is the check that caught k_match_mfma and
    k_harris sharing CUs)."""
    torch = pytest.importorskip("torch")
    from sfmfromscratch_amd import distributed as D
    U, n = 32, 128
    uq = torch.from_numpy(np.stack([synth.make_frame_u8(1080, 1920, 77, i) for i in range(U)])).cuda()
    ref = _clean_checksums(torch, uq)
    frames = uq[torch.arange(n, device="cuda") % U].contiguous()
    plan = D.GatherPlan(n, 1, 32, "consecutive")
    job = D.ChunkedGatherJob(P_1080, RATIO, plan, 0, 1080, 1920, inflight=2)
    for _ in range(2):
        job.run(frames)
        torch.cuda.synchronize()
        got = D.slot_checksums(torch, job.table)
        bad = (got != ref[torch.arange(n, device="cuda") % U]).any(1).nonzero().flatten().tolist()
        assert not bad, f"{len(bad)} gathered slots differ from a clean extraction: {bad[:10]}"


@pytest.mark.parametrize("gate", [False, True])
def test_pipeline_1080p_lanes_equal_clean_extraction(gate):
    """The headline pipeline (two 32 x 1080p batches in flight, each lane's matcher overlapping
    the other lane's extraction; with and without the lane gate): every lane's slots after
    every batch equal a clean single-frame extraction."""
    torch = pytest.importorskip("torch")
    from sfmfromscratch_amd import distributed as D
    from sfmfromscratch_amd.pipeline import BatchPipeline, consecutive_pairs
    B = 32
    u8 = torch.from_numpy(np.stack([synth.make_frame_u8(1080, 1920, 78, i) for i in range(B)])).cuda()
    ref = _clean_checksums(torch, u8)
    frames = torch.from_numpy(synth.u8_to_gray(u8.cpu().numpy())).cuda()
    pairs = torch.from_numpy(consecutive_pairs(B)).cuda()
    pipe = BatchPipeline(P_1080, RATIO, B, 1080, 1920, pairs, inflight=2, extra_slots=1, gate=gate)
    cks = []
    for _ in range(6):
        ln = pipe.submit(frames)
        with torch.cuda.stream(ln["stream"]):
            cks.append(D.slot_checksums(torch, ln["view"]))
    pipe.join()
    torch.cuda.synchronize()
    for s, ck in enumerate(cks):
        bad = (ck != ref).any(1).nonzero().flatten().tolist()
        assert not bad, f"batch {s}: {len(bad)} frames differ from a clean extraction: {bad[:10]}"
