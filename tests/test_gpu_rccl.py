"""RCCL code path of configs[3]'s exchange on the one GPU of the box (world size 1).

The multi-GPU bench (bench.py --gpus N, distributed.ChunkedGatherJob) gathers each chunk's
slot table with ONE coalesced RCCL group (torch's coalescing manager over three
all_gather_into_tensor calls of different dtypes), waited on a CUDA stream, on a process
group whose internal stream is high-priority.  Only the driver's 8-GPU run executes it with
several ranks; this test runs exactly those calls through RCCL with one rank, so the API
usage (coalescing manager, async work handles, the process-group options) is exercised on
the real backend, and the gathered table must equal what was sent bit for bit."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.mark.gpu
def test_rccl_coalesced_chunk_allgather_world1():
    import torch
    import torch.distributed as dist

    from sfmfromscratch_amd.distributed import GatherPlan, allgather_chunk, nccl_options
    from sfmfromscratch_amd.pipeline import SlotTable

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    store = dist.HashStore()
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, pg_options=nccl_options(dist),
                            device_id=dev)
    try:
        cap, chunk, n = 300, 8, 24
        plan = GatherPlan(n, 1, chunk)
        table = SlotTable(torch, n, cap, dev)
        g = torch.Generator(device="cpu").manual_seed(7)
        side = torch.cuda.Stream(device=dev)
        sent = []
        for c in range(plan.C):
            src = SlotTable(torch, chunk, cap, dev)
            src.desc.copy_(torch.rand(src.desc.shape, generator=g))
            src.xy.copy_(torch.randint(0, 4000, src.xy.shape, generator=g, dtype=torch.int32))
            src.count.copy_(torch.randint(0, cap + 1, src.count.shape, generator=g, dtype=torch.int32))
            sent.append((src.desc.cpu(), src.xy.cpu(), src.count.cpu()))
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                works = allgather_chunk(dist, table, plan, c, src, async_op=True, coalesce=True)
                assert len(works) == 1  # one grouped operation per chunk
                for w in works:
                    w.wait()
            torch.cuda.current_stream().wait_stream(side)
            src.desc.record_stream(side)
        torch.cuda.synchronize()
        for c, (d, xy, cnt) in enumerate(sent):
            b = plan.chunk_base(c)
            assert torch.equal(table.desc[b:b + chunk].cpu().view(torch.int32), d.view(torch.int32))
            assert torch.equal(table.xy[b:b + chunk].cpu(), xy)
            assert torch.equal(table.count[b:b + chunk].cpu(), cnt)
        assert np.array_equal(plan.slot_of(np.arange(n)), np.arange(n))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sfm_dist_abi_chunk_gather_and_halo_world1():
    """The C-ABI exchange (include/sfmfeat.h sfm_dist_*, RCCL bound at run time) on the box's one
    GPU: each chunk's slots gathered into the chunk-major table from separate buffers and in
    place (the own slots as the send buffer), bit for bit, on a side stream; the halo of a
    single rank moves nothing.  Several ranks need several GPUs (RCCL refuses two ranks on one
    device); the torch path's multi-rank schedule is covered over gloo (test_distributed_cpu)."""
    import torch

    from sfmfromscratch_amd._native import Dist
    from sfmfromscratch_amd.distributed import GatherPlan
    from sfmfromscratch_amd.pipeline import SlotTable

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    d = Dist(0, 0, 1, Dist.unique_id())
    try:
        cap, chunk, n = 300, 8, 24
        plan = GatherPlan(n, 1, chunk)
        table = SlotTable(torch, n, cap, dev)
        g = torch.Generator(device="cpu").manual_seed(11)
        side = torch.cuda.Stream(device=dev)
        sent = []
        for c in range(plan.C):
            src = SlotTable(torch, chunk, cap, dev)
            src.desc.copy_(torch.rand(src.desc.shape, generator=g))
            src.xy.copy_(torch.randint(0, 4000, src.xy.shape, generator=g, dtype=torch.int32))
            src.count.copy_(torch.randint(0, cap + 1, src.count.shape, generator=g, dtype=torch.int32))
            sent.append((src.desc.cpu(), src.xy.cpu(), src.count.cpu()))
            side.wait_stream(torch.cuda.current_stream())
            d.allgather_slots(table, plan.chunk_base(c), src, chunk, stream=side.cuda_stream)
            torch.cuda.current_stream().wait_stream(side)
            src.desc.record_stream(side)
        torch.cuda.synchronize()
        for c, (dd, xy, cnt) in enumerate(sent):
            b = plan.chunk_base(c)
            assert torch.equal(table.desc[b:b + chunk].cpu().view(torch.int32), dd.view(torch.int32))
            assert torch.equal(table.xy[b:b + chunk].cpu(), xy)
            assert torch.equal(table.count[b:b + chunk].cpu(), cnt)

        class View:  # the table's own slots of chunk 1 as the send buffer (in place)
            b = plan.chunk_base(1)
            xy, desc, count = table.xy[b:b + chunk], table.desc[b:b + chunk], table.count[b:b + chunk]

        before = (table.desc.cpu().clone(), table.xy.cpu().clone(), table.count.cpu().clone())
        d.allgather_slots(table, plan.chunk_base(1), View, chunk, stream=torch.cuda.current_stream().cuda_stream)
        d.halo(table, 0, stream=torch.cuda.current_stream().cuda_stream)  # one rank: nothing moves
        torch.cuda.synchronize()
        assert torch.equal(table.desc.cpu().view(torch.int32), before[0].view(torch.int32))
        assert torch.equal(table.xy.cpu(), before[1]) and torch.equal(table.count.cpu(), before[2])
        with pytest.raises(ValueError):
            d.allgather_slots(table, n - 4, src, chunk)  # past the table's end
    finally:
        d.close()
