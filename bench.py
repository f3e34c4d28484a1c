#!/usr/bin/env python3
"""bench.py — images/sec detect+describe+match at 1080p on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): per GPU, a batch of 32 synthetic 1080p frames
(uint8 -> float32 gray, device-resident before timing), ScaleRotInvSIFT with the
"octave" parameters (4 levels x 2, k 2500, ksize 3, 7x7 Gaussian sigma 6, alpha 0.05,
feature width 18), then NNRatioFeatureMatcher(0.85) over consecutive pairs — the
reference's schedule (Runner.py:183).  One step = extract the batch + match its pairs.
Steps go through pipeline.BatchPipeline with --inflight (default 2) batches on the GPU at
once: each in-flight batch has its own context, stream and slot table, so one batch's
small pyramid levels, descriptors and matcher overlap the next batch's Harris work.
Every batch is still fully extracted and matched; --inflight 1 serialises them.

Multi-GPU (weak scaling, one process per GPU, torchrun): rank r owns frames
[r*B, (r+1)*B) of one global sequence (sfmfromscratch_amd/distributed.py).  The only
exchange is the reference's consecutive pair that straddles two shards: rank r+1 sends
its first slot (xy, desc, count) to rank r over RCCL point-to-point, and rank r also
matches (its last frame, rank r+1's first frame).

Prints ONE JSON line (rank 0) with the driver's contract fields plus `roofline`
(dominant kernel, live HIP-event timing inside the timed region) and `cpu_baseline`
(the C restatement in oracle/, timed on a bounded sample on this host, rank 0, N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

P_OCT = {"num_interest_points": 2500, "ksize": 3, "gaussian_size": 7, "sigma": 6, "alpha": 0.05,
         "feature_width": 18, "pyramid_level": 4, "pyramid_scale_factor": 2}
RATIO = 0.85
H, W = 1080, 1920
PEAK_F32_TFLOPS = 157.3   # MI355X FP32 (vector == matrix) dense peak, MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0     # HBM3E spec
# The matcher's prefilter is split-f16 on the f16 MFMA (dense 2.5 PF): three f16 products
# (hi*hi, hi*lo, lo*hi) per f32-accurate product, so its algorithmic (GEMM-equivalent)
# rate is bounded by 2500 / 3 TFLOP/s.
PEAK_MATCH_TFLOPS = 2500.0 / 3

# algorithmic work: per pixel for the per-level stages, per pair element for
# the matcher (GEMM-equivalent 2 n1 n2 128 flop)
HARRIS_FLOP_PER_PX = 328   # Sobel 2x6 fma (24) + 3 products + 3x49 fma (294) + R (7)
MATCH_FLOP_PER_ELEM = 2    # GEMM-equivalent: one multiply-add per descriptor element pair
DESC_BYTES_PER_KP = 20 * 20 * 4 + 128 * 4 + 12   # level window + halo read, descriptor + xy/conf written
KERNELS = {"harris": "k_harris<7>", "match": "k_match_mfma", "describe": "k_describe_q",
           "nms": "k_nms_stream<8,256>", "median": "k_med_scan", "topk": "k_topk", "pyramid": "k_down2x3",
           "match_prep": "k_match_prep", "match_post": "k_match_compact"}
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")  # tools/pmc_traffic.py


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_threads() -> int:
    """Host cores this process may use (the GPU box's share is 16; os.cpu_count() there
    reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))


def cpu_baseline(frames_per_thread: int):
    """The C restatement in oracle/ (scalar code, one image per thread, ctypes releases
    the GIL) on `threads * frames_per_thread` 1080p frames and their consecutive pairs,
    each thread owning a contiguous block of frames; returns (images/s, seconds, threads,
    frames)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O
    from sfmfromscratch_amd import synth
    nt = cpu_threads()
    n = nt * frames_per_thread
    imgs = [synth.make_frame(H, W, 1234, i) for i in range(n)]

    def block(t):
        descs = [O.extract(imgs[i], P_OCT)[2] for i in range(t * frames_per_thread, (t + 1) * frames_per_thread)]
        for a, b in zip(descs, descs[1:]):
            O.match(a, b, RATIO)

    t0 = time.perf_counter()
    with ThreadPoolExecutor(nt) as pool:
        list(pool.map(block, range(nt)))
    dt = time.perf_counter() - t0
    return n / dt, dt, nt, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="frames per GPU per step")
    ap.add_argument("--cpu-sample", type=int, default=8,
                    help="frames per host thread in the CPU baseline sample (0 = skip)")
    ap.add_argument("--no-profile", action="store_true", help="disable the live per-stage HIP events")
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5"], default="c2",
                    help="c2 = BASELINE configs[1] (the headline line); c3 = configs[2] (256 frames, all "
                         "pairs); c4 = configs[3] (2048 frames sharded over the ranks, chunked RCCL all-gather "
                         "of the descriptor tables, pairwise match); c5 = configs[4]'s per-GPU share (4K, "
                         "5 octaves, k 8000)")
    ap.add_argument("--frames", type=int, default=None,
                    help="c3: frames in the all-pairs job (256); c4: global frames (strong: 2048) or frames "
                         "per GPU (weak: 256)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="c4: fixed global frame count (strong) or fixed frames per GPU (weak)")
    ap.add_argument("--pairs", default="consecutive",
                    help="c4 pair schedule: consecutive | window:W | all")
    ap.add_argument("--exchange", choices=["allgather", "halo"], default="allgather",
                    help="c4: chunked all-gather of every slot table (configs[3]) or, for consecutive pairs, "
                         "only the 1-slot point-to-point halo")
    ap.add_argument("--rgb-ingest", action="store_true",
                    help="c2: frames resident as decoded 2x-size RGB (3840x2160x3 u8); each step first runs "
                         "FeatureRunner's ingest on the device (PIL BICUBIC x0.5 + _rgb2gray, Runner.py:33-46)")
    ap.add_argument("--inflight", type=int, default=2,
                    help="batches in flight (double-buffered contexts / slot tables, pipeline.BatchPipeline)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ngpu = torch.cuda.device_count()
    torch.cuda.set_device(local % max(ngpu, 1))
    dev = torch.device("cuda", local % max(ngpu, 1))
    if world > 1:
        # BENCH_DIST_BACKEND=gloo: rehearsal of the multi-rank code paths with several ranks
        # on one GPU (RCCL needs one GPU per rank); measurements use RCCL
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    if args.workload == "c3":
        return run_all_pairs(args, torch, dev)
    if args.workload == "c4":
        return run_gather(args, torch, dist, dev, rank, world)
    if args.workload == "c5":
        global H, W, P_OCT
        H, W = 2160, 3840
        P_OCT = dict(P_OCT, num_interest_points=8000, pyramid_level=5)
        if args.batch == 32:
            args.batch = 8

    from sfmfromscratch_amd import distributed as D
    from sfmfromscratch_amd import synth
    from sfmfromscratch_amd.pipeline import BatchPipeline

    B = args.batch
    # device-resident float32 frames of this rank's shard of the global sequence
    rgb = None
    if args.rgb_ingest:  # decoded RGB at twice the size; the gray frames are made on the device
        uniq = [synth.make_frame_rgb_u8(2 * H, 2 * W, 1234, rank * B + i) for i in range(min(B, 8))]
        rgb = torch.from_numpy(np.stack([uniq[i % len(uniq)] for i in range(B)])).to(dev)
        del uniq
        frames = torch.empty((B, H, W), dtype=torch.float32, device=dev)
    else:
        frames_u8 = np.stack([synth.make_frame_u8(H, W, 1234, rank * B + i) for i in range(B)])
        frames = torch.from_numpy(synth.u8_to_gray(frames_u8)).to(dev)
        del frames_u8
    pairs_np = D.local_consecutive_pairs(B, rank, world)
    pairs = torch.from_numpy(pairs_np).to(dev)
    P = pairs.shape[0]
    # slot B of each lane's table = the next rank's first frame (halo)
    pipe = BatchPipeline(P_OCT, RATIO, B, H, W, pairs, inflight=args.inflight, device=dev.index, extra_slots=1)
    ctxs = pipe.contexts

    def halo(slots, n):
        D.halo_exchange(dist, slots, n, rank, world)

    if rgb is not None:
        from sfmfromscratch_amd.pipeline import ingest_rgb
        lane_frames = [torch.empty_like(frames) for _ in pipe.lanes]

        def step():  # ingest on the lane's stream, then extract + match there
            ln = pipe.lanes[pipe.n % pipe.inflight]
            f = lane_frames[pipe.n % pipe.inflight]
            ln["stream"].wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(ln["stream"]):
                ingest_rgb(ln["ex"].ctx, rgb, 0.5, out=f)
                pipe.submit(f, hook=halo)
    else:
        def step():
            pipe.submit(frames, hook=halo)

    for _ in range(args.warmup):
        step()
    pipe.join()
    torch.cuda.synchronize()

    def stage_work(counts, nsteps):
        """Algorithmic work of `nsteps` steps per stage:
        (bound, amount, unit, peak, algorithmic HBM bytes or None).  Latency-bound stages
        (describe, top-k, median) get no roofline."""
        levels = [(H >> l, W >> l) for l in range(P_OCT["pyramid_level"])]
        px = sum(h * w for h, w in levels) * B * nsteps
        pair_elems = sum(int(counts[i]) * int(counts[j]) for i, j in pairs_np) * 128 * nsteps
        # k_down2x3 reads level 0 once and writes levels 1..3 (one launch); a 5th level is
        # one k_down2 from level 3
        A = [h * w for h, w in levels]
        pyr_px = A[0] + sum(A[1:4]) + sum(A[l - 1] + A[l] for l in range(4, len(A)))
        pyr_bytes = 4.0 * pyr_px * B * nsteps
        return {
            # VALU-bound: 328 flop/px of separate mul/add-class ops; bytes: read
            # the level, write R
            "harris": ("valu", HARRIS_FLOP_PER_PX * px / 1e12, "TFLOP/s", PEAK_F32_TFLOPS, 8.0 * px),
            "match": ("mfma", MATCH_FLOP_PER_ELEM * pair_elems / 1e12, "TFLOP/s", PEAK_MATCH_TFLOPS, None),
            "nms": ("hbm", 4.0 * px / 1e9, "GB/s", PEAK_HBM_GBS, 4.0 * px),          # one read of R
            "pyramid": ("hbm", pyr_bytes / 1e9, "GB/s", PEAK_HBM_GBS, pyr_bytes),
        }

    def prof_enable(on):
        for c in ctxs:
            c.profile_enable(on)

    def prof_read():
        tot = {}
        for c in ctxs:
            for k, (ms, n) in c.profile_read(reset=True).items():
                a = tot.get(k, (0.0, 0))
                tot[k] = (a[0] + ms, a[1] + n)
        return tot

    def lane_counts():
        return pipe.lanes[0]["slots"].count.cpu().numpy()

    # Per-stage device times (every stage bracketed by HIP events) in an untimed pass with
    # one batch on the GPU at a time; it names the dominant stage, whose events alone
    # stay on during the timed run.
    stages, dom = {}, None
    if not args.no_profile:
        nprof = max(2, args.steps // 2)
        prof_enable(True)
        prof_read()
        for _ in range(nprof):
            step()
            pipe.join()
            torch.cuda.synchronize()
        prof_all = prof_read()
        work = stage_work(lane_counts(), nprof)
        for k, (ms, n) in prof_all.items():
            if not n:
                continue
            st = {"ms_per_step": round(ms / nprof, 4), "launches_per_step": n // nprof}
            if k in work:
                bound, amount, unit, peak, _ = work[k]
                ach = amount / (ms / 1e3)
                st.update({"bound": bound, "achieved": round(ach, 3), "unit": unit, "frac": round(ach / peak, 4)})
            stages[k] = st
        dom = max((k for k in prof_all if k in work and prof_all[k][1]), key=lambda k: prof_all[k][0])
        for c in ctxs:
            c.profile_stages([dom])
        prof_read()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    pipe.start()
    for _ in range(args.steps):
        step()
    pipe.join()
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    elapsed = max(wall, gpu_ms / 1e3)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    prof = prof_read() if dom else {}
    prof_enable(False)
    counts = lane_counts()
    nmatch = pipe.lanes[0]["mout"][2].cpu().numpy()

    images = world * B * args.steps
    value = images / elapsed
    roof = None
    if dom:
        # the dominant stage's launches inside the timed region, timed by their own events
        traffic = {}
        # the committed PMC traffic was measured on the headline workload (c2) only
        if os.path.exists(TRAFFIC_FILE) and args.workload == "c2" and not args.rgb_ingest:
            with open(TRAFFIC_FILE) as f:
                traffic = json.load(f).get("bytes_per_launch", {})
        bound, amount, unit, peak, abytes = stage_work(counts, args.steps)[dom]
        ms, n = prof[dom]
        achieved = amount / (ms / 1e3)
        kname = KERNELS[dom]
        tr = traffic.get(kname)
        alg_per_launch = abytes / max(n, 1) if abytes else None
        roof = {"kernel": kname, "stage": dom, "bound": bound, "achieved": round(achieved, 3), "peak": peak,
                "unit": unit, "frac": round(achieved / peak, 4), "traffic": tr,
                "algorithmic_bytes_per_launch": round(alg_per_launch) if alg_per_launch else None,
                "traffic_ratio": round(tr / alg_per_launch, 3) if tr and alg_per_launch else None,
                "avg_launch_ms": round(ms / max(n, 1), 4), "launches": n,
                "timing": "HIP events around each launch of the stage inside the timed region "
                          f"({args.inflight} batches in flight)"}
        if tr is not None:
            roof["traffic_note"] = "HBM bytes per launch, rocprofv3 PMC (profiles/pmc_traffic.json)"

    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0 and args.workload == "c2":
        v, dt, nt, nf = cpu_baseline(args.cpu_sample)
        cpu = {"value": round(v, 4), "unit": "images/sec", "cores": nt, "kind": "port",
               "sample": f"oracle/sfm_oracle.c (scalar C restatement) on {nt} host threads, each extracting "
                         f"{args.cpu_sample} synthetic 1080p frames and matching their consecutive pair "
                         f"({nf} frames, {nt * (args.cpu_sample - 1)} pairs) in {dt:.1f} s"}

    if rank == 0:
        out = {
            "metric": "images/sec detect+describe+match, 1080p, 1/2/4/8 MI355X" if args.workload == "c2"
                      else "images/sec detect+describe+match, 4K 5-octave k=8000",
            "value": round(value, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic (deterministic integer-generated textured {H}x{W} frames, device-resident f32)",
            "config": {"workload": ("BASELINE configs[1]: 32x 1080p per GPU, ScaleRotInvSIFT 4-level x2 octave "
                                    "pyramid, k=2500, fw 18, NNRatio 0.85 over consecutive pairs"
                                    + (" (+ device ingest from 3840x2160 RGB)" if args.rgb_ingest else ""))
                       if args.workload == "c2" else
                       (f"BASELINE configs[4] per-GPU share: {B}x 4K per step, ScaleRotInvSIFT 5-level x2 "
                        "octave pyramid, k=8000, fw 18, NNRatio 0.85 over consecutive pairs"),
                       "frames_per_gpu": B, "image": [H, W], "pairs_per_gpu": int(P),
                       "keypoints_mean": float(np.mean(counts[:B])),
                       "matches_mean": float(np.mean(nmatch[nmatch >= 0])) if (nmatch >= 0).any() else 0.0,
                       "parallelism": f"image-shard x{world}", "batches_in_flight": args.inflight},
            "roofline": roof,
            "cpu_baseline": cpu,
            "stages_ms": stages,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_all_pairs(args, torch, dev):
    """BASELINE configs[2]: N (256) device-resident 1080p frames extracted (32 per batch,
    two batches in flight), then every one of the N(N-1)/2 pairs matched (the matcher's
    split-f16 MFMA prefilter + exact f32 re-rank).  One step = the whole job."""
    from sfmfromscratch_amd import synth
    from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, SlotTable, all_pairs
    N, Bx = args.frames or 256, 32
    host = np.stack([synth.make_frame_u8(H, W, 1234 + 1000 * (i // 32), i % 32) for i in range(N)])
    frames = torch.from_numpy(synth.u8_to_gray(host)).to(dev)
    del host
    lanes = []
    for _ in range(max(1, args.inflight)):
        ex = BatchExtractor(P_OCT, device=dev.index)
        ex.reserve(Bx, H, W)
        lanes.append((ex, torch.cuda.Stream(device=dev)))
    cap = lanes[0][0].cap
    slots = SlotTable(torch, N, cap, dev)
    matcher = BatchMatcher(RATIO, device=dev.index, ctx=lanes[0][0].ctx)
    pairs_np = all_pairs(N)
    pairs = torch.from_numpy(pairs_np).to(dev)
    P = len(pairs_np)
    CH = 4096  # pairs per matcher launch
    out = (torch.zeros((P, cap, 2), dtype=torch.int32, device=dev),
           torch.zeros((P, cap), dtype=torch.float32, device=dev),
           torch.zeros((P,), dtype=torch.int32, device=dev))

    class View:
        pass

    def step():
        cur = torch.cuda.current_stream()
        for b0 in range(0, N, Bx):
            ex, stm = lanes[(b0 // Bx) % len(lanes)]
            stm.wait_stream(cur)
            v = View()
            v.xy, v.desc, v.count = slots.xy[b0:b0 + Bx], slots.desc[b0:b0 + Bx], slots.count[b0:b0 + Bx]
            with torch.cuda.stream(stm):
                ex.extract(frames[b0:b0 + Bx], out=v)
        for _, stm in lanes:
            cur.wait_stream(stm)
        matcher.prep(slots)  # operands of every slot once, then the pair chunks
        for a in range(0, P, CH):
            matcher.match(slots, pairs[a:a + CH], out=(out[0][a:a + CH], out[1][a:a + CH], out[2][a:a + CH]),
                          prepped=True)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ctx = matcher.ctx
    ctx.profile_enable(True)
    ctx.profile_stages(["match"])
    ctx.profile_read(reset=True)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    elapsed = max(time.perf_counter() - t0, ev0.elapsed_time(ev1) / 1e3)
    prof = ctx.profile_read(reset=True)
    ctx.profile_enable(False)
    counts = slots.count.cpu().numpy().astype(np.int64)
    nm = out[2].cpu().numpy()
    elems = int(sum(counts[i] * counts[j] for i, j in pairs_np)) * 128 * args.steps
    ms, n = prof.get("match", (0.0, 0))
    ach = MATCH_FLOP_PER_ELEM * elems / 1e12 / (ms / 1e3) if ms else None
    print(json.dumps({
        "metric": "images/sec detect+describe+match, 1080p, all pairs (BASELINE configs[2])",
        "value": round(N * args.steps / elapsed, 3), "unit": "images/sec", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (deterministic integer-generated textured 1080p frames, device-resident f32)",
        "config": {"workload": f"BASELINE configs[2]: {N}x 1080p, ScaleRotInvSIFT 4-level x2 octave pyramid, "
                               f"k=2500, NNRatio 0.85 over all {P} pairs",
                   "frames": N, "pairs": P, "pairs_per_sec": round(P * args.steps / elapsed, 1),
                   "keypoints_mean": float(counts.mean()), "matches_mean": float(nm[nm >= 0].mean()),
                   "parallelism": "single GPU"},
        "roofline": {"kernel": KERNELS["match"], "stage": "match", "bound": "mfma",
                     "achieved": round(ach, 3) if ach else None, "peak": round(PEAK_MATCH_TFLOPS, 1),
                     "unit": "TFLOP/s", "frac": round(ach / PEAK_MATCH_TFLOPS, 4) if ach else None, "traffic": None,
                     "avg_launch_ms": round(ms / max(n, 1), 4), "launches": n,
                     "note": "GEMM-equivalent 2*n1*n2*128 flop per pair (SURVEY.md §8d) against the split-f16 "
                             "MFMA bound 2500/3 TFLOP/s"},
        "cpu_baseline": None}), flush=True)


def run_gather(args, torch, dist, dev, rank, world):
    """BASELINE configs[3]: n_global 1080p frames sharded over the ranks (rank r owns
    [r*S, (r+1)*S)), each shard extracted in 32-frame chunks with --inflight chunks on the
    GPU at once; every chunk's slot table (xy, desc, count; fixed capacity) is all-gathered
    over RCCL as soon as it is extracted (distributed.GatherPlan: chunk-major global
    table), so the gather of chunk c overlaps the extraction of chunk c+1, and the pairs
    that become ready with chunk c are matched on their own stream while later chunks are
    still being extracted.  One step = the whole job: every frame extracted once, the
    rank's pairs matched.  --exchange halo replaces the all-gather by the 1-slot
    point-to-point halo (consecutive pairs only need rank r+1's first frame).

    strong scaling: n_global fixed (default 2048) for every world size; weak: 256 frames
    per GPU.  Frames are device-resident uint8 (the u8 -> f32 gray conversion runs inside
    extraction), tiled from up to 64 distinct synthetic frames per rank to bound host
    generation time."""
    from sfmfromscratch_amd import distributed as D
    from sfmfromscratch_amd import synth
    from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, SlotTable

    Bx = 32
    n_global = args.frames or (2048 if args.scaling == "strong" else 256)
    if args.scaling == "weak":
        n_global *= world
    plan = D.GatherPlan(n_global, world, Bx, args.pairs)
    S, C = plan.S, plan.C
    halo = args.exchange == "halo"
    if halo and args.pairs != "consecutive":
        raise SystemExit("--exchange halo serves consecutive pairs only")
    # this rank's frames, uint8, device-resident
    U = min(S, 64)
    uniq = np.stack([synth.make_frame_u8(H, W, 1234, rank * S + i) for i in range(U)])
    uq = torch.from_numpy(uniq).to(dev)
    del uniq
    frames = uq[torch.arange(S, device=dev) % U].contiguous()
    del uq

    lanes = []
    for _ in range(max(1, args.inflight)):
        ex = BatchExtractor(P_OCT, device=dev.index)
        ex.reserve(Bx, H, W)
        lanes.append({"ex": ex, "stream": torch.cuda.Stream(device=dev)})
    cap = lanes[0]["ex"].cap
    matcher = BatchMatcher(RATIO, device=dev.index)  # own context: matches run on their own stream
    mstream = torch.cuda.Stream(device=dev)

    if halo:
        # local table: slots [0, S) = own frames in order, slot S = rank r+1's first frame
        table = SlotTable(torch, S + 1, cap, dev)
        lp = D.local_consecutive_pairs(S, rank, world)
        ready = np.minimum(lp[:, 1] // Bx, C - 1)  # pair (l, l+1) is ready with l+1's chunk
        sched = [lp[ready == c] for c in range(C)]
        rank_pairs_n = len(lp)
        for ln in lanes:
            ln["slots"] = None
    else:
        table = SlotTable(torch, n_global, cap, dev)
        if args.pairs == "all":
            sched = None
            rank_pairs_n = None
        else:
            rp = plan.rank_pairs(rank)
            sched = plan.schedule(rp)
            rank_pairs_n = len(rp)
        for ln in lanes:
            ln["slots"] = SlotTable(torch, Bx, cap, dev) if world > 1 else None

    def view(tab, lo, n):
        v = SlotTable.__new__(SlotTable)
        v.B, v.cap = n, tab.cap
        v.xy, v.desc, v.count = tab.xy[lo:lo + n], tab.desc[lo:lo + n], tab.count[lo:lo + n]
        return v

    def new_out(P):
        P = max(P, 1)
        return (torch.zeros((P, cap, 2), dtype=torch.int32, device=dev),
                torch.zeros((P, cap), dtype=torch.float32, device=dev),
                torch.zeros((P,), dtype=torch.int32, device=dev))

    CH = 4096  # 'all': pairs per matcher launch (output buffer reused)
    if sched is not None:
        sched_dev = [torch.from_numpy(np.ascontiguousarray(p, np.int32)).to(dev) for p in sched]
        outs = [new_out(len(p)) for p in sched]
    else:
        out_all = new_out(CH)
    all_pairs_np = plan.global_pairs() if args.pairs == "all" else None
    comm_bytes = {"sent": 0, "gathered": 0}
    slot_bytes = cap * (128 * 4 + 2 * 4) + 4

    def step():
        cur = torch.cuda.current_stream()
        for ln in lanes:
            ln["stream"].wait_stream(cur)
            ln["pending"] = None
        mstream.wait_stream(cur)
        for c in range(C):
            ln = lanes[c % len(lanes)]
            bc = plan.chunk_size(c)
            l0 = c * Bx
            works = None
            with torch.cuda.stream(ln["stream"]):
                if ln["pending"]:  # the lane's slots are free again once their gather is done
                    for w in ln["pending"]:
                        w.wait()
                if halo:
                    ln["ex"].extract(frames[l0:l0 + bc], out=view(table, l0, bc))
                    if c == 0 and world > 1:
                        D.halo_exchange(dist, table, S, rank, world)
                elif world == 1:
                    ln["ex"].extract(frames[l0:l0 + bc], out=view(table, plan.chunk_base(c), bc))
                else:
                    ln["ex"].extract(frames[l0:l0 + bc], out=view(ln["slots"], 0, bc))
                    works = D.allgather_chunk(dist, table, plan, c, ln["slots"], async_op=True)
                    ln["pending"] = works
            if sched is None:
                continue
            with torch.cuda.stream(mstream):
                if works:
                    for w in works:
                        w.wait()
                elif halo and c == C - 1:  # the halo slot arrived on chunk 0's lane
                    for other in lanes:
                        mstream.wait_stream(other["stream"])
                else:
                    mstream.wait_stream(ln["stream"])
                # this chunk's slots get their matcher operands once; pairs of earlier
                # chunks' slots reuse theirs
                if halo:
                    matcher.prep(table, l0, bc + (1 if c == C - 1 and world > 1 else 0))
                else:
                    matcher.prep(table, plan.chunk_base(c), world * bc)
                if len(sched[c]):
                    matcher.match(table, sched_dev[c], out=outs[c], prepped=True)
        for ln in lanes:
            cur.wait_stream(ln["stream"])
            if ln["pending"]:
                for w in ln["pending"]:
                    w.wait()
        cur.wait_stream(mstream)
        if sched is None:  # 'all': deal by cost once the counts are gathered (host sync)
            counts = table.count.cpu().numpy()
            mine = D.weighted_deal(all_pairs_np, counts[plan.slot_of(np.arange(n_global))], world)[rank]
            sp = torch.from_numpy(plan.slot_of(mine).reshape(-1, 2)).to(dev)
            matcher.prep(table)
            for a in range(0, len(sp), CH):
                n = min(CH, len(sp) - a)
                matcher.match(table, sp[a:a + n], out=(out_all[0][:n], out_all[1][:n], out_all[2][:n]),
                              prepped=True)
            step.pairs = len(mine)

    step.pairs = rank_pairs_n
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # collectives alone (untimed): the chunked all-gather with nothing else on the GPU
    comm = None
    if world > 1 and not halo:
        src = lanes[0]["slots"]
        reps = 3
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            for c in range(C):
                for w in D.allgather_chunk(dist, table, plan, c, src, async_op=True):
                    w.wait()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        sent = S * slot_bytes
        gathered = n_global * slot_bytes
        comm = {"kind": f"all_gather_into_tensor x3 fields per chunk ({dist.get_backend()})", "chunks": C,
                "bytes_sent_per_rank": sent, "bytes_gathered_per_rank": gathered,
                "ms_alone": round(dt * 1e3, 3), "algbw_GBps": round(gathered / dt / 1e9, 1)}
    elif world > 1:
        comm = {"kind": f"halo: 1 slot point-to-point send/recv ({dist.get_backend()})",
                "bytes_sent_per_rank": slot_bytes}

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = max(time.perf_counter() - t0, ev0.elapsed_time(ev1) / 1e3)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    counts = table.count.cpu().numpy()
    nm = (torch.cat([o[2][:max(len(p), 1)] for o, p in zip(outs, sched)]).cpu().numpy()
          if sched is not None else out_all[2].cpu().numpy())
    pairs_total = torch.tensor([step.pairs or 0], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(pairs_total)
    if rank == 0:
        print(json.dumps({
            "metric": "images/sec detect+describe+match, 1080p, 1/2/4/8 MI355X",
            "value": round(n_global * args.steps / elapsed, 2), "unit": "images/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (deterministic integer-generated textured 1080p frames, device-resident uint8, "
                    f"{U} distinct per rank, tiled)",
            "config": {"workload": f"BASELINE configs[3]: {n_global}x 1080p sharded {S} per GPU, ScaleRotInvSIFT "
                                   "4-level x2 octave pyramid, k=2500, NNRatio 0.85, "
                                   + ("1-slot halo exchange" if halo else "chunked RCCL all-gather of the "
                                      "descriptor tables") + f", {args.pairs} pairs",
                       "frames_global": n_global, "frames_per_gpu": S, "chunk": Bx, "chunks": C,
                       "pairs_global": int(pairs_total.item()), "pair_schedule": args.pairs,
                       "exchange": args.exchange, "keypoints_mean": float(counts.mean()),
                       "matches_mean_rank0": float(nm[nm >= 0].mean()) if (nm >= 0).any() else 0.0,
                       "parallelism": f"image-shard x{world}", "batches_in_flight": args.inflight},
            "collective": comm,
            "roofline": None,
            "cpu_baseline": None}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
