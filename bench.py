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
           "nms": "k_nms_tile<1,0,true>", "median": "k_med_scan", "topk": "k_topk", "pyramid": "k_down2x3",
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
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="frames per GPU per step")
    ap.add_argument("--cpu-sample", type=int, default=2,
                    help="frames per host thread in the CPU baseline sample (0 = skip)")
    ap.add_argument("--no-profile", action="store_true", help="disable the live per-stage HIP events")
    ap.add_argument("--workload", choices=["c2", "c3", "c5"], default="c2",
                    help="c2 = BASELINE configs[1] (the headline line); c3 = configs[2] (256 frames, all "
                         "pairs); c5 = configs[4]'s per-GPU share (4K, 5 octaves, k 8000)")
    ap.add_argument("--frames", type=int, default=256, help="c3: frames in the all-pairs job")
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
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    if args.workload == "c3":
        return run_all_pairs(args, torch, dev)
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
    pipe = BatchPipeline(P_OCT, RATIO, B, H, W, pairs, inflight=args.inflight, device=local, extra_slots=1)
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
        """Algorithmic work of `nsteps` steps per stage: (bound, amount, unit, peak)."""
        levels = [(H >> l, W >> l) for l in range(P_OCT["pyramid_level"])]
        px = sum(h * w for h, w in levels) * B * nsteps
        px_lo = sum(h * w for h, w in levels[1:]) * B * nsteps
        pair_elems = sum(int(counts[i]) * int(counts[j]) for i, j in pairs_np) * 128 * nsteps
        kps = int(counts[:B].sum()) * nsteps
        return {
            "harris": ("mfma", HARRIS_FLOP_PER_PX * px / 1e12, "TFLOP/s", PEAK_F32_TFLOPS),
            "match": ("mfma", MATCH_FLOP_PER_ELEM * pair_elems / 1e12, "TFLOP/s", PEAK_MATCH_TFLOPS),
            "nms": ("hbm", 4.0 * px / 1e9, "GB/s", PEAK_HBM_GBS),          # one read of R
            "pyramid": ("hbm", 4.0 * px_lo * 5 / 1e9, "GB/s", PEAK_HBM_GBS),  # read 4 px, write 1
            "describe": ("hbm", DESC_BYTES_PER_KP * kps / 1e9, "GB/s", PEAK_HBM_GBS),
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
                bound, amount, unit, peak = work[k]
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
        if os.path.exists(TRAFFIC_FILE):
            with open(TRAFFIC_FILE) as f:
                traffic = json.load(f).get("bytes_per_launch", {})
        bound, amount, unit, peak = stage_work(counts, args.steps)[dom]
        ms, n = prof[dom]
        achieved = amount / (ms / 1e3)
        kname = KERNELS[dom]
        tr = traffic.get(kname)
        roof = {"kernel": kname, "stage": dom, "bound": bound, "achieved": round(achieved, 3), "peak": peak,
                "unit": unit, "frac": round(achieved / peak, 4), "traffic": tr,
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
    N, Bx = args.frames, 32
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
        for a in range(0, P, CH):
            matcher.match(slots, pairs[a:a + CH], out=(out[0][a:a + CH], out[1][a:a + CH], out[2][a:a + CH]))

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


if __name__ == "__main__":
    main()
