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

Multi-GPU (`--gpus N`, one process per GPU): without WORLD_SIZE in the environment,
bench.py starts N ranks itself (a child `torch.distributed.run`, before anything touches
a GPU) and relays rank 0's line; under an outer torchrun it checks WORLD_SIZE == N.  At
N > 1 the default workload is BASELINE configs[3] (`c4`): 2,048 1080p frames in all
(strong scaling), sharded over the ranks, each chunk's descriptor tables all-gathered over
RCCL while the next chunk is extracted (distributed.ChunkedGatherJob), pairs matched as
their chunks arrive.  The line reports the efficiency T1 / (N * TN) against the same job
timed alone on rank 0's GPU, the collective's bytes per rank against the xGMI bound and
the fraction of the gather hidden behind extraction.  `--workload c2` at N > 1 is the
weak-scaling halo variant (32 frames per GPU, 1-slot point-to-point exchange).

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
# Describe (k_describe_q): modelled algorithmic lane-ops per keypoint at window width ws
#  against the FP32 lane-op rate (1024 SIMDs x 16 lanes x 2.4 GHz; the
# orientation sort's float64 min/max count twice, the f64 vector rate being half).
VALU_LANE_OPS = 1024 * 16 * 2.4e9


def describe_ops(ws: int) -> float:
    """Lane-ops per keypoint of the reference's describe at window width ws
    (ScaleRotInvSIFT.py:33-87): per pixel Sobel (2 x 6 fma), |g| (4) and atan2 (~28); the
    bitwise-exact np.histogram path sorts the ws*ws orientation keys (bitonic, P = pow2 >= N,
    4 slots per f64 compare-exchange), a prefix sum and 37 bin-edge searches; 16 cells each
    sort, prefix-sum and bin their pixels; 128-D normalise + sqrt (RootSIFT)."""
    import math
    n = ws * ws
    p = max(1 << max(0, math.ceil(math.log2(n))), 16)
    lg = int(math.log2(p))
    ops = 44.0 * n + 4.0 * (p // 2) * lg * (lg + 1) / 2 + n + 37 * math.ceil(math.log2(n + 1))
    c = max(1, n // 16)
    pc = 1 << math.ceil(math.log2(c)) if c > 1 else 1
    lc = int(math.log2(pc))
    ops += 16 * (2.0 * (pc // 2) * lc * (lc + 1) / 2 + c + 9 * math.ceil(math.log2(c + 1)))
    return ops + 128 * 4


KERNELS = {"harris": "k_harris<7>", "match": "k_match_mfma", "describe": "k_describe_q",
           "nms": "k_nms_stream<8,256>", "median": "k_med_scan", "topk": "k_topk", "pyramid": "k_down2x3",
           "match_prep": "k_match_prep", "match_post": "k_match_compact"}
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")  # tools/pmc_traffic.py


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# Switches whose results are wrong by design (timing ablations).  Only the diagnostic build of
# the library (make ABLATIONS=1) reads them at all; bench.py refuses to run with any of them
# set unless --ablation-run marks the line as a diagnostic, not a measurement.
ABLATION_SWITCHES = ("SFMFEAT_SKIP", "SFMFEAT_NMS_DRY")
ENV_PREFIXES = ("SFMFEAT_", "SFM_", "HIP_", "GPU_", "HSA_", "ROCR_", "BENCH_", "NCCL_", "RCCL_")


def ablation_switches_set(environ=None) -> list:
    """Names of the results-wrong-by-design switches present in the environment."""
    environ = os.environ if environ is None else environ
    return sorted(k for k in environ if k in ABLATION_SWITCHES or (k.startswith("SFMFEAT_") and k.endswith("_ABL")))


def bench_env(environ=None) -> dict:
    """Every SFMFEAT_* / SFM_* / HIP_* / GPU_* / HSA_* / ROCR_* / BENCH_* / NCCL_* / RCCL_* variable
    set for this run (recorded in the JSON line, so an A/B switch is visible in the result)."""
    environ = os.environ if environ is None else environ
    return {k: environ[k] for k in sorted(environ) if k.startswith(ENV_PREFIXES)}


def emit(out: dict, args) -> None:
    """Print the one JSON line with its provenance: the environment's switches, the library
    and its build flags; a diagnostic (--ablation-run) line says so in its metric."""
    from sfmfromscratch_amd import _native
    out["env"] = bench_env()
    out["library"] = _native.library_info()
    out["ablation_run"] = bool(args.ablation_run)
    if args.ablation_run:
        out["metric"] = "DIAGNOSTIC ablation run, not a measurement: " + out["metric"]
    print(json.dumps(out), flush=True)


def default_workload(world: int) -> str:
    """The workload `--gpus N` resolves to without --workload: BASELINE configs[1] (`c2`, 32
    frames per GPU) on one GPU, configs[3] (`c4`, 2,048 frames in all, strong scaling) on N > 1.
    The N > 1 line carries its own same-workload N = 1 figure (scaling_detail.t1_*), which is
    the reference point of its efficiency — not the c2 line."""
    return "c2" if world == 1 else "c4"


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


def span_stats(spans, steps: int, flop: float, peak_tflops: float) -> dict:
    """Roofline timing of the dominant kernel from its kernel-active spans (sfm_profile_spans:
    per launch {earliest workgroup start, latest workgroup end} on the device's realtime clock;
    `spans` holds one [n, 2] ns array per context, i.e. per lane, all on the same clock).

    Two attributions of the kernel's time to the step, both over the timed region's launches:
      - `union`: the measure of the union of all launches' intervals over every lane — the
        time during which at least one launch of the kernel is active.  Non-overlapping:
        two lanes' launches running at once count once, so it never exceeds the region;
      - `launch_sum`: the sum of the launch durations (rocprofv3 --kernel-trace's per-launch
        view): counts twice the time in which two lanes' launches overlap.
    The roofline's `achieved` / `frac` use the union; the launch sum is reported beside it."""
    iv = [np.asarray(s, dtype=np.int64).reshape(-1, 2) for s in spans]
    iv = np.concatenate(iv) if iv else np.zeros((0, 2), np.int64)
    iv = iv[(iv[:, 0] >= 0) & (iv[:, 1] >= iv[:, 0])]
    n = int(len(iv))
    if n == 0:
        return {"launches": 0}
    dur = (iv[:, 1] - iv[:, 0]).astype(np.float64)
    order = np.argsort(iv[:, 0], kind="stable")
    union, cur0, cur1 = 0, int(iv[order[0], 0]), int(iv[order[0], 1])
    for k in order[1:]:
        a, b = int(iv[k, 0]), int(iv[k, 1])
        if a > cur1:
            union += cur1 - cur0
            cur0, cur1 = a, b
        else:
            cur1 = max(cur1, b)
    union += cur1 - cur0
    sum_ms, union_ms = float(dur.sum()) / 1e6, union / 1e6
    return {"launches": n, "avg_launch_ms": round(sum_ms / n, 4),
            "launch_sum_ms_per_step": round(sum_ms / steps, 4), "union_ms_per_step": round(union_ms / steps, 4),
            "overlap_ms_per_step": round((sum_ms - union_ms) / steps, 4),
            "first_to_last_ms": round((int(iv[:, 1].max()) - int(iv[:, 0].min())) / 1e6, 4),
            "achieved_union": flop / 1e12 / (union_ms / 1e3), "achieved_launch_sum": flop / 1e12 / (sum_ms / 1e3),
            "frac_union": flop / 1e12 / (union_ms / 1e3) / peak_tflops,
            "frac_launch_sum": flop / 1e12 / (sum_ms / 1e3) / peak_tflops}


def roofline_guard(roof: dict | None, ms_per_step: float, tol: float = 0.01) -> list:
    """Consistency checks of a roofline entry against its own line (bench.py exits 4 when any
    fails): the dominant kernel's attributed time per step must not exceed the step, and its
    launch count must be positive.  `tol` absorbs the difference between the device's
    realtime clock (spans) and the host / event clock of ms_per_step."""
    bad = []
    if not roof:
        return bad
    if not roof.get("launches"):
        bad.append("roofline: no launches of the dominant kernel were timed")
        return bad
    att = roof.get("ms_per_step")
    if att is None or att > ms_per_step * (1.0 + tol):
        bad.append(f"roofline: {roof.get('kernel')} takes {att} ms per step by its own timing, more than the "
                   f"{ms_per_step} ms step")
    return bad


def spin_until(ev):
    """Poll `ev` until the GPU has passed it, so the host sees the end of the timed work
    without a blocking wait's wake-up delay (measured up to ~3 ms on the box: a 20-step
    timed region of ~17.7 ms on the GPU's events read 20.9 ms on the host clock); the
    torch.cuda.synchronize() that follows is the contract's bracket and returns at once."""
    while not ev.query():
        pass


def free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`--gpus N` without an outer launcher: start N rank processes with
    torch.distributed.run (one per GPU, rendezvous on 127.0.0.1) as a CHILD process —
    this process never touches a GPU and never execs — relay their output (rank 0 prints
    the JSON line) and return their exit code.  Refuses N above the visible devices,
    except in the gloo rehearsal mode (BENCH_DIST_BACKEND=gloo: ranks share GPUs)."""
    import subprocess
    probe = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                           capture_output=True, text=True)
    ngpu = int(probe.stdout.strip() or 0) if probe.returncode == 0 else 0
    if n > ngpu and os.environ.get("BENCH_DIST_BACKEND", "nccl") == "nccl":
        log(f"bench.py: --gpus {n} needs {n} visible GPUs, this node shows {ngpu}")
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    log("bench.py: launching", " ".join(cmd[1:]))
    return subprocess.run(cmd).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="frames per GPU per step")
    ap.add_argument("--cpu-sample", type=int, default=8,
                    help="frames per host thread in the CPU baseline sample (0 = skip)")
    ap.add_argument("--no-profile", action="store_true", help="skip the untimed per-stage HIP-event pass (stages_ms)")
    ap.add_argument("--no-spans", action="store_true",
                    help="no kernel-active spans of the Harris launches in the timed region (no roofline)")
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5"], default=None,
                    help="default: c2 at one GPU, c4 at N > 1.  "
                         "c2 = BASELINE configs[1] (the headline line); c3 = configs[2] (256 frames, all "
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
    ap.add_argument("--inflight", type=int, default=int(os.environ.get("BENCH_INFLIGHT", "2")),
                    help="batches in flight (double-buffered contexts / slot tables, pipeline.BatchPipeline)")
    ap.add_argument("--ablation-run", action="store_true",
                    help="allow the timing-ablation switches (" + ", ".join(ABLATION_SWITCHES) + ", SFMFEAT_*_ABL; "
                         "diagnostic library only): the line is then marked as a diagnostic, not a measurement")
    ap.add_argument("--same-batch", action="store_true",
                    help="c2: submit the same 32 frames every step (default: two distinct batches alternate, so "
                         "no step re-reads the frames of the step before it)")
    ap.add_argument("--emulate-exchange", type=int, default=0, metavar="WG",
                    help="c4 at one GPU: a single-GPU rehearsal of one rank of an --emulate-world-rank job: after "
                         "each chunk's extraction a WG-workgroup device copy of the bytes that rank would receive "
                         "(count-compacted all-gather) on a high-priority stream beside the extraction; "
                         "reports the extraction slowdown and the hidden fraction of the emulated exchange")
    ap.add_argument("--emulate-world", type=int, default=8)
    ap.add_argument("--verify", action="store_true",
                    help="c4: after the timed run, re-extract a sample of frames and re-match a sample of this "
                         "rank's pairs with the plain (unchunked) calls and require bit-equal results")
    args = ap.parse_args()

    abl = ablation_switches_set()
    if abl and not args.ablation_run:
        log(f"bench.py: refusing to measure with timing-ablation switches set ({', '.join(abl)}): their results "
            "are wrong by design (pass --ablation-run for a diagnostic line)")
        sys.exit(3)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if args.workload is None:
        args.workload = default_workload(world)

    import torch
    import torch.distributed as dist

    ngpu = torch.cuda.device_count()
    if ngpu < 1:
        raise SystemExit("bench.py: no GPU visible")
    if world > 1:
        # BENCH_DIST_BACKEND=gloo: rehearsal of the multi-rank code paths with several ranks
        # on one GPU (RCCL needs one GPU per rank); measurements use RCCL
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
        if backend == "nccl" and world > ngpu:
            raise SystemExit(f"bench.py: {world} RCCL ranks need {world} GPUs, this node shows {ngpu}")
    torch.cuda.set_device(local % ngpu)
    dev = torch.device("cuda", local % ngpu)
    if world > 1:
        if backend == "nccl":
            from sfmfromscratch_amd.distributed import nccl_options
            dist.init_process_group("nccl", device_id=dev, pg_options=nccl_options(dist))
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
    batches = None
    if args.rgb_ingest:  # decoded RGB at twice the size; the gray frames are made on the device
        uniq = [synth.make_frame_rgb_u8(2 * H, 2 * W, 1234, rank * B + i) for i in range(min(B, 8))]
        rgb = torch.from_numpy(np.stack([uniq[i % len(uniq)] for i in range(B)])).to(dev)
        del uniq
        frames = torch.empty((B, H, W), dtype=torch.float32, device=dev)
    else:
        # two distinct batches (frames [2rB, 2rB + B) and [2rB + B, 2rB + 2B) of the global
        # sequence) alternate step by step, so no step re-reads the frames the step before it
        # read (one batch is 265 MB, the Infinity Cache 256 MB); --same-batch for the A/B
        nb = 1 if args.same_batch else 2
        batches = []
        for j in range(nb):
            frames_u8 = np.stack([synth.make_frame_u8(H, W, 1234, (rank * nb + j) * B + i) for i in range(B)])
            batches.append(torch.from_numpy(synth.u8_to_gray(frames_u8)).to(dev))
            del frames_u8
        frames = batches[0]
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
            pipe.submit(batches[pipe.n % len(batches)] if not same_batch[0] else frames, hook=halo)
    same_batch = [False]  # set for the same-batch comparison pass after the timed region

    def stage_work(counts, nsteps):
        """Algorithmic work of `nsteps` steps per stage:
        (bound, amount, unit, peak, algorithmic HBM bytes or None).  Latency-bound stages
        (describe, top-k, median) get no roofline.  `counts`: each lane's slot counts (the
        lanes take the steps in turn, and with alternating batches each lane its own batch)."""
        levels = [(H >> l, W >> l) for l in range(P_OCT["pyramid_level"])]
        px = sum(h * w for h, w in levels) * B * nsteps
        pair_elems = float(np.mean([sum(int(c[i]) * int(c[j]) for i, j in pairs_np) for c in counts])) * 128 * nsteps
        # k_down2x3 reads level 0 once and writes levels 1..3 (one launch); a 5th level is
        # one k_down2 from level 3.  Levels 1..3 exact 2x (H, W multiples of 8): the level-0
        # k_harris launch writes them from its image tiles (sfmfeat_api.hip, SFMFEAT_PYR_FUSED),
        # so their bytes move to the Harris stage and the pyramid stage keeps levels >= 4
        A = [h * w for h, w in levels]
        fused = (len(A) >= 4 and H % 8 == 0 and W % 8 == 0 and
                 os.environ.get("SFMFEAT_PYR_FUSED", "1") != "0")
        tail_px = sum(A[l - 1] + A[l] for l in range(4, len(A)))
        pyr_px = tail_px if fused else A[0] + sum(A[1:4]) + tail_px
        pyr_bytes = 4.0 * pyr_px * B * nsteps
        harris_bytes = 8.0 * px + (4.0 * sum(A[1:4]) * B * nsteps if fused else 0.0)
        work = {
            # VALU-bound: 328 flop/px of separate mul/add-class ops; bytes: read
            # the level, write R (+ the fused pyramid levels)
            "harris": ("valu", HARRIS_FLOP_PER_PX * px / 1e12, "TFLOP/s", PEAK_F32_TFLOPS, harris_bytes),
            "match": ("mfma", MATCH_FLOP_PER_ELEM * pair_elems / 1e12, "TFLOP/s", PEAK_MATCH_TFLOPS, None),
            "nms": ("hbm", 4.0 * px / 1e9, "GB/s", PEAK_HBM_GBS, 4.0 * px),          # one read of R
        }
        if pyr_px > 0:
            work["pyramid"] = ("hbm", pyr_bytes / 1e9, "GB/s", PEAK_HBM_GBS, pyr_bytes)
        return work

    def level_keypoints():
        """Keypoints per pyramid level over the batch (host-path extraction of the same frames,
        outside every timed region): the describe floor's keypoint counts."""
        if args.rgb_ingest:
            return None
        from sfmfromscratch_amd import _native, _abi
        ctx = _native.Context(_abi.params_from_dict(P_OCT, _abi.SFM_MODE_SCALEROT), device=dev.index)
        tot = np.zeros(P_OCT["pyramid_level"], np.int64)
        host = frames.cpu().numpy()
        for i in range(B):
            tot += ctx.extract(host[i])[4]
        ctx.close()
        return tot

    def describe_floor(lvl_kp, nsteps):
        """(floor ms, modelled lane-ops) of the describe stage over nsteps steps."""
        fws = [max(3, int(P_OCT["feature_width"] / (P_OCT["pyramid_scale_factor"] ** l)))
               for l in range(P_OCT["pyramid_level"])]
        ops = sum(int(k) * describe_ops(2 * (fw // 2)) for k, fw in zip(lvl_kp, fws)) * nsteps
        return ops / VALU_LANE_OPS * 1e3, ops

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
        return [ln["slots"].count.cpu().numpy() for ln in pipe.lanes]

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
        if "pyramid" in stages and "pyramid" not in work:
            stages["pyramid"]["note"] = ("levels 1-3 written by the level-0 k_harris launch (their bytes are "
                                         "in the harris stage); the stage's events bracket no launch here")
        if "topk" in stages:
            stages["topk"].update({"bound": "latency", "workgroups_per_launch": B,
                                   "note": "one 1,024-thread workgroup per plane and level: a dependent chain of "
                                           "barriers (radix digit passes, run sorts; the exact path's plane "
                                           "reads on exact levels); no byte or flop roofline applies"})
        dom = max((k for k in prof_all if k in work and prof_all[k][1]), key=lambda k: prof_all[k][0])
        prof_enable(False)
        prof_read()

    def run_steps(nsteps, step_events=None):
        """nsteps steps of the two-lane pipeline from an idle GPU; with step_events, one
        timing event per step on its lane's stream right after its match (the step's end)."""
        pipe.start()
        for _ in range(nsteps):
            h0 = time.perf_counter()
            step()
            if step_events is not None:
                host_ms.append((time.perf_counter() - h0) * 1e3)
                e = torch.cuda.Event(enable_timing=True)
                e.record(pipe.lanes[(pipe.n - 1) % pipe.inflight]["stream"])
                step_events.append(e)
        pipe.join()

    # W warm-up steps: the same two-lane pipeline as the timed steps, right before them
    run_steps(args.warmup)
    pipe.n = 0  # the timed steps start on lane 0 with the first batch
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    step_ev, host_ms = [], []
    # the roofline's timing: kernel-active spans of every Harris launch inside the timed
    # region itself (one atomic per workgroup; no events around the launches)
    span_on = not args.no_spans
    if span_on:
        for c in ctxs:
            c.profile_spans(P_OCT["pyramid_level"] * (args.steps + 4))
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    run_steps(args.steps, step_ev)
    t_sub = time.perf_counter() - t0
    ev1.record()
    spin_until(ev1)
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
    spans = []
    if span_on:
        for c in ctxs:
            sp, _, dropped = c.profile_spans_read()
            if dropped:
                raise SystemExit(f"bench.py: {dropped} Harris launches beyond the span capacity")
            spans.append(sp)
            c.profile_spans(0)
    # the timed region's workload (keypoints per slot, matches per pair), before any later pass
    # overwrites the lanes' tables
    counts_l = lane_counts()
    nmatch = np.concatenate([ln["mout"][2].cpu().numpy() for ln in pipe.lanes])
    # per-step end times inside the timed region (not part of `value`)
    step_end = [ev0.elapsed_time(e) for e in step_ev]
    step_detail = {"end_ms": [round(x, 4) for x in step_end],
                   "first_step_ms": round(step_end[0], 4) if step_end else None,
                   # period between the first and the second-to-last step ends: the last step
                   # ends early (its batch runs alone once the other lane has drained)
                   "steady_ms_per_step": (round((step_end[-2] - step_end[0]) / (len(step_end) - 2), 4)
                                          if len(step_end) > 3 else None),
                   "host_submit_ms": round(t_sub * 1e3, 3),
                   "host_step_submit_ms_max": round(max(host_ms), 3) if host_ms else None,
                   "host_step_submit_ms_median": round(float(np.median(host_ms)), 3) if host_ms else None}

    # the same K steps again with one batch submitted every step (the pre-round-5 workload): the
    # line reports its rate beside `value` (alternating batches) as the cost of never re-reading
    # the previous step's frames.  Right after the timed region and after its own warm-up, before
    # the host-path extraction below idles the GPU (a 20-step pass started on dropped clocks
    # read 10 % slow)
    same_value = None
    if batches is not None and len(batches) > 1:
        same_batch[0] = True
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        pipe.n = 0
        run_steps(args.warmup)  # untimed, like the headline's warm-up (clocks, caches, lanes)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        pipe.n = 0
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = time.perf_counter()
        s0.record()
        run_steps(args.steps)
        s1.record()
        spin_until(s1)
        torch.cuda.synchronize()
        el = max(time.perf_counter() - ts, s0.elapsed_time(s1) / 1e3)
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        same_value = world * B * args.steps / el
        same_batch[0] = False

    # the describe floor's keypoint counts: a host-path extraction (PCIe copies, the GPU
    # mostly idle), so after the timed region rather than between the profile pass and the
    # warm-up, where it would let the GPU's clocks drop right before timing
    if stages and "describe" in stages:
        lvl_kp = level_keypoints()
        if lvl_kp is not None:
            fl_ms, ops = describe_floor(lvl_kp, nprof)
            d = stages["describe"]
            d.update({"bound": "valu", "achieved": round(ops / (prof_all["describe"][0] / 1e3) / 1e12, 3),
                      "unit": "T lane-op/s", "floor_ms_per_step": round(fl_ms / nprof, 4),
                      "frac": round(fl_ms / prof_all["describe"][0], 4),
                      "keypoints_per_level": [int(v) for v in lvl_kp],
                      "note": "modelled lane-ops per keypoint (bench.describe_ops) / 39.3 T lane-op/s"})

    images = world * B * args.steps
    value = images / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    roof = None
    if spans:
        traffic = {}
        # the committed PMC traffic was measured on the headline workload (c2) only
        if os.path.exists(TRAFFIC_FILE) and args.workload == "c2" and not args.rgb_ingest:
            with open(TRAFFIC_FILE) as f:
                traffic = json.load(f).get("bytes_per_launch", {})
        bound, amount, unit, peak, abytes = stage_work(counts_l, args.steps)["harris"]
        st = span_stats(spans, args.steps, amount * 1e12, peak)
        n = st["launches"]
        kname = KERNELS["harris"]
        tr = traffic.get(kname)
        alg_per_launch = abytes / max(n, 1) if abytes and n else None
        roof = {"kernel": kname, "stage": "harris", "bound": bound,
                "achieved": round(st["achieved_union"], 3) if n else None, "peak": peak, "unit": unit,
                "frac": round(st["frac_union"], 4) if n else None, "traffic": tr,
                "algorithmic_bytes_per_launch": round(alg_per_launch) if alg_per_launch else None,
                "traffic_ratio": round(tr / alg_per_launch, 3) if tr and alg_per_launch else None,
                "ms_per_step": st.get("union_ms_per_step"), "avg_launch_ms": st.get("avg_launch_ms"),
                "launches": n,
                "launch_sum": ({"ms_per_step": st["launch_sum_ms_per_step"],
                                "achieved": round(st["achieved_launch_sum"], 3),
                                "frac": round(st["frac_launch_sum"], 4),
                                "overlap_ms_per_step": st["overlap_ms_per_step"],
                                "note": "sum of the launch durations (rocprofv3 --kernel-trace's per-launch view): "
                                        "counts twice the time two lanes' Harris launches overlap"} if n else None),
                "dominant_stage_by_events": dom,
                "timing": (f"kernel-active spans (sfm_profile_spans: earliest workgroup start to latest workgroup "
                           f"end of each launch, device realtime clock) of every Harris launch inside the timed "
                           f"region ({args.inflight} batches in flight); ms_per_step / achieved / frac = the "
                           f"union of the launches' intervals over all lanes (non-overlapping attribution)")}
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
            "ms_per_step": round(ms_per_step, 3),
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
                       "distinct_batches": len(batches) if batches is not None else 1,
                       "keypoints_mean": float(np.mean([c[:B].mean() for c in counts_l])),
                       "matches_mean": float(np.mean(nmatch[nmatch >= 0])) if (nmatch >= 0).any() else 0.0,
                       "parallelism": f"image-shard x{world}", "batches_in_flight": args.inflight},
            "roofline": roof,
            "cpu_baseline": cpu,
            "stages_ms": stages,
            "steps_detail": step_detail,
            "batches_detail": ({"distinct_batches": len(batches), "alternation": "step i submits batch i % 2 "
                                "(frames [2rB, 2rB+B) / [2rB+B, 2rB+2B)); lane i % 2 runs it",
                                "value_same_batch_every_step": round(same_value, 2),
                                "delta_pct_vs_same_batch": round(100.0 * (value - same_value) / same_value, 2)}
                               if same_value else None),
        }
        emit(out, args)
        bad = roofline_guard(roof, ms_per_step)
        if bad:
            log("bench.py: " + "; ".join(bad))
            sys.exit(4)
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
    spin_until(ev1)
    torch.cuda.synchronize()
    elapsed = max(time.perf_counter() - t0, ev0.elapsed_time(ev1) / 1e3)
    prof = ctx.profile_read(reset=True)
    ctx.profile_enable(False)
    counts = slots.count.cpu().numpy().astype(np.int64)
    nm = out[2].cpu().numpy()
    elems = int(sum(counts[i] * counts[j] for i, j in pairs_np)) * 128 * args.steps
    ms, n = prof.get("match", (0.0, 0))
    ach = MATCH_FLOP_PER_ELEM * elems / 1e12 / (ms / 1e3) if ms else None
    emit({
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
        "cpu_baseline": None}, args)


XGMI_LINK_GBS = 153.0  # per xGMI link per direction (task spec); the 8-GPU node is a full mesh


def run_gather(args, torch, dist, dev, rank, world):
    """BASELINE configs[3]: n_global 1080p frames sharded over the ranks (rank r owns
    [r*S, (r+1)*S)), extracted in 32-frame chunks, every chunk's slot table all-gathered
    over RCCL as soon as it is extracted and the pairs ready with it matched on their own
    stream (distributed.ChunkedGatherJob).  One step = the whole job: every frame
    extracted once, the rank's pairs matched.

    Reported next to the throughput (at N > 1):
      - efficiency = T1 / (N * TN): T1 is the same n_global-frame job timed alone on rank
        0's GPU (world 1: no exchange) before the multi-rank run;
      - collective: bytes per rank, the gather's time alone, its xGMI bound (full mesh, one
        link per peer) and `hidden_fraction` = 1 - (TN - T_compute) / T_gather_alone, with
        T_compute the same job with the collectives skipped;
      - the exchange is verified bit for bit once, after warm-up (per-frame checksums of
        what each owner sent vs. what every rank's table holds).
    strong scaling: n_global fixed (default 2048) for every N; weak: 256 frames per GPU.
    Frames are device-resident float32 gray (u8 / 255, converted before timing as for the
    configs[1] headline: until round 5 this job took u8 frames and timed the conversion,
    ~80 us per 32-frame chunk, which configs[1] does not), tiled from up to 64 distinct
    synthetic frames per rank."""
    from sfmfromscratch_amd import distributed as D
    from sfmfromscratch_amd import synth

    Bx = 32
    n_global = args.frames or (2048 if args.scaling == "strong" else 256)
    if args.scaling == "weak":
        n_global *= world
    plan = D.GatherPlan(n_global, world, Bx, args.pairs)
    S, C = plan.S, plan.C
    U = min(S, 64)

    def frames_of(r, n):  # rank r's first n local frames, device-resident float32 gray
        uniq = np.stack([synth.u8_to_gray(synth.make_frame_u8(H, W, 1234, r * S + i)) for i in range(min(U, n))])
        uq = torch.from_numpy(uniq).to(dev)
        return uq[torch.arange(n, device=dev) % uq.shape[0]].contiguous()

    def frame_of(r, l):  # rank r's local frame l, [1, H, W] u8 (the same tiling as frames_of)
        return torch.from_numpy(synth.make_frame_u8(H, W, 1234, r * S + l % U)[None]).to(dev)

    def timed(job, frames, steps, **kw):
        if job.plan.world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record()
        for _ in range(steps):
            job.run(frames, **kw)
        ev1.record()
        spin_until(ev1)
        torch.cuda.synchronize()
        if job.plan.world > 1:
            dist.barrier()
        el = max(time.perf_counter() - t0, ev0.elapsed_time(ev1) / 1e3)
        if job.plan.world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el / steps

    # T1: the same job on rank 0's GPU alone (the reference point of the efficiency)
    t1 = None
    if world > 1 and args.scaling == "strong":
        if rank == 0:
            plan1 = D.GatherPlan(n_global, 1, Bx, args.pairs)
            job1 = D.ChunkedGatherJob(P_OCT, RATIO, plan1, 0, H, W, inflight=args.inflight, device=dev.index)
            f1 = frames_of(0, n_global)
            job1.run(f1)
            t1 = timed(job1, f1, max(2, min(args.steps, 10)))
            del job1, f1
            torch.cuda.empty_cache()
            log(f"rank 0 alone: {n_global} frames in {t1 * 1e3:.2f} ms")
        dist.barrier()

    if args.emulate_exchange > 0:
        if world != 1:
            raise SystemExit("--emulate-exchange is a single-GPU rehearsal (run it with --gpus 1)")
        return run_emulated_exchange(args, torch, dev, D, plan, frames_of(rank, S), timed, n_global)
    job = D.ChunkedGatherJob(P_OCT, RATIO, plan, rank, H, W, dist=dist if world > 1 else None,
                             inflight=args.inflight, exchange=args.exchange, device=dev.index)
    frames = frames_of(rank, S)
    for _ in range(max(1, args.warmup)):
        job.run(frames, record_sent=world > 1)
    torch.cuda.synchronize()
    verified = None
    if world > 1 and not job.halo:
        bad = job.verify_exchange()
        if bad:  # a wrong exchange ends the run: no silent switch to another collective
            raise SystemExit(f"exchange check failed: {bad} of {n_global} gathered frames differ from their owner's "
                             f"({'coalesced' if job.coalesce else 'per-field'} all-gather)")
        verified = n_global

    comm = None
    t_compute = t_alone = None
    if world > 1:
        t_compute = timed(job, frames, max(2, min(args.steps, 10)), exchange=False)
        sent = S * job.slot_bytes
        if not job.halo:
            # bytes of the last (timed-shape) run: count-compacted rows, against full slots
            recv, recv_full = job.gathered_bytes()
            t_alone = job.gather_alone()
            gathered = recv * world // (world - 1)
            sent = recv // (world - 1)
            bound = recv / ((world - 1) * XGMI_LINK_GBS * 1e9)
            kind = ("count-compacted: counts, then each chunk's first M rows (M = its largest count), "
                    if job.compact else "full-capacity slots, ")
            kind += ("grouped all_gather_into_tensor per chunk" if job.coalesce else "one all_gather_into_tensor "
                     "per field per chunk") + f" ({dist.get_backend()})"
            comm = {"kind": kind, "chunks": C, "bytes_sent_per_rank": sent, "bytes_gathered_per_rank": gathered,
                    "bytes_received_per_rank": recv, "bytes_received_full_slots": recv_full,
                    "padding_bytes_saved_per_rank": recv_full - recv,
                    "rows_per_chunk_mean": round(float(np.mean(job.gathered_rows)), 1) if job.gathered_rows else None,
                    "ms_alone": round(t_alone * 1e3, 3),
                    "algbw_GBps": round(gathered / t_alone / 1e9, 1),
                    "xgmi_bound_ms": round(bound * 1e3, 3), "xgmi_bound_frac": round(bound / t_alone, 3),
                    "xgmi_bound_note": f"received bytes over (N-1) xGMI links at {XGMI_LINK_GBS:.0f} GB/s each "
                                       "(full mesh, one link per peer)",
                    "verified_frames": verified}
        else:
            comm = {"kind": f"halo: 1 slot point-to-point send/recv ({dist.get_backend()})",
                    "bytes_sent_per_rank": job.slot_bytes}

    # timed region; Harris (the dominant kernel) timed by its kernel-active spans on rank 0's lanes
    ctxs = [ln["ex"].ctx for ln in job.lanes]
    if not args.no_spans:
        for c in ctxs:
            c.profile_spans(P_OCT["pyramid_level"] * C * (args.steps + 1))
    tn = timed(job, frames, args.steps)
    roof = None
    if not args.no_spans:
        spans = []
        for c in ctxs:
            sp, _, dropped = c.profile_spans_read()
            spans.append(sp)
            c.profile_spans(0)
            if dropped:
                raise SystemExit(f"bench.py: {dropped} Harris launches beyond the span capacity")
        px = sum((H >> l) * (W >> l) for l in range(P_OCT["pyramid_level"])) * S * args.steps
        st = span_stats(spans, args.steps, HARRIS_FLOP_PER_PX * px, PEAK_F32_TFLOPS)
        if st["launches"]:
            roof = {"kernel": KERNELS["harris"], "stage": "harris", "bound": "valu",
                    "achieved": round(st["achieved_union"], 3), "peak": PEAK_F32_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(st["frac_union"], 4), "traffic": None, "ms_per_step": st["union_ms_per_step"],
                    "avg_launch_ms": st["avg_launch_ms"], "launches": st["launches"],
                    "launch_sum": {"ms_per_step": st["launch_sum_ms_per_step"],
                                   "frac": round(st["frac_launch_sum"], 4)},
                    "timing": "kernel-active spans of every Harris launch of this rank inside the timed region; "
                              "frac from the union of their intervals over the lanes"}

    if args.verify:
        verify_gather_job(args, torch, dist, dev, job, frame_of, world, rank)

    counts = job.table.count.cpu().numpy()
    nm = (torch.cat([o[2][:max(len(p), 1)] for o, p in zip(job.outs, job.sched)]).cpu().numpy()
          if job.sched is not None else job.out_all[2].cpu().numpy())
    pairs_total = torch.tensor([job.pairs_matched or 0], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(pairs_total)
    eff = None
    if t1 is not None:
        eff = {"efficiency": round(t1 / (world * tn), 4), "t1_ms": round(t1 * 1e3, 3), "tn_ms": round(tn * 1e3, 3),
               "t1_images_per_s": round(n_global / t1, 2), "tn_images_per_s": round(n_global / tn, 2),
               "definition": "T1 / (N * TN): T1 = the same job alone on rank 0's GPU (no exchange)",
               "note": "the N = 1 reference of this line is t1_images_per_s (the same configs[3] job on one GPU), "
                       "not the N = 1 headline line (configs[1], 32 frames per step)"}
    if comm is not None and t_compute is not None:
        comm["compute_only_ms"] = round(t_compute * 1e3, 3)
        if t_alone:
            comm["hidden_fraction"] = round(min(1.0, max(0.0, 1.0 - (tn - t_compute) / t_alone)), 4)
            comm["hidden_note"] = "1 - (TN - T_compute) / T_gather_alone; T_compute = the job with collectives skipped"
    if rank == 0:
        emit({
            "metric": "images/sec detect+describe+match, 1080p, 1/2/4/8 MI355X",
            "value": round(n_global / tn, 2), "unit": "images/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(tn * 1e3, 3),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (deterministic integer-generated textured 1080p frames, device-resident float32 "
                    f"gray (u8 / 255 before timing), {U} distinct per rank, tiled)",
            "config": {"workload": f"BASELINE configs[3]: {n_global}x 1080p sharded {S} per GPU, ScaleRotInvSIFT "
                                   "4-level x2 octave pyramid, k=2500, NNRatio 0.85, "
                                   + ("1-slot halo exchange" if job.halo else "chunked RCCL all-gather of the "
                                      "descriptor tables") + f", {args.pairs} pairs",
                       "frames_global": n_global, "frames_per_gpu": S, "chunk": Bx, "chunks": C,
                       "pairs_global": int(pairs_total.item()), "pair_schedule": args.pairs,
                       "exchange": args.exchange, "keypoints_mean": float(counts.mean()),
                       "matches_mean_rank0": float(nm[nm >= 0].mean()) if (nm >= 0).any() else 0.0,
                       "parallelism": f"image-shard x{world}", "batches_in_flight": args.inflight},
            "scaling_detail": eff,
            "collective": comm,
            "roofline": roof,
            "cpu_baseline": None}, args)
        bad = roofline_guard(roof, tn * 1e3)
        if bad:
            log("bench.py: " + "; ".join(bad))
            sys.exit(4)
    if world > 1:
        dist.destroy_process_group()


def run_emulated_exchange(args, torch, dev, D, plan, frames, timed, n_global):
    """--emulate-exchange WG (configs[3] readiness on one GPU): the job of one
    rank of an N-rank run (--frames = its shard, e.g. 256 = 2,048 / 8), first alone (T_compute),
    then with an emulated exchange per chunk (T_emu): a WG-workgroup copy of the bytes the rank
    would receive — (N - 1) x 32 frames x (M rows x 520 B + 4), M the largest keypoint count —
    on a high-priority stream beside the extraction; the rank's own pairs do not wait for it, as
    in the multi-rank job (distributed.ChunkedGatherJob `emulate`); the job ends after the last
    copy.  hidden_fraction = 1 - (T_emu - T_compute) / T_copies_alone.  It measures the
    collective's CU and HBM contention with extraction, not xGMI latency."""
    job = D.ChunkedGatherJob(P_OCT, RATIO, plan, 0, H, W, inflight=args.inflight, device=dev.index)
    for _ in range(max(1, args.warmup)):
        job.run(frames)
    torch.cuda.synchronize()
    rows = int(job.table.count.max().item())
    t_compute = timed(job, frames, args.steps)
    emu = {"world": args.emulate_world, "workgroups": args.emulate_exchange, "rows": rows}
    ejob = D.ChunkedGatherJob(P_OCT, RATIO, plan, 0, H, W, inflight=args.inflight, device=dev.index, emulate=emu)
    for _ in range(max(1, args.warmup)):
        ejob.run(frames)
    torch.cuda.synchronize()
    t_emu = timed(ejob, frames, args.steps)
    t_alone = ejob.emulated_gather_alone()
    t_compute2 = timed(job, frames, args.steps)  # again after, against drift
    t_c = min(t_compute, t_compute2)
    e = ejob.emulate
    comm = {"kind": (f"EMULATED exchange on one GPU: per chunk a {e['workgroups']}-workgroup device copy of the "
                     f"{e['bytes_per_chunk']} B one rank of a {e['world']}-rank job receives (count-compacted rows, "
                     f"M = {rows}) on a high-priority stream beside the extraction; the rank's own pairs do not "
                     "wait for it, the job ends after the last copy"),
            "emulated_world": e["world"], "workgroups": e["workgroups"], "rows": rows,
            "bytes_per_chunk": e["bytes_per_chunk"], "chunks": plan.C,
            "copies_alone_ms": round(t_alone * 1e3, 3),
            "copies_alone_GBps": round(e["bytes_per_chunk"] * plan.C / t_alone / 1e9, 1),
            "compute_only_ms": round(t_c * 1e3, 3), "compute_only_ms_runs": [round(t_compute * 1e3, 3),
                                                                             round(t_compute2 * 1e3, 3)],
            "job_with_emulated_exchange_ms": round(t_emu * 1e3, 3),
            "extraction_slowdown": round(t_emu / t_c, 4),
            "hidden_fraction": round(min(1.0, max(0.0, 1.0 - (t_emu - t_c) / t_alone)), 4),
            "hidden_note": "1 - (T_emu - T_compute) / T_copies_alone"}
    emit({
        "metric": "DIAGNOSTIC single-GPU rehearsal (emulated exchange), not a multi-GPU measurement: "
                  "images/sec detect+describe+match, 1080p, one rank's shard",
        "value": round(plan.S / t_emu, 2), "unit": "images/sec", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(t_emu * 1e3, 3), "higher_is_better": True,
        "scaling": args.scaling, "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (deterministic integer-generated textured 1080p frames, device-resident float32 gray)",
        "config": {"workload": f"BASELINE configs[3] readiness: one rank's {plan.S}-frame shard of an "
                               f"{e['world']}-rank job, 32-frame chunks, emulated all-gather per chunk",
                   "frames_per_gpu": plan.S, "chunk": plan.chunk, "parallelism": "single GPU (emulation)",
                   "batches_in_flight": args.inflight, "n_global_arg": n_global},
        "collective": comm, "roofline": None, "cpu_baseline": None}, args)


def verify_gather_job(args, torch, dist, dev, job, frame_of, world, rank):
    """--verify: sample frames (every rank's first and last) re-extracted here with a plain
    BatchExtractor must equal their gathered table slots bit for bit, and a sample of this
    rank's pairs re-matched with the plain (unprepped) matcher on copies of their gathered
    slots must equal the chunked job's matches.  No oracle: bench.py checks the chunked path against the
    single-call path (the GPU tests pin both to the oracle)."""
    from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, SlotTable
    plan = job.plan
    ex = BatchExtractor(P_OCT, device=dev.index)
    fr = {}
    for r in range(world):
        for l in sorted({0, plan.S - 1}):
            fr[r * plan.S + l] = frame_of(r, l)
    bad = 0
    for g, f in fr.items():
        s = ex.extract(f.contiguous())
        t = int(plan.slot_of(g)) if not job.halo else None
        if t is None:
            continue
        n = int(s.count[0])
        ok = (n == int(job.table.count[t]) and torch.equal(s.xy[0, :n], job.table.xy[t, :n])
              and torch.equal(s.desc[0, :n], job.table.desc[t, :n]))
        if not ok:
            log(f"verify: frame {g} (slot {t}): count {n} vs {int(job.table.count[t])}, xy equal "
                f"{torch.equal(s.xy[0, :n], job.table.xy[t, :n])}, desc equal {torch.equal(s.desc[0, :n], job.table.desc[t, :n])}")
        bad += 0 if ok else 1
    npairs = 0
    if job.sched is not None and not job.halo:
        m = BatchMatcher(RATIO, device=dev.index)
        for c in (0, plan.C - 1):
            sp = job.sched[c]
            for k in sorted({0, len(sp) - 1}) if len(sp) else []:
                a, b = (int(v) for v in sp[k])
                two = SlotTable(torch, 2, job.cap, dev)
                for d, src in ((0, a), (1, b)):
                    two.xy[d], two.desc[d], two.count[d] = job.table.xy[src], job.table.desc[src], job.table.count[src]
                mm, mc, nm = m.match(two, torch.tensor([[0, 1]], dtype=torch.int32, device=dev))
                o = job.outs[c]
                kk = int(nm[0])
                ok = kk == int(o[2][k]) and torch.equal(mm[0, :kk], o[0][k, :kk]) and torch.equal(mc[0, :kk], o[1][k, :kk])
                if not ok:
                    log(f"verify: chunk {c} pair {k} slots ({a}, {b}): nmatch {kk} vs {int(o[2][k])}, matches equal "
                        f"{torch.equal(mm[0, :kk], o[0][k, :kk])}, conf equal {torch.equal(mc[0, :kk], o[1][k, :kk])}")
                bad += 0 if ok else 1
                npairs += 1
    torch.cuda.synchronize()
    tot = torch.tensor([bad], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(tot)
    log(f"verify rank {rank}: {len(fr)} frames, {npairs} pairs checked, {bad} mismatches")
    if int(tot.item()):
        raise SystemExit(f"--verify: {int(tot.item())} mismatches over all ranks")


if __name__ == "__main__":
    main()
