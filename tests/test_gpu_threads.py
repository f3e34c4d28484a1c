"""GPU: the reference's own calling pattern — SFMRunner fans its consecutive pairs out over
a ThreadPoolExecutor(max_workers=8) (Runner.py:183-191), and every task constructs the
extractor class twice and the matcher once (corner_detect_and_matching_process,
Runner.py:336-355 -> FeatureRunner, Runner.py:22-73).  Eight Python threads run the drop-in
classes concurrently here, each on its own frames, and every result is checked bit for bit
against the C oracle.  The device memory the eight threads' contexts hold together is
measured (hipMemGetInfo through torch) and written to gpurun_out/threads_memory.json
(INTEGRATION.md §Threading quotes it)."""
from __future__ import annotations

import json
import os
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import ingest as I
from oracle import oracle as O
from sfmfromscratch_amd import NNRatioFeatureMatcher, ScaleRotInvSIFT, set_device, synth
from sfmfromscratch_amd.sift import current_device
from tests.golden_util import P_OCT, assert_matches_equal

pytestmark = pytest.mark.gpu

NT = 8  # Runner.py:186 max_workers=8
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_eight_threads_drop_in_classes_vs_oracle(tmp_path):
    torch = pytest.importorskip("torch")
    Image = pytest.importorskip("PIL.Image")
    from sfmfromscratch_amd.runner import FeatureRunner

    # per thread: one consecutive 1080p pair (the BASELINE frame size) for the extractor
    # classes + matcher, and one PNG pair for a FeatureRunner (ingest x0.5 -> 270 x 480)
    gray = [[synth.make_frame(1080, 1920, 4321, 2 * t + j) for j in range(2)] for t in range(NT)]
    rgb = [[synth.make_frame_rgb_u8(540, 960, 99, 2 * t + j) for j in range(2)] for t in range(NT)]
    paths = []
    for t in range(NT):
        pp = []
        for j in range(2):
            p = str(tmp_path / f"t{t}_{j}.png")
            Image.fromarray(rgb[t][j]).save(p)
            pp.append(p)
        paths.append(pp)
    small = dict(P_OCT, num_interest_points=800)

    torch.cuda.init()
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info(0)[0]
    start, held, measured = threading.Barrier(NT), threading.Barrier(NT + 1), threading.Barrier(NT + 1)
    res, errs = [None] * NT, []

    def worker(t):
        try:
            set_device(0)
            start.wait()  # all eight threads enter the library together
            e1 = ScaleRotInvSIFT(gray[t][0], P_OCT)
            e2 = ScaleRotInvSIFT(gray[t][1], P_OCT)
            X1, Y1 = e1.detect_keypoints()
            X2, Y2 = e2.detect_keypoints()
            D1, D2 = e1.extract_descriptors(), e2.extract_descriptors()
            m, c = NNRatioFeatureMatcher(0.85).match_features_ratio_test(D1, D2)
            fr = FeatureRunner(paths[t][0], paths[t][1], feature_extractor_class=ScaleRotInvSIFT,
                               extractor_params=small, match_threshold=0.85)
            res[t] = (X1, Y1, D1, X2, Y2, D2, m, c, fr, current_device())
        except BaseException as e:  # noqa: BLE001 (re-raised in the main thread)
            errs.append((t, e))
            start.abort()
        finally:
            # keep this thread's contexts alive until the main thread has read the memory
            try:
                held.wait(timeout=300)
                measured.wait(timeout=300)
            except threading.BrokenBarrierError:
                pass

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(NT)]
    for th in threads:
        th.start()
    held.wait(timeout=300)
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info(0)[0]
    measured.wait(timeout=300)
    for th in threads:
        th.join(timeout=300)
    if errs:
        raise errs[0][1]

    # the oracle on the same frames (C restatement; host threads, GIL released)
    def oracle_task(t):
        a, b = O.extract(gray[t][0], P_OCT), O.extract(gray[t][1], P_OCT)
        g = [I.ingest(rgb[t][j], 0.5) for j in range(2)]
        fa, fb = O.extract(g[0], small), O.extract(g[1], small)
        return a, b, O.match(a[2], b[2], 0.85), g, fa, fb, O.match(fa[2], fb[2], 0.85)

    with ThreadPoolExecutor(NT) as pool:
        oracle = list(pool.map(oracle_task, range(NT)))
    for t in range(NT):
        X1, Y1, D1, X2, Y2, D2, m, c, fr, dev = res[t]
        a, b, (om, oc), g, fa, fb, (fm, fc) = oracle[t]
        assert dev == 0
        for (X, Y, D), o in (((X1, Y1, D1), a), ((X2, Y2, D2), b)):
            assert np.array_equal(X, o[0]) and np.array_equal(Y, o[1]), f"thread {t}: keypoints"
            assert np.array_equal(D.view(np.uint32), o[2].view(np.uint32)), f"thread {t}: descriptors"
        assert_matches_equal(om, oc, m, c)
        assert np.array_equal(fr._image1_bw, g[0]) and np.array_equal(fr._image2_bw, g[1])
        assert np.array_equal(fr.X1, fa[0]) and np.array_equal(fr.Y2, fb[1])
        assert np.array_equal(np.asarray(fr.descriptors2).view(np.uint32), fb[2].view(np.uint32))
        assert_matches_equal(fm, fc, fr.matches, fr.confidences)

    used = free0 - free1
    rec = {"threads": NT, "device_bytes_all_threads": int(used), "device_bytes_per_thread": int(used // NT),
           "workload": "per thread: ScaleRotInvSIFT x2 on 1080x1920 (P-oct, k 2500) + NNRatioFeatureMatcher + "
                       "FeatureRunner on a 540x960 RGB PNG pair (k 800); contexts: one per thread and parameter set",
           "method": "torch.cuda.mem_get_info free bytes before the threads started minus while all eight "
                     "threads held their contexts"}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "threads_memory.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))
    assert used < 8 * (1 << 30), f"eight threads hold {used / 2**30:.2f} GiB of device memory"
