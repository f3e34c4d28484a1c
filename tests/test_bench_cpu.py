"""bench.py's launcher contract on a host without GPUs: `--gpus N` starts N ranks itself
(a child torch.distributed.run) and must refuse loudly — no JSON line, non-zero exit —
when the node shows fewer than N GPUs; under an outer launcher WORLD_SIZE must equal
--gpus.  (The multi-rank data path itself is covered by test_distributed_cpu.py over gloo
and by tests/test_gpu_gather.py on the GPU.)"""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "BENCH_DIST_BACKEND"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=env, timeout=180)


def test_gpus_n_refused_without_n_gpus():
    torch = pytest.importorskip("torch")
    if torch.cuda.device_count() >= 2:
        pytest.skip("this host has GPUs")
    r = _run(["--gpus", "2", "--steps", "1"])
    assert r.returncode == 2
    assert "needs 2 visible GPUs" in r.stderr
    assert '"metric"' not in r.stdout


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
    assert '"metric"' not in r.stdout


@pytest.mark.parametrize("switch", ["SFMFEAT_SKIP", "SFMFEAT_HARRIS_ABL", "SFMFEAT_SELECT_ABL", "SFMFEAT_DQ_ABL",
                                    "SFMFEAT_NMS_DRY"])
def test_ablation_switch_refused(switch):
    """A results-wrong-by-design timing switch in the environment ends the run before any GPU
    work: non-zero exit, no JSON line (only --ablation-run, a marked diagnostic, accepts it)."""
    r = _run(["--gpus", "1", "--steps", "1"], {switch: "1"})
    assert r.returncode == 3, r.stderr
    assert switch in r.stderr and "refusing" in r.stderr
    assert '"metric"' not in r.stdout


def test_bench_env_and_workload_resolution():
    """The JSON line's `env` holds every run switch; `--gpus N` resolves to configs[1] (c2) at
    N = 1 and to configs[3] (c4, whose line carries its own N = 1 figure) at N > 1."""
    sys.path.insert(0, ROOT)
    import bench
    env = {"SFMFEAT_HARRIS_SLOTS": "448", "HIP_VISIBLE_DEVICES": "0", "GPU_MAX_HW_QUEUES": "4",
           "HSA_ENABLE_IPC_MODE_LEGACY": "0", "HOME": "/root", "PATH": "/bin"}
    assert bench.bench_env(env) == {k: env[k] for k in ("GPU_MAX_HW_QUEUES", "HIP_VISIBLE_DEVICES",
                                                        "HSA_ENABLE_IPC_MODE_LEGACY", "SFMFEAT_HARRIS_SLOTS")}
    assert bench.ablation_switches_set(env) == []
    assert bench.ablation_switches_set(dict(env, SFMFEAT_SKIP="8", SFMFEAT_MATCH_ABL="2")) == \
        ["SFMFEAT_MATCH_ABL", "SFMFEAT_SKIP"]
    assert bench.default_workload(1) == "c2"
    assert [bench.default_workload(n) for n in (2, 4, 8)] == ["c4"] * 3


def test_shipped_library_has_no_ablations():
    """The product library is the build without timing ablations: sfm_build_flags() is 0 and the
    ablation switches' names do not occur in it (only `make ABLATIONS=1` compiles them in)."""
    sys.path.insert(0, ROOT)
    from sfmfromscratch_amd import _native
    lib = os.path.join(ROOT, "sfmfromscratch_amd", "lib", "libsfmfeat.so")
    if not os.path.exists(lib):
        pytest.skip("libsfmfeat.so not built")
    assert _native.load_library(lib).sfm_build_flags() == 0
    data = open(lib, "rb").read()
    for name in (b"SFMFEAT_SKIP", b"SFMFEAT_HARRIS_ABL", b"SFMFEAT_SELECT_ABL", b"SFMFEAT_DQ_ABL", b"SFMFEAT_MATCH_ABL",
                 b"SFMFEAT_NMS_DRY"):
        assert name not in data, name


def test_span_stats_union_and_launch_sum():
    """The roofline's timing from kernel-active spans: two lanes' launches that overlap count
    once in the union (non-overlapping attribution) and twice in the launch sum."""
    sys.path.insert(0, ROOT)
    import numpy as np

    import bench
    ms = 1_000_000  # ns
    lane_a = np.array([[0, 4 * ms], [10 * ms, 12 * ms]], np.int64)
    lane_b = np.array([[3 * ms, 6 * ms], [20 * ms, 21 * ms], [-1, -1]], np.int64)  # an unused slot is dropped
    st = bench.span_stats([lane_a, lane_b], steps=2, flop=2e12, peak_tflops=100.0)
    assert st["launches"] == 4
    assert st["launch_sum_ms_per_step"] == 5.0          # (4 + 2 + 3 + 1) / 2
    assert st["union_ms_per_step"] == 4.5              # ([0, 6] + [10, 12] + [20, 21]) / 2
    assert st["overlap_ms_per_step"] == 0.5
    assert st["first_to_last_ms"] == 21.0
    assert abs(st["achieved_union"] - 2.0 / 9e-3) < 1e-6   # 2 TFLOP over 9 ms
    assert abs(st["frac_launch_sum"] - 2.0 / 10e-3 / 100.0) < 1e-9
    assert bench.span_stats([np.zeros((0, 2), np.int64)], 1, 1.0, 1.0) == {"launches": 0}


def test_roofline_guard_rejects_more_kernel_time_than_the_step():
    """bench.py exits 4 when the dominant kernel's attributed time per step exceeds the step
    (the round-5 line implied 0.948 ms of Harris per 0.812 ms step) or nothing was timed."""
    sys.path.insert(0, ROOT)
    import bench
    ok = {"kernel": "k_harris<7>", "launches": 80, "ms_per_step": 0.70}
    assert bench.roofline_guard(ok, 0.812) == []
    assert bench.roofline_guard(None, 0.812) == []
    assert bench.roofline_guard(dict(ok, ms_per_step=0.948), 0.812)
    assert bench.roofline_guard(dict(ok, ms_per_step=0.815), 0.812) == []   # within the clock tolerance
    assert bench.roofline_guard(dict(ok, launches=0), 0.812)


def test_shipped_library_reads_only_product_switches():
    """Every SFMFEAT_* name in the shipped library is a product switch that
    tests/test_gpu_switches.py runs against the default bit for bit; the diagnostic A/B
    switches (slower Harris forms, NMS strip shapes, stream-schedule experiments) exist only
    in the diagnostic build (SFM_DIAG_ENV)."""
    import re
    sys.path.insert(0, ROOT)
    from tests.test_gpu_switches import PRODUCT_SWITCHES
    lib = os.path.join(ROOT, "sfmfromscratch_amd", "lib", "libsfmfeat.so")
    if not os.path.exists(lib):
        pytest.skip("libsfmfeat.so not built")
    names = set(m.decode() for m in re.findall(rb"SFMFEAT_[A-Z0-9_]+", open(lib, "rb").read()))
    assert names, "no switch names found (string scan broken?)"
    assert names <= set(PRODUCT_SWITCHES), sorted(names - set(PRODUCT_SWITCHES))
    for diag in ("SFMFEAT_HARRIS_MF", "SFMFEAT_HARRIS_PP", "SFMFEAT_HARRIS_NPAIR", "SFMFEAT_NMS_BAND",
                 "SFMFEAT_SELECT_CALLER", "SFMFEAT_RERANK8_MAX", "SFMFEAT_MATCH_UNITS"):
        assert diag not in names
