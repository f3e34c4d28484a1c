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
