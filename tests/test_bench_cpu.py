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
