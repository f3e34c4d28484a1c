"""Every product switch of the shipped library against the default path, bit for bit.

The shipped libsfmfeat.so reads exactly the switches in PRODUCT_SWITCHES (a CPU test,
tests/test_bench_cpu.py::test_shipped_library_reads_only_product_switches, checks the
library's strings against this list); the alternatives measured slower for good
(Harris forms 1/3/4/5, NMS strip shapes, stream-schedule and launch-shape A/Bs) are read only
by the diagnostic build (make ABLATIONS=1, SFM_DIAG_ENV).  The library reads its switches
once per process (or per context), so each group of alternatives runs in one child process
(same GPU, same inputs) and this process holds the defaults:
  group "paths":
    SFMFEAT_PYR_FUSED=0       pyramid levels 1-3 by k_down2x3 instead of the level-0 k_harris launch
    SFMFEAT_RERANK2=0         one query row per wavefront in the matcher's exact re-rank
    SFMFEAT_EXACT_PX=64       4K level 3 tries certification before its exact path
    SFMFEAT_SELECT_SUBSET=0   certified top-k always from the full candidate list
    SFMFEAT_MATCH_STAGE=1     the one-workgroup-per-CU matcher sweep (256-row query blocks)
    SFMFEAT_NMS_TILE=1        the tiled certified-NMS kernel instead of the streaming band kernel
    SFMFEAT_HARRIS_SLOTS=320  another resident-workgroup budget (tiles per workgroup change)
    SFMFEAT_MATCH_BUDGET_MB=8 the matcher's pairs in many small sub-launches
  group "exact":
    SFMFEAT_MATCH_DIRECT=1    the all-pairs exact VALU matcher instead of the MFMA prefilter
    SFMFEAT_DESCRIBE=wave     k_describe (one wavefront per keypoint) at every level
    SFMFEAT_SELECT=exact      the exact median + full NMS predicate on every plane
    SFMFEAT_SERIAL=1          every extraction stage on the caller's stream
Cases: 4 x 1080p at P-oct (four exact 2x levels: the fused pyramid) and 2 x 4K at five
levels, k = 8000 (fused levels 1-3 plus a trailing k_down2, exact level 3).
"""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np
import pytest

from sfmfromscratch_amd import synth
from tests.golden_util import P_OCT

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = {"1080p": (4, 1080, 1920, dict(P_OCT, num_interest_points=2500)),
         "4k": (2, 2160, 3840, dict(P_OCT, num_interest_points=8000, pyramid_level=5))}
ALT_GROUPS = {
    "paths": {"SFMFEAT_PYR_FUSED": "0", "SFMFEAT_RERANK2": "0", "SFMFEAT_EXACT_PX": "64",
              "SFMFEAT_SELECT_SUBSET": "0", "SFMFEAT_MATCH_STAGE": "1", "SFMFEAT_NMS_TILE": "1",
              "SFMFEAT_HARRIS_SLOTS": "320", "SFMFEAT_MATCH_BUDGET_MB": "8"},
    "exact": {"SFMFEAT_MATCH_DIRECT": "1", "SFMFEAT_DESCRIBE": "wave", "SFMFEAT_SELECT": "exact",
              "SFMFEAT_SERIAL": "1"},
}
# every SFMFEAT_* switch the shipped library reads (SFMFEAT_DEVICE / SFMFEAT_LIB and the
# pipeline's SFMFEAT_LANE_* are read by the Python package, not the library)
PRODUCT_SWITCHES = sorted({k for g in ALT_GROUPS.values() for k in g})


def run_cases() -> dict:
    """Extract and match every case's frames on cuda:0; numpy results by name."""
    import torch

    from sfmfromscratch_amd.pipeline import BatchExtractor, BatchMatcher, consecutive_pairs
    out = {}
    for name, (B, H, W, pp) in CASES.items():
        u8 = np.stack([synth.make_frame_u8(H, W, 404, i) for i in range(B)])
        frames = torch.from_numpy(u8).cuda()
        ex = BatchExtractor(pp)
        slots = ex.extract(frames)
        pairs = torch.from_numpy(consecutive_pairs(B)).cuda()
        m, c, n = BatchMatcher(0.85, ctx=ex.ctx).match(slots, pairs)
        torch.cuda.synchronize()
        out[f"{name}_count"] = slots.count.cpu().numpy()
        out[f"{name}_xy"] = slots.xy.cpu().numpy()
        out[f"{name}_desc"] = slots.desc.cpu().numpy().view(np.uint32)
        out[f"{name}_nmatch"] = n.cpu().numpy()
        out[f"{name}_m"] = m.cpu().numpy()
        out[f"{name}_c"] = c.cpu().numpy().view(np.uint32)
    return out


@pytest.mark.parametrize("group", sorted(ALT_GROUPS))
def test_default_paths_equal_alternatives(tmp_path, group):
    path = str(tmp_path / "alt.npz")
    env = dict(os.environ, **ALT_GROUPS[group])
    code = ("import sys, numpy as np; sys.path.insert(0, %r); from tests import test_gpu_switches as t; "
            "np.savez(%r, **t.run_cases())" % (ROOT, path))
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    alt = np.load(path)
    mine = run_cases()
    for name in CASES:
        cnt = mine[f"{name}_count"]
        assert np.array_equal(cnt, alt[f"{name}_count"]), name
        assert cnt.min() > 0, name
        for b, k in enumerate(cnt):
            assert np.array_equal(mine[f"{name}_xy"][b, :k], alt[f"{name}_xy"][b, :k]), (name, b)
            assert np.array_equal(mine[f"{name}_desc"][b, :k], alt[f"{name}_desc"][b, :k]), (name, b)
        nm = mine[f"{name}_nmatch"]
        assert np.array_equal(nm, alt[f"{name}_nmatch"]), name
        assert nm.min() > 0, name
        for p, k in enumerate(nm):
            # identical kernels order equal-nndr runs identically, so whole arrays compare
            assert np.array_equal(mine[f"{name}_m"][p, :k], alt[f"{name}_m"][p, :k]), (name, p)
            assert np.array_equal(mine[f"{name}_c"][p, :k], alt[f"{name}_c"][p, :k]), (name, p)
