"""CPU: the C-ABI exchange's entry points (include/sfmfeat.h sfm_dist_*) validate their
arguments before touching RCCL or a device, report through sfm_dist_last_error, and bind RCCL
at run time (the library itself has no link-time RCCL dependency, so hosts that never call them
load none).  The collectives themselves run in tests/test_gpu_rccl.py."""
import ctypes
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sfmfromscratch_amd import _abi, _native  # noqa: E402


def test_dist_argument_errors_before_any_device_call():
    L = _native.load_library()
    h = _native._vp()
    uid = (ctypes.c_uint8 * 128)()
    for dev, rank, world in ((0, 2, 2), (0, -1, 1), (0, 0, 0), (-1, 0, 1)):
        assert L.sfm_dist_create(dev, rank, world, uid, ctypes.byref(h)) == _abi.SFM_EINVAL
        assert b"rank" in L.sfm_dist_last_error(None)
        assert not h.value
    assert L.sfm_dist_create(0, 0, 1, None, ctypes.byref(h)) == _abi.SFM_EINVAL
    assert L.sfm_dist_unique_id(None) == _abi.SFM_EINVAL
    assert L.sfm_dist_allgather_slots_dev(None, 1, 1, None, None, None, None, None, None, 0, None) == _abi.SFM_EINVAL
    assert L.sfm_dist_halo_dev(None, 1, None, None, None, None, None, None, None) == _abi.SFM_EINVAL
    assert L.sfm_dist_destroy(None) == _abi.SFM_OK
    with pytest.raises(ValueError):
        _native.Dist(0, 0, 1, b"short")


def test_library_has_no_link_time_rccl_dependency():
    out = subprocess.run(["readelf", "-d", _native.LIB_PATH], capture_output=True, text=True).stdout
    assert "librccl" not in out
    syms = subprocess.run(["nm", "-D", "--undefined-only", _native.LIB_PATH], capture_output=True, text=True).stdout
    assert "nccl" not in syms


def test_unique_ids_are_128_distinct_bytes():
    pytest.importorskip("torch")  # the RCCL bound here is PyTorch's copy (or the system's)
    a, b = _native.Dist.unique_id(), _native.Dist.unique_id()
    assert len(a) == len(b) == 128 and a != b
