"""CPU-side checks of the boundary: the C-ABI library loads and exports every symbol the
header declares, the parameter mirror matches the reference defaults, and the host
logic that needs no device behaves like the reference."""
from __future__ import annotations

import ctypes
import os
import re

import numpy as np
import pytest

from sfmfromscratch_amd import _abi, _native
from sfmfromscratch_amd.matcher import ratio_as_float32
from sfmfromscratch_amd.pipeline import all_pairs, consecutive_pairs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sfmfeat.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sfm_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    lib = _native.load_library()
    names = header_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
        assert n in _native.SIGNATURES, f"{n} not bound in _native.SIGNATURES"


def test_struct_layout_matches_header(tmp_path):
    """ctypes mirror == the C compiler's layout of sfm_params (offsets and size)."""
    import subprocess
    fields = [f[0] for f in _abi.SfmParams._fields_]
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "sfmfeat.h"\nint main(void){\n'
                   + "".join(f'printf("%zu\\n", offsetof(sfm_params, {f}));\n' for f in fields)
                   + 'printf("%zu\\n", sizeof(sfm_params));return 0;}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert out[:-1] == [getattr(_abi.SfmParams, f).offset for f in fields]
    assert out[-1] == ctypes.sizeof(_abi.SfmParams)


def test_params_defaults_match_reference_and_native():
    lib = _native.load_library()
    for mode in (_abi.SFM_MODE_SCALEROT, _abi.SFM_MODE_NAIVE):
        p = _abi.SfmParams()
        lib.sfm_params_default(ctypes.byref(p), mode)
        q = _abi.params_from_dict({}, mode)
        for f in ("num_interest_points", "ksize", "gaussian_size", "feature_width", "sigma", "alpha",
                  "pyramid_level", "pyramid_scale_factor"):
            assert getattr(p, f) == getattr(q, f), f
        assert p.num_interest_points == 2500 and p.ksize == 7 and p.feature_width == 16


def test_capacity_and_pyramid_dims():
    lib = _native.load_library()
    p = _abi.params_from_dict({"num_interest_points": 2500, "pyramid_level": 3, "pyramid_scale_factor": 1.1},
                              _abi.SFM_MODE_SCALEROT)
    assert lib.sfm_keypoint_capacity(ctypes.byref(p)) == 3 * 833
    d = np.zeros(6, np.int32)
    assert lib.sfm_pyramid_dims(ctypes.byref(p), 480, 640, d.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))) == 0
    assert d.tolist() == [480, 640, 436, 581, 396, 528]
    p4 = _abi.params_from_dict({"pyramid_level": 4}, _abi.SFM_MODE_SCALEROT)
    d = np.zeros(8, np.int32)
    lib.sfm_pyramid_dims(ctypes.byref(p4), 1080, 1920, d.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    assert d.tolist() == [1080, 1920, 540, 960, 270, 480, 135, 240]


def test_gaussian_taps_are_numpys():
    p = _abi.params_from_dict({"gaussian_size": 7, "sigma": 6}, _abi.SFM_MODE_SCALEROT)
    g = np.array(p.gauss_kernel[:49], np.float32)
    ref = _abi.generate_gaussian_kernel(7, 6).astype(np.float32).ravel()
    assert np.array_equal(g, ref)
    assert p.gauss_kernel_set == 1


def test_ratio_threshold_semantics():
    # python float: NEP 50 weak scalar -> compared in float32
    assert ratio_as_float32(0.85) == np.float32(0.85)
    # numpy float64: strong -> float64 compare == compare with the largest f32 <= r
    r = np.float64(0.85)
    t = ratio_as_float32(r)
    assert np.float64(t) <= r and np.float64(np.nextafter(t, np.float32(1))) > r


def test_pair_schedules():
    assert consecutive_pairs(4).tolist() == [[0, 1], [1, 2], [2, 3]]
    assert len(all_pairs(5)) == 10


def test_naive_descriptors_before_detect_raises_like_reference():
    from sfmfromscratch_amd import NaiveSIFT
    ns = NaiveSIFT(np.zeros((16, 16), np.float32), {})
    with pytest.raises(RuntimeError, match="Keypoints not detected"):
        ns.extract_descriptors()


def test_matcher_index_error_before_device():
    from sfmfromscratch_amd import NNRatioFeatureMatcher
    m = NNRatioFeatureMatcher(0.8)
    with pytest.raises(IndexError):
        m.match_features_ratio_test(np.zeros((3, 128), np.float32), np.zeros((1, 128), np.float32))
    a, b = m.match_features_ratio_test(np.zeros((0, 128), np.float32), np.zeros((5, 128), np.float32))
    assert a.shape == (0,) and b.shape == (0,)


def test_product_fails_loudly_without_device_or_library(monkeypatch):
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is visible")
    from sfmfromscratch_amd import ScaleRotInvSIFT
    with pytest.raises(RuntimeError):
        ScaleRotInvSIFT(np.zeros((64, 64), np.float32), {})
    with pytest.raises(_native.NativeLibraryMissing):
        _native.load_library("/nonexistent/libsfmfeat.so")


def test_resize_dims_like_runner():
    """sfm_resize_dims == (int(H * s), int(W * s)) of Runner.py:37-42 (host arithmetic only)."""
    from sfmfromscratch_amd._native import resize_dims
    for H, W, s in [(2160, 3840, 0.5), (481, 641, 0.5), (90, 60, 0.75), (7, 9, 0.3), (100, 100, 1.7)]:
        assert resize_dims(H, W, s) == (int(H * s), int(W * s))
    with pytest.raises(ValueError):
        resize_dims(1, 1, 0.5)


def test_set_device_is_thread_local():
    """set_device (the drop-in classes' device) belongs to the calling thread: the reference
    drives the classes from 8 threads (Runner.py:183-191), so one thread's choice must not move
    another's work.  No device call is made."""
    import threading

    from sfmfromscratch_amd import set_device
    from sfmfromscratch_amd.sift import current_device
    base = current_device()
    seen = {}

    def other():
        seen["before"] = current_device()
        set_device(5)
        seen["after"] = current_device()

    set_device(3)
    try:
        th = threading.Thread(target=other)
        th.start()
        th.join()
        assert seen == {"before": base, "after": 5}
        assert current_device() == 3
    finally:
        set_device(base)
