"""ctypes binding of libsfmfeat.so (include/sfmfeat.h).

The product path has no CPU fallback: if the HIP library is missing or no GPU is
visible, the calls raise.  Contexts are per thread (the reference drives extractor and
matcher from 8 threads, Runner.py:183-191) and per parameter set.
"""
from __future__ import annotations

import ctypes
import os
import sys
import threading

import numpy as np

from . import _abi
from ._abi import SfmParams

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SFMFEAT_LIB", os.path.join(_HERE, "lib", "libsfmfeat.so"))

_lib = None
_lib_lock = threading.Lock()

_fp = ctypes.POINTER(ctypes.c_float)
_i64p = ctypes.POINTER(ctypes.c_int64)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p

# exported symbol -> (restype, argtypes); every symbol of include/sfmfeat.h
SIGNATURES = {
    "sfm_params_default": (None, [ctypes.POINTER(SfmParams), ctypes.c_int32]),
    "sfm_abi_version": (ctypes.c_int32, []),
    "sfm_build_flags": (ctypes.c_int32, []),
    "sfm_keypoint_capacity": (ctypes.c_int64, [ctypes.POINTER(SfmParams)]),
    "sfm_pyramid_dims": (ctypes.c_int32, [ctypes.POINTER(SfmParams), ctypes.c_int32, ctypes.c_int32, _i32p]),
    "sfm_ctx_create": (ctypes.c_int32, [ctypes.c_int32, ctypes.POINTER(SfmParams), ctypes.POINTER(_vp)]),
    "sfm_ctx_destroy": (ctypes.c_int32, [_vp]),
    "sfm_last_error": (ctypes.c_char_p, [_vp]),
    "sfm_extract": (ctypes.c_int32, [_vp, _fp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, _i64p, _i64p,
                                     _fp, _fp, ctypes.c_int64, _i64p, _i32p]),
    "sfm_match": (ctypes.c_int32, [_vp, _fp, ctypes.c_int64, _fp, ctypes.c_int64, ctypes.c_float, _i64p, _fp,
                                   ctypes.c_int64, _i64p]),
    "sfm_reserve": (ctypes.c_int32, [_vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "sfm_ingest_rgb": (ctypes.c_int32, [_vp, _u8p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                        _fp]),
    "sfm_resize_dims": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, ctypes.c_double, _i32p, _i32p]),
    "sfm_ransac_find_inliers": (ctypes.c_int32, [_vp, _i64p, _i64p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double,
                                                 _i64p, _i64p, _i64p, _i32p]),
    "sfm_ransac_sample_indices": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _i32p]),
    "sfm_ransac_find_inliers_dev": (ctypes.c_int32, [_vp, _vp, _vp, _i32p, ctypes.c_int32, ctypes.c_int32,
                                                     ctypes.c_int32, ctypes.c_double, _vp, _vp, _vp, _vp]),
    "sfm_ingest_rgb_dev": (ctypes.c_int32, [_vp, _vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_int32, ctypes.c_int32, _vp, _vp]),
    "sfm_extract_batch_dev": (ctypes.c_int32, [_vp, _vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _vp, _vp,
                                               _vp, ctypes.c_int64, _vp]),
    "sfm_extract_batch_u8_dev": (ctypes.c_int32, [_vp, _vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _vp,
                                                  _vp, _vp, ctypes.c_int64, _vp]),
    "sfm_match_pairs_dev": (ctypes.c_int32, [_vp, _vp, _vp, ctypes.c_int32, ctypes.c_int64, _vp, ctypes.c_int32,
                                             ctypes.c_float, _vp, _vp, _vp, _vp]),
    "sfm_match_prep_dev": (ctypes.c_int32, [_vp, _vp, _vp, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                                            ctypes.c_int32, _vp]),
    "sfm_match_pairs_prepped_dev": (ctypes.c_int32, [_vp, _vp, _vp, ctypes.c_int32, ctypes.c_int64, _vp,
                                                     ctypes.c_int32, ctypes.c_float, _vp, _vp, _vp, _vp]),
    "sfm_ctx_stream": (ctypes.c_int32, [_vp, ctypes.POINTER(_vp)]),
    "sfm_ctx_set_serial": (ctypes.c_int32, [_vp, ctypes.c_int32]),
    "sfm_ctx_set_fused_prep": (ctypes.c_int32, [_vp, ctypes.c_int32]),
    "sfm_ctx_set_priority": (ctypes.c_int32, [_vp, ctypes.c_int32]),
    "sfm_gate_create": (ctypes.c_int32, [ctypes.c_int32, ctypes.POINTER(_vp)]),
    "sfm_gate_destroy": (ctypes.c_int32, [_vp]),
    "sfm_ctx_set_gate": (ctypes.c_int32, [_vp, _vp]),
    "sfm_profile_enable": (ctypes.c_int32, [_vp, ctypes.c_int32]),
    "sfm_profile_stages": (ctypes.c_int32, [_vp, ctypes.c_int32]),
    "sfm_profile_read": (ctypes.c_int32, [_vp, ctypes.POINTER(ctypes.c_double), _i64p, ctypes.c_int32]),
    "sfm_profile_spans": (ctypes.c_int32, [_vp, ctypes.c_int64]),
    "sfm_profile_spans_read": (ctypes.c_int32, [_vp, _i64p, _i32p, ctypes.c_int64, _i64p, _i64p, ctypes.c_int32]),
    "sfm_debug_time_harris": (ctypes.c_float, [ctypes.c_int32] * 6),
    "sfm_debug_harris_stamps": (ctypes.c_float, [ctypes.c_int32] * 6 + [ctypes.c_void_p, ctypes.c_int64]),
    "sfm_debug_match_stamps": (ctypes.c_int64, [ctypes.c_void_p, ctypes.c_int64]),
    "sfm_debug_select_stats": (ctypes.c_int32, [_vp, _i32p, _i32p]),
    "sfm_copy_wg": (ctypes.c_int32, [_vp, _vp, ctypes.c_int64, ctypes.c_int32, _vp]),
    "sfm_dist_unique_id": (ctypes.c_int32, [_u8p]),
    "sfm_dist_create": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _u8p, ctypes.POINTER(_vp)]),
    "sfm_dist_destroy": (ctypes.c_int32, [_vp]),
    "sfm_dist_last_error": (ctypes.c_char_p, [_vp]),
    "sfm_dist_rank": (ctypes.c_int32, [_vp, _i32p, _i32p]),
    "sfm_dist_allgather_slots_dev": (ctypes.c_int32, [_vp, ctypes.c_int32, ctypes.c_int32, _vp, _vp, _vp, _vp, _vp,
                                                      _vp, ctypes.c_int64, _vp]),
    "sfm_dist_halo_dev": (ctypes.c_int32, [_vp, ctypes.c_int32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),

    "sfm_debug_copy_level": (ctypes.c_int32, [_vp, ctypes.c_int32, ctypes.c_int32, _vp, _vp]),
    "sfm_debug_atan2": (ctypes.c_int32, [ctypes.c_int32, _fp, _fp, _fp, ctypes.c_int64]),
    "sfm_debug_harris": (ctypes.c_int32, [ctypes.c_int32, _fp, ctypes.c_int32, ctypes.c_double, ctypes.c_int32,
                                          _fp, ctypes.c_int32, ctypes.c_int32, _fp, _fp, _i64p]),
    "sfm_debug_nms": (ctypes.c_int32, [ctypes.c_int32, _fp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_int32, _vp, ctypes.c_int32, _vp, _i64p]),
}


class NativeLibraryMissing(ImportError):
    pass


def _preload_torch_hip_runtime():
    """If PyTorch-ROCm is installed, load ITS libamdhip64 first (without importing torch).

    torch bundles its own HIP runtime with the same SONAME as /opt/rocm's; whichever is
    loaded first serves the whole process.  Loading torch's copy up front keeps one
    runtime for both libsfmfeat and torch whatever the import order (device pointers and
    streams are then shared); without torch the system runtime is used."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    for d in spec.submodule_search_locations:
        cand = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(cand):
            try:
                ctypes.CDLL(cand, mode=ctypes.RTLD_GLOBAL)
            except OSError:
                pass
            return


def _preload_torch_rccl():
    """sfm_dist_* bind the librccl.so.1 already in the process: when PyTorch is installed its
    copy must be that one (one collective runtime per process), so torch is imported first and
    loads it in its own order.  (Loading torch's librccl.so by path before `import torch`
    aborts the interpreter at exit: a double free in the libraries' teardown.)  Without torch
    the library path's RCCL is used."""
    import importlib.util
    if "torch" not in sys.modules and importlib.util.find_spec("torch") is not None:
        import torch  # noqa: F401


def load_library(path: str | None = None):
    """Load libsfmfeat.so and bind every C-ABI symbol (no device call is made)."""
    global _lib
    with _lib_lock:
        if _lib is not None and path is None:
            return _lib
        _preload_torch_hip_runtime()
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise NativeLibraryMissing(
                f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(hipcc --offload-arch=gfx950); there is no CPU fallback")
        L = ctypes.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.sfm_abi_version() != 1:
            raise NativeLibraryMissing("libsfmfeat ABI version mismatch")
        if path is None:
            _lib = L
        return L


SFM_BUILD_ABLATIONS = 1  # include/sfmfeat.h


def library_info() -> dict:
    """Path and build flags of the loaded library (bench lines record them): `ablations` is
    True only for the diagnostic build (make ABLATIONS=1), whose timing switches skip work."""
    L = load_library()
    flags = int(L.sfm_build_flags())
    return {"path": os.path.relpath(LIB_PATH, os.path.dirname(_HERE)) if os.path.isabs(LIB_PATH) else LIB_PATH,
            "build_flags": flags, "ablations": bool(flags & SFM_BUILD_ABLATIONS)}


def check(rc: int, ctx=None):
    if rc == _abi.SFM_OK:
        return
    msg = ""
    if ctx is not None and ctx.value:
        m = load_library().sfm_last_error(ctx)
        msg = m.decode() if m else ""
    if rc == _abi.SFM_EINVAL:
        raise ValueError(msg or "invalid argument")
    if rc == _abi.SFM_EINDEX:
        raise IndexError(msg or "index 1 is out of bounds")
    if rc == _abi.SFM_ESTATE:
        raise RuntimeError(msg or "call out of order")
    if rc == _abi.SFM_ERANGE:
        raise ValueError(msg or "output capacity too small")
    raise RuntimeError(f"sfmfeat device error: {msg}")


def _params_key(p: SfmParams) -> bytes:
    return bytes(memoryview(p))


def resize_dims(H: int, W: int, scale: float = 0.5) -> tuple[int, int]:
    """(int(H * scale), int(W * scale)), the PIL target size of Runner.py:37-42."""
    h2, w2 = ctypes.c_int32(0), ctypes.c_int32(0)
    rc = load_library().sfm_resize_dims(H, W, ctypes.c_double(scale), ctypes.byref(h2), ctypes.byref(w2))
    if rc != _abi.SFM_OK:
        raise ValueError(f"bad resize: {H}x{W} * {scale}")
    return int(h2.value), int(w2.value)


class Context:
    """One sfm_ctx (device workspace + HIP stream) for a fixed parameter set."""

    def __init__(self, params: SfmParams, device: int = 0):
        self.lib = load_library()
        self.params = params
        self.device = device
        h = _vp()
        rc = self.lib.sfm_ctx_create(device, ctypes.byref(params), ctypes.byref(h))
        if rc != _abi.SFM_OK:
            if rc == _abi.SFM_EINVAL:
                raise ValueError("unsupported extractor parameters for the HIP path")
            raise RuntimeError("sfm_ctx_create failed: no usable MI355X (HIP) device")
        self.handle = h
        self.capacity = int(self.lib.sfm_keypoint_capacity(ctypes.byref(params)))
        self.levels = 1 if params.mode == _abi.SFM_MODE_NAIVE else int(params.pyramid_level)

    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            self.lib.sfm_ctx_destroy(self.handle)
            self.handle = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stream(self) -> int:
        """The context's own HIP stream (hipStream_t as an int), created on first use."""
        h = _vp()
        check(self.lib.sfm_ctx_stream(self.handle, ctypes.byref(h)), self.handle)
        return int(h.value or 0)

    def set_priority(self, priority: int):
        """HIP priority of the context's streams (lower = higher); before they exist."""
        check(self.lib.sfm_ctx_set_priority(self.handle, int(priority)), self.handle)

    def set_fused_prep(self, on: bool):
        """Batch extractions write the matcher's operands of their slots (sfm_ctx_set_fused_prep)."""
        check(self.lib.sfm_ctx_set_fused_prep(self.handle, 1 if on else 0), self.handle)

    def set_serial(self, serial: bool):
        """Every extraction stage on the caller's stream (no aux-stream overlap)."""
        check(self.lib.sfm_ctx_set_serial(self.handle, 1 if serial else 0), self.handle)

    def select_stats(self):
        """(planes that took the exact-median path, planes) of the last extraction."""
        fb, tot = ctypes.c_int32(0), ctypes.c_int32(0)
        check(self.lib.sfm_debug_select_stats(self.handle, ctypes.byref(fb), ctypes.byref(tot)), self.handle)
        return int(fb.value), int(tot.value)

    def copy_level(self, level: int, what: int, out_ptr: int, stream: int):
        """Level `level`'s R maps (what 0) / images (what 1) of the last extraction -> out."""
        check(self.lib.sfm_debug_copy_level(self.handle, int(level), int(what), ctypes.c_void_p(out_ptr),
                                            ctypes.c_void_p(stream)), self.handle)

    # -------- host-pointer API (drop-in path) --------
    def extract(self, img: np.ndarray):
        """-> X (n,) int64, Y (n,) int64, desc (n,128) float32, conf (n,) float32, level_counts"""
        if img.dtype != np.float32:
            img = img.astype(np.float32)
        if img.strides[1] != 4:
            img = np.ascontiguousarray(img)
        H, W = img.shape
        cap = max(self.capacity, 1)
        X = np.empty(cap, np.int64)
        Y = np.empty(cap, np.int64)
        D = np.empty((cap, 128), np.float32)
        C = np.empty(cap, np.float32)
        lc = np.zeros(self.levels, np.int32)
        n = ctypes.c_int64(0)
        rc = self.lib.sfm_extract(self.handle, img.ctypes.data_as(_fp), H, W, img.strides[0] // 4,
                                  X.ctypes.data_as(_i64p), Y.ctypes.data_as(_i64p), D.ctypes.data_as(_fp),
                                  C.ctypes.data_as(_fp), cap, ctypes.byref(n), lc.ctypes.data_as(_i32p))
        check(rc, self.handle)
        k = n.value
        return X[:k], Y[:k], D[:k], C[:k], lc

    def match(self, d1: np.ndarray, d2: np.ndarray, ratio32: np.float32):
        d1 = np.ascontiguousarray(d1, dtype=np.float32)
        d2 = np.ascontiguousarray(d2, dtype=np.float32)
        n1, n2 = d1.shape[0], d2.shape[0]
        cap = max(n1, 1)
        m = np.empty((cap, 2), np.int64)
        c = np.empty(cap, np.float32)
        k = ctypes.c_int64(0)
        rc = self.lib.sfm_match(self.handle, d1.ctypes.data_as(_fp), n1, d2.ctypes.data_as(_fp), n2,
                                ctypes.c_float(ratio32), m.ctypes.data_as(_i64p), c.ctypes.data_as(_fp), cap,
                                ctypes.byref(k))
        check(rc, self.handle)
        return m[:k.value], c[:k.value]

    def ingest_rgb(self, rgb: np.ndarray, scale: float = 0.5) -> np.ndarray:
        """FeatureRunner's ingest (Runner.py:33-46) of one decoded [H, W, 3] uint8 RGB frame:
        PIL BICUBIC resize to int(shape * scale), /255, _rgb2gray -> [H2, W2] float32."""
        rgb = np.ascontiguousarray(rgb)
        if rgb.dtype != np.uint8 or rgb.ndim != 3 or rgb.shape[2] != 3:
            raise ValueError("ingest_rgb expects an [H, W, 3] uint8 RGB frame")
        H, W = rgb.shape[:2]
        H2, W2 = resize_dims(H, W, scale)
        out = np.empty((H2, W2), np.float32)
        check(self.lib.sfm_ingest_rgb(self.handle, rgb.ctypes.data_as(_u8p), H, W, H2, W2, out.ctypes.data_as(_fp)),
              self.handle)
        return out

    def ransac_find_inliers(self, p1: np.ndarray, p2: np.ndarray, threshold: float, iters: int):
        """-> (in1 (k,2) int64, in2 (k,2) int64, best_iter) or None when n < 8."""
        p1 = np.ascontiguousarray(p1, np.int64).reshape(-1, 2)
        p2 = np.ascontiguousarray(p2, np.int64).reshape(-1, 2)
        n = p1.shape[0]
        o1 = np.empty((max(n, 1), 2), np.int64)
        o2 = np.empty((max(n, 1), 2), np.int64)
        k = ctypes.c_int64(0)
        bi = ctypes.c_int32(-1)
        check(self.lib.sfm_ransac_find_inliers(self.handle, p1.ctypes.data_as(_i64p), p2.ctypes.data_as(_i64p), n,
                                               int(iters), ctypes.c_double(threshold), o1.ctypes.data_as(_i64p),
                                               o2.ctypes.data_as(_i64p), ctypes.byref(k), ctypes.byref(bi)),
              self.handle)
        if k.value < 0:
            return None
        return o1[:k.value], o2[:k.value], int(bi.value)

    # -------- device-pointer API (throughput path; pointers are ints) --------
    def ingest_rgb_dev(self, rgb_ptr: int, B: int, H: int, W: int, H2: int, W2: int, gray_ptr: int,
                       stream: int = 0):
        check(self.lib.sfm_ingest_rgb_dev(self.handle, rgb_ptr, B, H, W, H2, W2, gray_ptr, stream or None),
              self.handle)

    def reserve(self, B: int, H: int, W: int):
        check(self.lib.sfm_reserve(self.handle, B, H, W), self.handle)

    def extract_batch_dev(self, imgs_ptr: int, B: int, H: int, W: int, xy_ptr: int, desc_ptr: int,
                          count_ptr: int, cap: int, stream: int = 0, u8: bool = False):
        fn = self.lib.sfm_extract_batch_u8_dev if u8 else self.lib.sfm_extract_batch_dev
        check(fn(self.handle, imgs_ptr, B, H, W, xy_ptr, desc_ptr, count_ptr, cap, stream or None), self.handle)

    PROF_STAGES = ["pyramid", "harris", "median", "nms", "topk", "describe", "match_prep", "match",
                   "match_post"]

    def profile_enable(self, on: bool = True):
        check(self.lib.sfm_profile_enable(self.handle, 1 if on else 0), self.handle)

    def profile_stages(self, names):
        """Bracket only the named stages (PROF_STAGES) with events; [] turns profiling off."""
        mask = 0
        for k in names:
            mask |= 1 << self.PROF_STAGES.index(k)
        check(self.lib.sfm_profile_stages(self.handle, mask), self.handle)

    def profile_read(self, reset: bool = True) -> dict:
        ms = np.zeros(len(self.PROF_STAGES), np.float64)
        n = np.zeros(len(self.PROF_STAGES), np.int64)
        check(self.lib.sfm_profile_read(self.handle, ms.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                        n.ctypes.data_as(_i64p), 1 if reset else 0), self.handle)
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(self.PROF_STAGES)}

    def profile_spans(self, capacity: int):
        """Record the kernel-active span of each of the next `capacity` Harris launches (0: off)."""
        check(self.lib.sfm_profile_spans(self.handle, int(capacity)), self.handle)

    def profile_spans_read(self, reset: bool = True):
        """-> (spans [n, 2] int64 ns on the device clock, first level [n], dropped launches)."""
        n, dropped = ctypes.c_int64(0), ctypes.c_int64(0)
        check(self.lib.sfm_profile_spans_read(self.handle, None, None, 0, ctypes.byref(n), ctypes.byref(dropped), 0),
              self.handle)
        k = int(n.value)
        sp = np.zeros((max(k, 1), 2), np.int64)
        lv = np.zeros(max(k, 1), np.int32)
        check(self.lib.sfm_profile_spans_read(self.handle, sp.ctypes.data_as(_i64p), lv.ctypes.data_as(_i32p), k,
                                              ctypes.byref(n), ctypes.byref(dropped), 1 if reset else 0), self.handle)
        return sp[:k], lv[:k], int(dropped.value)

    def match_pairs_dev(self, desc_ptr: int, count_ptr: int, nimg: int, cap: int, pairs_ptr: int, P: int,
                        ratio32: float, matches_ptr: int, conf_ptr: int, nmatch_ptr: int, stream: int = 0,
                        prepped: bool = False):
        fn = self.lib.sfm_match_pairs_prepped_dev if prepped else self.lib.sfm_match_pairs_dev
        check(fn(self.handle, desc_ptr, count_ptr, nimg, cap, pairs_ptr, P, ctypes.c_float(ratio32), matches_ptr,
                 conf_ptr, nmatch_ptr, stream or None), self.handle)

    def match_prep_dev(self, desc_ptr: int, count_ptr: int, nimg: int, cap: int, slot_lo: int, slot_n: int,
                       stream: int = 0):
        check(self.lib.sfm_match_prep_dev(self.handle, desc_ptr, count_ptr, nimg, cap, slot_lo, slot_n,
                                          stream or None), self.handle)


def copy_wg(dst_ptr: int, src_ptr: int, nbytes: int, workgroups: int, stream: int = 0):
    """sfm_copy_wg: a `workgroups`-workgroup device copy on `stream` (exchange emulation)."""
    check(load_library().sfm_copy_wg(dst_ptr, src_ptr, int(nbytes), int(workgroups), stream or None))


def debug_atan2(y: np.ndarray, x: np.ndarray, device: int = 0) -> np.ndarray:
    y = np.ascontiguousarray(y, dtype=np.float32)
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(y)
    check(load_library().sfm_debug_atan2(device, y.ctypes.data_as(_fp), x.ctypes.data_as(_fp),
                                         out.ctypes.data_as(_fp), y.size))
    return out


def debug_harris(img: np.ndarray, params: SfmParams, device: int = 0):
    """-> (R map float32, median float32, candidate count) of one plane."""
    img = np.ascontiguousarray(img, dtype=np.float32)
    H, W = img.shape
    gs = int(params.gaussian_size)
    g = np.array(params.gauss_kernel[: gs * gs], np.float32)
    R = np.empty_like(img)
    med = np.zeros(1, np.float32)
    nc = ctypes.c_int64(0)
    check(load_library().sfm_debug_harris(device, g.ctypes.data_as(_fp), gs, params.alpha, params.ksize,
                                          img.ctypes.data_as(_fp), H, W, R.ctypes.data_as(_fp),
                                          med.ctypes.data_as(_fp), ctypes.byref(nc)))
    return R, med[0], nc.value


def debug_nms(R: np.ndarray, tnms, ksize: int = 3, tile: bool = False, device: int = 0):
    """Certified-mode NMS of B planes R [B, H, W] f32 with per-plane key thresholds tnms [B]
    -> list of B sorted uint64 key arrays (~fkey(R) << 32 | raster index)."""
    R = np.ascontiguousarray(R, dtype=np.float32)
    B, H, W = R.shape
    t = np.ascontiguousarray(tnms, dtype=np.uint32)
    keys = np.zeros(B * H * W, np.uint64)
    cnt = np.zeros(B, np.int64)
    check(load_library().sfm_debug_nms(device, R.ctypes.data_as(_fp), B, H, W, ksize, t.ctypes.data,
                                       int(tile), keys.ctypes.data, cnt.ctypes.data_as(_i64p)))
    return [np.sort(keys[b * H * W: b * H * W + cnt[b]]) for b in range(B)]


class Gate:
    """sfm_gate: serialises the Harris phases of the contexts that share it (batches in
    flight, pipeline.BatchPipeline)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = _vp()
        if self.lib.sfm_gate_create(device, ctypes.byref(h)) != _abi.SFM_OK:
            raise RuntimeError("sfm_gate_create failed: no usable MI355X (HIP) device")
        self.handle = h

    def attach(self, ctx: Context):
        check(self.lib.sfm_ctx_set_gate(ctx.handle, self.handle), ctx.handle)

    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            self.lib.sfm_gate_destroy(self.handle)
            self.handle = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Dist:
    """sfm_dist: one rank's RCCL communicator for the sharded jobs' exchange (include/sfmfeat.h
    sfm_dist_*): the consecutive schedule's halo slot and configs[3]'s per-chunk
    slot gather, enqueued on a stream, without torch.distributed.  One rank makes the id
    (`unique_id`) and hands it to the others over any channel; `from_process_group` uses a
    torch.distributed group's broadcast for that."""

    def __init__(self, device: int, rank: int, world: int, uid: bytes):
        self.lib = load_library()
        _preload_torch_rccl()
        if len(uid) != 128:
            raise ValueError("the RCCL unique id is 128 bytes")
        ub = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        h = _vp()
        rc = self.lib.sfm_dist_create(int(device), int(rank), int(world), ub, ctypes.byref(h))
        if rc != _abi.SFM_OK:
            msg = (self.lib.sfm_dist_last_error(None) or b"").decode()
            if rc == _abi.SFM_EINVAL:
                raise ValueError(msg)
            raise RuntimeError(f"sfm_dist_create: {msg}")
        self.handle, self.device, self.rank, self.world = h, int(device), int(rank), int(world)

    @staticmethod
    def unique_id() -> bytes:
        lib = load_library()
        _preload_torch_rccl()
        buf = (ctypes.c_uint8 * 128)()
        if lib.sfm_dist_unique_id(buf) != _abi.SFM_OK:
            raise RuntimeError(f"sfm_dist_unique_id: {(lib.sfm_dist_last_error(None) or b'').decode()}")
        return bytes(buf)

    @classmethod
    def from_process_group(cls, dist, device: int, group=None) -> "Dist":
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        box = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0, group=group)
        return cls(device, rank, world, box[0])

    def _check(self, rc: int):
        if rc == _abi.SFM_OK:
            return
        msg = (self.lib.sfm_dist_last_error(self.handle) or b"").decode()
        if rc == _abi.SFM_EINVAL:
            raise ValueError(msg)
        raise RuntimeError(f"sfm_dist: {msg}")

    def allgather_slots(self, table, base: int, src, bc: int, stream: int = 0):
        """Every rank's src slots [0, bc) -> table slots [base + r * bc, ...) (pipeline.SlotTable
        fields; in place when src is the table's own slots base + rank * bc)."""
        cap = int(table.xy.shape[1])
        if int(src.xy.shape[1]) != cap or base + self.world * bc > int(table.xy.shape[0]) or bc > int(src.xy.shape[0]):
            raise ValueError("allgather_slots: slot shapes do not fit")
        self._check(self.lib.sfm_dist_allgather_slots_dev(
            self.handle, int(bc), cap, src.xy.data_ptr(), src.desc.data_ptr(), src.count.data_ptr(),
            table.xy.data_ptr(), table.desc.data_ptr(), table.count.data_ptr(), int(base), stream or None))

    def halo(self, slots, n_local: int, stream: int = 0):
        """distributed.halo_exchange's move: rank r + 1's slot 0 into this rank's slot n_local."""
        cap = int(slots.xy.shape[1])
        recvs = self.rank < self.world - 1
        if recvs and n_local >= int(slots.xy.shape[0]):
            raise ValueError("halo: the slot table has no slot n_local")
        dst = (slots.xy[n_local].data_ptr(), slots.desc[n_local].data_ptr(), slots.count[n_local:].data_ptr()) \
            if recvs else (None, None, None)
        self._check(self.lib.sfm_dist_halo_dev(self.handle, cap, slots.xy.data_ptr(), slots.desc.data_ptr(),
                                               slots.count.data_ptr(), *dst, stream or None))

    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            self.lib.sfm_dist_destroy(self.handle)
            self.handle = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_tls = threading.local()


def context_for(params: SfmParams, device: int = 0) -> Context:
    """Thread-local context cache keyed by (device, parameter bytes)."""
    cache = getattr(_tls, "cache", None)
    if cache is None:
        cache = _tls.cache = {}
    key = (device, _params_key(params))
    ctx = cache.get(key)
    if ctx is None:
        ctx = cache[key] = Context(params, device)
    return ctx
