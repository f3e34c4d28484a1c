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


def test_integration_c_snippet_compiles_against_the_header(tmp_path):
    """INTEGRATION.md §3's C use of the exchange beside the batch calls (one rank's chunk:
    extract into the table's own slots, gather in place, match) compiles against
    include/sfmfeat.h with -Werror: the documented binding matches the declared signatures."""
    src = tmp_path / "rank.c"
    src.write_text(r'''
#include <stdint.h>
#include "sfmfeat.h"
int rank_chunk(sfm_ctx* ctx, const float* frames, int32_t B, int32_t H, int32_t W, int32_t rank,
               int32_t world, int32_t device, int64_t base, int64_t cap, int32_t n_slots, int32_t* xy,
               float* desc, int32_t* count, const int32_t* pairs, int32_t P, int32_t* m, float* conf,
               int32_t* nm, void* stream) {
  uint8_t id[SFM_DIST_ID_BYTES];
  if (rank == 0 && sfm_dist_unique_id(id) != SFM_OK) return -1;   /* then broadcast id */
  sfm_dist* d = 0;
  if (sfm_dist_create(device, rank, world, id, &d) != SFM_OK) return -2;
  const int64_t own = base + (int64_t)rank * B;
  int rc = sfm_extract_batch_dev(ctx, frames, B, H, W, xy + own * cap * 2, desc + own * cap * 128,
                                 count + own, cap, stream);
  if (rc == SFM_OK)
    rc = sfm_dist_allgather_slots_dev(d, B, (int32_t)cap, xy + own * cap * 2, desc + own * cap * 128,
                                      count + own, xy, desc, count, base, stream);
  if (rc == SFM_OK)
    rc = sfm_match_pairs_dev(ctx, desc, count, n_slots, cap, pairs, P, 0.85f, m, conf, nm, stream);
  int32_t r = -1, w = -1;
  sfm_dist_rank(d, &r, &w);
  if (rc != SFM_OK) (void)sfm_dist_last_error(d);
  sfm_dist_destroy(d);
  return rc;
}
''')
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-c", "-I", os.path.join(ROOT, "include"), str(src),
                    "-o", str(tmp_path / "rank.o")], check=True)
