// dist.hip — sfm_dist_*: the sharded jobs' exchange over RCCL (include/sfmfeat.h; SURVEY.md
// §8b "sfm_dist_*", §8e).  Host code only: one communicator per rank, the halo slot of the
// consecutive schedule (distributed.py halo_exchange) and configs[3]'s per-chunk slot gather
// (distributed.py allgather_chunk) as grouped RCCL operations on the caller's stream.
//
// RCCL is bound at run time, not linked: a process that already holds an RCCL (PyTorch-ROCm
// loads its own copy, with the same soname as /opt/rocm's) must use that one — two copies of
// the collective runtime in one process would each own bootstrap threads and device state —
// and a host that never calls sfm_dist_* loads none.
#include <dlfcn.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <string>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "../../include/sfmfeat.h"

namespace {

struct RcclApi {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::string why;  // empty when every entry point resolved
};

template <typename F>
bool bind(void* h, const char* name, F& f, std::string& why) {
  f = reinterpret_cast<F>(dlsym(h, name));
  if (f == nullptr && why.empty()) why = std::string("RCCL without ") + name;
  return f != nullptr;
}

const RcclApi& rccl() {
  static const RcclApi api = [] {
    RcclApi a;
    // the copy already in the process first (RTLD_NOLOAD matches it by soname), else the
    // library path's
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (h == nullptr) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (h == nullptr) {
      const char* e = dlerror();
      a.why = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
      return a;
    }
    bind(h, "ncclGetUniqueId", a.get_unique_id, a.why);
    bind(h, "ncclCommInitRank", a.init_rank, a.why);
    bind(h, "ncclCommDestroy", a.destroy, a.why);
    bind(h, "ncclAllGather", a.all_gather, a.why);
    bind(h, "ncclSend", a.send, a.why);
    bind(h, "ncclRecv", a.recv, a.why);
    bind(h, "ncclGroupStart", a.group_start, a.why);
    bind(h, "ncclGroupEnd", a.group_end, a.why);
    bind(h, "ncclGetErrorString", a.error_string, a.why);
    return a;
  }();
  return api;
}

// failures before a communicator exists (sfm_dist_last_error(NULL))
std::mutex g_err_mu;
std::string g_err;

void set_global_error(const std::string& m) {
  std::lock_guard<std::mutex> lk(g_err_mu);
  g_err = m;
}

}  // namespace

struct sfm_dist {
  ncclComm_t comm = nullptr;
  int32_t rank = 0, world = 1, device = 0;
  std::string err;
};

namespace {

int32_t fail(sfm_dist* d, int32_t code, const std::string& m) {
  if (d != nullptr) d->err = m;
  else set_global_error(m);
  return code;
}

int32_t nccl_fail(sfm_dist* d, const char* what, ncclResult_t r) {
  const char* s = rccl().error_string ? rccl().error_string(r) : "?";
  return fail(d, SFM_EDEVICE, std::string(what) + ": " + s);
}

// the communicator's device current on this host thread for the enqueue
int32_t use_device(sfm_dist* d) {
  const hipError_t e = hipSetDevice(d->device);
  if (e != hipSuccess) return fail(d, SFM_EDEVICE, std::string("hipSetDevice: ") + hipGetErrorString(e));
  return SFM_OK;
}

}  // namespace

extern "C" {

int32_t sfm_dist_unique_id(uint8_t* id) {
  if (id == nullptr) return fail(nullptr, SFM_EINVAL, "sfm_dist_unique_id: id is NULL");
  const RcclApi& r = rccl();
  if (!r.why.empty()) return fail(nullptr, SFM_EDEVICE, r.why);
  static_assert(sizeof(ncclUniqueId) == SFM_DIST_ID_BYTES, "RCCL unique id size");
  ncclUniqueId u;
  const ncclResult_t rc = r.get_unique_id(&u);
  if (rc != ncclSuccess) return nccl_fail(nullptr, "ncclGetUniqueId", rc);
  memcpy(id, &u, sizeof(u));
  return SFM_OK;
}

int32_t sfm_dist_create(int32_t device, int32_t rank, int32_t world, const uint8_t* id, sfm_dist** out) {
  if (out == nullptr || id == nullptr) return fail(nullptr, SFM_EINVAL, "sfm_dist_create: NULL argument");
  *out = nullptr;
  if (world < 1 || rank < 0 || rank >= world || device < 0)
    return fail(nullptr, SFM_EINVAL, "sfm_dist_create: need 0 <= rank < world and device >= 0");
  const RcclApi& r = rccl();
  if (!r.why.empty()) return fail(nullptr, SFM_EDEVICE, r.why);
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return fail(nullptr, SFM_EDEVICE, std::string("hipSetDevice: ") + hipGetErrorString(e));
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t comm = nullptr;
  const ncclResult_t rc = r.init_rank(&comm, world, u, rank);
  if (rc != ncclSuccess) return nccl_fail(nullptr, "ncclCommInitRank", rc);
  sfm_dist* d = new sfm_dist;
  d->comm = comm;
  d->rank = rank;
  d->world = world;
  d->device = device;
  *out = d;
  return SFM_OK;
}

int32_t sfm_dist_destroy(sfm_dist* d) {
  if (d == nullptr) return SFM_OK;
  int32_t st = SFM_OK;
  if (d->comm != nullptr && rccl().destroy != nullptr) {
    const ncclResult_t rc = rccl().destroy(d->comm);
    if (rc != ncclSuccess) st = nccl_fail(nullptr, "ncclCommDestroy", rc);
  }
  delete d;
  return st;
}

const char* sfm_dist_last_error(const sfm_dist* d) {
  if (d != nullptr) return d->err.c_str();
  // the text of a failure before any communicator: stable until the next such failure
  static thread_local std::string copy;
  std::lock_guard<std::mutex> lk(g_err_mu);
  copy = g_err;
  return copy.c_str();
}

int32_t sfm_dist_rank(const sfm_dist* d, int32_t* rank, int32_t* world) {
  if (d == nullptr) return SFM_EINVAL;
  if (rank) *rank = d->rank;
  if (world) *world = d->world;
  return SFM_OK;
}

int32_t sfm_dist_allgather_slots_dev(sfm_dist* d, int32_t bc, int32_t cap, const int32_t* src_xy,
                                     const float* src_desc, const int32_t* src_count, int32_t* tab_xy,
                                     float* tab_desc, int32_t* tab_count, int64_t base, void* stream) {
  if (d == nullptr) return fail(nullptr, SFM_EINVAL, "sfm_dist_allgather_slots_dev: no communicator");
  if (bc < 0 || cap < 1 || base < 0)
    return fail(d, SFM_EINVAL, "sfm_dist_allgather_slots_dev: need bc >= 0, cap >= 1, base >= 0");
  if (bc == 0) return SFM_OK;
  if (!src_xy || !src_desc || !src_count || !tab_xy || !tab_desc || !tab_count)
    return fail(d, SFM_EINVAL, "sfm_dist_allgather_slots_dev: NULL buffer");
  if (int32_t s = use_device(d)) return s;
  const RcclApi& r = rccl();
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const size_t nxy = (size_t)bc * cap * 2, nd = (size_t)bc * cap * 128;
  ncclResult_t rc = r.group_start();
  if (rc != ncclSuccess) return nccl_fail(d, "ncclGroupStart", rc);
  // the descriptors first: the largest transfer starts first inside the fused launch
  ncclResult_t a = r.all_gather(src_desc, tab_desc + (size_t)base * cap * 128, nd, ncclFloat32, d->comm, st);
  ncclResult_t b = r.all_gather(src_xy, tab_xy + (size_t)base * cap * 2, nxy, ncclInt32, d->comm, st);
  ncclResult_t c = r.all_gather(src_count, tab_count + base, (size_t)bc, ncclInt32, d->comm, st);
  rc = r.group_end();
  if (a != ncclSuccess) return nccl_fail(d, "ncclAllGather (desc)", a);
  if (b != ncclSuccess) return nccl_fail(d, "ncclAllGather (xy)", b);
  if (c != ncclSuccess) return nccl_fail(d, "ncclAllGather (count)", c);
  if (rc != ncclSuccess) return nccl_fail(d, "ncclGroupEnd", rc);
  return SFM_OK;
}

int32_t sfm_dist_halo_dev(sfm_dist* d, int32_t cap, const int32_t* src_xy, const float* src_desc,
                          const int32_t* src_count, int32_t* dst_xy, float* dst_desc, int32_t* dst_count,
                          void* stream) {
  if (d == nullptr) return fail(nullptr, SFM_EINVAL, "sfm_dist_halo_dev: no communicator");
  if (cap < 1) return fail(d, SFM_EINVAL, "sfm_dist_halo_dev: cap must be >= 1");
  const bool sends = d->rank > 0, recvs = d->rank < d->world - 1;
  if (!sends && !recvs) return SFM_OK;
  if (sends && (!src_xy || !src_desc || !src_count)) return fail(d, SFM_EINVAL, "sfm_dist_halo_dev: NULL source");
  if (recvs && (!dst_xy || !dst_desc || !dst_count))
    return fail(d, SFM_EINVAL, "sfm_dist_halo_dev: NULL destination");
  if (int32_t s = use_device(d)) return s;
  const RcclApi& r = rccl();
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const size_t nxy = (size_t)cap * 2, nd = (size_t)cap * 128;
  ncclResult_t rc = r.group_start();
  if (rc != ncclSuccess) return nccl_fail(d, "ncclGroupStart", rc);
  ncclResult_t bad = ncclSuccess;
  auto chk = [&](ncclResult_t x) { if (bad == ncclSuccess) bad = x; };
  if (sends) {
    const int p = d->rank - 1;
    chk(r.send(src_desc, nd, ncclFloat32, p, d->comm, st));
    chk(r.send(src_xy, nxy, ncclInt32, p, d->comm, st));
    chk(r.send(src_count, 1, ncclInt32, p, d->comm, st));
  }
  if (recvs) {
    const int p = d->rank + 1;
    chk(r.recv(dst_desc, nd, ncclFloat32, p, d->comm, st));
    chk(r.recv(dst_xy, nxy, ncclInt32, p, d->comm, st));
    chk(r.recv(dst_count, 1, ncclInt32, p, d->comm, st));
  }
  rc = r.group_end();
  if (bad != ncclSuccess) return nccl_fail(d, "ncclSend / ncclRecv", bad);
  if (rc != ncclSuccess) return nccl_fail(d, "ncclGroupEnd", rc);
  return SFM_OK;
}

}  // extern "C"
