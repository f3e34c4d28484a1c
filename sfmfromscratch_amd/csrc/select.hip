// select.hip — keypoint selection per plane (NaiveSIFT.py:90-120), one 1024-thread
// workgroup per plane, one launch per pyramid level:
//   certified select : the k smallest 64-bit candidate keys of the certified NMS pass
//                      (sort_filter = argsort(conf)[::-1][:k]); final when the k-th key
//                      reaches tcert (kernels.h, MedianState);
//   exact path       : planes that do not certify (and levels too small to, and forced
//                      exact mode) continue in the same workgroup — np.median by radix
//                      select (:91), the full NMS predicate with that median (:77-97), then
//                      the same top-k over those candidates;
//   edge filter      : h <= y < H-h, h <= x < W-h (h = feature_width // 2), applied AFTER
//                      top-k; keys stay in ascending key order (confidence descending).
// Up to max(kTopkDirect, next_pow2(k)) candidates are sorted directly in LDS; beyond that a block radix select
// on the confidence half of the key finds the k-th key (ties on confidence resolved by
// raster index, exactly), and only the selected k keys are sorted.
//
// The exact path used to be four launches per level (median collect, median final, NMS,
// top-k) that exited at once on certified planes; a plane's exact path now runs in the
// workgroup that found it uncertified, so a certified level costs one launch in all.
#include <stdlib.h>

#include "kernels.h"

namespace sfm {

constexpr int kTopkDirect = 2048;  // candidates sorted whole; above: radix select first
constexpr int kTieLdsCap = 2048;   // confidence ties of the k-th key sorted in LDS; more: radix in global

// LDS histogram add (pred lanes add 1 to h[bin]); agg: the lanes on the first active lane's
// bin fold into one add by that lane (planes where many keys share a bin, e.g. R == 0 runs,
// otherwise serialise up to 64 same-address atomics per wavefront instruction).
SFM_DEV void hist_add(uint32_t* h, uint32_t bin, bool pred, bool agg) {
  if (!agg) {
    if (pred) atomicAdd(&h[bin], 1u);
    return;
  }
  const uint64_t act = __ballot(pred);
  if (act == 0) return;
  const int leader = __ffsll((unsigned long long)act) - 1;
  const uint32_t b0 = (uint32_t)__shfl((int)bin, leader);
  const uint64_t same = __ballot(pred && bin == b0);
  if (pred && bin != b0) atomicAdd(&h[bin], 1u);
  if (__lane_id() == leader) atomicAdd(&h[b0], (uint32_t)__popcll(same));
}

// Block radix select over a global array of 64-bit keys on one 32-bit half.
// use_lo = false: value = key >> 32 over all keys.  use_lo = true: value = key & ~0u over
// keys whose high half == match_hi.  Finds the value of 0-based rank `rank`; returns it
// and the residual rank among equal values in *rank_io.
SFM_DEV uint32_t radix_select_u32(const uint64_t* arr, int64_t m, bool use_lo, uint32_t match_hi,
                                  uint32_t* rank_io, uint32_t* s_h, uint32_t* s_scan,
                                  uint32_t* s_out, bool agg = false) {
  const int tid = threadIdx.x, nt = blockDim.x;
  uint32_t prefix = 0, mask = 0, rank = *rank_io;
  const int shifts[3] = {20, 8, 0};
  const uint32_t dmasks[3] = {0xfffu, 0xfffu, 0xffu};
  for (int d = 0; d < 3; ++d) {
    for (int i = tid; i < kHistBins; i += nt) s_h[i] = 0u;
    __syncthreads();
    constexpr int U = 8;  // loads in flight per thread
    for (int64_t base = 0; base < m; base += (int64_t)nt * U) {
      uint64_t kb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = base + tid + (int64_t)nt * u;
        kb[u] = i < m ? arr[i] : 0ull;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t key = kb[u];
        const uint32_t hi = (uint32_t)(key >> 32);
        const uint32_t v = use_lo ? (uint32_t)key : hi;
        const bool in = base + tid + (int64_t)nt * u < m && (!use_lo || hi == match_hi) && (v & mask) == prefix;
        hist_add(s_h, (v >> shifts[d]) & dmasks[d], in, agg);
      }
    }
    __syncthreads();
    find_bin(s_h, kHistBins, rank, s_scan, s_out);
    prefix |= s_out[0] << shifts[d];
    mask |= dmasks[d] << shifts[d];
    rank -= s_out[1];
    __syncthreads();
  }
  *rank_io = rank;
  return prefix;
}

// As radix_select_u32 (use_lo = false) over keys held in registers: thread t holds keys
// t + 1024 j (j < R; absent keys are ~0 and never counted: their rank lies above every
// real key's).  No global re-reads between the digit passes.
template <int R>
SFM_DEV uint32_t radix_select_regs(const uint64_t (&kr)[R], int64_t m, uint32_t* rank_io, uint32_t* s_h,
                                   uint32_t* s_scan, uint32_t* s_out, bool agg = false) {
  const int tid = threadIdx.x, nt = blockDim.x;
  uint32_t prefix = 0, mask = 0, rank = *rank_io;
  const int shifts[3] = {20, 8, 0};
  const uint32_t dmasks[3] = {0xfffu, 0xfffu, 0xffu};
  for (int d = 0; d < 3; ++d) {
    for (int i = tid; i < kHistBins; i += nt) s_h[i] = 0u;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t v = (uint32_t)(kr[j] >> 32);
      hist_add(s_h, (v >> shifts[d]) & dmasks[d], (int64_t)tid + (int64_t)nt * j < m && (v & mask) == prefix, agg);
    }
    __syncthreads();
    find_bin(s_h, kHistBins, rank, s_scan, s_out);
    prefix |= s_out[0] << shifts[d];
    mask |= dmasks[d] << shifts[d];
    rank -= s_out[1];
    __syncthreads();
  }
  *rank_io = rank;
  return prefix;
}

constexpr int kRegKeys = 8;  // keys per thread held in registers by the top-k (C <= 8192)

// The workgroup's LDS is sized per launch from k (select_sel_cap): a bitonic sort of n > 2048
// keys runs over next_pow2(n) slots, so the sel area holds max(next_pow2(k), kTopkDirect) keys
// (4096 at k = 2500: 68 KB in all, against 100 KB for the largest k), and a select workgroup
// fits on a CU beside one k_harris workgroup (78.8 KB).  Its VGPRs are kept at <= 88 for the
// same reason: 4 waves per SIMD x 88 + one k_harris wave (160) = 512, the SIMD's register file
// (tests/test_isa_guard_cpu.py pins both budgets).
struct SelectLds {
  uint64_t* sel;   // sel_cap
  uint64_t* tie;   // kTieLdsCap
  uint32_t* h;     // kHistBins
  uint32_t* scan;  // 1024
  uint32_t* out;   // 2
  uint32_t* cnt;   // 2
  int med_cap;     // u32 median-list keys held over the sel + tie areas
  int sel_cap;     // keys the sel area holds (>= kTopkDirect): lists up to it are sorted whole
};

// The kk (>= 1) smallest of the C keys cp[0..C) into L.sel[0..kk), ascending (tp: per-plane
// scratch for tie lists that overflow LDS).
// abl (timing ablations, results wrong by design; SFMFEAT_SELECT_ABL): 1 no final sort, 2 no
// radix select (every key counts as below the k-th); k_select: 4 no exact median, 8 no exact NMS;
// 16 (a correct variant, A/B): wave-aggregated histogram adds (hist_add); 32 (correct, A/B,
// SFMFEAT_SELECT_SUBSET=0): no subset fast path (topk_subset)
SFM_DEV void topk_sorted(const uint64_t* cp, int64_t C, int kk, uint64_t* tp, const SelectLds& L, int abl = 0) {
  const int tid = threadIdx.x, nt = blockDim.x;
  // up to sel_cap keys: sorted whole (for k > kTopkDirect the k-key sort below runs over the
  // same next_pow2 slots, so the radix select would only add to it)
  if (C <= L.sel_cap) {
    for (int i = tid; i < C; i += nt) L.sel[i] = cp[i];
    __syncthreads();
    sort_keys_u64(L.sel, (int)C);
    return;
  }
  uint32_t rank = (uint32_t)(kk - 1);
  uint32_t T;  // confidence half of the k-th key
  auto part = [&](uint64_t key) {  // keys below the k-th's confidence; its ties
    const uint32_t hi = (uint32_t)(key >> 32);
    if (hi < T) {
      L.sel[atomicAdd(&L.cnt[0], 1u)] = key;
    } else if (hi == T) {
      const uint32_t t = atomicAdd(&L.cnt[1], 1u);
      if (t < kTieLdsCap) L.tie[t] = key;
      tp[t] = key;
    }
  };
  if (C <= (int64_t)kRegKeys * nt) {
    // every key read once into registers (all loads in flight together)
    uint64_t kr[kRegKeys];
#pragma unroll
    for (int j = 0; j < kRegKeys; ++j) {
      const int64_t i = tid + (int64_t)nt * j;
      kr[j] = i < C ? cp[i] : ~0ull;
    }
    T = (abl & 2) ? 0xffffffffu : radix_select_regs(kr, C, &rank, L.h, L.scan, L.out, (abl & 16) != 0);
    if (tid == 0) {
      L.cnt[0] = 0u;
      L.cnt[1] = 0u;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kRegKeys; ++j)
      if (tid + (int64_t)nt * j < C) part(kr[j]);
  } else {
    T = radix_select_u32(cp, C, false, 0u, &rank, L.h, L.scan, L.out, (abl & 16) != 0);
    if (tid == 0) {
      L.cnt[0] = 0u;
      L.cnt[1] = 0u;
    }
    __syncthreads();
    constexpr int U = 8;  // loads in flight per thread
    for (int64_t base = 0; base < C; base += (int64_t)nt * U) {
      uint64_t kb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = base + tid + (int64_t)nt * u;
        kb[u] = i < C ? cp[i] : 0ull;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (base + tid + (int64_t)nt * u < C) part(kb[u]);
    }
  }
  __syncthreads();
  const uint32_t nless = (abl & 2) ? min(L.cnt[0], (uint32_t)kk) : L.cnt[0];
  const uint32_t ntie = L.cnt[1];
  const uint32_t need = (abl & 2) ? 0u : rank + 1;  // ties taken, by ascending raster index
  if (ntie <= (uint32_t)kTieLdsCap) {
    sort_keys_u64(L.tie, (int)ntie);
    for (uint32_t i = tid; i < need; i += nt) L.sel[nless + i] = L.tie[i];
  } else {
    uint32_t r2 = rank;
    const uint32_t Tlo = radix_select_u32(tp, ntie, true, T, &r2, L.h, L.scan, L.out, (abl & 16) != 0);
    for (int64_t i = tid; i < ntie; i += nt) {
      const uint64_t key = tp[i];
      if ((uint32_t)key <= Tlo) L.sel[atomicAdd(&L.cnt[0], 1u)] = key;
    }
  }
  __syncthreads();
  if (abl & 1) return;
  sort_keys_u64(L.sel, kk);
}

// Wave-aggregated append to an LDS counter: the lane's slot, or -1 without pred.
SFM_DEV int lds_wave_append(uint32_t* counter, bool pred) {
  const uint64_t mask = __ballot(pred);
  if (mask == 0) return -1;
  const int lane = __lane_id();
  const int leader = __ffsll((unsigned long long)mask) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(mask));
  base = __shfl(base, leader);
  const uint64_t lower = mask & ((lane == 0) ? 0ull : (~0ull >> (64 - lane)));
  return pred ? (int)(base + (uint32_t)__popcll(lower)) : -1;
}

// Certified planes with more than L.sel_cap candidates: the candidates at or above a higher
// threshold tsub[t] (MedianState) — the 3 vmin / 8-th or vmin / 2-th largest value's bucket,
// about 1-3k keys at vmin = 128 k instead of 3-7k — when at least kk (and at most L.sel_cap:
// kTopkDirect, or next_pow2(k) above it) of them exist.  Every candidate outside that subset
// lies below its threshold, i.e. below each of its members, so its kk best keys are the whole
// list's kk best (the caller's certification test then applies unchanged).  Sorted whole in L.sel; true when taken, false
// (nothing written) when neither subset fits: the caller runs the full top-k.
SFM_DEV bool topk_subset(const uint64_t* cp, int64_t C, int kk, const uint32_t (&tsub)[2], uint32_t tnms,
                         const SelectLds& L) {
  const int tid = threadIdx.x, nt = blockDim.x;
  // (tsub[0] >= tsub[1] >= tnms: when tsub[0] == tnms both subsets are the whole list)
  if (C <= L.sel_cap || C > (int64_t)kRegKeys * nt || tsub[0] <= tnms) return false;
  uint64_t kr[kRegKeys];
#pragma unroll
  for (int j = 0; j < kRegKeys; ++j) {
    const int64_t i = tid + (int64_t)nt * j;
    kr[j] = i < C ? cp[i] : ~0ull;  // ~0: high half 0xffffffff, below every threshold
  }
  // candidate keys hold ~fkey(R) in their high half: fkey(R) >= t  <=>  hi <= ~t
  const uint32_t h0 = ~tsub[0], h1 = ~tsub[1];
  if (tid < 2) L.cnt[tid] = 0u;
  __syncthreads();
  uint32_t c0 = 0, c1 = 0;
#pragma unroll
  for (int j = 0; j < kRegKeys; ++j) {
    const uint32_t hi = (uint32_t)(kr[j] >> 32);
    c0 += (uint32_t)__popcll(__ballot(hi <= h0));
    c1 += (uint32_t)__popcll(__ballot(hi <= h1));
  }
  if ((tid & 63) == 0) {
    atomicAdd(&L.cnt[0], c0);
    atomicAdd(&L.cnt[1], c1);
  }
  __syncthreads();
  const uint32_t n0 = L.cnt[0], n1 = L.cnt[1];
  const uint32_t cap = (uint32_t)L.sel_cap;
  const int t = (n0 >= (uint32_t)kk && n0 <= cap) ? 0 : (tsub[1] > tnms && n1 >= (uint32_t)kk && n1 <= cap) ? 1 : -1;
  if (t < 0) return false;  // (uniform)
  const uint32_t ht = t == 0 ? h0 : h1;
  __syncthreads();
  if (tid == 0) L.cnt[0] = 0u;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kRegKeys; ++j) {
    const bool in = (uint32_t)(kr[j] >> 32) <= ht;
    const int slot = lds_wave_append(&L.cnt[0], in);
    if (in) L.sel[slot] = kr[j];
  }
  __syncthreads();
  sort_keys_u64(L.sel, (int)(t == 0 ? n0 : n1));
  return true;
}

// Edge filter with order-preserving compaction of L.sel[0..nsel) into the plane's list.
SFM_DEV void emit_keypoints(const SelectLds& L, int nsel, KpList kp, int b, int kcap, int H, int W, int hw) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const int per = (nsel + nt - 1) / nt;
  const int beg = tid * per;
  uint32_t local = 0;
  for (int i = beg; i < beg + per && i < nsel; ++i) {
    const uint32_t idx = (uint32_t)L.sel[i];
    const int y = (int)(idx / (uint32_t)W), x = (int)(idx % (uint32_t)W);
    local += (y >= hw && y < H - hw && x >= hw && x < W - hw) ? 1u : 0u;
  }
  uint32_t total;
  uint32_t pos = block_exclusive_scan(local, L.scan, &total);
  for (int i = beg; i < beg + per && i < nsel; ++i) {
    const uint64_t key = L.sel[i];
    const uint32_t idx = (uint32_t)key;
    const int y = (int)(idx / (uint32_t)W), x = (int)(idx % (uint32_t)W);
    if (y >= hw && y < H - hw && x >= hw && x < W - hw) {
      const int64_t o = (int64_t)b * kcap + pos;
      kp.x[o] = x;
      kp.y[o] = y;
      kp.conf[o] = fkey_inv(~(uint32_t)(key >> 32));
      ++pos;
    }
  }
  if (tid == 0) kp.count[b] = (int32_t)total;
}

// Both middle keys from the collected list at once: digit 2 (11 bits) of rank r1 in bucket b1
// and of rank r2 in bucket b2 histogrammed in the two halves of s_h in one list pass, then
// digit 3 (10 bits) likewise (as select_in_list twice, in half the passes).
// The list's first L.med_cap keys live in LDS (ll), the rest in global memory (lp, same index).

SFM_DEV void select_pair_in_list(const uint32_t* ll, const uint32_t* lp, int64_t m, uint32_t b1, uint32_t r1,
                                 uint32_t b2, uint32_t r2, const SelectLds& L, uint32_t* key1, uint32_t* key2,
                                 bool agg) {
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int i = tid; i < kHistBins; i += nt) L.h[i] = 0u;
  __syncthreads();
  for (int64_t i = tid; i < m; i += nt) {
    const uint32_t k = i < L.med_cap ? ll[i] : lp[i];
    const bool in2 = (k >> 21) == b2;  // b1 == b2 is possible: both halves count the key
    hist_add(L.h, (k >> 10) & 0x7ffu, (k >> 21) == b1, agg);
    hist_add(L.h, 2048 + ((k >> 10) & 0x7ffu), in2, agg);
  }
  __syncthreads();
  find_bin(L.h, 2048, r1, L.scan, L.out);
  const uint32_t pre1 = (b1 << 11) | L.out[0];
  r1 -= L.out[1];
  __syncthreads();
  find_bin(L.h + 2048, 2048, r2, L.scan, L.out);
  const uint32_t pre2 = (b2 << 11) | L.out[0];
  r2 -= L.out[1];
  __syncthreads();
  for (int i = tid; i < 2048; i += nt) L.h[i] = 0u;
  __syncthreads();
  for (int64_t i = tid; i < m; i += nt) {
    const uint32_t k = i < L.med_cap ? ll[i] : lp[i];
    hist_add(L.h, k & 0x3ffu, (k >> 10) == pre1, agg);
    hist_add(L.h, 1024 + (k & 0x3ffu), (k >> 10) == pre2, agg);
  }
  __syncthreads();
  find_bin(L.h, 1024, r1, L.scan, L.out);
  *key1 = (pre1 << 10) | L.out[0];
  __syncthreads();
  find_bin(L.h + 1024, 1024, r2, L.scan, L.out);
  *key2 = (pre2 << 10) | L.out[0];
  __syncthreads();
}

// np.median of the plane (NaiveSIFT.py:91): the keys of the two digit-1 buckets holding the
// middle ranks (from the Harris histogram's select scan) are collected into a list whose
// first L.med_cap keys stay in LDS (the top-k areas are free until the exact NMS), the rest
// in `list`; then digits 2 and 3 are resolved from it.  Even n: float32 (v[n/2-1] + v[n/2]) / 2.
// The plane is read with 16-B loads (8 per thread in flight) when it is 16-B aligned.
SFM_DEV float exact_median(const float* Rp, int64_t n, const MedianState& s, uint32_t* list, const SelectLds& L,
                           bool agg) {
  const int tid = threadIdx.x, nt = blockDim.x;
  uint32_t* const ll = reinterpret_cast<uint32_t*>(L.sel);
  if (tid == 0) L.cnt[0] = 0u;
  __syncthreads();
  const uint32_t b1 = s.bucket[0], b2 = s.bucket[1];
  auto put = [&](uint32_t key, bool valid) {
    const uint32_t d = key >> (32 - kMedBits1);
    const bool in = valid && (d == b1 || d == b2);
    const int slot = lds_wave_append(&L.cnt[0], in);
    if (in) {
      if (slot < L.med_cap) ll[slot] = key;
      else list[slot] = key;
    }
  };
  constexpr int U = 4;  // loads in flight per thread (8 float4 loads cost k_select 10 VGPRs)
  if ((n & 3) == 0 && (reinterpret_cast<uintptr_t>(Rp) & 15) == 0) {
    const float4* R4 = reinterpret_cast<const float4*>(Rp);
    const int64_t n4 = n >> 2;
    for (int64_t base = 0; base < n4; base += (int64_t)nt * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = base + tid + (int64_t)nt * u;
        v[u] = i < n4 ? R4[i] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = base + tid + (int64_t)nt * u < n4;
        put(fkey(v[u].x), ok);
        put(fkey(v[u].y), ok);
        put(fkey(v[u].z), ok);
        put(fkey(v[u].w), ok);
      }
    }
  } else {
    for (int64_t base = 0; base < n; base += (int64_t)nt * U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = base + tid + (int64_t)nt * u;
        v[u] = i < n ? Rp[i] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) put(fkey(v[u]), base + tid + (int64_t)nt * u < n);
    }
  }
  __syncthreads();
  const int64_t m = (int64_t)L.cnt[0];
  __syncthreads();
  uint32_t key1, key2;
  if (s.odd) {  // one middle rank: the pair search on (b1, rank) twice
    select_pair_in_list(ll, list, m, b1, s.rank[0], b1, s.rank[0], L, &key1, &key2, agg);
    return fkey_inv(key1);
  }
  select_pair_in_list(ll, list, m, b1, s.rank[0], b2, s.rank[1], L, &key1, &key2, agg);
  const float v1 = fkey_inv(key1);
  const float v2 = fkey_inv(key2);
  const float sum = v1 + v2;
  return sum / 2.0f;
}

// The reference's NMS predicate with the exact median, over one plane inside the workgroup
// (nms.hip, mode 1): candidate <=> (R >= med && no cell of the clipped window is larger) ||
// (R < med && R == 0) (:92, :95); appended to cp in any order (top-k orders them).
// 3 x 3: wavefront rows of four 64-column chunks (RB rows per iteration), every load in
// flight together; the column maxima's neighbours come from the adjacent lanes (the
// chunk's edge lanes load theirs); out-of-image cells are -inf, so v == window max <=>
// none larger.  Other windows: a clipped-window loop per pixel.
SFM_DEV int64_t exact_nms(const float* Rp, int H, int W, int kh, float med, uint64_t* cp, const SelectLds& L) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nw = blockDim.x >> 6;
  if (tid == 0) L.cnt[1] = 0u;
  __syncthreads();
  auto pred_of = [&](float v, float m) { return (v < med) ? (v == 0.0f) : (v == m); };
  if (kh == 1 && (W & 3) == 0 && (reinterpret_cast<uintptr_t>(Rp) & 15) == 0) {
    // as below with 16-B loads: lane l of chunk ch owns columns x0 .. x0 + 3 (x0 = xb + 256 ch
    // + 4 l); the window's outer columns come from the neighbouring lanes' column maxima
    // (the chunk's edge lanes load the column beyond it)
    constexpr int NCH = 1, RB = 3;  // RB = 4: 90 VGPRs for the whole kernel, above its budget
    for (int y0 = wid * RB; y0 < H; y0 += nw * RB) {
      for (int xb = 0; xb < W; xb += 256 * NCH) {
        float4 c[RB + 2][NCH];
        float e[RB + 2][NCH];
#pragma unroll
        for (int rr = 0; rr < RB + 2; ++rr) {
          const int yy = y0 - 1 + rr;
          const bool rok = yy >= 0 && yy < H;
#pragma unroll
          for (int ch = 0; ch < NCH; ++ch) {
            const int x0 = xb + 256 * ch + 4 * lane;
            const int xe = lane == 0 ? x0 - 1 : x0 + 4;  // edge lanes: the column beyond the chunk
            c[rr][ch] = (rok && x0 < W) ? *reinterpret_cast<const float4*>(Rp + (int64_t)yy * W + x0)
                                        : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
            e[rr][ch] = (rok && (lane == 0 || lane == 63) && xe >= 0 && xe < W) ? Rp[(int64_t)yy * W + xe] : -INFINITY;
          }
        }
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
          for (int ch = 0; ch < NCH; ++ch) {
            const int y = y0 + rb;
            const int x0 = xb + 256 * ch + 4 * lane;
            const float4 a = c[rb][ch], m = c[rb + 1][ch], z = c[rb + 2][ch];
            const float c0 = fmaxf(fmaxf(a.x, m.x), z.x), c1 = fmaxf(fmaxf(a.y, m.y), z.y);
            const float c2 = fmaxf(fmaxf(a.z, m.z), z.z), c3 = fmaxf(fmaxf(a.w, m.w), z.w);
            const float em = fmaxf(fmaxf(e[rb][ch], e[rb + 1][ch]), e[rb + 2][ch]);
            const float up = __shfl_up(c3, 1), dn = __shfl_down(c0, 1);
            const float l = lane == 0 ? em : up, r = lane == 63 ? em : dn;
            const float w0 = fmaxf(fmaxf(l, c0), c1), w1 = fmaxf(fmaxf(c0, c1), c2);
            const float w2 = fmaxf(fmaxf(c1, c2), c3), w3 = fmaxf(fmaxf(c2, c3), r);
            const bool rowok = y < H && x0 < W;
            const float vv[4] = {m.x, m.y, m.z, m.w}, ww[4] = {w0, w1, w2, w3};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const bool pred = rowok && pred_of(vv[j], ww[j]);
              const int slot = lds_wave_append(&L.cnt[1], pred);
              if (pred) cp[slot] = ((uint64_t)(~fkey(vv[j])) << 32) | (uint32_t)(y * W + x0 + j);
            }
          }
      }
    }
  } else if (kh == 1) {
    // RB output rows per wavefront iteration from RB + 2 image rows loaded once (every load
    // of the iteration in flight together)
    constexpr int NCH = 2, RB = 2;  // NCH = 2, RB = 4: 106 VGPRs
    for (int y0 = wid * RB; y0 < H; y0 += nw * RB) {
      for (int xb = 0; xb < W; xb += 64 * NCH) {
        float c[RB + 2][NCH], e[RB + 2][NCH];
#pragma unroll
        for (int rr = 0; rr < RB + 2; ++rr) {
          const int yy = y0 - 1 + rr;
          const bool rok = yy >= 0 && yy < H;
#pragma unroll
          for (int ch = 0; ch < NCH; ++ch) {
            const int x = xb + 64 * ch + lane;
            const int xe = lane == 0 ? x - 1 : x + 1;  // edge lanes: the column beyond the chunk
            c[rr][ch] = (rok && x < W) ? Rp[(int64_t)yy * W + x] : -INFINITY;
            e[rr][ch] = (rok && (lane == 0 || lane == 63) && xe >= 0 && xe < W) ? Rp[(int64_t)yy * W + xe] : -INFINITY;
          }
        }
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
          for (int ch = 0; ch < NCH; ++ch) {
            const int y = y0 + rb;
            const int x = xb + 64 * ch + lane;
            const float cm = fmaxf(fmaxf(c[rb][ch], c[rb + 1][ch]), c[rb + 2][ch]);
            const float em = fmaxf(fmaxf(e[rb][ch], e[rb + 1][ch]), e[rb + 2][ch]);
            const float up = __shfl_up(cm, 1), dn = __shfl_down(cm, 1);
            const float l = lane == 0 ? em : up, r = lane == 63 ? em : dn;
            const float v = c[rb + 1][ch];
            const bool pred = y < H && x < W && pred_of(v, fmaxf(fmaxf(l, cm), r));
            const int slot = lds_wave_append(&L.cnt[1], pred);
            if (pred) cp[slot] = ((uint64_t)(~fkey(v)) << 32) | (uint32_t)(y * W + x);
          }
      }
    }
  } else {
    for (int y = wid; y < H; y += nw) {
      const int y0 = max(y - kh, 0), y1 = min(y + kh, H - 1);
      for (int xb = 0; xb < W; xb += 64) {
        const int x = xb + lane;
        bool pred = false;
        float v = 0.0f;
        if (x < W) {
          v = Rp[(int64_t)y * W + x];
          if (v < med) {
            pred = v == 0.0f;  // R_maxpool[R < median] = 0 (:92)
          } else {
            const int x0 = max(x - kh, 0), x1 = min(x + kh, W - 1);
            bool ismax = true;
            for (int yy = y0; yy <= y1; ++yy) {
              const float* row = Rp + (int64_t)yy * W;
              for (int xx = x0; xx <= x1; ++xx) ismax &= !(row[xx] > v);
            }
            pred = ismax;
          }
        }
        const int slot = lds_wave_append(&L.cnt[1], pred);
        if (pred) cp[slot] = ((uint64_t)(~fkey(v)) << 32) | (uint32_t)(y * W + x);
      }
    }
  }
  __syncthreads();
  const int64_t C = (int64_t)L.cnt[1];
  __syncthreads();
  return C;
}

__global__ void __launch_bounds__(1024) k_select(SelectLevels g, int kcap, int k, int kh, int B, int abl,
                                                  int sel_cap) {
  // this workgroup's level and plane (levels are B workgroups each, level-major)
  const int li = (int)blockIdx.x / B;
  const SelectLevels::Level& lv = g.l[li];
  const float* __restrict__ R = lv.R;
  uint64_t* __restrict__ cand = lv.cand;
  const unsigned long long* __restrict__ cand_count = lv.cand_count;
  uint32_t* __restrict__ medlist = lv.medlist;
  uint64_t* __restrict__ scratch = lv.scratch;
  const KpList kp = lv.kp;
  MedianState* __restrict__ state = lv.state;
  const int H = lv.H, W = lv.W, hw = lv.hw;
  extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
  __shared__ uint32_t s_out[2];
  __shared__ uint32_t s_cnt[2];
  SelectLds L;
  L.sel = reinterpret_cast<uint64_t*>(s_raw);
  L.tie = L.sel + sel_cap;
  L.h = reinterpret_cast<uint32_t*>(L.tie + kTieLdsCap);
  L.scan = L.h + kHistBins;
  L.out = s_out;
  L.cnt = s_cnt;
  L.med_cap = (sel_cap + kTieLdsCap) * 2;
  L.sel_cap = sel_cap;

  const int tid = threadIdx.x;
  const int b = (int)blockIdx.x - li * B;
  const int64_t n = (int64_t)H * W;
  uint64_t* cp = cand + (int64_t)b * n;
  uint64_t* tp = scratch + (int64_t)b * n;
  const MedianState s = state[b];
  if (k <= 0) {
    if (tid == 0) kp.count[b] = 0;
    return;
  }
  if (!s.fallback) {
    const int64_t C = (int64_t)cand_count[(int64_t)b * kCounterStride];  // certified NMS's candidates
    if (C >= (int64_t)k) {
      // SFMFEAT_SELECT_SUBSET=0 (A/B): always the full candidate list
      bool done = false;
      if (!(abl & 32)) done = topk_subset(cp, C, k, s.tsub, s.tnms, L);
      asm volatile("" ::: "memory");  // topk_sorted re-reads the keys: no 16 VGPRs held across
      if (!done) topk_sorted(cp, C, k, tp, L, abl);
      if ((abl & 3) || ~(uint32_t)(L.sel[k - 1] >> 32) >= s.tcert) {  // k-th candidate above the median's bucket
        emit_keypoints(L, k, kp, b, kcap, H, W, hw);
        return;
      }
    }
    // cannot certify (fewer than k candidates, or the k-th not above the median's bucket)
    if (tid == 0) state[b].fallback = 1u;
  }
  // abl 4: no exact median (the median's bucket start instead), 8: no exact NMS (no candidates)
  const float med = (abl & 4) ? fkey_inv(s.bucket[0] << (32 - kMedBits1))
                              : exact_median(R + (int64_t)b * n, n, s, medlist + (int64_t)b * n, L, (abl & 16) != 0);
  if (tid == 0) state[b].median = med;
  const int64_t C = (abl & 8) ? 0 : exact_nms(R + (int64_t)b * n, H, W, kh, med, cp, L);
  const int kk = (int)((int64_t)k < C ? (int64_t)k : C);
  if (kk <= 0) {
    if (tid == 0) kp.count[b] = 0;
    return;
  }
  topk_sorted(cp, C, kk, tp, L);
  emit_keypoints(L, kk, kp, b, kcap, H, W, hw);
}

static int select_sel_cap(int k) {
  int p = kTopkDirect;
  while (p < k) p <<= 1;
  return p;
}

static size_t select_lds_bytes(int sel_cap) {
  return (size_t)sel_cap * 8 + (size_t)kTieLdsCap * 8 + (size_t)kHistBins * 4 + 1024 * 4;
}

size_t topk_lds_bytes() { return select_lds_bytes(select_sel_cap(kTopkLdsCap)); }

void launch_select_levels(const SelectLevels& g, int kcap, int k, int B, int ksize, hipStream_t st) {
  if (g.n < 1 || g.n > kSelectMaxLevels || B < 1) return;
  static const int abl = [] {
    const char* e = SFM_ABLATION_ENV("SFMFEAT_SELECT_ABL");
    const char* sb = getenv("SFMFEAT_SELECT_SUBSET");  // a correct variant (A/B): 0 = full list always
    return (e ? atoi(e) : 0) | ((sb && atoi(sb) == 0) ? 32 : 0);
  }();
  const int sel_cap = select_sel_cap(k < 1 ? 1 : k);
  hipLaunchKernelGGL(k_select, dim3(B * g.n), dim3(1024), select_lds_bytes(sel_cap), st, g, kcap, k, ksize / 2, B,
                     abl, sel_cap);
}

void launch_select(const float* R, uint64_t* cand, const unsigned long long* cand_count, uint32_t* medlist,
                   uint64_t* scratch, KpList kp, int kcap, int k, int B, int H, int W, int ksize, int half_window,
                   MedianState* state, hipStream_t st) {
  SelectLevels g{};
  g.n = 1;
  g.l[0] = SelectLevels::Level{R, cand, cand_count, medlist, scratch, kp, state, H, W, half_window};
  launch_select_levels(g, kcap, k, B, ksize, st);
}

void init_topk_attributes() {
  (void)hipFuncSetAttribute((const void*)k_select, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)topk_lds_bytes());
}

}  // namespace sfm
