// select.hip — top-k + edge filter per plane (NaiveSIFT.py:99-120):
//   sort_filter = argsort(conf)[::-1][:k]   -> k smallest 64-bit candidate keys
//   edge filter h <= y < H-h, h <= x < W-h  (h = feature_width // 2), applied AFTER top-k
//   re-sort descending                      -> keys stay in ascending key order
// One 1024-thread workgroup per plane.  Up to kTopkDirect candidates are sorted directly
// in LDS; beyond that a block radix select on the confidence half of the key finds the
// k-th key (ties on confidence resolved by raster index, exactly), and only the
// selected k keys are sorted.
//
// mode 0 (certified select, kernels.h MedianState): a plane is final when it has at least
// k candidates and the k-th key reaches tcert; otherwise it is flagged `fallback` and left
// to mode 1, which runs after the exact median + NMS on the flagged planes only.
#include "kernels.h"

namespace sfm {

constexpr int kTieLdsCap = 4096;
constexpr int kTopkDirect = 2048;  // candidates sorted whole; above: radix select first

// Block radix select over a global array of 64-bit keys on one 32-bit half.
// use_lo = false: value = key >> 32 over all keys.  use_lo = true: value = key & ~0u over
// keys whose high half == match_hi.  Finds the value of 0-based rank `rank`; returns it
// and the residual rank among equal values in *rank_io.
SFM_DEV uint32_t radix_select_u32(const uint64_t* arr, int64_t m, bool use_lo, uint32_t match_hi,
                                  uint32_t* rank_io, uint32_t* s_h, uint32_t* s_scan,
                                  uint32_t* s_out) {
  const int tid = threadIdx.x, nt = blockDim.x;
  uint32_t prefix = 0, mask = 0, rank = *rank_io;
  const int shifts[3] = {20, 8, 0};
  const uint32_t dmasks[3] = {0xfffu, 0xfffu, 0xffu};
  for (int d = 0; d < 3; ++d) {
    for (int i = tid; i < kHistBins; i += nt) s_h[i] = 0u;
    __syncthreads();
    for (int64_t i = tid; i < m; i += nt) {
      uint64_t key = arr[i];
      uint32_t hi = (uint32_t)(key >> 32);
      uint32_t v;
      if (use_lo) {
        if (hi != match_hi) continue;
        v = (uint32_t)key;
      } else {
        v = hi;
      }
      if ((v & mask) == prefix) atomicAdd(&s_h[(v >> shifts[d]) & dmasks[d]], 1u);
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

__global__ void __launch_bounds__(1024) k_topk(const uint64_t* __restrict__ cand,
                                               const unsigned long long* __restrict__ cand_count,
                                               uint64_t* __restrict__ scratch, KpList kp, int kcap,
                                               int k, int H, int W, int hw,
                                               MedianState* __restrict__ state, int mode) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
  uint64_t* s_sel = reinterpret_cast<uint64_t*>(s_raw);               // kTopkLdsCap
  uint64_t* s_tie = s_sel + kTopkLdsCap;                               // kTieLdsCap
  uint32_t* s_h = reinterpret_cast<uint32_t*>(s_tie + kTieLdsCap);     // kHistBins
  uint32_t* s_scan = s_h + kHistBins;                                  // 1024
  __shared__ uint32_t s_out[2];
  __shared__ uint32_t s_cnt[2];

  const int tid = threadIdx.x, nt = blockDim.x;
  const int b = blockIdx.x;
  const int64_t n = (int64_t)H * W;
  const uint64_t* cp = cand + (int64_t)b * n;
  const int64_t C = (int64_t)cand_count[(int64_t)b * kCounterStride];
  if (mode == 0) {
    if (state[b].fallback) return;
    if (C < (int64_t)k) {  // cannot certify: the exact path decides this plane
      if (tid == 0) state[b].fallback = 1u;
      return;
    }
  } else if (!state[b].fallback) {
    return;
  }
  const int kk = (int)((int64_t)k < C ? (int64_t)k : C);
  if (kk <= 0) {
    if (tid == 0) kp.count[b] = 0;
    return;
  }
  int nsel;
  if (C <= kTopkDirect) {
    const int P = next_pow2((int)C);
    for (int i = tid; i < P; i += nt) s_sel[i] = (i < C) ? cp[i] : ~0ull;
    __syncthreads();
    bitonic_sort_u64(s_sel, P);
    nsel = kk;
  } else {
    uint32_t rank = (uint32_t)(kk - 1);
    const uint32_t T = radix_select_u32(cp, C, false, 0u, &rank, s_h, s_scan, s_out);
    if (tid == 0) { s_cnt[0] = 0u; s_cnt[1] = 0u; }
    __syncthreads();
    uint64_t* tp = scratch + (int64_t)b * n;
    for (int64_t i = tid; i < C; i += nt) {
      uint64_t key = cp[i];
      uint32_t hi = (uint32_t)(key >> 32);
      if (hi < T) {
        s_sel[atomicAdd(&s_cnt[0], 1u)] = key;
      } else if (hi == T) {
        uint32_t t = atomicAdd(&s_cnt[1], 1u);
        if (t < kTieLdsCap) s_tie[t] = key;
        tp[t] = key;
      }
    }
    __syncthreads();
    const uint32_t nless = s_cnt[0];
    const uint32_t ntie = s_cnt[1];
    const uint32_t need = rank + 1;  // ties taken, by ascending raster index
    if (ntie <= (uint32_t)kTieLdsCap) {
      const int P = next_pow2((int)ntie);
      for (int i = tid; i < P; i += nt)
        if (i >= (int)ntie) s_tie[i] = ~0ull;
      __syncthreads();
      bitonic_sort_u64(s_tie, P);
      for (uint32_t i = tid; i < need; i += nt) s_sel[nless + i] = s_tie[i];
    } else {
      uint32_t r2 = rank;
      const uint32_t Tlo = radix_select_u32(tp, ntie, true, T, &r2, s_h, s_scan, s_out);
      for (int64_t i = tid; i < ntie; i += nt) {
        uint64_t key = tp[i];
        if ((uint32_t)key <= Tlo) s_sel[atomicAdd(&s_cnt[0], 1u)] = key;
      }
    }
    __syncthreads();
    nsel = kk;
    const int P = next_pow2(nsel);
    for (int i = tid; i < P; i += nt)
      if (i >= nsel) s_sel[i] = ~0ull;
    __syncthreads();
    bitonic_sort_u64(s_sel, P);
  }
  __syncthreads();
  if (mode == 0 && kk > 0 && ~(uint32_t)(s_sel[kk - 1] >> 32) < state[b].tcert) {
    if (tid == 0) state[b].fallback = 1u;  // k-th candidate not above the median's bucket
    return;
  }
  // edge filter with order-preserving compaction
  const int per = (nsel + nt - 1) / nt;
  const int beg = tid * per;
  uint32_t local = 0;
  for (int i = beg; i < beg + per && i < nsel; ++i) {
    uint32_t idx = (uint32_t)s_sel[i];
    int y = (int)(idx / (uint32_t)W), x = (int)(idx % (uint32_t)W);
    local += (y >= hw && y < H - hw && x >= hw && x < W - hw) ? 1u : 0u;
  }
  uint32_t total;
  uint32_t pos = block_exclusive_scan(local, s_scan, &total);
  for (int i = beg; i < beg + per && i < nsel; ++i) {
    uint64_t key = s_sel[i];
    uint32_t idx = (uint32_t)key;
    int y = (int)(idx / (uint32_t)W), x = (int)(idx % (uint32_t)W);
    if (y >= hw && y < H - hw && x >= hw && x < W - hw) {
      int64_t o = (int64_t)b * kcap + pos;
      kp.x[o] = x;
      kp.y[o] = y;
      kp.conf[o] = fkey_inv(~(uint32_t)(key >> 32));
      ++pos;
    }
  }
  if (tid == 0) kp.count[b] = (int32_t)total;
}

size_t topk_lds_bytes() {
  return (size_t)kTopkLdsCap * 8 + (size_t)kTieLdsCap * 8 + (size_t)kHistBins * 4 + 1024 * 4;
}

void launch_topk(const uint64_t* cand, const unsigned long long* cand_count, uint64_t* scratch,
                 KpList kp, int kcap, int k, int B, int H, int W, int half_window,
                 MedianState* state, int mode, hipStream_t st) {
  hipLaunchKernelGGL(k_topk, dim3(B), dim3(1024), topk_lds_bytes(), st, cand, cand_count, scratch, kp,
                     kcap, k, H, W, half_window, state, mode);
}

void init_topk_attributes() {
  (void)hipFuncSetAttribute((const void*)k_topk, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)topk_lds_bytes());
}

}  // namespace sfm
