// median.hip — exact np.median of each R plane (NaiveSIFT.py:91), by radix select on
// order-preserving 32-bit keys of the float32 values.
//   even H*W: float32 (v[k1] + v[k2]) / 2 with k1 = n/2-1, k2 = n/2
//   odd  H*W: v[n/2]
// Digit 1 (top 11 bits) is histogrammed inside the Harris kernel.  Then:
//   k_med_scan    : one block per plane finds the digit-1 bucket of each rank and the
//                   certified-select threshold (kernels.h, MedianState)
//   k_med_collect : grid pass over R appending the keys that fall in those buckets
//   k_med_final   : one block per plane resolves digits 2 (11 bits) and 3 (10 bits)
// collect / final run only for planes flagged `fallback` (the exact path).
#include <algorithm>

#include "kernels.h"

namespace sfm {

// Stand-alone select scan (the diagnostic path; extraction fuses it into k_harris).
__global__ void __launch_bounds__(256) k_med_scan(const uint32_t* __restrict__ hist,
                                                  MedianState* __restrict__ st,
                                                  unsigned long long* __restrict__ list_count,
                                                  int64_t n, int64_t vmin, int force_exact) {
  __shared__ uint32_t s_red[10];
  const int b = blockIdx.x;
  select_scan_plane(hist + (int64_t)b * kMedBins1, st + b, list_count + (int64_t)b * kCounterStride, n, vmin,
                    force_exact, s_red);
}

constexpr int kCollectPerThread = 16;
constexpr int kCollectBlocksPerPlane = 64;

// Each workgroup scans chunks of 256 * 16 consecutive keys and appends the ones in the two
// target buckets with one global atomic per chunk (block_append).  Certified planes exit.
__global__ void __launch_bounds__(256) k_med_collect(const float* __restrict__ R,
                                                     const MedianState* __restrict__ st,
                                                     uint32_t* __restrict__ list,
                                                     unsigned long long* __restrict__ list_count,
                                                     int64_t n) {
  __shared__ uint32_t s_wsum[4];
  __shared__ unsigned long long s_base;
  const int b = blockIdx.y;
  if (!st[b].fallback) return;
  const uint32_t b1 = st[b].bucket[0], b2 = st[b].bucket[1];
  const float* Rp = R + (int64_t)b * n;
  const int64_t nchunks = (n + 256 * kCollectPerThread - 1) / (256 * kCollectPerThread);
  for (int64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    const int64_t base = chunk * 256 * kCollectPerThread;
    uint32_t keys[kCollectPerThread];
    uint32_t mask = 0;
#pragma unroll
    for (int q = 0; q < kCollectPerThread; ++q) {
      int64_t i = base + (int64_t)q * 256 + threadIdx.x;  // coalesced
      keys[q] = 0;
      if (i < n) {
        uint32_t key = fkey(Rp[i]);
        uint32_t d = key >> (32 - kMedBits1);
        keys[q] = key;
        if (d == b1 || d == b2) mask |= 1u << q;
      }
    }
    int64_t slot = block_append(&list_count[(int64_t)b * kCounterStride], (uint32_t)__popc(mask), s_wsum,
                                &s_base);
    uint32_t* lp = list + (int64_t)b * n + slot;
#pragma unroll
    for (int q = 0; q < kCollectPerThread; ++q)
      if (mask & (1u << q)) *lp++ = keys[q];
  }
}

__global__ void __launch_bounds__(1024) k_med_final(MedianState* __restrict__ st,
                                                    const uint32_t* __restrict__ list,
                                                    const unsigned long long* __restrict__ list_count,
                                                    int64_t n) {
  __shared__ uint32_t s_h[kHistBins];
  __shared__ uint32_t s_scan[1024];
  __shared__ uint32_t s_out[2];
  const int b = blockIdx.x;
  if (!st[b].fallback) return;
  const uint32_t* lp = list + (int64_t)b * n;
  const int64_t m = (int64_t)list_count[(int64_t)b * kCounterStride];
  MedianState s = st[b];
  uint32_t key1 = select_in_list(lp, m, s.bucket[0], s.rank[0], s_h, s_scan, s_out);
  float v1 = fkey_inv(key1);
  float med;
  if (s.odd) {
    med = v1;
  } else {
    uint32_t key2 = select_in_list(lp, m, s.bucket[1], s.rank[1], s_h, s_scan, s_out);
    float v2 = fkey_inv(key2);
    float sum = v1 + v2;
    med = sum / 2.0f;
  }
  if (threadIdx.x == 0) st[b].median = med;
}

void launch_select_scan(const uint32_t* hist, MedianState* state, unsigned long long* list_count, int B,
                        int H, int W, int64_t vmin, int force_exact, hipStream_t st) {
  int64_t n = (int64_t)H * W;
  hipLaunchKernelGGL(k_med_scan, dim3(B), dim3(256), 0, st, hist, state, list_count, n, vmin, force_exact);
}

void launch_median_exact(const float* R, MedianState* state, uint32_t* list, unsigned long long* list_count,
                         int B, int H, int W, hipStream_t st) {
  int64_t n = (int64_t)H * W;
  int64_t nchunks = (n + 256 * kCollectPerThread - 1) / (256 * kCollectPerThread);
  int gx = (int)std::min<int64_t>(nchunks, kCollectBlocksPerPlane);
  hipLaunchKernelGGL(k_med_collect, dim3(gx, B), dim3(256), 0, st, R, state, list, list_count, n);
  hipLaunchKernelGGL(k_med_final, dim3(B), dim3(1024), 0, st, state, list, list_count, n);
}

}  // namespace sfm
