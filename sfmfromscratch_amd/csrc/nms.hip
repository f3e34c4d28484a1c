// nms.hip — max-pool NMS + median threshold + candidate compaction
// (NaiveSIFT.py:77-97):
//   R_maxpool[r,c] = max of R over the ksize x ksize window clipped to the image (:85-88)
//   R_maxpool[R < median] = 0                                                    (:92)
//   candidate  <=> R == R_maxpool                                                (:95)
// i.e. (R >= med && R == window max) || (R < med && R == 0).  Candidates are appended
// per plane as 64-bit keys ~fkey(R) << 32 | raster index, so ascending key order is the
// reference's confidence-descending order with ties broken by raster index.
//
// Max is exact, so the window max is computed separably (row max, then column max) on an
// LDS tile; out-of-image cells hold -inf and never win (the window is clipped).
#include "kernels.h"

namespace sfm {

constexpr int kNT_W = 64;
constexpr int kNT_H = 32;
constexpr int kRowsPerThread = kNT_H / 4;  // 256 threads = 64 columns x 4 row groups

template <int KH>  // KH = ksize // 2 (KH_MAX = SFM_NMS_MAX_HALF when instantiated generic)
__global__ void __launch_bounds__(256) k_nms(const float* __restrict__ R,
                                             const MedianState* __restrict__ st,
                                             uint64_t* __restrict__ cand,
                                             unsigned long long* __restrict__ cand_count, int H,
                                             int W, int kh, int tiles_x) {
  constexpr int KM = KH;  // LDS sized for the template half-width
  __shared__ float s_r[kNT_H + 2 * KM][kNT_W + 2 * KM];
  __shared__ float s_m[kNT_H + 2 * KM][kNT_W];
  __shared__ uint32_t s_wsum[4];
  __shared__ unsigned long long s_base;
  const int tid = threadIdx.x;
  const int b = blockIdx.y;
  const int tx0 = (blockIdx.x % tiles_x) * kNT_W;
  const int ty0 = (blockIdx.x / tiles_x) * kNT_H;
  const int64_t n = (int64_t)H * W;
  const float* Rp = R + (int64_t)b * n;
  const int TWh = kNT_W + 2 * kh, THh = kNT_H + 2 * kh;
  for (int idx = tid; idx < THh * TWh; idx += 256) {
    int iy = idx / TWh, ix = idx - iy * TWh;
    int gy = ty0 - kh + iy, gx = tx0 - kh + ix;
    float v = -INFINITY;  // outside the image: never the (clipped) window max
    if (gy >= 0 && gy < H && gx >= 0 && gx < W) v = Rp[(int64_t)gy * W + gx];
    s_r[iy][ix] = v;
  }
  __syncthreads();
  for (int idx = tid; idx < THh * kNT_W; idx += 256) {
    int iy = idx / kNT_W, ix = idx - iy * kNT_W;
    float m = s_r[iy][ix];
    for (int d = 1; d <= 2 * kh; ++d) m = fmaxf(m, s_r[iy][ix + d]);
    s_m[iy][ix] = m;
  }
  __syncthreads();
  const float med = st[b].median;
  const int c = tid & 63;
  const int rg = tid >> 6;
  uint32_t flags = 0;
#pragma unroll
  for (int q = 0; q < kRowsPerThread; ++q) {
    const int r = rg * kRowsPerThread + q;
    const int gy = ty0 + r, gx = tx0 + c;
    if (gy < H && gx < W) {
      float m = s_m[r][c];
      for (int d = 1; d <= 2 * kh; ++d) m = fmaxf(m, s_m[r + d][c]);
      const float v = s_r[r + kh][c + kh];
      const bool pred = (v < med) ? (v == 0.0f) : (v == m);
      flags |= pred ? (1u << q) : 0u;
    }
  }
  const int64_t slot = block_append(&cand_count[(int64_t)b * kCounterStride], (uint32_t)__popc(flags), s_wsum,
                                    &s_base);
  uint64_t* out = cand + (int64_t)b * n + slot;
#pragma unroll
  for (int q = 0; q < kRowsPerThread; ++q) {
    if (flags & (1u << q)) {
      const int r = rg * kRowsPerThread + q;
      const int gy = ty0 + r, gx = tx0 + c;
      const float v = s_r[r + kh][c + kh];
      *out++ = ((uint64_t)(~fkey(v)) << 32) | (uint32_t)(gy * W + gx);
    }
  }
}

void launch_nms(const float* R, const MedianState* state, uint64_t* cand,
                unsigned long long* cand_count, int B, int H, int W, int ksize, hipStream_t st) {
  int kh = ksize / 2;
  int tiles_x = (W + kNT_W - 1) / kNT_W;
  int tiles_y = (H + kNT_H - 1) / kNT_H;
  dim3 grid(tiles_x * tiles_y, B);
  switch (kh) {
    case 0: hipLaunchKernelGGL(k_nms<0>, grid, dim3(256), 0, st, R, state, cand, cand_count, H, W, kh, tiles_x); break;
    case 1: hipLaunchKernelGGL(k_nms<1>, grid, dim3(256), 0, st, R, state, cand, cand_count, H, W, kh, tiles_x); break;
    case 2: hipLaunchKernelGGL(k_nms<2>, grid, dim3(256), 0, st, R, state, cand, cand_count, H, W, kh, tiles_x); break;
    case 3: hipLaunchKernelGGL(k_nms<3>, grid, dim3(256), 0, st, R, state, cand, cand_count, H, W, kh, tiles_x); break;
    default:
      hipLaunchKernelGGL(k_nms<SFM_NMS_MAX_HALF>, grid, dim3(256), 0, st, R, state, cand, cand_count, H, W, kh, tiles_x);
      break;
  }
}

}  // namespace sfm
