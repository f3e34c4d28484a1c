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
constexpr int kNT_H = 16;
constexpr int kMaxHalf = SFM_NMS_MAX_HALF;

__global__ void __launch_bounds__(256) k_nms(const float* __restrict__ R,
                                             const MedianState* __restrict__ st,
                                             uint64_t* __restrict__ cand,
                                             unsigned long long* __restrict__ cand_count, int H,
                                             int W, int kh, int tiles_x) {
  __shared__ float s_r[kNT_H + 2 * kMaxHalf][kNT_W + 2 * kMaxHalf];
  __shared__ float s_m[kNT_H + 2 * kMaxHalf][kNT_W];
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
    float v = -INFINITY;
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
  uint64_t keys[4];
  bool flag[4];
  uint32_t cnt = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = rg * 4 + q;
    const int gy = ty0 + r, gx = tx0 + c;
    flag[q] = false;
    keys[q] = 0;
    if (gy < H && gx < W) {
      float m = s_m[r][c];
      for (int d = 1; d <= 2 * kh; ++d) m = fmaxf(m, s_m[r + d][c]);
      float v = s_r[r + kh][c + kh];
      flag[q] = (v < med) ? (v == 0.0f) : (v == m);
      keys[q] = ((uint64_t)(~fkey(v)) << 32) | (uint32_t)(gy * W + gx);
    }
    cnt += flag[q] ? 1u : 0u;
  }
  __shared__ uint32_t s_wsum[4];
  __shared__ unsigned long long s_base;
  int64_t slot = block_append(&cand_count[(int64_t)b * kCounterStride], cnt, s_wsum, &s_base);
  uint64_t* out = cand + (int64_t)b * n + slot;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (flag[q]) *out++ = keys[q];
}

void launch_nms(const float* R, const MedianState* state, uint64_t* cand,
                unsigned long long* cand_count, int B, int H, int W, int ksize, hipStream_t st) {
  int kh = ksize / 2;
  int tiles_x = (W + kNT_W - 1) / kNT_W;
  int tiles_y = (H + kNT_H - 1) / kNT_H;
  hipLaunchKernelGGL(k_nms, dim3(tiles_x * tiles_y, B), dim3(256), 0, st, R, state, cand, cand_count,
                     H, W, kh, tiles_x);
}

}  // namespace sfm
