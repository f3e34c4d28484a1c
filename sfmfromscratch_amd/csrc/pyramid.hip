// pyramid.hip — image ingest and the resize pyramid (ScaleRotInvSIFT._build_image_pyramid,
// ScaleRotInvSIFT.py:109-115: level i = cv2.resize(level i-1, (int(w/s), int(h/s)))).
//
// HBM-bound streaming kernels.  Two resize rules (the restatement of cv2.resize
// INTER_LINEAR on float32):
//   * exact 2x in both axes -> OpenCV's INTER_AREA-fast switch: ((a00+a01)+(a10+a11))*0.25
//   * otherwise half-pixel bilinear with OpenCV's coefficient rule.
// Planes of all B images of one level are contiguous: [B][h][w] float32.
#include <algorithm>

#include "kernels.h"

namespace sfm {

static int grid_for(int64_t n, int per_thread);

// uint8 -> float32 value/255 (Runner.py:521).  4 pixels per thread, 16-byte stores.
__global__ void __launch_bounds__(256) k_u8_to_f32(const uint8_t* __restrict__ src,
                                                   float* __restrict__ dst, int64_t n) {
  int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (; i + 3 < n; i += stride) {
    uchar4 v = *reinterpret_cast<const uchar4*>(src + i);
    float4 o;
    o.x = (float)v.x / 255.0f;
    o.y = (float)v.y / 255.0f;
    o.z = (float)v.z / 255.0f;
    o.w = (float)v.w / 255.0f;
    *reinterpret_cast<float4*>(dst + i) = o;
  }
  for (; i < n; ++i) dst[i] = (float)src[i] / 255.0f;
}

// Exact 2x downscale: each thread produces 2 horizontally adjacent outputs.
__global__ void __launch_bounds__(256) k_down2(const float* __restrict__ src, int sh, int sw,
                                               float* __restrict__ dst, int dh, int dw, int B) {
  int half = (dw + 1) >> 1;
  int64_t total = (int64_t)B * dh * half;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    int xh = (int)(t % half);
    int64_t r = t / half;
    int y = (int)(r % dh);
    int b = (int)(r / dh);
    const float* s0 = src + ((int64_t)b * sh + 2 * y) * sw;
    const float* s1 = s0 + sw;
    float* d = dst + ((int64_t)b * dh + y) * dw;
    int x = 2 * xh;
    {
      float t0 = s0[2 * x] + s0[2 * x + 1];
      float t1 = s1[2 * x] + s1[2 * x + 1];
      d[x] = (t0 + t1) * 0.25f;
    }
    if (x + 1 < dw) {
      float t0 = s0[2 * x + 2] + s0[2 * x + 3];
      float t1 = s1[2 * x + 2] + s1[2 * x + 3];
      d[x + 1] = (t0 + t1) * 0.25f;
    }
  }
}

// Three exact 2x levels in one pass (level l -> l+1, l+2, l+3): each thread reads one
// 8 x 8 block of level l with 16-B loads and writes its 4 x 4, 2 x 2 and 1 x 1 blocks,
// every value ((a00 + a01) + (a10 + a11)) * 0.25 of the level above, exactly k_down2's
// expression, so the levels are bit-identical to three k_down2 launches — without
// re-reading levels l+1 and l+2.  Needs sh, sw divisible by 8 and 16-B aligned planes.
__global__ void __launch_bounds__(256) k_down2x3(const float* __restrict__ src, int sh, int sw,
                                                 float* __restrict__ d1, float* __restrict__ d2,
                                                 float* __restrict__ d3, int B, uint4* __restrict__ z0,
                                                 int64_t n0, uint4* __restrict__ z1, int64_t n1) {
  // side job: zero the extraction's histograms and counters (z0 / z1, 16-B units), so the
  // step needs no separate fill launches ahead of Harris
  {
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, gs = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = i0; i < n0; i += gs) z0[i] = make_uint4(0u, 0u, 0u, 0u);
    for (int64_t i = i0; i < n1; i += gs) z1[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  const int bw = sw >> 3, bh = sh >> 3;
  const int64_t total = (int64_t)B * bh * bw;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int bx = (int)(t % bw);
    const int64_t r = t / bw;
    const int by = (int)(r % bh);
    const int b = (int)(r / bh);
    const float* s = src + ((int64_t)b * sh + 8 * by) * sw + 8 * bx;
    float a[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float4 lo = *reinterpret_cast<const float4*>(s + (int64_t)i * sw);
      const float4 hi = *reinterpret_cast<const float4*>(s + (int64_t)i * sw + 4);
      a[i][0] = lo.x; a[i][1] = lo.y; a[i][2] = lo.z; a[i][3] = lo.w;
      a[i][4] = hi.x; a[i][5] = hi.y; a[i][6] = hi.z; a[i][7] = hi.w;
    }
    down2x3_block(a, d1, d2, d3, b, sh, sw, by, bx);
  }
}

bool launch_down2x3(const float* src, int sh, int sw, float* d1, float* d2, float* d3, int B, hipStream_t st,
                    void* z0, size_t z0_bytes, void* z1, size_t z1_bytes) {
  const bool ok = sh % 8 == 0 && sw % 8 == 0 && sh >= 8 && sw >= 8 && ((uintptr_t)src & 15) == 0 &&
                  ((uintptr_t)d1 & 15) == 0 && ((uintptr_t)d2 & 7) == 0 && ((uintptr_t)z0 & 15) == 0 &&
                  ((uintptr_t)z1 & 15) == 0 && z0_bytes % 16 == 0 && z1_bytes % 16 == 0;
  if (!ok) return false;
  const int64_t n = (int64_t)B * (sh / 8) * (sw / 8);
  const int64_t n0 = z0 ? (int64_t)(z0_bytes / 16) : 0, n1 = z1 ? (int64_t)(z1_bytes / 16) : 0;
  hipLaunchKernelGGL(k_down2x3, dim3(grid_for(std::max(n, std::max(n0, n1)), 1)), dim3(256), 0, st, src, sh, sw,
                     d1, d2, d3, B, static_cast<uint4*>(z0), n0, static_cast<uint4*>(z1), n1);
  return true;
}

struct LinCoef {
  int s;
  float a0, a1;
  bool single;
};

// OpenCV INTER_LINEAR coefficient rule (resize.cpp, float path), restated.
SFM_DEV LinCoef lin_coef(int d, int sn, double scale) {
  LinCoef c;
  float f = (float)(((double)d + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f -= (float)s;
  c.single = false;
  if (s < 0) { s = 0; f = 0.0f; }
  if (s + 1 >= sn) {
    c.single = true;
    if (s >= sn - 1) { s = sn - 1; f = 0.0f; }
  }
  c.s = s;
  c.a0 = 1.0f - f;
  c.a1 = f;
  return c;
}

__global__ void __launch_bounds__(256) k_resize_linear(const float* __restrict__ src, int sh, int sw,
                                                       float* __restrict__ dst, int dh, int dw, int B,
                                                       double scale_x, double scale_y) {
  int64_t total = (int64_t)B * dh * dw;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    int x = (int)(t % dw);
    int64_t r = t / dw;
    int y = (int)(r % dh);
    int b = (int)(r / dh);
    LinCoef cx = lin_coef(x, sw, scale_x);
    LinCoef cy = lin_coef(y, sh, scale_y);
    int sy1 = cy.s + 1 < sh ? cy.s + 1 : sh - 1;
    const float* base = src + (int64_t)b * sh * sw;
    const float* rows[2] = {base + (int64_t)cy.s * sw, base + (int64_t)sy1 * sw};
    float h[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const float* S = rows[k];
      if (cx.single) {
        h[k] = S[cx.s];
      } else {
        float p = S[cx.s] * cx.a0;
        float q = S[cx.s + 1] * cx.a1;
        h[k] = p + q;
      }
    }
    float p = h[0] * cy.a0;
    float q = h[1] * cy.a1;
    dst[t] = p + q;
  }
}

static int grid_for(int64_t n, int per_thread) {
  int64_t blocks = (n / per_thread + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 8192) blocks = 8192;
  return (int)blocks;
}

void launch_u8_to_f32(const uint8_t* src, float* dst, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(k_u8_to_f32, dim3(grid_for(n, 4)), dim3(256), 0, st, src, dst, n);
}

void launch_resize(const float* src, int sh, int sw, float* dst, int dh, int dw, int B,
                   hipStream_t st) {
  if (sh == 2 * dh && sw == 2 * dw) {
    int64_t n = (int64_t)B * dh * ((dw + 1) / 2);
    hipLaunchKernelGGL(k_down2, dim3(grid_for(n, 1)), dim3(256), 0, st, src, sh, sw, dst, dh, dw, B);
  } else {
    double scale_x = 1.0 / ((double)dw / (double)sw);
    double scale_y = 1.0 / ((double)dh / (double)sh);
    int64_t n = (int64_t)B * dh * dw;
    hipLaunchKernelGGL(k_resize_linear, dim3(grid_for(n, 1)), dim3(256), 0, st, src, sh, sw, dst, dh,
                       dw, B, scale_x, scale_y);
  }
}

}  // namespace sfm
