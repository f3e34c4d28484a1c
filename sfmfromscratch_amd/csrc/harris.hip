// harris.hip — fused Harris response (NaiveSIFT._find_harris_interest_points,
// NaiveSIFT.py:59-74): Sobel gradients -> Ix^2, Iy^2, IxIy -> three 2-D Gaussian
// window sums -> R = det - alpha * trace^2, plus the first radix digit histogram of R
// for the exact median (NaiveSIFT.py:91).
//
// One workgroup (256 threads, 4 waves) owns a 64 x 32 output tile of one plane.  The
// image tile (+ Sobel and window halo) and the three product planes live in LDS; each
// thread then accumulates a 1 x 4 horizontal strip for two rows.  The 2-D window is the
// reference's full KS x KS correlation (not separable: a separable sum would round
// differently and move keypoints), accumulated per pixel as an fma chain
// in row-major tap order (OpenCV FilterVec_32f's v_muladd chain).
// VALU-bound by design.
#include <algorithm>

#include "kernels.h"

namespace sfm {

constexpr int kHT_W = 64;
constexpr int kHT_H = 32;

template <int KS>
__global__ void __launch_bounds__(256) k_harris(const float* __restrict__ lvl, float* __restrict__ Rout,
                                                uint32_t* __restrict__ hist_g, int H, int W,
                                                int tiles_x, int ntiles,
                                                const float* __restrict__ gk, float alpha) {
  constexpr int GA = KS / 2;
  constexpr int PW = kHT_W + KS - 1;
  constexpr int PH = kHT_H + KS - 1;
  constexpr int IW = PW + 2;
  constexpr int IH = PH + 2;
  __shared__ float s_prod[3][PH][PW];
  __shared__ float s_img[IH * IW];
  __shared__ uint32_t s_hist[kHistBins];  // digit-1 histogram, flushed once per workgroup

  const int tid = threadIdx.x;
  const int b = blockIdx.y;
  const float* img = lvl + (int64_t)b * H * W;
  for (int i = tid; i < kHistBins; i += 256) s_hist[i] = 0u;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
  const int tx0 = (tile % tiles_x) * kHT_W;
  const int ty0 = (tile / tiles_x) * kHT_H;
  __syncthreads();  // previous tile's LDS reads are done

  // 1. image tile with zero border (BORDER_CONSTANT)
  for (int idx = tid; idx < IH * IW; idx += 256) {
    int iy = idx / IW, ix = idx - iy * IW;
    int gy = ty0 - GA - 1 + iy, gx = tx0 - GA - 1 + ix;
    float v = 0.0f;
    if (gy >= 0 && gy < H && gx >= 0 && gx < W) v = img[(int64_t)gy * W + gx];
    s_img[idx] = v;
  }
  __syncthreads();

  // 2. gradients (NaiveSIFT.py:201-213): fma chain over the non-zero taps in row-major order
  //    from acc = +0 (k*p is exact for the Sobel taps) and products
  for (int idx = tid; idx < PH * PW; idx += 256) {
    int py = idx / PW, px = idx - py * PW;
    int gy = ty0 - GA + py, gx = tx0 - GA + px;
    float pxx = 0.0f, pyy = 0.0f, pxy = 0.0f;
    if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
      const float* c = s_img + (py + 1) * IW + (px + 1);
      float a00 = c[-IW - 1], a01 = c[-IW], a02 = c[-IW + 1];
      float a10 = c[-1], a12 = c[1];
      float a20 = c[IW - 1], a21 = c[IW], a22 = c[IW + 1];
      float ix = 0.0f;
      ix = __builtin_fmaf(-1.0f, a00, ix);
      ix = __builtin_fmaf(1.0f, a02, ix);
      ix = __builtin_fmaf(-2.0f, a10, ix);
      ix = __builtin_fmaf(2.0f, a12, ix);
      ix = __builtin_fmaf(-1.0f, a20, ix);
      ix = __builtin_fmaf(1.0f, a22, ix);
      float iy = 0.0f;
      iy = __builtin_fmaf(-1.0f, a00, iy);
      iy = __builtin_fmaf(-2.0f, a01, iy);
      iy = __builtin_fmaf(-1.0f, a02, iy);
      iy = __builtin_fmaf(1.0f, a20, iy);
      iy = __builtin_fmaf(2.0f, a21, iy);
      iy = __builtin_fmaf(1.0f, a22, iy);
      pxx = ix * ix;  // Ix ** 2  :61
      pyy = iy * iy;  // Iy ** 2  :62
      pxy = ix * iy;  // Ix * Iy  :63
    }
    s_prod[0][py][px] = pxx;
    s_prod[1][py][px] = pyy;
    s_prod[2][py][px] = pxy;
  }
  __syncthreads();

  // 3. window sums: thread owns columns 4*tq .. 4*tq+3 of rows ry and ry+16; the three
  //    planes are accumulated together, taps in row-major order per pixel
  const int tq = tid & 15;
  const int ry0 = tid >> 4;
#pragma unroll 1
  for (int half = 0; half < 2; ++half) {
    const int r = ry0 + half * 16;
    float acc[3][4];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[pl][q] = 0.0f;
#pragma unroll 1
    for (int i = 0; i < KS; ++i) {
      float v[3][4 + KS - 1];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        const float* row = &s_prod[pl][r + i][4 * tq];
#pragma unroll
        for (int j = 0; j < 4 + KS - 1; ++j) v[pl][j] = row[j];
      }
#pragma unroll
      for (int j = 0; j < KS; ++j) {
        const float kk = gk[i * KS + j];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            acc[pl][q] = __builtin_fmaf(kk, v[pl][q + j], acc[pl][q]);
          }
      }
    }
    const int gy = ty0 + r;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int gx = tx0 + 4 * tq + q;
      float sxx = acc[0][q], syy = acc[1][q], sxy = acc[2][q];
      float t1 = sxx * syy;
      float t2 = sxy * sxy;
      float det = t1 - t2;     // :71
      float tr = sxx + syy;    // :72
      float tr2 = tr * tr;
      float at = alpha * tr2;
      float Rv = det - at;     // :74
      if (gy < H && gx < W) {
        Rout[(int64_t)b * H * W + (int64_t)gy * W + gx] = Rv;
        atomicAdd(&s_hist[fkey(Rv) >> (32 - kHistBits)], 1u);
      }
    }
  }
  }  // tile loop
  __syncthreads();
  uint32_t* hg = hist_g + (int64_t)b * kHistBins;
  for (int i = tid; i < kHistBins; i += 256) {
    uint32_t c = s_hist[i];
    if (c) atomicAdd(&hg[i], c);
  }
}

template <int KS>
static void launch_ks(const float* lvl, float* R, uint32_t* hist, int B, int H, int W,
                      const float* gk, float alpha, hipStream_t st) {
  int tiles_x = (W + kHT_W - 1) / kHT_W;
  int tiles_y = (H + kHT_H - 1) / kHT_H;
  int ntiles = tiles_x * tiles_y;
  // ~4 resident workgroups per CU over the whole batch; each loops over tiles so the
  // digit histogram is flushed once per workgroup instead of once per tile
  int per_plane = std::max(1, std::min(ntiles, 512 / std::max(B, 1)));
  hipLaunchKernelGGL(k_harris<KS>, dim3(per_plane, B), dim3(256), 0, st, lvl, R, hist, H, W, tiles_x,
                     ntiles, gk, alpha);
}

void launch_harris(const float* lvl, float* R, uint32_t* hist, int B, int H, int W,
                   const float* d_gauss, int ks, float alpha, hipStream_t st) {
  switch (ks) {
    case 1: launch_ks<1>(lvl, R, hist, B, H, W, d_gauss, alpha, st); break;
    case 2: launch_ks<2>(lvl, R, hist, B, H, W, d_gauss, alpha, st); break;
    case 3: launch_ks<3>(lvl, R, hist, B, H, W, d_gauss, alpha, st); break;
    case 4: launch_ks<4>(lvl, R, hist, B, H, W, d_gauss, alpha, st); break;
    case 5: launch_ks<5>(lvl, R, hist, B, H, W, d_gauss, alpha, st); break;
    case 6: launch_ks<6>(lvl, R, hist, B, H, W, d_gauss, alpha, st); break;
    case 7: launch_ks<7>(lvl, R, hist, B, H, W, d_gauss, alpha, st); break;
    case 8: launch_ks<8>(lvl, R, hist, B, H, W, d_gauss, alpha, st); break;
    case 9: launch_ks<9>(lvl, R, hist, B, H, W, d_gauss, alpha, st); break;
    case 11: launch_ks<11>(lvl, R, hist, B, H, W, d_gauss, alpha, st); break;
    case 13: launch_ks<13>(lvl, R, hist, B, H, W, d_gauss, alpha, st); break;
    case 15: launch_ks<15>(lvl, R, hist, B, H, W, d_gauss, alpha, st); break;
    default: break;  // rejected at context creation
  }
}

}  // namespace sfm
