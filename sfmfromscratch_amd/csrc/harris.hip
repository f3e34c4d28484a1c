// harris.hip — fused Harris response (NaiveSIFT._find_harris_interest_points,
// NaiveSIFT.py:59-74): Sobel gradients -> Ix^2, Iy^2, IxIy -> three 2-D Gaussian
// window sums -> R = det - alpha * trace^2, plus the first radix digit histogram of R
// for the exact median (NaiveSIFT.py:91).
//
// One workgroup (256 threads, 4 waves) walks 64 x 32 output tiles of one plane.  The three
// product planes of a tile (+ window halo) live in LDS; each thread accumulates an 8-pixel
// row segment (14-float windows read with 16-B LDS loads: ~0.07 LDS reads per fma).  The 2-D window is the
// reference's full KS x KS correlation (not separable: a separable sum would round
// differently and move keypoints), accumulated per pixel as an fma chain
// in row-major tap order (OpenCV FilterVec_32f's v_muladd chain).
// VALU-bound by design.
#include <algorithm>

#include "kernels.h"

namespace sfm {

constexpr int kHT_W = 64;   // output tile width  (8 threads x 8 pixels)
constexpr int kHT_H = 32;   // output tile height (32 thread rows)

template <int KS>
__global__ void __launch_bounds__(256) k_harris(const float* __restrict__ lvl, float* __restrict__ Rout,
                                                uint32_t* __restrict__ hist_g, int H, int W,
                                                int tiles_x, int ntiles,
                                                const float* __restrict__ gk, float alpha) {
  constexpr int GA = KS / 2;
  constexpr int PW = kHT_W + KS - 1;        // product tile width
  constexpr int PH = kHT_H + KS - 1;        // product tile height
  // row stride S = PW rounded up to S % 4 == 2 floats.  Lanes walk rows fastest
  // (r = tid & 31), so a 16-lane LDS group reads 16 rows whose 8-B words sit at
  // bank offsets r*S mod 32 = distinct even banks (S/2 odd) -> conflict-free b64 reads
  constexpr int PWP = (PW % 4 == 2) ? PW : PW + ((6 - PW % 4) % 4);
  constexpr int NV = 8 + KS - 1;            // window values per row per plane
  constexpr int NV2 = (NV + 1) / 2;         // float2 loads per row per plane
  constexpr int NVP = 2 * NV2;
  static_assert(PWP % 4 == 2 && PWP >= PW && 56 + NVP <= PWP + 2, "harris LDS row stride");
  __shared__ __attribute__((aligned(16))) float s_prod[3][PH][PWP];  // rows 8-B aligned
  __shared__ uint32_t s_hist[kHistBins];  // digit-1 histogram, flushed once per workgroup

  const int tid = threadIdx.x;
  const int b = blockIdx.y;
  const float* img = lvl + (int64_t)b * H * W;
  for (int i = tid; i < kHistBins; i += 256) s_hist[i] = 0u;
  const int r = tid & 31;      // output row in the tile (fastest across lanes)
  const int tq = tid >> 5;     // 8 pixel columns 8*tq .. 8*tq+7
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int tx0 = (tile % tiles_x) * kHT_W;
    const int ty0 = (tile / tiles_x) * kHT_H;
    __syncthreads();  // previous tile's LDS reads are done
    // 1. gradients (NaiveSIFT.py:201-213, fma chain over the non-zero taps in row-major
    //    order from +0; k*p is exact for the Sobel taps) and products Ix^2, Iy^2, IxIy
    //    (:61-63).  Image taps come straight from global memory (L1-resident tile).
    for (int idx = tid; idx < PH * PW; idx += 256) {
      const int py = idx / PW, px = idx - py * PW;
      const int gy = ty0 - GA + py, gx = tx0 - GA + px;
      float pxx = 0.0f, pyy = 0.0f, pxy = 0.0f;
      const bool inside = gy >= 0 && gy < H && gx >= 0 && gx < W;
      {
        // branch-free taps: clamped (always valid) addresses, all nine loads issued before
        // one wait, zero outside the image (BORDER_CONSTANT)
        float t[9];
        bool ok[9];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
          const int yy = gy + dy - 1;
          const int yc = min(max(yy, 0), H - 1);
#pragma unroll
          for (int dx = 0; dx < 3; ++dx) {
            const int xx = gx + dx - 1;
            const int xc = min(max(xx, 0), W - 1);
            t[dy * 3 + dx] = img[(int64_t)yc * W + xc];
            ok[dy * 3 + dx] = yy >= 0 && yy < H && xx >= 0 && xx < W;
          }
        }
        asm volatile("" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]),
                     "+v"(t[6]), "+v"(t[7]), "+v"(t[8]));
        float a[3][3];
#pragma unroll
        for (int q = 0; q < 9; ++q) a[q / 3][q % 3] = ok[q] ? t[q] : 0.0f;
        float ix = 0.0f;
        ix = __builtin_fmaf(-1.0f, a[0][0], ix);
        ix = __builtin_fmaf(1.0f, a[0][2], ix);
        ix = __builtin_fmaf(-2.0f, a[1][0], ix);
        ix = __builtin_fmaf(2.0f, a[1][2], ix);
        ix = __builtin_fmaf(-1.0f, a[2][0], ix);
        ix = __builtin_fmaf(1.0f, a[2][2], ix);
        float iy = 0.0f;
        iy = __builtin_fmaf(-1.0f, a[0][0], iy);
        iy = __builtin_fmaf(-2.0f, a[0][1], iy);
        iy = __builtin_fmaf(-1.0f, a[0][2], iy);
        iy = __builtin_fmaf(1.0f, a[2][0], iy);
        iy = __builtin_fmaf(2.0f, a[2][1], iy);
        iy = __builtin_fmaf(1.0f, a[2][2], iy);
        pxx = inside ? ix * ix : 0.0f;
        pyy = inside ? iy * iy : 0.0f;
        pxy = inside ? ix * iy : 0.0f;
      }
      s_prod[0][py][px] = pxx;
      s_prod[1][py][px] = pyy;
      s_prod[2][py][px] = pxy;
    }
    __syncthreads();

    // 2. window sums (:67-69): per pixel an fma chain over the KS x KS taps in row-major
    //    order; each thread accumulates an 8-pixel row segment for the three planes.
    float acc[3][8];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[pl][q] = 0.0f;
#pragma unroll 2
    for (int i = 0; i < KS; ++i) {
      float v[3][NVP];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        const float2* row = reinterpret_cast<const float2*>(&s_prod[pl][r + i][8 * tq]);
#pragma unroll
        for (int c2 = 0; c2 < NV2; ++c2) {
          const float2 t = row[c2];
          v[pl][2 * c2 + 0] = t.x;
          v[pl][2 * c2 + 1] = t.y;
        }
      }
#pragma unroll
      for (int j = 0; j < KS; ++j) {
        const float kk = gk[i * KS + j];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[pl][q] = __builtin_fmaf(kk, v[pl][q + j], acc[pl][q]);
      }
    }
    // 3. R = det - alpha * trace^2 (:71-74), digit-1 histogram of R
    const int gy = ty0 + r;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int gx = tx0 + 8 * tq + q;
      const float sxx = acc[0][q], syy = acc[1][q], sxy = acc[2][q];
      const float t1 = sxx * syy;
      const float t2 = sxy * sxy;
      const float det = t1 - t2;
      const float tr = sxx + syy;
      const float tr2 = tr * tr;
      const float at = alpha * tr2;
      const float Rv = det - at;
      if (gy < H && gx < W) {
        Rout[(int64_t)b * H * W + (int64_t)gy * W + gx] = Rv;
        atomicAdd(&s_hist[fkey(Rv) >> (32 - kHistBits)], 1u);
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
  int per_plane = std::max(1, std::min(ntiles, 768 / std::max(B, 1)));
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
