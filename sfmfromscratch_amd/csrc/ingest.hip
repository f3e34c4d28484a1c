// ingest.hip — FeatureRunner's frame ingest (Runner.py:33-46) on the device: decoded RGB
// frames -> PIL BICUBIC resize (Runner.py:37-42, _PIL_resize :481-493) -> /255 ->
// _rgb2gray (:467-478) -> the float32 gray frames the extractor takes.
//
// The resize is Pillow's 8-bit resampler (libImaging/Resample.c; Pillow 11.0.0 pinned at
// requirements.txt:27): per output column / row a window of double-precision bicubic
// taps (a = -0.5, support 2 x the downscale factor, normalised by their sum), converted
// to 22-bit fixed point (normalize_coeffs_8bpc), then a horizontal pass over every source
// row and a vertical pass, each (1 << 21) + sum(u8 * tap) in int32, clipped to u8
// (clip8).  The tap tables are built on the host with the same double arithmetic
// (build_resample_table); both passes run here in integers, so the u8 result is exactly
// PIL's.  The gray conversion is float32 u8/255 (_PIL_image_to_numpy_arr) then
// (r*0.299f + g*0.587f) + b*0.114f with each product rounded (NEP 50 weak scalars).
//
// HBM-bound: the horizontal pass reads the RGB frame once and writes an RGB temp of
// H x W2; the vertical pass reads it once and writes the gray frame (4K -> 1080p:
// 24.9 + 12.4 + 12.4 + 8.3 MB per frame).
#include <math.h>

#include <vector>

#include "kernels.h"

namespace sfm {

constexpr int kResPrec = 22;  // PRECISION_BITS = 32 - 8 - 2

SFM_DEV uint32_t clip8(int ss) {
  if (ss >= (1 << kResPrec << 8)) return 255u;
  if (ss <= 0) return 0u;
  return (uint32_t)(ss >> kResPrec);
}

// table row o: [xmin, count, tap_0 .. tap_{ksize-1}] (int32)
__global__ void __launch_bounds__(256) k_resample_h(const uint8_t* __restrict__ rgb, uint8_t* __restrict__ tmp,
                                                    const int32_t* __restrict__ tab, int ksize, int H, int W,
                                                    int W2) {
  const int x2 = blockIdx.x * 256 + threadIdx.x;
  const int y = blockIdx.y, b = blockIdx.z;
  if (x2 >= W2) return;
  const int32_t* t = tab + (int64_t)x2 * (2 + ksize);
  const int xmin = t[0], cnt = t[1];
  const uint8_t* src = rgb + (((int64_t)b * H + y) * W + xmin) * 3;
  int s0 = 1 << (kResPrec - 1), s1 = s0, s2 = s0;
  for (int k = 0; k < cnt; ++k) {
    const int w = t[2 + k];
    s0 += (int)src[3 * k + 0] * w;
    s1 += (int)src[3 * k + 1] * w;
    s2 += (int)src[3 * k + 2] * w;
  }
  uint8_t* dst = tmp + (((int64_t)b * H + y) * W2 + x2) * 3;
  dst[0] = (uint8_t)clip8(s0);
  dst[1] = (uint8_t)clip8(s1);
  dst[2] = (uint8_t)clip8(s2);
}

__global__ void __launch_bounds__(256) k_resample_v_gray(const uint8_t* __restrict__ tmp, float* __restrict__ gray,
                                                         const int32_t* __restrict__ tab, int ksize, int H, int W2,
                                                         int H2) {
  const int x2 = blockIdx.x * 256 + threadIdx.x;
  const int y2 = blockIdx.y, b = blockIdx.z;
  if (x2 >= W2) return;
  const int32_t* t = tab + (int64_t)y2 * (2 + ksize);
  const int ymin = t[0], cnt = t[1];
  const uint8_t* src = tmp + (((int64_t)b * H + ymin) * W2 + x2) * 3;
  const int64_t rs = (int64_t)W2 * 3;
  int s0 = 1 << (kResPrec - 1), s1 = s0, s2 = s0;
  for (int k = 0; k < cnt; ++k) {
    const int w = t[2 + k];
    s0 += (int)src[k * rs + 0] * w;
    s1 += (int)src[k * rs + 1] * w;
    s2 += (int)src[k * rs + 2] * w;
  }
  const float r = (float)clip8(s0) / 255.0f, g = (float)clip8(s1) / 255.0f, bl = (float)clip8(s2) / 255.0f;
  const float t0 = r * 0.299f, t1 = g * 0.587f, t2 = bl * 0.114f;
  gray[((int64_t)b * H2 + y2) * W2 + x2] = (t0 + t1) + t2;
}

// bicubic_filter of Resample.c (a = -0.5)
static double bicubic_tap(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

// precompute_coeffs (box [0, in)) + normalize_coeffs_8bpc; out == in gives the identity
// (PIL skips that pass; a single tap of 1.0 reproduces the input exactly)
int build_resample_table(int in, int out, std::vector<int32_t>& tab) {
  if (in == out) {
    tab.assign((size_t)out * 3, 0);
    for (int o = 0; o < out; ++o) {
      tab[(size_t)o * 3 + 0] = o;
      tab[(size_t)o * 3 + 1] = 1;
      tab[(size_t)o * 3 + 2] = 1 << kResPrec;
    }
    return 1;
  }
  double scale = (double)(in - 0) / out, filterscale = scale;
  if (filterscale < 1.0) filterscale = 1.0;
  const double support = 2.0 * filterscale;
  const int ksize = (int)ceil(support) * 2 + 1;
  tab.assign((size_t)out * (2 + ksize), 0);
  std::vector<double> k(ksize);
  for (int xx = 0; xx < out; ++xx) {
    const double center = 0 + (xx + 0.5) * scale;
    double ww = 0.0;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in) xmax = in;
    xmax -= xmin;
    for (int x = 0; x < ksize; ++x) k[x] = 0.0;
    for (int x = 0; x < xmax; ++x) {
      const double w = bicubic_tap((x + xmin - center + 0.5) * ss);
      k[x] = w;
      ww += w;
    }
    for (int x = 0; x < xmax; ++x)
      if (ww != 0.0) k[x] /= ww;
    int32_t* t = &tab[(size_t)xx * (2 + ksize)];
    t[0] = xmin;
    t[1] = xmax;
    for (int x = 0; x < ksize; ++x)
      t[2 + x] = k[x] < 0 ? (int32_t)(-0.5 + k[x] * (1 << kResPrec)) : (int32_t)(0.5 + k[x] * (1 << kResPrec));
  }
  return ksize;
}

void launch_ingest_rgb(const uint8_t* rgb, uint8_t* tmp, float* gray, const int32_t* tab_h, int ks_h,
                       const int32_t* tab_v, int ks_v, int B, int H, int W, int H2, int W2, hipStream_t st) {
  hipLaunchKernelGGL(k_resample_h, dim3((W2 + 255) / 256, H, B), dim3(256), 0, st, rgb, tmp, tab_h, ks_h, H, W, W2);
  hipLaunchKernelGGL(k_resample_v_gray, dim3((W2 + 255) / 256, H2, B), dim3(256), 0, st, tmp, gray, tab_v, ks_v, H,
                     W2, H2);
}

}  // namespace sfm
