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
// HBM-bound, two passes through an RGB temp of H x W2 (4K -> 1080p per frame: 24.9 MB
// read + 12.4 written, 12.4 read (L2-assisted) + 8.3 written).  k_rows_h / k_rows_v
// stream whole rows (below); other shapes take the per-pixel k_resample_h /
// k_resample_v_gray.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "kernels.h"

namespace sfm {

constexpr int kResPrec = 22;  // PRECISION_BITS = 32 - 8 - 2

// u8 x 22-bit tap + acc: both factors fit 24-bit signed, so one full-rate v_mad_i32_i24
// (a 32-bit integer multiply runs at a quarter of the VALU rate); exact int32 as in PIL
SFM_DEV int mad24(int a, int b, int c) { return __mul24(a, b) + c; }

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
    s0 = mad24((int)src[3 * k + 0], w, s0);
    s1 = mad24((int)src[3 * k + 1], w, s1);
    s2 = mad24((int)src[3 * k + 2], w, s2);
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
    s0 = mad24((int)src[k * rs + 0], w, s0);
    s1 = mad24((int)src[k * rs + 1], w, s1);
    s2 = mad24((int)src[k * rs + 2], w, s2);
  }
  const float r = (float)clip8(s0) / 255.0f, g = (float)clip8(s1) / 255.0f, bl = (float)clip8(s2) / 255.0f;
  const float t0 = r * 0.299f, t1 = g * 0.587f, t2 = bl * 0.114f;
  gray[((int64_t)b * H2 + y2) * W2 + x2] = (t0 + t1) + t2;
}

// Row-streaming two-pass path (W % 4 == 0, W2 % 4 == 0).
//
// k_rows_h: persistent workgroups walk source rows; a whole RGB row (W*3 bytes) is staged
// in LDS with 4-byte loads, the next row's words prefetched into registers while the
// current row computes.  Each output column reads its KS taps from a deduplicated tap-set
// table in LDS (for a x0.5 resize all interior columns share one set, so the reads are
// broadcasts), and the u8 results are packed in an LDS output row and stored as words.
// k_rows_v: one thread per 4 output columns of one output row: KS temp rows x 12 bytes,
// the row's taps uniform (scalar loads), gray via per-channel lookup tables.
constexpr int kRowsMaxW = 4096;      // source row width staged in LDS (pixels)
constexpr int kRowsMaxW2 = 4096;
constexpr int kRowsMaxSets = 64;

template <int KS>
__global__ void __launch_bounds__(256) k_rows_h(const uint8_t* __restrict__ rgb, uint8_t* __restrict__ tmp,
                                                const int32_t* __restrict__ colmap, const int32_t* __restrict__ sets,
                                                int nsets, int nrows, int W, int W2) {
  constexpr int NW = kRowsMaxW * 3 / 4;            // words of a staged source row
  constexpr int kPer = (NW + 255) / 256;
  __shared__ __attribute__((aligned(16))) uint32_t s_row[NW + 2 * KS + 2];
  __shared__ __attribute__((aligned(16))) uint32_t s_out[kRowsMaxW2 * 3 / 4];
  __shared__ int32_t s_map[kRowsMaxW2];
  __shared__ int32_t s_sets[kRowsMaxSets][KS];
  const int tid = threadIdx.x;
  const int nw = W * 3 / 4, nwo = W2 * 3 / 4;
  for (int i = tid; i < W2; i += 256) s_map[i] = colmap[i];
  for (int i = tid; i < nsets * KS; i += 256) (&s_sets[0][0])[i] = sets[i];
  uint32_t v[kPer];
  auto fetch = [&](int row) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(rgb + (int64_t)row * W * 3);
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int w = tid + 256 * q;
      v[q] = src[min(w, nw - 1)];
    }
  };
  if ((int)blockIdx.x < nrows) fetch(blockIdx.x);
  for (int row = blockIdx.x; row < nrows; row += gridDim.x) {
    __syncthreads();  // the previous row's LDS reads are done
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int w = tid + 256 * q;
      if (w < nw) s_row[w] = v[q];
    }
    __syncthreads();
    if (row + (int)gridDim.x < nrows) fetch(row + gridDim.x);
    uint8_t* po = reinterpret_cast<uint8_t*>(s_out);
    constexpr int NWD = (3 * KS + 3) / 4;  // words holding the 3*KS window bytes
    for (int x = tid; x < W2; x += 256) {
      const int m = s_map[x];
      const int xmin = m & 0xfffff, set = m >> 20;
      // the window's bytes as NWD + 1 word reads realigned by v_alignbyte (byte picks
      // then fold into the multiply's operand select) instead of 3*KS byte reads
      const int boff = 3 * xmin, w0 = boff >> 2, sh = boff & 3;
      uint32_t wd[NWD + 1], al[NWD];
#pragma unroll
      for (int i = 0; i <= NWD; ++i) wd[i] = s_row[w0 + i];
#pragma unroll
      for (int i = 0; i < NWD; ++i) al[i] = __builtin_amdgcn_alignbyte(wd[i + 1], wd[i], sh);
      auto byte = [&](int j) { return (int)((al[j >> 2] >> (8 * (j & 3))) & 255u); };
      int s0 = 1 << (kResPrec - 1), s1 = s0, s2 = s0;
#pragma unroll
      for (int i = 0; i < KS; ++i) {
        const int k = s_sets[set][i];
        s0 = mad24(byte(3 * i + 0), k, s0);
        s1 = mad24(byte(3 * i + 1), k, s1);
        s2 = mad24(byte(3 * i + 2), k, s2);
      }
      po[3 * x + 0] = (uint8_t)clip8(s0);
      po[3 * x + 1] = (uint8_t)clip8(s1);
      po[3 * x + 2] = (uint8_t)clip8(s2);
    }
    __syncthreads();
    uint32_t* dst = reinterpret_cast<uint32_t*>(tmp + (int64_t)row * W2 * 3);
    for (int w = tid; w < nwo; w += 256) dst[w] = s_out[w];
  }
}

template <int KS>
__global__ void __launch_bounds__(256) k_rows_v(const uint8_t* __restrict__ tmp, float* __restrict__ gray,
                                                const int32_t* __restrict__ tab, int ks, int H, int W2, int H2) {
  __shared__ float s_lut[3 * 256];
  for (int i = threadIdx.x; i < 3 * 256; i += 256) {
    const float wgt = i < 256 ? 0.299f : (i < 512 ? 0.587f : 0.114f);
    s_lut[i] = ((float)(i & 255) / 255.0f) * wgt;  // float32 u / 255 times the gray weight
  }
  __syncthreads();
  const int q = blockIdx.x * 256 + threadIdx.x;  // output columns 4q .. 4q+3
  const int y2 = blockIdx.y, b = blockIdx.z;
  if (4 * q >= W2) return;
  const int32_t* t = tab + (int64_t)y2 * (2 + ks);  // uniform: scalar loads
  const int ymin = t[0], cnt = t[1];
  const int64_t rw = (int64_t)W2 * 3 / 4;          // words per temp row
  const uint32_t* src = reinterpret_cast<const uint32_t*>(tmp) + ((int64_t)b * H + ymin) * rw + 3 * q;
  uint32_t wv[KS][3];
#pragma unroll
  for (int i = 0; i < KS; ++i) {
    const int ii = i < cnt ? i : 0;  // zero-weight taps re-read row ymin (in range)
#pragma unroll
    for (int j = 0; j < 3; ++j) wv[i][j] = src[ii * rw + j];
  }
  int acc[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) acc[j] = 1 << (kResPrec - 1);
#pragma unroll
  for (int i = 0; i < KS; ++i) {
    const int w = i < cnt ? t[2 + i] : 0;
#pragma unroll
    for (int j = 0; j < 12; ++j) acc[j] = mad24((int)((wv[i][j >> 2] >> (8 * (j & 3))) & 255u), w, acc[j]);
  }
  float g[4];
#pragma unroll
  for (int o = 0; o < 4; ++o)
    g[o] = (s_lut[clip8(acc[3 * o])] + s_lut[256 + clip8(acc[3 * o + 1])]) + s_lut[512 + clip8(acc[3 * o + 2])];
  *reinterpret_cast<float4*>(gray + ((int64_t)b * H2 + y2) * W2 + 4 * q) = make_float4(g[0], g[1], g[2], g[3]);
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

// Row path: column map (xmin | set << 20) + deduplicated tap sets of the horizontal table.
bool ingest_rows_tables(const std::vector<int32_t>& tab_h, int ks_h, int W, int W2, int ks,
                        std::vector<int32_t>& colmap, std::vector<int32_t>& sets) {
  if ((W & 3) || (W2 & 3) || W > kRowsMaxW || W2 > kRowsMaxW2 || ks_h > ks) return false;
  const int th = 2 + ks_h;
  colmap.assign(W2, 0);
  sets.clear();
  int nsets = 0;
  for (int x = 0; x < W2; ++x) {
    std::vector<int32_t> k(ks, 0);
    const int cnt = tab_h[(size_t)x * th + 1];
    for (int i = 0; i < cnt && i < ks; ++i) k[i] = tab_h[(size_t)x * th + 2 + i];
    int id = -1;
    for (int sidx = 0; sidx < nsets && id < 0; ++sidx)
      if (std::equal(k.begin(), k.end(), sets.begin() + (size_t)sidx * ks)) id = sidx;
    if (id < 0) {
      if (nsets == kRowsMaxSets) return false;
      sets.insert(sets.end(), k.begin(), k.end());
      id = nsets++;
    }
    colmap[x] = tab_h[(size_t)x * th] | (id << 20);
  }
  return true;
}

int ingest_rows_ks(int ks_h, int ks_v) {
  const int ks = std::max(ks_h, ks_v);
  return ks <= 5 ? 5 : (ks <= 7 ? 7 : (ks <= 9 ? 9 : 0));
}

void launch_ingest_rgb(const uint8_t* rgb, uint8_t* tmp, float* gray, const int32_t* tab_h, int ks_h,
                       const int32_t* tab_v, int ks_v, const int32_t* colmap, const int32_t* sets, int nsets,
                       int B, int H, int W, int H2, int W2, hipStream_t st) {
  const int ks = colmap ? ingest_rows_ks(ks_h, ks_v) : 0;
  if (ks) {
    const int nrows = B * H;
    const dim3 gh(std::min(nrows, 1536)), gv((W2 / 4 + 255) / 256, H2, B);
#define SFM_ROWS_KS(K)                                                                                   \
  hipLaunchKernelGGL(k_rows_h<K>, gh, dim3(256), 0, st, rgb, tmp, colmap, sets, nsets, nrows, W, W2);      \
  hipLaunchKernelGGL(k_rows_v<K>, gv, dim3(256), 0, st, tmp, gray, tab_v, ks_v, H, W2, H2)
    if (ks == 5) { SFM_ROWS_KS(5); }
    else if (ks == 7) { SFM_ROWS_KS(7); }
    else { SFM_ROWS_KS(9); }
#undef SFM_ROWS_KS
    return;
  }
  hipLaunchKernelGGL(k_resample_h, dim3((W2 + 255) / 256, H, B), dim3(256), 0, st, rgb, tmp, tab_h, ks_h, H, W, W2);
  hipLaunchKernelGGL(k_resample_v_gray, dim3((W2 + 255) / 256, H2, B), dim3(256), 0, st, tmp, gray, tab_v, ks_v, H,
                     W2, H2);
}

}  // namespace sfm
