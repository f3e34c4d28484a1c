// describe.hip — 128-D descriptors, one wavefront per keypoint.
//   rotate = 1: ScaleRotInvSIFT._get_SIFT_descriptors (ScaleRotInvSIFT.py:33-87)
//   rotate = 0: NaiveSIFT._get_SIFT_descriptors       (NaiveSIFT.py:122-173)
// Window rows/cols [y-h+1, y+h+1), h = fw // 2 (:53-56).  Gradients are the exact
// Sobel restatement, magnitude sqrt(Ix^2 + Iy^2), orientation = numpy's SVML atan2f.
// Every histogram is np.histogram's cumulative path: stable sort of the values, sequential
// float32 prefix sum of the weights, float64 bin-edge search ('left', last edge 'right'),
// bin = difference of prefix sums.  RootSIFT: w / ||w|| then sqrt (:82-85), with the
// fixed-order norm of DESIGN.md §Numerics.
#include "kernels.h"

#include <stdlib.h>

namespace sfm {

// numpy.linspace(-pi, pi, num)[i]: i*step + start, last element = stop exactly.
SFM_DEV double pi_edge(int i, int num) {
  const double start = -3.141592653589793, stop = 3.141592653589793;
  if (i == num - 1) return stop;
  double step = (stop - start) / (double)(num - 1);
  return (double)i * step + start;
}

struct DescLayout {
  int ws, n, n4, pw, P;
  size_t off_keys, off_patch, off_ori, off_mag, off_sw, off_cw, off_cellw, off_wgh, total;
};

__host__ __device__ inline DescLayout desc_layout(int fw, int rotate) {
  DescLayout L;
  int h = fw / 2;
  L.ws = 2 * h;
  L.n = L.ws * L.ws;
  L.pw = L.ws + 2;
  int P = 1;
  while (P < L.n) P <<= 1;
  L.P = P;
  L.n4 = (L.n + 3) & ~3;
  size_t o = 0;
  L.off_keys = o;  o += rotate ? (size_t)P * 8 : 0;
  L.off_patch = o; o += (size_t)L.pw * L.pw * 4;
  L.off_ori = o;   o += (size_t)L.n * 4;
  L.off_mag = o;   o += (size_t)L.n * 4;
  o = (o + 15) & ~(size_t)15;
  L.off_sw = o;    o += rotate ? (size_t)L.n4 * 4 : 0;        // weights in sorted order
  L.off_cw = o;    o += rotate ? (size_t)(L.n4 + 1) * 4 : 0;  // their prefix sums
  L.off_cellw = o; o += 16 * 17 * 4;
  L.off_wgh = o;   o += 128 * 4;
  o = (o + 15) & ~(size_t)15;
  L.total = o;
  return L;
}

// Keys (fkey(ori[e]) << 32 | e, padding ~0) sorted by one wavefront in registers, then
// written to s_keys in sorted order (16-B stores).
template <int E>
SFM_DEV void wave_sort_to_lds(const float* s_ori, int n, uint64_t* s_keys) {
  const int lane = threadIdx.x & 63;
  uint64_t k[E];
#pragma unroll
  for (int r = 0; r < E; ++r) {
    const int e = lane * E + r;
    k[r] = (e < n) ? (((uint64_t)fkey(s_ori[e]) << 32) | (uint32_t)e) : ~0ull;
  }
  wave_bitonic_sort_u64<E>(k);
#pragma unroll
  for (int r = 0; r < E; ++r) s_keys[lane * E + r] = k[r];
  __syncthreads();
}

__global__ void __launch_bounds__(64) k_describe(const float* __restrict__ lvl, int H, int W, int fw,
                                                 int rotate, KpList kp, int kcap,
                                                 const int32_t* __restrict__ lc_all, int level, int B,
                                                 double scale, int32_t* __restrict__ out_xy,
                                                 float* __restrict__ out_desc, float* __restrict__ out_conf,
                                                 int64_t out_cap) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
  const int b = blockIdx.y;
  const int kpi = blockIdx.x;
  const int count = kp.count[b];
  if (kpi >= count) return;
  const int lane = threadIdx.x;
  const DescLayout Ly = desc_layout(fw, rotate);
  uint64_t* s_keys = reinterpret_cast<uint64_t*>(s_raw + Ly.off_keys);
  float* s_patch = reinterpret_cast<float*>(s_raw + Ly.off_patch);
  float* s_ori = reinterpret_cast<float*>(s_raw + Ly.off_ori);
  float* s_mag = reinterpret_cast<float*>(s_raw + Ly.off_mag);
  float* s_sw = reinterpret_cast<float*>(s_raw + Ly.off_sw);
  float* s_cw = reinterpret_cast<float*>(s_raw + Ly.off_cw);
  float* s_cellw = reinterpret_cast<float*>(s_raw + Ly.off_cellw);
  float* s_wgh = reinterpret_cast<float*>(s_raw + Ly.off_wgh);
  __shared__ int s_idx[37];

  const int64_t ko = (int64_t)b * kcap + kpi;
  const int x = kp.x[ko], y = kp.y[ko];
  const int h = fw / 2, ws = Ly.ws, n = Ly.n, pw = Ly.pw;
  const float* img = lvl + (int64_t)b * H * W;

  // 1. image patch with one pixel of Sobel halo, zero outside the image
  for (int e = lane; e < pw * pw; e += 64) {
    int pr = e / pw, pc = e - pr * pw;
    int gy = y - h + pr, gx = x - h + pc;
    float v = 0.0f;
    if (gy >= 0 && gy < H && gx >= 0 && gx < W) v = img[(int64_t)gy * W + gx];
    s_patch[e] = v;
  }
  __syncthreads();
  // 2. magnitude / orientation over the 2h x 2h window (ScaleRotInvSIFT.py:40-42)
  for (int e = lane; e < n; e += 64) {
    int i = e / ws, j = e - i * ws;
    const float* c = s_patch + (i + 1) * pw + (j + 1);
    float a00 = c[-pw - 1], a01 = c[-pw], a02 = c[-pw + 1];
    float a10 = c[-1], a12 = c[1];
    float a20 = c[pw - 1], a21 = c[pw], a22 = c[pw + 1];
    float gx = 0.0f;
    gx = __builtin_fmaf(-1.0f, a00, gx);
    gx = __builtin_fmaf(1.0f, a02, gx);
    gx = __builtin_fmaf(-2.0f, a10, gx);
    gx = __builtin_fmaf(2.0f, a12, gx);
    gx = __builtin_fmaf(-1.0f, a20, gx);
    gx = __builtin_fmaf(1.0f, a22, gx);
    float gy = 0.0f;
    gy = __builtin_fmaf(-1.0f, a00, gy);
    gy = __builtin_fmaf(-2.0f, a01, gy);
    gy = __builtin_fmaf(-1.0f, a02, gy);
    gy = __builtin_fmaf(1.0f, a20, gy);
    gy = __builtin_fmaf(2.0f, a21, gy);
    gy = __builtin_fmaf(1.0f, a22, gy);
    float sx = gx * gx;
    float sy = gy * gy;
    float s = sx + sy;
    s_mag[e] = sqrtf(s);
    s_ori[e] = svml_atan2f(gy, gx);
  }
  __syncthreads();

  // 3. dominant orientation (ScaleRotInvSIFT.py:24-31), 36 bins over the whole window
  double dom = 0.0;
  if (rotate) {
    // sort (fkey(orientation), raster index): np.histogram's sort, made stable
    if (Ly.P == 512) {
      wave_sort_to_lds<8>(s_ori, n, s_keys);
    } else if (Ly.P == 256) {
      wave_sort_to_lds<4>(s_ori, n, s_keys);
    } else if (Ly.P == 128) {
      wave_sort_to_lds<2>(s_ori, n, s_keys);
    } else if (Ly.P == 64) {
      wave_sort_to_lds<1>(s_ori, n, s_keys);
    } else {
      for (int e = lane; e < Ly.P; e += 64)
        s_keys[e] = (e < n) ? (((uint64_t)fkey(s_ori[e]) << 32) | (uint32_t)e) : ~0ull;
      __syncthreads();
      bitonic_sort_u64(s_keys, Ly.P);
    }
    // weights in sorted order (parallel gather), zero-padded to a multiple of 4
    for (int m = lane; m < Ly.n4; m += 64) s_sw[m] = (m < n) ? s_mag[(uint32_t)s_keys[m]] : 0.0f;
    __syncthreads();
    // np.histogram's float32 cumulative sum: inherently sequential, so one lane adds in
    // sorted order while its 16-B loads run one step ahead (zero padding adds exactly 0)
    if (lane == 0) {
      const float4* w4 = reinterpret_cast<const float4*>(s_sw);
      const int nq = Ly.n4 >> 2;
      float acc = 0.0f;
      s_cw[0] = 0.0f;
      float4 nxt = w4[0];
      for (int q = 0; q < nq; ++q) {
        const float4 cur = nxt;
        if (q + 1 < nq) nxt = w4[q + 1];
        acc = acc + cur.x;
        s_cw[4 * q + 1] = acc;
        acc = acc + cur.y;
        s_cw[4 * q + 2] = acc;
        acc = acc + cur.z;
        s_cw[4 * q + 3] = acc;
        acc = acc + cur.w;
        s_cw[4 * q + 4] = acc;
      }
    }
    if (lane < 37) {
      double e = pi_edge(lane, 37);
      int lo = 0, hi = n;  // first position whose value fails the predicate
      while (lo < hi) {
        int mid = (lo + hi) >> 1;
        double v = (double)fkey_inv((uint32_t)(s_keys[mid] >> 32));
        bool pass = (lane < 36) ? (v < e) : (v <= e);
        if (pass) lo = mid + 1; else hi = mid;
      }
      s_idx[lane] = lo;
    }
    __syncthreads();
    float hb = -INFINITY;
    int bi = 64;
    if (lane < 36) {
      hb = s_cw[s_idx[lane + 1]] - s_cw[s_idx[lane]];
      bi = lane;
    }
    // first argmax: larger value wins, equal values -> smaller bin index
    for (int off = 32; off >= 1; off >>= 1) {
      float ov = __shfl_xor(hb, off);
      int oi = __shfl_xor(bi, off);
      if (ov > hb || (ov == hb && oi < bi)) { hb = ov; bi = oi; }
    }
    dom = (pi_edge(bi, 37) + pi_edge(bi + 1, 37)) / 2.0;
  }

  // 4. 4 x 4 cells of 4 x 4 px from the window's top-left (:68-76), 8 bins each.  One lane
  //    per cell holds its (up to) 16 values in registers in raster order; a Batcher
  //    odd-even merge network on (value, raster slot) is the stable sort np.histogram's
  //    cumulative path needs; empty slots (+inf) sort last.
  if (lane < 16) {
    const int r = lane >> 2, cc = lane & 3;
    double cv[16];
    float wt[16];
    int sl[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int i = 4 * r + (t >> 2), j = 4 * cc + (t & 3);
      const bool ok = i < ws && j < ws;
      const int e = ok ? i * ws + j : 0;
      const double ov = (double)s_ori[e];
      cv[t] = ok ? (rotate ? ov - dom : ov) : INFINITY;  // float64 relative angle (:62)
      wt[t] = ok ? s_mag[e] : 0.0f;
      sl[t] = t;
    }
#pragma unroll
    for (int p = 1; p < 16; p <<= 1)
#pragma unroll
      for (int k = p; k >= 1; k >>= 1)
#pragma unroll
        for (int j = k % p; j + k < 16; j += 2 * k)
#pragma unroll
          for (int i = 0; i < k; ++i) {
            const int a = i + j, c = i + j + k;
            if (c < 16 && a / (2 * p) == c / (2 * p)) {
              const bool sw = cv[a] > cv[c] || (cv[a] == cv[c] && sl[a] > sl[c]);
              const double tv = cv[a];
              cv[a] = sw ? cv[c] : tv;
              cv[c] = sw ? tv : cv[c];
              const float tw = wt[a];
              wt[a] = sw ? wt[c] : tw;
              wt[c] = sw ? tw : wt[c];
              const int ts = sl[a];
              sl[a] = sw ? sl[c] : ts;
              sl[c] = sw ? ts : sl[c];
            }
          }
    float* cw = s_cellw + lane * 17;
    float acc = 0.0f;
    cw[0] = 0.0f;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      acc = acc + wt[m];  // empty slots (weight 0) sit after every real value
      cw[m + 1] = acc;
    }
    int idx[9];
#pragma unroll
    for (int eb = 0; eb < 9; ++eb) {
      const double e = pi_edge(eb, 9);
      int c = 0;
#pragma unroll
      for (int m = 0; m < 16; ++m) c += (eb < 8) ? (cv[m] < e ? 1 : 0) : (cv[m] <= e ? 1 : 0);
      idx[eb] = c;
    }
#pragma unroll
    for (int bb = 0; bb < 8; ++bb) s_wgh[lane * 8 + bb] = cw[idx[bb + 1]] - cw[idx[bb]];
  }
  __syncthreads();

  // 5. fixed-order L2 norm, normalise, RootSIFT
  float w0 = s_wgh[lane], w1 = s_wgh[lane + 64];
  float a = w0 * w0;
  float c = w1 * w1;
  float s = a + c;
  for (int off = 32; off >= 1; off >>= 1) {
    float o = __shfl_down(s, off);
    s = s + o;
  }
  float nrm = sqrtf(__shfl(s, 0));
  int64_t off0 = 0;
  for (int l = 0; l < level; ++l) off0 += lc_all[(int64_t)l * B + b];
  const int64_t slot = (int64_t)b * out_cap + off0 + kpi;
  float v0 = w0, v1 = w1;
  if (nrm > 0.0f) {
    v0 = v0 / nrm;
    v1 = v1 / nrm;
  }
  out_desc[slot * 128 + lane] = sqrtf(v0);
  out_desc[slot * 128 + lane + 64] = sqrtf(v1);
  if (lane == 0) {
    if (out_conf) out_conf[slot] = kp.conf[ko];
    out_xy[slot * 2 + 0] = (int32_t)((double)x * scale);  // (x * scale).astype(int) :101
    out_xy[slot * 2 + 1] = (int32_t)((double)y * scale);  // :102
  }
}

__global__ void k_finalize_counts(const int32_t* __restrict__ lc_all, int B, int L,
                                  int32_t* __restrict__ out_count) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  int32_t s = 0;
  for (int l = 0; l < L; ++l) s += lc_all[(int64_t)l * B + b];
  out_count[b] = s;
}

size_t describe_lds_bytes(int fw, int rotate) { return desc_layout(fw, rotate).total; }

void init_describe_attributes(size_t max_lds) {
  (void)hipFuncSetAttribute((const void*)k_describe, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)max_lds);
}

bool launch_describe(const float* lvl, int B, int H, int W, int fw, int rotate, KpList kp,
                     int kcap, const int32_t* level_counts_all, int level, int L, double scale,
                     int32_t* out_xy, float* out_desc, float* out_conf, int64_t out_cap,
                     int32_t* out_count, const MatchOperands& mo, bool* operands_written, hipStream_t st) {
  if (operands_written) *operands_written = false;
  if (kcap <= 0) return false;
  static const bool one_per_wave = [] {
    const char* v = getenv("SFMFEAT_DESCRIBE");
    return v && v[0] == 'w';  // "wave": the one-keypoint-per-wavefront kernel (A/B timing)
  }();
  if (!one_per_wave && launch_describe_quad(lvl, B, H, W, fw, rotate, kp, kcap, level_counts_all, level,
                                            scale, out_xy, out_desc, out_conf, out_cap, out_count, L, mo, st)) {
    if (operands_written) *operands_written = mo.hi != nullptr;
    return out_count != nullptr;
  }
  size_t lds = describe_lds_bytes(fw, rotate);
  hipLaunchKernelGGL(k_describe, dim3(kcap, B), dim3(64), lds, st, lvl, H, W, fw, rotate, kp, kcap,
                     level_counts_all, level, B, scale, out_xy, out_desc, out_conf, out_cap);
  return false;
}

void launch_finalize_counts(const int32_t* level_counts_all, int B, int L, int32_t* out_count,
                            hipStream_t st) {
  hipLaunchKernelGGL(k_finalize_counts, dim3((B + 255) / 256), dim3(256), 0, st, level_counts_all, B, L,
                     out_count);
}

}  // namespace sfm
