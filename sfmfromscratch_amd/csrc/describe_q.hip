// describe_q.hip — 128-D descriptors, four keypoints per 64-lane wavefront.
//
// Same arithmetic as describe.hip (ScaleRotInvSIFT.py:33-87 / NaiveSIFT.py:122-173, the
// np.histogram cumulative path, RootSIFT with the fixed-order norm) and bit-identical
// results, laid out so that one instruction serves four keypoints: keypoint g of the
// workgroup owns lanes [16g, 16g+16), exactly one DPP row, so every cross-lane step is a
// row-local DPP move and the serial parts (the float32 prefix sums, the per-cell sorts)
// run in four keypoints at once.  Compiled per window width ws = 2*(fw//2) in [2, 22].
//
//   1. image patch (+1 px Sobel halo) -> LDS;  2. Sobel, |g|, SVML atan2 for the ws x ws
//   window, each lane owning pixels e = 16 r + lane;  3. (rotate) the (fkey(ori), e) keys
//   sorted in registers by a 16-lane bitonic network (E keys per lane, DPP exchanges),
//   sorted weights gathered, the sequential prefix sum carried lane to lane, the 37 bin
//   boundaries found by integer binary search against the exact float images of the
//   float64 edges, first argmax -> dominant orientation;  4. one lane per 4x4 cell: its
//   16 pixels ordered by (relative angle, raster slot) — for rotate, by their rank in the
//   global order, which is the same order (a float pair that the float64 subtraction
//   could merge has both |ori| < 2^-25: such keypoints take the exact double-key network)
//   — prefix sum, 9 edge boundaries, 8 bins;  5. norm over the same reduction tree as the
//   one-keypoint kernel, normalise, sqrt.
#include "kernels.h"

#include <stdlib.h>
#include <string.h>

#include <mutex>

namespace sfm {
namespace dq {

constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int pow2ceil(int v) { return v <= 1 ? 1 : 2 * pow2ceil((v + 1) / 2); }

template <int WS, int ROT>
struct Geo {
  static constexpr int N = WS * WS, PW = WS + 2, NP = PW * PW;
  static constexpr int P = cmax(pow2ceil(N), 16), E = P / 16;   // sort slots, keys per lane
  static constexpr int RN = (N + 15) / 16;                      // pixels per lane
  static constexpr int A = (cmax(cmax(NP, N + 4), 16 * 17) + 3) & ~3;  // patch | prefix sums
  static constexpr int NQ = (N + 3) & ~3;
  static constexpr int OFF_M = A;                               // |g| -> sorted weights
  static constexpr int OFF_K = OFF_M + NQ;                      // sorted keys (rotate) / ori
  static constexpr int OFF_R = OFF_K + NQ;                      // rank of each pixel (u16)
  static constexpr int OFF_I = OFF_R + (ROT ? (NQ / 2 + 3) & ~3 : 0);  // 37 boundaries
  static constexpr int OFF_T = OFF_I + (ROT ? 40 : 0);          // 9 cell-edge keys
  static constexpr int G = OFF_T + 12;                          // floats per keypoint
};

SFM_DEV double pi_edge(int i, int num) {  // numpy.linspace(-pi, pi, num)[i]
  const double start = -3.141592653589793, stop = 3.141592653589793;
  if (i == num - 1) return stop;
  const double step = (stop - start) / (double)(num - 1);
  return (double)i * step + start;
}

// fkey of the smallest float o with fl((double)o - sh) >= e (or > e when `strict`): for
// float keys v, (double)v - sh < e  <=>  fkey(v) < result, since the map is monotone.
SFM_DEV uint32_t edge_key(double e, double sh, bool strict) {
  uint32_t kc = fkey((float)(e + sh));
  auto pass = [&](uint32_t kk) {
    const double d = (double)fkey_inv(kk) - sh;
    return strict ? d > e : d >= e;
  };
  for (int it = 0; it < 64 && pass(kc); ++it) --kc;
  for (int it = 0; it < 64 && !pass(kc); ++it) ++kc;
  return kc;
}

// Bin-edge keys, the same for every keypoint, computed once per device by the host (the same
// IEEE double arithmetic as pi_edge / edge_key above, fp-contract off on both sides):
// c_ori[j] = edge_key(linspace(-pi, pi, 37)[j], 0, j == 36) (orientation histogram) and
// c_cell[bi][t] = edge_key(linspace(-pi, pi, 9)[t], dom_bi, t == 8) with dom_bi the centre of
// orientation bin bi (bi < 36), dom = 0 in row 36 (the non-rotated NaiveSIFT path).
__constant__ uint32_t c_ori[37];
__constant__ uint32_t c_cell[37][9];

// ---- row-local (16-lane) exchanges --------------------------------------------------
template <int CTRL>
SFM_DEV uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}
// the value held by lane (lane ^ X) of the same row
template <int X>
SFM_DEV uint32_t rxor(uint32_t v) {
  if constexpr (X == 1) return dpp<0xB1>(v);        // quad_perm [1,0,3,2]
  else if constexpr (X == 2) return dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  else if constexpr (X == 3) return dpp<0x1B>(v);   // quad_perm [3,2,1,0]
  else if constexpr (X == 4) return dpp<0x1B>(dpp<0x141>(v));  // half-mirror, then ^3
  else if constexpr (X == 7) return dpp<0x141>(v);  // row_half_mirror
  else if constexpr (X == 8) return dpp<0x128>(v);  // row_ror:8
  else {
    static_assert(X == 15, "row-local xor");
    return dpp<0x140>(v);                           // row_mirror
  }
}
template <int X>
SFM_DEV float rxorf(float v) { return __uint_as_float(rxor<X>(__float_as_uint(v))); }
template <int X>
SFM_DEV double rxord(double v) {
  const uint64_t u = __double_as_longlong(v);
  return __longlong_as_double((long long)(((uint64_t)rxor<X>((uint32_t)(u >> 32)) << 32) | rxor<X>((uint32_t)u)));
}

// Sort keys as doubles: kBias + (fkey << 9 | pixel) is a positive normal double for every
// 41-bit payload, so the double order is the payload order and a compare-exchange is one
// v_min_f64 + one v_max_f64 (no lane masks; the file is built with -fno-honor-nans so
// they are not preceded by canonicalisations).  kPad sorts after every key.
constexpr uint64_t kBias = 1ull << 52;
constexpr uint64_t kPad = kBias + (1ull << 41);
SFM_DEV double dkey(uint64_t payload) { return __longlong_as_double((long long)(kBias + payload)); }
SFM_DEV uint64_t dpayload(double k) { return (uint64_t)__double_as_longlong(k) - kBias; }

SFM_DEV void cas_up(double& a, double& b) {
  const double lo = __builtin_fmin(a, b), hi = __builtin_fmax(a, b);
  a = lo;
  b = hi;
}
SFM_DEV double keep_or_take(bool lower, double mine, double other) {
  const double lo = __builtin_fmin(mine, other), hi = __builtin_fmax(mine, other);
  return lower ? lo : hi;
}

// Bitonic sort (all comparators ascending: each merge starts with the mirrored compare)
// of 16*E keys held as lane gl, register r <-> position gl*E + r of one 16-lane row.
template <int E, int S>
SFM_DEV void half_clean(double (&k)[E], int gl) {
  if constexpr (S >= 1) {
    if constexpr (S < E) {
#pragma unroll
      for (int r = 0; r < E; ++r)
        if ((r & S) == 0) cas_up(k[r], k[r + S]);
    } else {
      constexpr int X = S / E;
      const bool lower = (gl & X) == 0;
#pragma unroll
      for (int r = 0; r < E; ++r) k[r] = keep_or_take(lower, k[r], rxord<X>(k[r]));
    }
    half_clean<E, S / 2>(k, gl);
  }
}
template <int E, int SIZE>
SFM_DEV void merge_level(double (&k)[E], int gl) {
  if constexpr (SIZE <= 16 * E) {
    if constexpr (SIZE <= E) {
#pragma unroll
      for (int r = 0; r < E; ++r)
        if ((r & (SIZE / 2)) == 0) cas_up(k[r], k[r ^ (SIZE - 1)]);
    } else {
      constexpr int X = SIZE / E - 1;
      const bool lower = (gl & ((X + 1) >> 1)) == 0;
      if constexpr (E == 1) {
        k[0] = keep_or_take(lower, k[0], rxord<X>(k[0]));
      } else {
#pragma unroll
        for (int r = 0; r < E / 2; ++r) {
          const double oa = rxord<X>(k[E - 1 - r]);
          const double ob = rxord<X>(k[r]);
          k[r] = keep_or_take(lower, k[r], oa);
          k[E - 1 - r] = keep_or_take(lower, k[E - 1 - r], ob);
        }
      }
    }
    half_clean<E, SIZE / 4>(k, gl);
    merge_level<E, SIZE * 2>(k, gl);
  }
}

// Sobel (the fmaf chains of describe.hip), magnitude and SVML orientation at c.
SFM_DEV void grad_at(const float* c, int pw, float& mag, float& ori) {
  const float a00 = c[-pw - 1], a01 = c[-pw], a02 = c[-pw + 1];
  const float a10 = c[-1], a12 = c[1];
  const float a20 = c[pw - 1], a21 = c[pw], a22 = c[pw + 1];
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
  const float sx = gx * gx;
  const float sy = gy * gy;
  const float s = sx + sy;
  mag = sqrtf(s);
  ori = svml_atan2f(gy, gx);
}

SFM_DEV void cas_up(uint32_t& a, uint32_t& b) {
  const uint32_t lo = min(a, b), hi = max(a, b);
  a = lo;
  b = hi;
}

// Batcher odd-even merge network over 16 register slots (ascending).
template <typename T>
SFM_DEV void batcher16(T (&q)[16]) {
#pragma unroll
  for (int p = 1; p < 16; p <<= 1)
#pragma unroll
    for (int kk = p; kk >= 1; kk >>= 1)
#pragma unroll
      for (int j = kk % p; j + kk < 16; j += 2 * kk)
#pragma unroll
        for (int i = 0; i < kk; ++i) {
          const int a = i + j, c = i + j + kk;
          if (c < 16 && a / (2 * p) == c / (2 * p)) cas_up(q[a], q[c]);
        }
}

// ABL (timing ablations, results invalid): 1 no sort, 2 no prefix chain, 4 no cells, 8 no gradients,
// 16 no orientation-edge search, 32 no cell-edge keys, 64 no patch loads
template <int WS, int ROT, int ABL = 0>
__global__ void __launch_bounds__(64) k_describe_q(const float* __restrict__ lvl, int H, int W, KpList kp,
                                                   int kcap, const int32_t* __restrict__ lc_all, int level,
                                                   int B, double scale, int32_t* __restrict__ out_xy,
                                                   float* __restrict__ out_desc, float* __restrict__ out_conf,
                                                   int64_t out_cap, int32_t* __restrict__ out_count, int L,
                                                   MatchOperands mo) {
  using C = Geo<WS, ROT>;
  constexpr int N = C::N, PW = C::PW, NP = C::NP, E = C::E, RN = C::RN, h = WS / 2;
  __shared__ __attribute__((aligned(16))) float s_all[4 * C::G];
  const int b = blockIdx.y;
  // the last level's launch also writes the slot's keypoint count (sum over the levels), so
  // no separate one-workgroup finalize launch trails the extraction
  if (out_count != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {
    int32_t s = 0;
    for (int l = 0; l < L; ++l) s += lc_all[(int64_t)l * B + b];
    out_count[b] = s;
  }
  // fused matcher operands: the last level's launch carries kPadBlocks extra workgroups per
  // image that write the padding rows [count, capP) (norm2 = +inf, hi = lo = 0), as
  // k_match_prep does, so the sweep needs no bounds checks
  const int nkb = (kcap + 3) / 4;
  if ((int)blockIdx.x >= nkb) {
    int32_t s = 0;
    for (int l = 0; l < L; ++l) s += lc_all[(int64_t)l * B + b];
    const int nt = ((int)gridDim.x - nkb) * 64;
    for (int64_t r = s + ((int)blockIdx.x - nkb) * 64 + threadIdx.x; r < mo.capP; r += nt) {
      const int64_t mr = (int64_t)b * mo.capP + r;
      uint4* hz = reinterpret_cast<uint4*>(mo.hi + mr * 128);
      uint4* lz = reinterpret_cast<uint4*>(mo.lo + mr * 128);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        hz[q] = make_uint4(0u, 0u, 0u, 0u);
        lz[q] = make_uint4(0u, 0u, 0u, 0u);
      }
      mo.norm2[mr] = INFINITY;
      mo.rnorm[mr] = 0.0f;
    }
    return;
  }
  const int count = kp.count[b];
  const int kbase = blockIdx.x * 4;
  if (kbase >= count) return;
  const int lane = threadIdx.x, g = lane >> 4, gl = lane & 15;
  const int kpi = kbase + g;
  const bool valid = kpi < count;
  const int64_t ko = (int64_t)b * kcap + (valid ? kpi : kbase);
  const int x = kp.x[ko], y = kp.y[ko];
  float* sA = s_all + g * C::G;                                     // patch, prefix sums
  float* sM = sA + C::OFF_M;                                        // |g|, sorted weights
  uint32_t* sK = reinterpret_cast<uint32_t*>(sA + C::OFF_K);        // sorted keys / ori
  uint16_t* sR = reinterpret_cast<uint16_t*>(sA + C::OFF_R);        // pixel -> sorted rank
  int32_t* sI = reinterpret_cast<int32_t*>(sA + C::OFF_I);          // 37 boundaries
  uint32_t* sT = reinterpret_cast<uint32_t*>(sA + C::OFF_T);        // 9 cell-edge keys

  // 1. patch with one pixel of Sobel halo, zero outside the image (loads unconditional)
  const float* img = lvl + (int64_t)b * H * W;
#pragma unroll
  for (int it = 0; it < (NP + 15) / 16; ++it) {
    const int e0 = it * 16 + gl;
    const int e = e0 < NP ? e0 : NP - 1;
    const int pr = e / PW, pc = e - pr * PW;
    const int gy = y - h + pr, gx = x - h + pc;
    const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
    const int cy = min(max(gy, 0), H - 1), cx = min(max(gx, 0), W - 1);
    const float v = (ABL & 64) ? (float)(cy + cx) : img[(int64_t)cy * W + cx];
    if (e0 < NP) sA[e] = in ? v : 0.0f;
  }
  __syncthreads();

  // 2. gradient magnitude / orientation (ScaleRotInvSIFT.py:40-42)
  double k[E];
  bool tiny = false;
#pragma unroll
  for (int r = 0; r < E; ++r) k[r] = __longlong_as_double((long long)kPad);
#pragma unroll
  for (int r = 0; r < RN; ++r) {
    const int e0 = r * 16 + gl;
    const bool ok = (N % 16 == 0) || e0 < N;
    const int e = ok ? e0 : N - 1;
    const int i = e / WS, j = e - i * WS;
    float mag, ori;
    if constexpr ((ABL & 8) != 0) {
      mag = sA[(i + 1) * PW + (j + 1)];
      ori = sA[(i + 1) * PW + j] - 100.0f;
    } else {
      grad_at(sA + (i + 1) * PW + (j + 1), PW, mag, ori);
    }
    if (ok) {
      sM[e] = mag;
      if (!ROT) sK[e] = __float_as_uint(ori);
    }
    if (ROT) {
      k[r] = ok ? dkey(((uint64_t)fkey(ori) << 9) | (uint32_t)e) : __longlong_as_double((long long)kPad);
      tiny |= ok && ori != 0.0f && fabsf(ori) < 0x1p-25f;
    }
  }
  __syncthreads();

  double dom = 0.0;
  int dom_bin = 36;  // row of c_cell (36: dom = 0)
  if constexpr (ROT) {
    // 3. dominant orientation (ScaleRotInvSIFT.py:24-31): np.histogram's cumulative path
    if constexpr ((ABL & 1) == 0) merge_level<E, 2>(k, gl);
    float w[E];
    uint32_t ke[E], kf[E];  // pixel and fkey at sorted position gl*E + r
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const int p = gl * E + r;
      const uint64_t pl = dpayload(k[r]);
      ke[r] = p < N ? (uint32_t)(pl & 511u) : 0u;
      kf[r] = (uint32_t)(pl >> 9);
      w[r] = p < N ? sM[ke[r]] : 0.0f;
    }
    __syncthreads();  // every gather done before sM is overwritten with sorted weights
    // float32 prefix sum in sorted order: lane s adds its E weights, then hands the
    // running total to lane s+1 (the four rows advance together)
    float cw[E];
#pragma unroll
    for (int r = 0; r < E; ++r) cw[r] = 0.0f;
    float carry = 0.0f;
    constexpr int NL = (N + E - 1) / E;
    if constexpr ((ABL & 2) != 0) {
#pragma unroll
      for (int r = 0; r < E; ++r) cw[r] = w[r];
    }
    for (int s = 0; s < ((ABL & 2) ? 0 : NL); ++s) {
      if (gl == s) {
        float acc = carry;
#pragma unroll
        for (int r = 0; r < E; ++r) {
          acc = acc + w[r];
          cw[r] = acc;
        }
      }
      const float nxt = __uint_as_float(dpp<0x111>(__float_as_uint(cw[E - 1])));  // row_shr:1
      if (gl == s + 1) carry = nxt;
    }
#pragma unroll
    for (int r = 0; r < E; r += (E >= 4 ? 4 : 1)) {
      const int p = gl * E + r;
      if (p < N) {
        if constexpr (E >= 4) {
          *reinterpret_cast<uint4*>(sK + p) = make_uint4(kf[r], kf[r + 1], kf[r + 2], kf[r + 3]);
          *reinterpret_cast<float4*>(sM + p) = make_float4(w[r], w[r + 1], w[r + 2], w[r + 3]);
          *reinterpret_cast<float4*>(sA + 4 + p) = make_float4(cw[r], cw[r + 1], cw[r + 2], cw[r + 3]);
        } else {
          sK[p] = kf[r];
          sM[p] = w[r];
          sA[4 + p] = cw[r];
        }
      }
    }
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const int p = gl * E + r;
      if (p < N) sR[ke[r]] = (uint16_t)p;
    }
    if (gl == 0) sA[3] = 0.0f;  // cw[q] lives at sA[3 + q]
    __syncthreads();
    // bin boundaries: count of sorted values < edge j (<= for the last edge)
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int j = gl + 16 * t;
      if ((ABL & 16) != 0 && j <= 36) {
        sI[j] = j * N / 37;
      } else if (j <= 36) {
        const uint32_t T = c_ori[j];
        int lo = 0;
        constexpr int S0 = pow2ceil(N + 1) / 2;
#pragma unroll
        for (int s = S0; s >= 1; s >>= 1) {
          const int q = lo + s;
          const uint32_t v = sK[(q <= N ? q : N) - 1];
          if (q <= N && v < T) lo = q;
        }
        sI[j] = lo;
      }
    }
    __syncthreads();
    float hb = -INFINITY;
    int bi = 64;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int j = gl + 16 * t;
      if (j < 36) {
        const float v = sA[3 + sI[j + 1]] - sA[3 + sI[j]];
        if (v > hb) { hb = v; bi = j; }
      }
    }
    // first argmax over the row: larger value wins, equal values -> smaller bin index
    {
      float ov; int oi;
      ov = rxorf<8>(hb); oi = (int)rxor<8>((uint32_t)bi);
      if (ov > hb || (ov == hb && oi < bi)) { hb = ov; bi = oi; }
      ov = rxorf<4>(hb); oi = (int)rxor<4>((uint32_t)bi);
      if (ov > hb || (ov == hb && oi < bi)) { hb = ov; bi = oi; }
      ov = rxorf<2>(hb); oi = (int)rxor<2>((uint32_t)bi);
      if (ov > hb || (ov == hb && oi < bi)) { hb = ov; bi = oi; }
      ov = rxorf<1>(hb); oi = (int)rxor<1>((uint32_t)bi);
      if (ov > hb || (ov == hb && oi < bi)) { hb = ov; bi = oi; }
    }
    dom = (pi_edge(bi, 37) + pi_edge(bi + 1, 37)) / 2.0;
    dom_bin = bi;
  }

  // 4. the 4 x 4 cells of 4 x 4 px from the window's top-left (:68-76), 8 bins each
  if (gl < 9) sT[gl] = (ABL & 32) ? 0x80000000u + (uint32_t)(dom * 1e6) * gl : c_cell[dom_bin][gl];
  __syncthreads();  // (also: the rotate prefix sums in sA are no longer read)
  float hv[8];
  if constexpr ((ABL & 4) != 0) {
#pragma unroll
    for (int bb = 0; bb < 8; ++bb) hv[bb] = sM[gl * 8 + bb] + __uint_as_float(sT[bb & 7]);
  } else {
  const int r4 = gl >> 2, c4 = gl & 3;
  float wv[16];
  uint32_t hk[16];
  const bool grp_tiny = ROT && ((__ballot(tiny) >> (16 * g)) & 0xFFFFull) != 0;
  if (ROT && !grp_tiny) {
    // the cell's pixels in global sorted order (= by relative angle, then raster slot)
    uint32_t q[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int i = 4 * r4 + (t >> 2), j = 4 * c4 + (t & 3);
      const bool ok = i < WS && j < WS;
      q[t] = ok ? (uint32_t)sR[ok ? i * WS + j : 0] : 0xFFFFFFFFu;
    }
    batcher16(q);
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const bool ok = q[m] != 0xFFFFFFFFu;
      const uint32_t p = ok ? q[m] : 0u;
      wv[m] = ok ? sM[p] : 0.0f;
      hk[m] = ok ? sK[p] : 0xFFFFFFFFu;
    }
  } else {
    // (fkey(ori), slot) keys; for rotate (rare: some 0 < |ori| < 2^-25) the exact
    // float64 relative angle decides, as in describe.hip
    uint64_t q[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int i = 4 * r4 + (t >> 2), j = 4 * c4 + (t & 3);
      const bool ok = i < WS && j < WS;
      const int e = ok ? i * WS + j : 0;
      const uint32_t key = ROT ? sK[sR[e]] : fkey(__uint_as_float(sK[e]));
      q[t] = ok ? (((uint64_t)key << 32) | (uint32_t)t) : ~0ull;
    }
    if (!ROT) {
      double dq16[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) dq16[t] = q[t] == ~0ull ? __longlong_as_double((long long)kPad)
                                                           : dkey(((q[t] >> 32) << 4) | (uint32_t)t);
      batcher16(dq16);
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const uint64_t pl = dpayload(dq16[t]);
        q[t] = pl >= (1ull << 36) ? ~0ull : (((pl >> 4) << 32) | (pl & 15u));
      }
    } else {
      double cv[16];
      int sl[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        cv[t] = q[t] == ~0ull ? INFINITY : (double)fkey_inv((uint32_t)(q[t] >> 32)) - dom;
        sl[t] = t;
      }
#pragma unroll
      for (int p = 1; p < 16; p <<= 1)
#pragma unroll
        for (int kk = p; kk >= 1; kk >>= 1)
#pragma unroll
          for (int j = kk % p; j + kk < 16; j += 2 * kk)
#pragma unroll
            for (int i = 0; i < kk; ++i) {
              const int a = i + j, c = i + j + kk;
              if (c < 16 && a / (2 * p) == c / (2 * p)) {
                const bool sw = cv[a] > cv[c] || (cv[a] == cv[c] && sl[a] > sl[c]);
                const double tv = cv[a];
                cv[a] = sw ? cv[c] : tv;
                cv[c] = sw ? tv : cv[c];
                const uint64_t tq = q[a];
                q[a] = sw ? q[c] : tq;
                q[c] = sw ? tq : q[c];
                const int ts = sl[a];
                sl[a] = sw ? sl[c] : ts;
                sl[c] = sw ? ts : sl[c];
              }
            }
    }
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const bool ok = q[m] != ~0ull;
      const int t = ok ? (int)(uint32_t)q[m] : 0;
      const int e = (4 * r4 + (t >> 2)) * WS + 4 * c4 + (t & 3);
      wv[m] = ok ? (ROT ? sM[sR[e]] : sM[e]) : 0.0f;
      hk[m] = ok ? (uint32_t)(q[m] >> 32) : 0xFFFFFFFFu;
    }
  }
  // prefix sums (empty slots add exactly 0 after every real value), 9 edge boundaries
  float* cc = sA + gl * 17;
  float acc = 0.0f;
  cc[0] = 0.0f;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    acc = acc + wv[m];
    cc[m + 1] = acc;
  }
  int bidx[9];
#pragma unroll
  for (int eb = 0; eb < 9; ++eb) {
    const uint32_t T = sT[eb];
    int c = 0;
#pragma unroll
    for (int m = 0; m < 16; ++m) c += hk[m] < T ? 1 : 0;
    bidx[eb] = c;
  }
#pragma unroll
  for (int bb = 0; bb < 8; ++bb) hv[bb] = cc[bidx[bb + 1]] - cc[bidx[bb]];

  }
  // 5. fixed-order L2 norm: the one-keypoint kernel's tree (lane i holds bins i, i+64,
  //    then halving strides 32..1) — bin 8*cell + t lives in lane `cell`, register t
  float tr[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const float a = hv[t] * hv[t];
    tr[t] = a + rxorf<8>(a);
  }
#pragma unroll
  for (int t = 0; t < 8; ++t) tr[t] = tr[t] + rxorf<4>(tr[t]);
#pragma unroll
  for (int t = 0; t < 8; ++t) tr[t] = tr[t] + rxorf<2>(tr[t]);
#pragma unroll
  for (int t = 0; t < 8; ++t) tr[t] = tr[t] + rxorf<1>(tr[t]);
#pragma unroll
  for (int t = 0; t < 4; ++t) tr[t] = tr[t] + tr[t + 4];
  tr[0] = tr[0] + tr[2];
  tr[1] = tr[1] + tr[3];
  tr[0] = tr[0] + tr[1];
  const float nrm = sqrtf(__shfl(tr[0], g * 16));
  if (!valid) return;
  int64_t off0 = 0;
  for (int l = 0; l < level; ++l) off0 += lc_all[(int64_t)l * B + b];
  const int64_t slot = (int64_t)b * out_cap + off0 + kpi;
  float o[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) o[t] = sqrtf(nrm > 0.0f ? hv[t] / nrm : hv[t]);
  float4* dst = reinterpret_cast<float4*>(out_desc + slot * 128 + gl * 8);
  dst[0] = make_float4(o[0], o[1], o[2], o[3]);
  dst[1] = make_float4(o[4], o[5], o[6], o[7]);
  if (mo.hi != nullptr) {
    // the matcher's operands of this row (k_match_prep's arithmetic: the same hi / lo of each
    // element; the squared norm summed in double over the row's 16 lanes)
    const int64_t r = off0 + kpi, mr = (int64_t)b * mo.capP + r;
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    h8 hh, ll;
    double s = 0.0;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float xs = o[t] * kMatchScale;
      const _Float16 hv16 = (_Float16)xs;
      const float rr = (xs - (float)hv16) * kMatchLoScale;  // exact difference, exact scaling
      hh[t] = hv16;
      ll[t] = (_Float16)rr;
      s += (double)o[t] * (double)o[t];
    }
    *reinterpret_cast<h8*>(mo.hi + mr * 128 + gl * 8) = hh;
    *reinterpret_cast<h8*>(mo.lo + mr * 128 + gl * 8) = ll;
    s += rxord<8>(s);
    s += rxord<4>(s);
    s += rxord<2>(s);
    s += rxord<1>(s);
    if (gl == 0) {
      const float n2 = (float)s, rn = (float)sqrt(s);
      mo.norm2[mr] = n2;
      mo.rnorm[mr] = rn;
      // per-16-row maxima (non-negative floats order as their bit patterns)
      float2* pm = mo.pmax + (int64_t)b * (mo.capP / kPrepRows) + r / kPrepRows;
      atomicMax(reinterpret_cast<unsigned int*>(&pm->x), __float_as_uint(n2));
      atomicMax(reinterpret_cast<unsigned int*>(&pm->y), __float_as_uint(rn));
    }
  }
  if (gl == 0) {
    if (out_conf) out_conf[slot] = kp.conf[ko];
    out_xy[slot * 2 + 0] = (int32_t)((double)x * scale);  // (x * scale).astype(int) :101
    out_xy[slot * 2 + 1] = (int32_t)((double)y * scale);  // :102
  }
}

}  // namespace dq

namespace {
uint32_t fkey_h(float v) {
  uint32_t b;
  memcpy(&b, &v, 4);
  if (b == 0x80000000u) b = 0u;
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
float fkey_inv_h(uint32_t k) {
  const uint32_t b = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  float f;
  memcpy(&f, &b, 4);
  return f;
}
double pi_edge_h(int i, int num) {  // = dq::pi_edge
  const double start = -3.141592653589793, stop = 3.141592653589793;
  if (i == num - 1) return stop;
  const double step = (stop - start) / (double)(num - 1);
  return (double)i * step + start;
}
uint32_t edge_key_h(double e, double sh, bool strict) {  // = dq::edge_key
  uint32_t kc = fkey_h((float)(e + sh));
  auto pass = [&](uint32_t kk) {
    const double d = (double)fkey_inv_h(kk) - sh;
    return strict ? d > e : d >= e;
  };
  for (int it = 0; it < 64 && pass(kc); ++it) --kc;
  for (int it = 0; it < 64 && !pass(kc); ++it) ++kc;
  return kc;
}
}  // namespace

void init_describe_quad_tables() {
  static std::mutex mu;
  static bool done[256] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 256) return;
  std::lock_guard<std::mutex> lk(mu);
  if (done[dev]) return;
  uint32_t ori[37], cell[37][9];
  for (int j = 0; j < 37; ++j) ori[j] = edge_key_h(pi_edge_h(j, 37), 0.0, j == 36);
  for (int bi = 0; bi < 37; ++bi) {
    const double dom = bi < 36 ? (pi_edge_h(bi, 37) + pi_edge_h(bi + 1, 37)) / 2.0 : 0.0;
    for (int t = 0; t < 9; ++t) cell[bi][t] = edge_key_h(pi_edge_h(t, 9), dom, t == 8);
  }
  done[dev] = hipMemcpyToSymbol(HIP_SYMBOL(dq::c_ori), ori, sizeof(ori)) == hipSuccess &&
              hipMemcpyToSymbol(HIP_SYMBOL(dq::c_cell), cell, sizeof(cell)) == hipSuccess;
}

#define SFM_DQ_BODY(WS)                                                                              \
    if (rotate)                                                                                      \
      hipLaunchKernelGGL((dq::k_describe_q<WS, 1>), grid, dim3(64), 0, st, lvl, H, W, kp, kcap, lc,  \
                         level, B, scale, out_xy, out_desc, out_conf, out_cap, out_count, L, mo);        \
    else                                                                                             \
      hipLaunchKernelGGL((dq::k_describe_q<WS, 0>), grid, dim3(64), 0, st, lvl, H, W, kp, kcap, lc,  \
                         level, B, scale, out_xy, out_desc, out_conf, out_cap, out_count, L, mo);        \
    return true;
#define SFM_DQ_CASE(WS) \
  case WS:              \
    SFM_DQ_BODY(WS)

bool launch_describe_quad(const float* lvl, int B, int H, int W, int fw, int rotate, KpList kp, int kcap,
                          const int32_t* lc, int level, double scale, int32_t* out_xy, float* out_desc,
                          float* out_conf, int64_t out_cap, int32_t* out_count, int L, const MatchOperands& mo,
                          hipStream_t st) {
  // (+ the padding-row workgroups of the fused matcher operands in the last level's launch)
  constexpr int kPadBlocks = 8;
  const dim3 grid((kcap + 3) / 4 + (mo.hi != nullptr && out_count != nullptr ? kPadBlocks : 0), B);
  switch (2 * (fw / 2)) {
    SFM_DQ_CASE(2)
    SFM_DQ_CASE(4)
    SFM_DQ_CASE(6)
    SFM_DQ_CASE(8)
    SFM_DQ_CASE(10)
    SFM_DQ_CASE(12)
    SFM_DQ_CASE(14)
    SFM_DQ_CASE(16)
    case 18:
#ifdef SFM_ABLATIONS  // timing ablations: the diagnostic build only
      if (rotate) {
        static const int abl = [] {
          const char* v = SFM_ABLATION_ENV("SFMFEAT_DQ_ABL");
          return v ? atoi(v) : 0;
        }();
        switch (abl) {
#define SFM_DQ_ABL(A)                                                                                     \
  case A:                                                                                                \
    hipLaunchKernelGGL((dq::k_describe_q<18, 1, A>), grid, dim3(64), 0, st, lvl, H, W, kp, kcap, lc, level, \
                       B, scale, out_xy, out_desc, out_conf, out_cap, out_count, L, mo);                     \
    return true;
          SFM_DQ_ABL(1)
          SFM_DQ_ABL(2)
          SFM_DQ_ABL(4)
          SFM_DQ_ABL(8)
          SFM_DQ_ABL(7)
          SFM_DQ_ABL(16)
          SFM_DQ_ABL(32)
          SFM_DQ_ABL(64)
          SFM_DQ_ABL(55)
          SFM_DQ_ABL(127)
          default:
            break;
        }
      }
#endif
      SFM_DQ_BODY(18)
    SFM_DQ_CASE(20)
    SFM_DQ_CASE(22)
    default:
      return false;
  }
}

}  // namespace sfm
