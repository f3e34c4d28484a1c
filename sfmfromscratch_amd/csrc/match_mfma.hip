// match_mfma.hip — exact NN-ratio matching with an MFMA prefilter.
//
// The reference's distances (NNRatioFeatureMatcher.py:31-34) are float32 pairwise sums;
// its result only depends on, per query row, the two smallest distances and the argmin.
// Those are found EXACTLY in three steps inside one workgroup of 128 query rows:
//   1. approximate d^2 = |a|^2 + |b|^2 - 2 a.b for every target with fp16 split operands
//      (a = hi + lo * 2^-11, three f16 MFMA products hi.hi + (hi.lo + lo.hi), f32
//      accumulation, operands pre-scaled by 2^8 to keep them out of the f16 subnormal
//      range), tracking each row's second-smallest approximate value D2~ (sweep 1);
//   2. a second sweep collects every target with d~ <= D2~ + 2 E_i, where E_i bounds
//      |d~ - d_ref| rigorously (fp16 representation, dropped lo.lo term, f32 accumulation
//      error <= K u sum|ab|, f32 rounding of d~ and of the reference's own pairwise sum):
//      any target outside that window is strictly farther than the second nearest;
//   3. recompute the window with the reference's exact float32 pairwise order (8
//      accumulators) and take (distance, index) minima -> ratio test.
// Rows whose window overflows the per-row LDS list (runs of near-identical target
// descriptors) are recomputed exactly over all targets by k_match_overflow.
#include <stdlib.h>

#include <type_traits>

#include "kernels.h"

namespace sfm {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kQW = 32;                // query rows per wave
constexpr int kWaves = 4;              // waves per workgroup
constexpr int kQB = kQW * kWaves;      // 128 query rows per workgroup
constexpr int kRowH = 128 + 8;         // padded fp16 row in LDS (272 B): conflict-free b128 reads
constexpr int kCandCap = 128;          // window members per query row kept in LDS
constexpr float kScale = 256.0f;       // operand pre-scale (2^8)
constexpr float kLoScale = 2048.0f;    // lo part scale (2^11)

// Per image: fp16 hi / lo (scaled) copies, squared norms (float32 of the float64 sum),
// norms, and per-image maxima for the error bound.
__global__ void __launch_bounds__(256) k_match_prep(const float* __restrict__ desc,
                                                   const int32_t* __restrict__ count, int64_t cap,
                                                   int64_t capP, _Float16* __restrict__ hi,
                                                   _Float16* __restrict__ lo,
                                                   float* __restrict__ norm2,
                                                   float* __restrict__ rnorm) {
  const int img = blockIdx.y;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);  // one wave per row
  const int lane = threadIdx.x & 63;
  const int n = count[img];
  const int64_t o = ((int64_t)img * capP + row) * 128;
  float a0 = 0.0f, a1 = 0.0f;
  if (row < n) {
    const float* src = desc + ((int64_t)img * cap + row) * 128;
    a0 = src[lane];
    a1 = src[lane + 64];
  }
  float v[2] = {a0, a1};
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    float x = v[q] * kScale;
    _Float16 h = (_Float16)x;
    float r = (x - (float)h) * kLoScale;  // exact difference, exact power-of-two scaling
    hi[o + lane + 64 * q] = h;
    lo[o + lane + 64 * q] = (_Float16)r;
    s += (double)v[q] * (double)v[q];
  }
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) {
    float n2 = (float)s;
    float rn = (float)sqrt(s);
    // padding rows: +inf squared norm, so their approximate distance is +inf and the
    // sweep needs no bounds checks (never admitted, never in the top 2)
    norm2[(int64_t)img * capP + row] = row < n ? n2 : INFINITY;
    rnorm[(int64_t)img * capP + row] = rn;
  }
}

// Per-image maxima of the squared norms and norms (block reduction, no atomics).
__global__ void __launch_bounds__(256) k_match_imgmax(const int32_t* __restrict__ count, int64_t capP,
                                                      const float* __restrict__ norm2,
                                                      const float* __restrict__ rnorm,
                                                      unsigned int* __restrict__ imgmax) {
  __shared__ float s_a[256], s_b[256];
  const int img = blockIdx.x, tid = threadIdx.x;
  const int n = count[img];
  float a = 0.0f, b = 0.0f;
  for (int r = tid; r < n; r += 256) {
    a = fmaxf(a, norm2[(int64_t)img * capP + r]);
    b = fmaxf(b, rnorm[(int64_t)img * capP + r]);
  }
  s_a[tid] = a;
  s_b[tid] = b;
  __syncthreads();
  for (int off = 128; off >= 1; off >>= 1) {
    if (tid < off) {
      s_a[tid] = fmaxf(s_a[tid], s_a[tid + off]);
      s_b[tid] = fmaxf(s_b[tid], s_b[tid + off]);
    }
    __syncthreads();
  }
  if (tid == 0) {
    imgmax[img * 2 + 0] = __float_as_uint(s_a[0]);
    imgmax[img * 2 + 1] = __float_as_uint(s_b[0]);
  }
}

// Reference-order exact squared distance (numpy pairwise, 8 accumulators).
SFM_DEV float exact_sqdist(const float* __restrict__ a, const float* __restrict__ b) {
  float r[8];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float4 a0 = *reinterpret_cast<const float4*>(a + 8 * i);
    float4 a1 = *reinterpret_cast<const float4*>(a + 8 * i + 4);
    float4 b0 = *reinterpret_cast<const float4*>(b + 8 * i);
    float4 b1 = *reinterpret_cast<const float4*>(b + 8 * i + 4);
    float d[8] = {a0.x - b0.x, a0.y - b0.y, a0.z - b0.z, a0.w - b0.w,
                  a1.x - b1.x, a1.y - b1.y, a1.z - b1.z, a1.w - b1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float sq = d[j] * d[j];
      r[j] = (i == 0) ? sq : r[j] + sq;
    }
  }
  float t01 = r[0] + r[1], t23 = r[2] + r[3], t45 = r[4] + r[5], t67 = r[6] + r[7];
  float u0 = t01 + t23, u1 = t45 + t67;
  return u0 + u1;
}

SFM_DEV void top2_merge(float& b1, int& j1, float& b2, float ob1, int oj1, float ob2) {
  if (ob1 < b1 || (ob1 == b1 && oj1 < j1)) {
    b2 = fminf(b1, ob2);
    b1 = ob1;
    j1 = oj1;
  } else {
    b2 = fminf(b2, ob1);
  }
}

constexpr int kTT2 = 64;               // targets per LDS stage (two 32-target MFMA sub-tiles)
constexpr int kStageHalves = kTT2 * kRowH;  // f16 elements per array per stage
constexpr int kScr = 2 * kStageHalves / 2;  // re-rank scratch floats in the stage buffers (8704)

// One workgroup = 4 waves x 32 query rows; two sweeps over the target table of the pair, in
// 64-row LDS stages (the next stage's hi/lo rows are loaded into registers while the
// current stage's MFMAs run, then stored into the single LDS stage buffer):
//   sweep 1: the running top-2 of d~ per row (two v_med3 per element) -> the row's FINAL
//            window thr = b2~ + 2E (both halves of the wave merged);
//   sweep 2: the same MFMAs; every target with d~ <= thr is appended to the row's LDS list
//            (index only: the window is exact, so no approximate distance is kept and no
//            post-filter runs; a ballot skips the append code for stages where no lane of
//            the wave admits anything).
// Every target inside the window is re-ranked with the reference's exact float32 distance
// (flattened over the workgroup, in chunks through the stage buffers).  A row whose window
// holds more than kCandCap targets is handed to k_match_overflow (global list).
// The window argument: the targets achieving b1~ and b2~ have exact distances <= b1~ + E and
// <= b2~ + E, so the exact second-smallest D2 <= b2~ + E; a target with exact d <= D2 has
// d~ <= d + E <= b2~ + 2E.  Targets outside the window are strictly farther than D2.
// ABL (timing builds only; results are wrong unless 0): 6 = no re-rank, 8 = no sweep 2
template <int ABL>
__global__ void __launch_bounds__(256, 2) k_match_mfma(
    const float* __restrict__ desc, const int32_t* __restrict__ count, int64_t cap, int64_t capP,
    const _Float16* __restrict__ hi, const _Float16* __restrict__ lo, const float* __restrict__ norm2,
    const float* __restrict__ rnorm, const unsigned int* __restrict__ imgmax,
    const int32_t* __restrict__ pairs, int P, float ratio, RowBest* __restrict__ rows_out, int max_rows,
    int* __restrict__ ovf_count, int2* __restrict__ ovf_list) {
  // stage buffer [hi|lo][64][kRowH]; after the sweeps the space holds the re-rank scratch
  __shared__ __attribute__((aligned(16))) _Float16 sT[2][kStageHalves];
  __shared__ __attribute__((aligned(16))) float sN[kTT2];
  __shared__ uint16_t sCand[kQB][kCandCap];
  __shared__ int sCnt[kQB];
  __shared__ int sOff[kQB + 1];
  float* sDex = reinterpret_cast<float*>(&sT[0][0]);
  static_assert(sizeof(sT) >= (size_t)kScr * 4, "re-rank scratch fits");

  // XCD-aware mapping (workgroups b and b + 8 share an XCD and its L2): group g = b % 8
  // takes the pairs p = g (mod 8), so all query blocks of a pair stream its target table
  // through one L2
  const int QB = (max_rows + kQB - 1) / kQB;
  const int grp = blockIdx.x & 7, slot8 = blockIdx.x >> 3;
  const int p = grp + 8 * (slot8 / QB);
  if (p >= P) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int i1 = pairs[2 * p], i2 = pairs[2 * p + 1];
  const int n1 = count[i1], n2 = count[i2];
  const int row0 = (slot8 % QB) * kQB;
  if (row0 >= n1 || n2 < 1) return;

  // this lane's query row (column of the MFMA output) and its fragments, kept in registers
  const int ql = wid * kQW + (lane & 31);           // local query row 0..127
  const int qi = row0 + ql;                          // query row in image i1
  const int half = lane >> 5;
  const int64_t qo = ((int64_t)i1 * capP + qi) * 128;
  h8 qhi[8], qlo[8];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    qhi[kk] = *reinterpret_cast<const h8*>(hi + qo + kk * 16 + 8 * half);
    qlo[kk] = *reinterpret_cast<const h8*>(lo + qo + kk * 16 + 8 * half);
  }
  const float na = norm2[(int64_t)i1 * capP + qi];
  const float ra = rnorm[(int64_t)i1 * capP + qi];
  const float maxn2 = __uint_as_float(imgmax[i2 * 2 + 0]);
  const float maxrn = __uint_as_float(imgmax[i2 * 2 + 1]);
  // rigorous |d~ - d_ref| bound (matcher exactness)
  const float E = 3.0517578125e-05f * ra * maxrn + 4e-6f * (na + maxn2) + 1.25e-4f;
  for (int i = tid; i < kQB; i += 256) sCnt[i] = 0;

  const int nst = (n2 + kTT2 - 1) / kTT2;
  const int64_t to = (int64_t)i2 * capP * 128;
  // stage loader: 64 rows x (hi, lo) x 256 B = 32 KB; thread -> (row, 32-B column chunk)
  const int lr = tid >> 2, lc = (tid & 3) * 32;   // row 0..63, halves 0..127 step 32
  h8 g[8];
  auto load_stage = [&](int st) {
    const int64_t gofs = to + (int64_t)(st * kTT2 + lr) * 128 + lc;  // rows < capP: in bounds
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      g[q] = *reinterpret_cast<const h8*>(hi + gofs + 8 * q);
      g[4 + q] = *reinterpret_cast<const h8*>(lo + gofs + 8 * q);
    }
  };
  auto store_stage = [&]() {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      *reinterpret_cast<h8*>(&sT[0][lr * kRowH + lc + 8 * q]) = g[q];
      *reinterpret_cast<h8*>(&sT[1][lr * kRowH + lc + 8 * q]) = g[4 + q];
    }
  };

  float b1 = INFINITY, b2 = INFINITY, thr = INFINITY;
  const bool live = qi < n1;
  // one sweep over the pair's targets; PH 0 tracks the running top-2, PH 1 appends the
  // final window
  auto sweep = [&](auto phc) {
    constexpr int PH = decltype(phc)::value;
    load_stage(0);
    const float nrm_t0 = (tid < kTT2) ? norm2[(int64_t)i2 * capP + tid] : 0.0f;
    store_stage();
    if (tid < kTT2) sN[tid] = nrm_t0;
    for (int st = 0; st < nst; ++st) {
      __syncthreads();  // stage st visible
      float nrm_next = 0.0f;
      if (st + 1 < nst) {
        load_stage(st + 1);
        if (tid < kTT2) nrm_next = norm2[(int64_t)i2 * capP + (st + 1) * kTT2 + tid];
      }
      const _Float16* tH = &sT[0][0];
      const _Float16* tL = &sT[1][0];
      uint32_t mm = 0;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        // 32 targets x 32 queries: hi.hi into ahh, hi.lo + lo.hi into ax (one chain each)
        f32x16 ahh = {}, ax = {};
        const int trow = (32 * sub + (lane & 31)) * kRowH;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const int ko = kk * 16 + 8 * half;
          const h8 thi = *reinterpret_cast<const h8*>(tH + trow + ko);
          const h8 tlo = *reinterpret_cast<const h8*>(tL + trow + ko);
          ahh = __builtin_amdgcn_mfma_f32_32x32x16_f16(thi, qhi[kk], ahh, 0, 0, 0);
          ax = __builtin_amdgcn_mfma_f32_32x32x16_f16(thi, qlo[kk], ax, 0, 0, 0);
          ax = __builtin_amdgcn_mfma_f32_32x32x16_f16(tlo, qhi[kk], ax, 0, 0, 0);
        }
        // d~ = na + nb - 2 a.b with a.b = (ahh + ax 2^-11) 2^-16: two fmas by exact powers
        // of two (each rounding is covered by E's 4e-6 (na + nb) term);
        // targets past n2 are padding rows with norm2 = +inf: d~ = +inf
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const float4 nb4 = *reinterpret_cast<const float4*>(&sN[32 * sub + 8 * g4 + 4 * half]);
          const float nbv[4] = {nb4.x, nb4.y, nb4.z, nb4.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int rr = 4 * g4 + e;
            const float t2 = na + nbv[e];
            const float dv = __builtin_fmaf(ax[rr], -1.4901161193847656e-08f /* -2^-26 */,
                                            __builtin_fmaf(ahh[rr], -3.0517578125e-05f /* -2^-15 */, t2));
            if (PH == 0) {  // running top-2 (b1 <= b2): b2 = med3(b1, b2, d), b1 = min(b1, d)
              b2 = __builtin_amdgcn_fmed3f(b1, b2, dv);
              b1 = __builtin_amdgcn_fmed3f(b1, dv, -INFINITY);
            } else {
              mm |= (dv <= thr) ? (1u << (16 * sub + rr)) : 0u;
            }
          }
        }
      }
      if (PH == 1 && __any(mm != 0u)) {  // wave-uniform: skip when no lane admits
        if (live && mm) {  // reserve this lane's slots with one LDS atomic, then fill them
          int slot = atomicAdd(&sCnt[ql], __popc(mm));
          for (; mm; mm &= mm - 1, ++slot) {
            const int bit = __builtin_ctz(mm), rr = bit & 15;
            const int j = st * kTT2 + 32 * (bit >> 4) + 4 * half + (rr & 3) + 8 * (rr >> 2);
            if (slot < kCandCap) sCand[ql][slot] = (uint16_t)j;
          }
        }
      }
      if (st + 1 < nst) {
        __syncthreads();  // every wave is done with this stage's LDS rows
        store_stage();
        if (tid < kTT2) sN[tid] = nrm_next;
      }
    }
  };
  sweep(std::integral_constant<int, 0>{});
  {  // the row's final window (both halves of the wave merged)
    const float ob1 = __shfl_xor(b1, 32), ob2 = __shfl_xor(b2, 32);
    thr = fminf(fmaxf(b1, ob1), fminf(b2, ob2)) + 2.0f * E;
  }
  __syncthreads();  // sweep 1's last stage consumed before sweep 2 overwrites the buffer
  if (ABL == 8) {
    if (thr == -1.0f) rows_out[0].col = 1;  // defeats dead-code elimination
    return;
  }
  sweep(std::integral_constant<int, 1>{});
  __syncthreads();  // sweeps done: the stage buffers become the re-rank scratch
  if (ABL != 0) return;

  // exact re-rank of every window member, flattened over the workgroup: row rl owns
  // entries [sOff[rl], sOff[rl+1]); a row whose window overflowed its list goes to the
  // overflow kernel instead
  if (tid < kQB) {
    const int c = sCnt[tid];
    const bool ok = row0 + tid < n1 && c <= kCandCap;
    sOff[tid + 1] = ok ? c : 0;
    if (row0 + tid < n1 && c > kCandCap) {
      const int k = atomicAdd(ovf_count, 1);
      ovf_list[k] = make_int2(p, row0 + tid);
    }
  }
  if (tid == 0) sOff[0] = 0;
  __syncthreads();
  if (tid < 64) {  // inclusive scan of the 128 counts by one wave (2 per lane)
    int a = sOff[2 * tid + 1], b = sOff[2 * tid + 2];
    int x = a + b;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off);
      if (tid >= off) x += y;
    }
    sOff[2 * tid + 1] = x - b;
    sOff[2 * tid + 2] = x;
  }
  __syncthreads();
  const int total = sOff[kQB];
  const float* A = desc + (int64_t)i1 * cap * 128;
  const float* Bd = desc + (int64_t)i2 * cap * 128;
  float e1 = INFINITY, e2 = INFINITY;
  int j1 = 0x7fffffff;
  for (int c0 = 0; c0 < total; c0 += kScr) {
    const int c1 = min(total, c0 + kScr);
    for (int e = c0 + tid; e < c1; e += 256) {
      int lo_ = 0, hi_ = kQB;  // the row with sOff[row] <= e < sOff[row + 1]
      while (hi_ - lo_ > 1) {
        const int mid = (lo_ + hi_) >> 1;
        if (sOff[mid] <= e) lo_ = mid; else hi_ = mid;
      }
      const int rl = lo_, slot = e - sOff[rl];
      sDex[e - c0] = exact_sqdist(A + (int64_t)(row0 + rl) * 128, Bd + (int64_t)sCand[rl][slot] * 128);
    }
    __syncthreads();
    if (tid < kQB) {  // this row's entries inside the chunk, (distance, index) order
      const int s0 = max(sOff[tid], c0), s1 = min(sOff[tid + 1], c1);
      for (int e = s0; e < s1; ++e) {
        const float dd = sDex[e - c0];
        const int j = sCand[tid][e - sOff[tid]];
        if (dd < e1 || (dd == e1 && j < j1)) { e2 = e1; e1 = dd; j1 = j; }
        else if (dd < e2) e2 = dd;
      }
    }
    __syncthreads();
  }
  if (tid < kQB && row0 + tid < n1 && sCnt[tid] <= kCandCap) {
    RowBest rb;
    rb.col = -1;
    rb.nndr = 0.0f;
    const float d1 = sqrtf(e1), d2 = sqrtf(e2);
    if (d2 > 0.0f) {
      const float nndr = d1 / d2;
      if (nndr <= ratio) { rb.col = j1; rb.nndr = nndr; }
    }
    rows_out[(int64_t)p * max_rows + row0 + tid] = rb;
  }
}

// Rows whose window overflowed the LDS list (long runs of near-identical target
// descriptors): exact distances to every target, one wavefront per row — lanes stride the
// targets (the query row is a wave-uniform broadcast load), per-lane (distance, index)
// top-2, then a shuffle merge.  Grid-stride over the list, so the launch needs no host
// read of its length.
__global__ void __launch_bounds__(256) k_match_overflow(const float* __restrict__ desc,
                                                        const int32_t* __restrict__ count, int64_t cap,
                                                        const int32_t* __restrict__ pairs, float ratio,
                                                        RowBest* __restrict__ rows_out, int max_rows,
                                                        const int* __restrict__ ovf_count,
                                                        const int2* __restrict__ ovf_list) {
  const int nov = *ovf_count;
  const int lane = threadIdx.x & 63;
  for (int w = blockIdx.x * 4 + (threadIdx.x >> 6); w < nov; w += gridDim.x * 4) {
    const int2 ent = ovf_list[w];
    const int p = ent.x, row = ent.y;
    const int i1 = pairs[2 * p], i2 = pairs[2 * p + 1];
    const int n2 = count[i2];
    const float* A = desc + ((int64_t)i1 * cap + row) * 128;
    const float* Bd = desc + (int64_t)i2 * cap * 128;
    float e1 = INFINITY, e2 = INFINITY;
    int j1 = 0x7fffffff;
    for (int j = lane; j < n2; j += 64) {
      const float dd = exact_sqdist(A, Bd + (int64_t)j * 128);
      if (dd < e1 || (dd == e1 && j < j1)) { e2 = e1; e1 = dd; j1 = j; }
      else if (dd < e2) e2 = dd;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const float o1 = __shfl_xor(e1, off), o2 = __shfl_xor(e2, off);
      const int oj = __shfl_xor(j1, off);
      top2_merge(e1, j1, e2, o1, oj, o2);
    }
    if (lane == 0) {
      RowBest rb;
      rb.col = -1;
      rb.nndr = 0.0f;
      const float d1 = sqrtf(e1), d2 = sqrtf(e2);
      if (d2 > 0.0f) {
        const float nndr = d1 / d2;
        if (nndr <= ratio) { rb.col = j1; rb.nndr = nndr; }
      }
      rows_out[(int64_t)p * max_rows + row] = rb;
    }
  }
}

void launch_match_prep(const float* desc, const int32_t* count, int nimg, int64_t cap, int64_t capP,
                       _Float16* hi, _Float16* lo, float* norm2, float* rnorm, unsigned int* imgmax,
                       hipStream_t st) {
  hipLaunchKernelGGL(k_match_prep, dim3((unsigned)(capP / 4), nimg), dim3(256), 0, st, desc, count, cap, capP, hi,
                     lo, norm2, rnorm);
  hipLaunchKernelGGL(k_match_imgmax, dim3(nimg), dim3(256), 0, st, count, capP, norm2, rnorm, imgmax);
}

void launch_match_mfma(const float* desc, const int32_t* count, int64_t cap, int64_t capP,
                       const _Float16* hi, const _Float16* lo, const float* norm2, const float* rnorm,
                       const unsigned int* imgmax, const int32_t* pairs, int P, float ratio,
                       RowBest* rows, int max_rows, int* ovf_count, int2* ovf_list, hipStream_t st) {
  static const int abl = [] {
    const char* e = getenv("SFMFEAT_MATCH_ABL");  // diagnostics only (tools/bench_match.py)
    return e ? atoi(e) : 0;
  }();
  const int qb = (max_rows + kQB - 1) / kQB;
  const dim3 grid((unsigned)(8 * ((P + 7) / 8) * qb));
  (void)hipMemsetAsync(ovf_count, 0, sizeof(int), st);
  if (abl == 6)
    hipLaunchKernelGGL(k_match_mfma<6>, grid, dim3(256), 0, st, desc, count, cap, capP, hi, lo, norm2, rnorm, imgmax,
                       pairs, P, ratio, rows, max_rows, ovf_count, ovf_list);
  else if (abl == 8)
    hipLaunchKernelGGL(k_match_mfma<8>, grid, dim3(256), 0, st, desc, count, cap, capP, hi, lo, norm2, rnorm, imgmax,
                       pairs, P, ratio, rows, max_rows, ovf_count, ovf_list);
  else
    hipLaunchKernelGGL(k_match_mfma<0>, grid, dim3(256), 0, st, desc, count, cap, capP, hi, lo, norm2, rnorm, imgmax,
                       pairs, P, ratio, rows, max_rows, ovf_count, ovf_list);
  // the overflow list's length stays on the device: a fixed grid strides over it
  hipLaunchKernelGGL(k_match_overflow, dim3(256), dim3(256), 0, st, desc, count, cap, pairs, ratio, rows, max_rows,
                     ovf_count, ovf_list);
}

}  // namespace sfm
