// common.h — device helpers shared by the gfx950 kernels of libsfmfeat.
//
// Numeric contract: every kernel is compiled with
// -ffp-contract=off and correctly rounded f32 division / sqrt, so each arithmetic
// expression below is one IEEE binary32 (or binary64) operation; fused multiply-adds
// appear only as explicit __builtin_fmaf where the contract prescribes them.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define SFM_DEV __device__ __forceinline__

// Timing ablations (results wrong by design: SFMFEAT_SKIP, SFMFEAT_HARRIS_ABL,
// SFMFEAT_SELECT_ABL, SFMFEAT_DQ_ABL, SFMFEAT_NMS_DRY) exist only in a diagnostic build of the
// library (make ABLATIONS=1: -DSFM_ABLATIONS, its own output directory).  The shipped
// libsfmfeat.so never reads those switches, so no environment can make it skip work;
// sfm_build_flags() tells the two builds apart.
#ifdef SFM_ABLATIONS
#define SFM_ABLATION_ENV(name) getenv(name)
#else
#define SFM_ABLATION_ENV(name) ((const char*)nullptr)
#endif
// Diagnostic A/B switches (alternative layouts, launch shapes and stream schedules that were
// measured slower and are kept for experiments): like the ablations, read only by the
// diagnostic build.  The shipped library reads only the product switches, each of which
// tests/test_gpu_switches.py runs against the default bit for bit (PRODUCT_SWITCHES there).
#define SFM_DIAG_ENV(name) SFM_ABLATION_ENV(name)

namespace sfm {

constexpr int kWave = 64;

SFM_DEV uint32_t fbits(float f) { return __float_as_uint(f); }
SFM_DEV float ffrom(uint32_t u) { return __uint_as_float(u); }

// Exact 2x downscale of one value (OpenCV's INTER_AREA-fast rule for exact 2x resizes,
// pyramid.hip): ((a00 + a01) + (a10 + a11)) * 0.25
SFM_DEV float down2_px(float a00, float a01, float a10, float a11) {
  const float t0 = a00 + a01;
  const float t1 = a10 + a11;
  return (t0 + t1) * 0.25f;
}
// One 8 x 8 block (block row by, column bx) of plane b of a level of size sh x sw -> its
// 4 x 4, 2 x 2 and 1 x 1 blocks of the next three exact 2x levels (16-B stores into d1)
SFM_DEV void down2x3_block(const float (&a)[8][8], float* d1, float* d2, float* d3, int b, int sh, int sw,
                           int by, int bx) {
  const int w1 = sw >> 1, w2 = sw >> 2, w3 = sw >> 3;
  const int h1 = sh >> 1, h2 = sh >> 2, h3 = sh >> 3;
  float l1[4][4], l2[2][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      l1[i][j] = down2_px(a[2 * i][2 * j], a[2 * i][2 * j + 1], a[2 * i + 1][2 * j], a[2 * i + 1][2 * j + 1]);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      l2[i][j] = down2_px(l1[2 * i][2 * j], l1[2 * i][2 * j + 1], l1[2 * i + 1][2 * j], l1[2 * i + 1][2 * j + 1]);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    *reinterpret_cast<float4*>(d1 + ((int64_t)b * h1 + 4 * by + i) * w1 + 4 * bx) =
        make_float4(l1[i][0], l1[i][1], l1[i][2], l1[i][3]);
#pragma unroll
  for (int i = 0; i < 2; ++i)
    *reinterpret_cast<float2*>(d2 + ((int64_t)b * h2 + 2 * by + i) * w2 + 2 * bx) = make_float2(l2[i][0], l2[i][1]);
  d3[((int64_t)b * h3 + by) * w3 + bx] = down2_px(l2[0][0], l2[0][1], l2[1][0], l2[1][1]);
}

// Order-preserving map float -> uint32 (ascending), -0 folded onto +0 (numpy compares
// them equal; the median/selection only ever needs the value back).
SFM_DEV uint32_t fkey(float v) {
  uint32_t b = __float_as_uint(v);
  if (b == 0x80000000u) b = 0u;
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
// fkey for values that are never -0 (three VALU ops, no compare): b ^ m with m = 0x80000000
// for b >= 0 (b | 0x80000000) and m = 0xffffffff for b < 0 (~b).  Harris's R is never -0
// (det = t1 - t2 of non-negative products, at = alpha tr^2 >= +0, and x - x = +0), so its
// digit-1 histogram takes this form (tests/test_gpu_parity.py pins the R map and median).
SFM_DEV uint32_t fkey_nz(float v) {
  const uint32_t b = __float_as_uint(v);
  return b ^ ((uint32_t)((int32_t)b >> 31) | 0x80000000u);
}
SFM_DEV float fkey_inv(uint32_t k) {
  uint32_t b = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(b);
}

// np.arctan2 on float32 as numpy's bundled SVML __svml_atan2f16 computes it
// (transcription pinned bit-exactly against numpy; oracle/sfm_oracle.c orc_atan2f).
SFM_DEV float svml_atan2f(float y, float x) {
  const float PI = __uint_as_float(0x40490fdbu), PI_2 = __uint_as_float(0x3fc90fdbu);
  float ax = fabsf(x), ay = fabsf(y);
  uint32_t sy = __float_as_uint(y) & 0x80000000u;
  uint32_t sx = __float_as_uint(x) & 0x80000000u;
  if (ay == 0.0f) return __uint_as_float((sx ? __float_as_uint(PI) : 0u) | sy);
  if (ax == 0.0f) return __uint_as_float(__float_as_uint(PI_2) | sy);
  bool k = ay < ax;
  float num = k ? ay : -ax;
  float den = k ? ax : ay;
  float off = k ? 0.0f : PI_2;
  float q = num / den;
  float z2 = q * q;
  float z4 = z2 * z2;
  const float c0 = __uint_as_float(0x3b322cc0u), c1 = __uint_as_float(0xbc7f2631u),
              c2 = __uint_as_float(0x3d2bc384u), c3 = __uint_as_float(0xbd987629u),
              c4 = __uint_as_float(0x3dd96474u), c5 = __uint_as_float(0xbe1161f8u),
              c6 = __uint_as_float(0x3e4cb79fu), c7 = __uint_as_float(0xbeaaaa49u);
  float A = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(__builtin_fmaf(c0, z4, c2), z4, c4), z4, c6), z4, 1.0f);
  float B = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(c1, z4, c3), z4, c5), z4, c7);
  float r = __builtin_fmaf(__builtin_fmaf(B, z2, A), q, off);
  if (sx) {
    r = __uint_as_float(__float_as_uint(r) | 0x80000000u);
    r = r + PI;
  }
  return __uint_as_float(__float_as_uint(r) | sy);
}

// Wave-aggregated append: every lane with `pred` gets a unique slot in [0, *counter).
// Returns the slot (or -1 for lanes without pred).  One atomic per wave.
SFM_DEV int64_t wave_append(unsigned long long* counter, bool pred) {
  uint64_t mask = __ballot(pred);
  if (mask == 0) return -1;
  int lane = __lane_id();
  int leader = __ffsll((unsigned long long)mask) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(counter, (unsigned long long)__popcll(mask));
  base = __shfl(base, leader);
  uint64_t lower = mask & ((lane == 0) ? 0ull : (~0ull >> (64 - lane)));
  return pred ? (int64_t)(base + __popcll(lower)) : -1;
}

// Block-wide append with ONE global atomic per workgroup (same-address atomics serialise
// at ~88/us on MI355X, MI355X_MICROARCH.md 'dequeue'): every thread contributes `cnt`
// items; returns the thread's first slot.  Item order inside the block is thread order.
// s_wsum: >= blockDim.x/64 uint32; s_base: one uint64.  Every thread must call it.
SFM_DEV int64_t block_append(unsigned long long* counter, uint32_t cnt, uint32_t* s_wsum,
                             unsigned long long* s_base) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nw = blockDim.x >> 6;
  uint32_t x = cnt;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    uint32_t y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_wsum[wid] = x;
  __syncthreads();
  if (tid == 0) {
    uint32_t run = 0;
    for (int w = 0; w < nw; ++w) {
      uint32_t t = s_wsum[w];
      s_wsum[w] = run;
      run += t;
    }
    *s_base = run ? atomicAdd(counter, (unsigned long long)run) : 0ull;
  }
  __syncthreads();
  int64_t r = (int64_t)(*s_base + s_wsum[wid] + (x - cnt));
  __syncthreads();
  return r;
}

// Inclusive prefix sum of one uint32 per lane across the wavefront (shuffles, no LDS).
SFM_DEV uint32_t wave_inclusive_scan(uint32_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  return x;
}

// Block-wide: given a histogram of `nb` bins in LDS (nb a multiple of blockDim.x, blockDim.x
// a multiple of 64), find the bin holding 0-based rank `rank`; s_out = {bin, count before
// bin}.  s_scan holds >= blockDim.x / 64 uint32 (wave totals).  Every thread calls it.
// Wave-shuffle scan: two block barriers.
SFM_DEV void find_bin(const uint32_t* s_h, int nb, uint32_t rank, uint32_t* s_scan,
                      uint32_t* s_out) {
  const int tid = threadIdx.x, nt = blockDim.x, wid = tid >> 6;
  const int per = nb / nt;
  uint32_t local = 0;
  for (int i = 0; i < per; ++i) local += s_h[tid * per + i];
  const uint32_t x = wave_inclusive_scan(local);
  if ((tid & 63) == 63) s_scan[wid] = x;
  __syncthreads();
  uint32_t base = 0;
  for (int w = 0; w < wid; ++w) base += s_scan[w];
  const uint32_t excl = base + x - local, incl = excl + local;
  if (rank >= excl && rank < incl) {
    uint32_t c = excl;
    for (int i = 0; i < per; ++i) {
      uint32_t h = s_h[tid * per + i];
      if (rank < c + h) {
        s_out[0] = (uint32_t)(tid * per + i);
        s_out[1] = c;
        break;
      }
      c += h;
    }
  }
  __syncthreads();
}

// Block-wide exclusive scan of one uint32 per thread; returns the exclusive prefix and
// writes the block total to *total.  s_scan holds >= blockDim.x / 64 + 1 uint32.
SFM_DEV uint32_t block_exclusive_scan(uint32_t v, uint32_t* s_scan, uint32_t* total) {
  const int tid = threadIdx.x, nt = blockDim.x, wid = tid >> 6, nw = nt >> 6;
  const uint32_t x = wave_inclusive_scan(v);
  if ((tid & 63) == 63) s_scan[wid] = x;
  __syncthreads();
  uint32_t base = 0, all = 0;
  for (int w = 0; w < nw; ++w) {
    const uint32_t t = s_scan[w];
    base += w < wid ? t : 0u;
    all += t;
  }
  *total = all;
  __syncthreads();
  return base + x - v;
}

// Block-wide ascending bitonic sort of P (power of two) uint64 keys in LDS (blockDim.x a
// multiple of 64).  Stages with stride < 64 stay inside an aligned 128-key chunk that one
// wave owns (pair i of chunk i / 64), so they need only wave-level ordering; the larger
// strides are separated by block barriers.
SFM_DEV void bitonic_sort_u64(uint64_t* s, int P) {
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const bool wide = stride >= 64;
      if (wide) __syncthreads();
      for (int i = tid; i < (P >> 1); i += nt) {
        int pos = 2 * i - (i & (stride - 1));
        int partner = pos + stride;
        bool asc = (pos & size) == 0;
        uint64_t a = s[pos], b = s[partner];
        if ((a > b) == asc) {
          s[pos] = b;
          s[partner] = a;
        }
      }
      if (wide) {
        __syncthreads();
      } else {  // LDS ops of one wave are processed in order; keep the compiler from reordering
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
  }
  __syncthreads();
}

// One wavefront sorts N = 64 * E u64 keys held in registers, blocked layout (element m in
// lane m / E, slot m % E), ascending.  Bitonic network with compile-time stages: strides
// below E compare-exchange inside a lane, larger strides exchange with lane ^ (stride / E).
template <int E>
SFM_DEV void wave_bitonic_sort_u64(uint64_t (&k)[E]) {
  const int lane = threadIdx.x & 63;
  constexpr int N = 64 * E;
#pragma unroll
  for (int size = 2; size <= N; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride >= E) {
        const int lm = stride / E;
        const bool lower = (lane & lm) == 0;
#pragma unroll
        for (int r = 0; r < E; ++r) {
          const bool asc = ((lane * E + r) & size) == 0;
          const uint32_t olo = __shfl_xor((uint32_t)k[r], lm);
          const uint32_t ohi = __shfl_xor((uint32_t)(k[r] >> 32), lm);
          const uint64_t o = ((uint64_t)ohi << 32) | olo;
          const bool take_min = (asc == lower);
          const bool lt = o < k[r];
          k[r] = (take_min == lt) ? o : k[r];
        }
      } else {
#pragma unroll
        for (int r = 0; r < E; ++r) {
          if ((r & stride) == 0) {
            const bool asc = ((lane * E + r) & size) == 0;
            const uint64_t a = k[r], b = k[r + stride];
            const bool sw = (a > b) == asc;
            k[r] = sw ? b : a;
            k[r + stride] = sw ? a : b;
          }
        }
      }
    }
  }
}

SFM_DEV int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

// The n (<= blockDim.x) keys of s[0..n) in ascending order, by runs: each wave sorts its 64
// keys in registers (shuffle bitonic, no LDS), the sorted runs go back to LDS, and every key's
// final position is its place in its run plus, for each other run, the number of that run's
// keys below it (a 64-entry binary search; the runs' searches are independent).  The keys are
// distinct (their low half is the raster index); padding (~0) sorts after every key and is not
// stored.  Three barriers instead of the bitonic network's ~55 stages (10 block-wide).
template <int E>  // keys per lane: runs of 64 E keys, n <= E * blockDim.x
SFM_DEV void run_merge_sort_u64(uint64_t* s, int n) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int RL = 64 * E;  // run length
  const int nruns = (n + RL - 1) / RL;
  uint64_t k[E];
#pragma unroll
  for (int r = 0; r < E; ++r) {
    const int i = w * RL + lane * E + r;
    k[r] = i < n ? s[i] : ~0ull;
  }
  if (w < nruns) wave_bitonic_sort_u64<E>(k);
  __syncthreads();
  if (w < nruns) {
#pragma unroll
    for (int r = 0; r < E; ++r) s[w * RL + lane * E + r] = k[r];
  }
  __syncthreads();
  uint32_t pos[E];
#pragma unroll
  for (int r = 0; r < E; ++r) pos[r] = (uint32_t)(lane * E + r);
  if (w < nruns) {
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      if (v < nruns && v != w) {
        const uint64_t* run = s + RL * v;
#pragma unroll
        for (int r = 0; r < E; ++r) {
          int lo = 0;  // keys of run v below k[r] (RL - 1 at most, then the last entry)
#pragma unroll
          for (int step = RL / 2; step >= 1; step >>= 1)
            if (run[lo + step - 1] < k[r]) lo += step;
          lo += (lo == RL - 1 && run[lo] < k[r]) ? 1 : 0;
          pos[r] += (uint32_t)lo;
        }
      }
    }
  }
  __syncthreads();
  if (w < nruns) {
#pragma unroll
    for (int r = 0; r < E; ++r)
      if (k[r] != ~0ull) s[pos[r]] = k[r];
  }
  __syncthreads();
}

// ascending sort of s[0..n) (distinct keys; padding ~0 sorts last): runs for n <= 2 blockDim.x,
// else the LDS bitonic network over next_pow2(n) slots (s must hold them)
SFM_DEV void sort_keys_u64(uint64_t* s, int n) {
  const int tid = threadIdx.x, nt = blockDim.x;
  if (n <= nt && nt <= 1024) {
    run_merge_sort_u64<1>(s, n);
  } else if (n <= 2 * nt && nt <= 1024) {
    run_merge_sort_u64<2>(s, n);
  } else {
    const int P = next_pow2(n);
    for (int i = tid; i < P; i += nt)
      if (i >= n) s[i] = ~0ull;
    __syncthreads();
    bitonic_sort_u64(s, P);
  }
}



}  // namespace sfm
