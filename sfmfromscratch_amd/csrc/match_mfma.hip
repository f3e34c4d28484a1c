// match_mfma.hip — exact NN-ratio matching with an MFMA prefilter.
//
// The reference's distances (NNRatioFeatureMatcher.py:31-34) are float32 pairwise sums;
// its result only depends on, per query row, the two smallest distances and the argmin.
// Those are found EXACTLY by:
//   1. k_match_mfma: ONE sweep per (pair, 256 query rows) over the target table computing
//      approximate d~ = |a|^2 + |b|^2 - 2 a.b with fp16 split operands (a = hi + lo 2^-11,
//      three f16 MFMA products hi.hi + (hi.lo + lo.hi), f32 accumulation, operands
//      pre-scaled by 2^8 out of the f16 subnormal range).  Each row keeps a running top-2
//      of d~ and appends to its window list every target with d~ <= b2~(so far) + 2 E_i,
//      where E_i bounds |d~ - d_ref| rigorously (fp16 representation, dropped lo.lo term,
//      f32 accumulation error, f32 rounding of d~ and of the reference's own pairwise
//      sum); any target outside the final window is strictly farther than the second
//      nearest (argument above k_match_mfma);
//   2. k_match_rerank: the list entries within the row's final threshold recomputed with the
//      reference's exact float32 pairwise order (8 accumulators), (distance, index) top-2,
//      ratio test;
//   3. k_match_overflow: rows whose list overflowed (runs of near-identical target
//      descriptors) recomputed exactly over every target.
#include <stdlib.h>

#include <type_traits>

#include "kernels.h"

namespace sfm {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kQW = 32;                // query rows per wave
constexpr int kWaves = 8;              // waves per workgroup (two per SIMD: one workgroup per CU)
constexpr int kQB = kQW * kWaves;      // 256 query rows per workgroup
constexpr int kNT = 64 * kWaves;       // threads per workgroup
constexpr int kRowH = 128 + 8;         // padded fp16 row in LDS (272 B): conflict-free b128 reads
constexpr int kCandCap = kMatchCandCap;  // admitted targets per query row (global list)
constexpr int kHalfCap = kCandCap / 2;   // each half-wave's share of a row's list
constexpr float kScale = kMatchScale;      // operand pre-scale (2^8)
constexpr float kLoScale = kMatchLoScale;  // lo part scale (2^11)

// Per image: fp16 hi / lo (scaled) copies, squared norms (float32 of the float64 sum),
// norms, and per-block maxima of both for the error bound (16 rows per workgroup, one wave
// per row; the sweep reduces a pair's target-image maxima itself, so no extra launch).
__global__ void __launch_bounds__(256) k_match_prep(const float* __restrict__ desc,
                                                   const int32_t* __restrict__ count, int64_t cap,
                                                   int64_t capP, _Float16* __restrict__ hi,
                                                   _Float16* __restrict__ lo,
                                                   float* __restrict__ norm2,
                                                   float* __restrict__ rnorm,
                                                   float2* __restrict__ pmax) {
  __shared__ float2 s_m[4];
  const int img = blockIdx.y;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = count[img];
  float m2 = 0.0f, mr = 0.0f;  // this wave's rows: maxima (lane 0)
#pragma unroll
  for (int k = 0; k < kPrepRows / 4; ++k) {
    const int row = blockIdx.x * kPrepRows + wv * (kPrepRows / 4) + k;
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
      if (row < n) {
        m2 = fmaxf(m2, n2);
        mr = fmaxf(mr, rn);
      }
    }
  }
  if (lane == 0) s_m[wv] = make_float2(m2, mr);
  __syncthreads();
  if (threadIdx.x == 0) {
    float2 r = s_m[0];
    for (int w = 1; w < 4; ++w) r = make_float2(fmaxf(r.x, s_m[w].x), fmaxf(r.y, s_m[w].y));
    pmax[(int64_t)img * gridDim.x + blockIdx.x] = r;
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

// d~ rounded DOWN to bf16 (kept as its top 16 bits): truncation for positive values;
// negative values (|d~| within E of 0) become -inf, which always passes the filter
SFM_DEV uint16_t bf16_down(float v) {
  return v >= 0.0f ? (uint16_t)(__float_as_uint(v) >> 16) : (uint16_t)0xFF80u;
}

// (m & a) | (~m & b) as one v_bfi_b32 (asm: the compiler turns a select tree over an array
// back into a dynamically indexed stack array)
SFM_DEV uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}
// all ones when bit `bit` of x is set, else 0 (v_bfe_i32: the bit, sign-extended)
SFM_DEV uint32_t lane_bit_mask(int x, int bit) { return (uint32_t)__builtin_amdgcn_sbfe(x, bit, 1); }

// x of the lane 32 away (the other half of the wavefront): one v_permlane32_swap + a select,
// instead of a ds_bpermute through the LDS crossbar
SFM_DEV float other_half(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}
SFM_DEV int other_half(int x) { return __float_as_int(other_half(__int_as_float(x))); }

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
// LDS of one sweep workgroup (one __shared__ array; carved per staging form below): stage
// buffers (hi, lo), target norms of the stages in use, the per-wave d~ staging of the appends:
// what the three-buffer LDS-DMA pipeline of one 512-thread workgroup per CU (two waves per
// SIMD) needs.  (Round 3 sized it to keep the sweep off CUs running k_harris: the two
// together changed Harris results.  The cause is a gfx950 hazard of packed-FP32 forms that
// read src1's high half beside MFMA (tools/pk_mfma_hazard.hip, DESIGN.md §7 Co-residency);
// Harris no longer uses them and tests/test_isa_guard_cpu.py keeps every kernel clear of
// them, so co-residency is safe and the size is a performance choice.)
constexpr int kDmaBufs = 3, kDmaNormBufs = 4;  // LDS-DMA staging: stage s + 2 in flight over s
constexpr int kRegBufs = 2, kRegNormBufs = 3;  // register staging
constexpr size_t kDBytes = (size_t)kWaves * 64 * 16 * 4;  // per-wave d~ staging of the appends
constexpr size_t kSweepLds = (size_t)kDmaBufs * 2 * kTT2 * 256 + kDmaNormBufs * kTT2 * 4 + kDBytes;
static_assert(kSweepLds >= (size_t)kRegBufs * 2 * kTT2 * kRowH * 2 + kRegNormBufs * kTT2 * 4 + kDBytes,
              "one LDS array serves both staging forms");
static_assert(kSweepLds <= 160 * 1024, "LDS per CU");
// STAGE 3 (the half-CU form): 4 waves x 32 query rows, two LDS-DMA stage buffers, no LDS
// staging of the appends: 65 KB of LDS and <= 256 VGPRs at one wave per SIMD, so a k_harris
// workgroup (80 KB, one wave per SIMD) fits beside it on the same CU — the matcher's MFMAs
// and Harris's VALU then share the SIMDs instead of taking CUs in turn
constexpr int kWaves3 = 4;
constexpr size_t kSweepLds3 = (size_t)2 * 2 * kTT2 * 256 + 3 * kTT2 * 4 + 256;
// (the Harris side is checked on the built code objects: tests/test_isa_guard_cpu.py
// test_half_cu_sweep_fits_beside_one_harris_workgroup reads both kernels' LDS from the
// metadata; this bound only keeps the sweep within half of the CU's LDS)
static_assert(kSweepLds3 <= 80 * 1024, "half-CU sweep: at most half of the CU's LDS");
constexpr int sweep_waves(int stage) { return stage == 3 ? kWaves3 : kWaves; }
constexpr int sweep_rows(int stage) { return kQW * sweep_waves(stage); }

// LDS-DMA (global_load_lds) issued from inline asm, M0 = the wave-uniform LDS destination:
// hipcc's own waitcnt pass then does not see them (it would wait vmcnt(0) ahead of every LDS
// read while one is in flight, draining the prefetch); the sweep counts them itself
__device__ __forceinline__ void glds_x4(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}
__device__ __forceinline__ void glds_x1(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

// One workgroup = 8 waves x 32 query rows; ONE sweep over the target table of the pair in
// 64-row LDS stages, software-pipelined by 32-target sub-tile: the MFMAs of one sub-tile run
// beside the epilogue of the previous one.  Staging (STAGE):
//   1 (default): LDS-DMA.  Each wave issues its share of a stage as global_load_lds_dwordx4
//     (1 KB = 4 target rows per instruction, no VGPRs, no ds_write); rows are 256 B with the
//     16-B pieces XOR-swizzled by row (the swizzle is on the per-lane SOURCE address: the DMA
//     destination is lane-linear) so the fragment reads are conflict-free.  Three buffers:
//     stage s + 2 is issued at the end of iteration s and stays in flight across the next
//     barrier (counted vmcnt, raw s_barrier); the appends' stores come before it in issue
//     order, so the count stays static.
//   0: register staging (global -> VGPRs -> ds_write into padded rows), two buffers (A/B).
// Per element the epilogue forms d~; per sub-tile a tournament gives the lane's two smallest,
// merged into the row's running top-2, and a target is admitted when d~ <= thr,
// thr = b2~(so far) + 2E: this lane's own b2~ after the sub-tile,
// capped by the wave-merged b2~ of the previous stage.  b2~ only decreases, so every running
// thr >= the final one and the admitted set contains the row's final window (argument
// below).  thr uses the row's b2~ over both half-waves (merged after every sub-tile).
// Admitted target indices go to the row's list in global memory: each half-wave lane appends
// to its own kHalfCap entries with a register count (no LDS atomics), and the row's count
// word holds both (low / high 16 bits); k_match_rerank recomputes them with the reference's
// exact float32 distance; a row whose list overflowed goes to k_match_overflow (exact over
// all targets).
// The window argument: the targets achieving b1~ and b2~ have exact distances <= b1~ + E and
// <= b2~ + E, so the exact second-smallest D2 <= b2~ + E; a target with exact d <= D2 has
// d~ <= d + E <= b2~ + 2E.  Targets outside the window are strictly farther than D2.
// ABL (diagnostic build only, SFMFEAT_MATCH_ABL; results wrong by design): 1 no epilogue
// (MFMAs, fragment reads, stages and barriers only), 2 no MFMAs (the epilogue on unchanged
// accumulators), 4 no admission masks / appends, 16 fragment reads of k-step 0 only (reused
// for all eight: no LDS latency inside a sub-tile), 32 full sweep + clock stamps (below)
// The sweep's work units: one per (pair, 256-row query block) that holds query rows of a pair
// whose target image has keypoints, in pair order: units[0] = their number U, units[1 + u] =
// p | block << 20.  The sweep gives each XCD a contiguous run of ceil(U / 8) of them (below), so
// every XCD gets the same number of workgroups and a pair's blocks still share one L2.  (The
// grid is sized on the host for the capacity, P x ceil(cap / 256) slots; per-pair block counts
// live on the device.)
__global__ void __launch_bounds__(1024) k_match_units(const int32_t* __restrict__ count,
                                                      const int32_t* __restrict__ pairs, int P, int max_rows,
                                                      int qbr, int32_t* __restrict__ units) {
  __shared__ uint32_t s_w[16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint32_t base = 0;
  for (int c0 = 0; c0 < P; c0 += 1024) {
    const int p = c0 + tid;
    uint32_t q = 0;
    if (p < P) {
      const int n1 = min(count[pairs[2 * p]], max_rows), n2 = count[pairs[2 * p + 1]];
      q = (n1 > 0 && n2 > 0) ? (uint32_t)((n1 + qbr - 1) / qbr) : 0u;
    }
    const uint32_t x = wave_inclusive_scan(q);
    if (lane == 63) s_w[wid] = x;
    __syncthreads();
    uint32_t before = 0, tot = 0;
    for (int w = 0; w < 16; ++w) {
      const uint32_t t = s_w[w];
      before += w < wid ? t : 0u;
      tot += t;
    }
    const uint32_t first = base + before + x - q;
    for (uint32_t j = 0; j < q; ++j) units[1 + first + j] = (int32_t)((uint32_t)p | (j << kMatchUnitPairBits));
    base += tot;
    __syncthreads();
  }
  if (tid == 0) units[0] = (int32_t)base;
}

// ABL & 32 (diagnostic build): per-wave shader-clock stamps of the first kStampSt stages of
// workgroups 0 .. kStampWg-1 (after the stage barrier, after each sub-tile region, after the
// DMA issue), kept in LDS and copied out at the end (sfm_debug_match_stamps)
constexpr int kStampWg = 16, kStampSt = 40;
__device__ uint64_t g_match_stamps[kStampWg][kWaves][kStampSt + 1][4];
// and for every workgroup of the launch (up to kStampAll): start / end realtime, __smid(),
// pair | row0 << 32 (0 for workgroups that exit at once)
constexpr int kStampAll = 1024;
__device__ uint64_t g_match_wg[kStampAll][4];

template <int STAGE, int ABL = 0>
__global__ void __launch_bounds__(64 * sweep_waves(STAGE), STAGE == 3 ? 2 : 1) k_match_mfma(
    const int32_t* __restrict__ count, int64_t capP, const _Float16* __restrict__ hi,
    const _Float16* __restrict__ lo, const float* __restrict__ norm2, const float* __restrict__ rnorm,
    const float2* __restrict__ pmax, const int32_t* __restrict__ pairs, int P, int max_rows,
    uint32_t* __restrict__ cand, int32_t* __restrict__ cand_n, float* __restrict__ cand_thr,
    int* __restrict__ ovf_count, int2* __restrict__ ovf_list, const int32_t* __restrict__ units) {
  constexpr bool DMA = STAGE >= 1;
  constexpr bool H3 = STAGE == 3;                // the half-CU form
  constexpr int NW = sweep_waves(STAGE), NTH = 64 * NW, QBR = sweep_rows(STAGE);
  constexpr int NBUF = H3 ? 2 : DMA ? kDmaBufs : kRegBufs;
  constexpr int NNB = H3 ? 3 : DMA ? kDmaNormBufs : kRegNormBufs;
  constexpr int ROWB = DMA ? 256 : kRowH * 2;  // bytes per staged target row
  constexpr int ARRB = kTT2 * ROWB;            // one array (hi or lo) of a stage
  constexpr int BUFB = 2 * ARRB;
  constexpr int OFF_N = NBUF * BUFB;
  constexpr int OFF_D = OFF_N + NNB * kTT2 * 4;
  constexpr size_t LDSB = H3 ? kSweepLds3 : kSweepLds;
  static_assert((size_t)OFF_D + (H3 ? 256 : kDBytes) <= LDSB, "LDS carve");
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDSB];
  float* const sNb = reinterpret_cast<float*>(smem + OFF_N);  // [NNB][kTT2]
  float* const sDb = reinterpret_cast<float*>(smem + OFF_D);  // [kWaves][8][64] float2
  constexpr bool STAMP = (ABL & 32) != 0;
  __shared__ uint64_t s_stamp[STAMP ? kWaves * (kStampSt + 1) * 4 : 1];
  auto stamp = [&](int st, int k) {
    if constexpr (STAMP) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      if ((threadIdx.x & 63) == 0 && st < kStampSt) s_stamp[((threadIdx.x >> 6) * (kStampSt + 1) + st) * 4 + k] = t;
    }
  };

  // XCD-aware mapping (workgroups b and b + 8 share an XCD and its L2): group g = b % 8
  // takes the pairs p = g (mod 8), so all query blocks of a pair stream its target table
  // through one L2
  const int QB = (max_rows + QBR - 1) / QBR;
  if constexpr ((ABL & 32) != 0) {
    if (threadIdx.x == 0 && blockIdx.x < kStampAll) {
      g_match_wg[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();
      g_match_wg[blockIdx.x][1] = 0;
      g_match_wg[blockIdx.x][2] = (uint64_t)__smid();
      g_match_wg[blockIdx.x][3] = 0;
    }
  }
  const int grp = blockIdx.x & 7, slot8 = blockIdx.x >> 3;
  int p, row0;
  if (units) {  // XCD grp takes units [grp * cu, grp * cu + cu) (k_match_units)
    const int U = units[0], cu = (U + 7) >> 3;
    const int u = grp * cu + slot8;
    if (slot8 >= cu || u >= U) return;
    const int code = units[1 + u];
    p = code & ((1 << kMatchUnitPairBits) - 1);
    row0 = (code >> kMatchUnitPairBits) * QBR;
  } else {  // SFMFEAT_MATCH_UNITS=0: pairs p = grp (mod 8) on XCD grp, every block slot (A/B)
    p = grp + 8 * (slot8 / QB);
    row0 = (slot8 % QB) * QBR;
    if (p >= P) return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int i1 = pairs[2 * p], i2 = pairs[2 * p + 1];
  const int n1 = count[i1], n2 = count[i2];
  if (row0 >= n1 || n2 < 1) return;

  // this lane's query row (column of the MFMA output) and its fragments, kept in registers
  const int ql = wid * kQW + (lane & 31);           // local query row 0..255
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
  // the target image's maxima of norm2 / norm: reduced here from k_match_prep's per-block
  // maxima (capP / kPrepRows of them), through the d~ staging area before its first use
  float maxn2, maxrn;
  {
    const int nblk = (int)(capP / kPrepRows);
    float m2 = 0.0f, mr = 0.0f;
    for (int t = tid; t < nblk; t += NTH) {
      const float2 v = pmax[(int64_t)i2 * nblk + t];
      m2 = fmaxf(m2, v.x);
      mr = fmaxf(mr, v.y);
    }
    for (int off = 32; off >= 1; off >>= 1) {
      m2 = fmaxf(m2, __shfl_xor(m2, off));
      mr = fmaxf(mr, __shfl_xor(mr, off));
    }
    if (lane == 0) {
      sDb[2 * wid] = m2;
      sDb[2 * wid + 1] = mr;
    }
    __syncthreads();
    maxn2 = sDb[0];
    maxrn = sDb[1];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      maxn2 = fmaxf(maxn2, sDb[2 * w]);
      maxrn = fmaxf(maxrn, sDb[2 * w + 1]);
    }
    __syncthreads();  // the d~ staging area is free again
  }
  // rigorous |d~ - d_ref| bound (matcher exactness)
  const float E = 3.0517578125e-05f * ra * maxrn + 4e-6f * (na + maxn2) + 1.25e-4f;
  const float E2 = 2.0f * E;
  const bool live = qi < n1;
  uint32_t* my_list = cand + ((int64_t)p * max_rows + qi) * kCandCap + half * kHalfCap;
  int cnt = 0;  // this lane's appended targets (its half of the row)

  const int nst = (n2 + kTT2 - 1) / kTT2;
  const int64_t to = (int64_t)i2 * capP * 128;
  const float* const nrm_t = norm2 + (int64_t)i2 * capP;

  // ---- LDS-DMA staging (STAGE 1): wave w fetches chunks w and w + 8 (4 rows each) of both
  //      arrays; lane l of a chunk: row 4 ci + l / 16, LDS piece l % 16 = global piece
  //      (l % 16) ^ (row % 16).  Wave 0 also fetches the stage's 64 target norms.
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  const uint32_t smem_lds = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) unsigned char*)smem);
  auto issue_stage = [&](int stg, int buf, int nbuf) {
    const int64_t rb = (int64_t)stg * kTT2;  // rows < capP: in bounds
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int a = j >> 1, ci = (j & 1) * 8 + wid;
      const int ciu = (j & 1) * 8 + wid_u;
      const int row = 4 * ci + (lane >> 4);
      const int c = (lane & 15) ^ (row & 15);
      const _Float16* src = (a ? lo : hi) + to + (rb + row) * 128 + c * 8;
      glds_x4(src, smem_lds + (uint32_t)(buf * BUFB + a * ARRB + ciu * 1024));
    }
    if (wid_u == 0) glds_x1(nrm_t + rb + lane, smem_lds + (uint32_t)(OFF_N + nbuf * kTT2 * 4));
  };
  // STAGE 3: a stage's 32 pieces over 4 waves: wave w fetches chunks 4 k + w (k = 0..3) of
  // both arrays, in two parts (one per sub-tile region; part 0 also carries wave 0's norms)
  auto issue_part3 = [&](int stg, int buf, int nbuf, int part) {
    const int64_t rb = (int64_t)stg * kTT2;  // rows < capP: in bounds
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = 4 * part + jj;
      const int a = j >> 2, ci = 4 * (j & 3) + wid, ciu = 4 * (j & 3) + wid_u;
      const int row = 4 * ci + (lane >> 4);
      const int c = (lane & 15) ^ (row & 15);
      const _Float16* src = (a ? lo : hi) + to + (rb + row) * 128 + c * 8;
      glds_x4(src, smem_lds + (uint32_t)(buf * BUFB + a * ARRB + ciu * 1024));
    }
    if (part == 0 && wid_u == 0) glds_x1(nrm_t + rb + lane, smem_lds + (uint32_t)(OFF_N + nbuf * kTT2 * 4));
  };
  // this wave's share of the stage issued two iterations ago has landed (the last stage's
  // share stays in flight); then every wave's
  auto stage_barrier = [&]() {
    if constexpr (H3) {  // this wave's pieces of stage st (issued one stage ago) have landed
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else if constexpr (DMA) {
      if (wid_u == 0) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      __syncthreads();
    }
  };

  // ---- register staging (STAGE 0): thread t -> row 32 q + t / 16, halves 8 (t % 16)
  const int lr = tid >> 4, lc = (tid & 15) * 8;
  h8 g[DMA ? 1 : 4];
  auto load_stage = [&](int st) {
    if constexpr (!DMA) {
      const int64_t gofs = to + (int64_t)(st * kTT2) * 128 + tid * 8;  // rows < capP: in bounds
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        g[q] = *reinterpret_cast<const h8*>(hi + gofs + 4096 * q);
        g[2 + q] = *reinterpret_cast<const h8*>(lo + gofs + 4096 * q);
      }
    }
  };
  auto store_stage = [&](int buf) {
    if constexpr (!DMA) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        *reinterpret_cast<h8*>(smem + buf * BUFB + ((32 * q + lr) * kRowH + lc) * 2) = g[q];
        *reinterpret_cast<h8*>(smem + buf * BUFB + ARRB + ((32 * q + lr) * kRowH + lc) * 2) = g[2 + q];
      }
    }
  };

  // fragment byte offsets of k-step kk inside a stage buffer (sub-tile 0, hi array)
  int frag[8];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    if constexpr (DMA) frag[kk] = (lane & 31) * 256 + (((2 * kk + half) ^ (lane & 15)) << 4);
    else frag[kk] = ((lane & 31) * kRowH + kk * 16 + 8 * half) * 2;
  }
  // 32 targets x 32 queries of sub-tile `sub` of the stage at byte offset `bofs`: hi.hi into
  // ahh, hi.lo + lo.hi into ax (one accumulation chain each)
  auto mfma_sub = [&](const int (&vb)[8], int sub, f32x16& ahh, f32x16& ax) {
    if constexpr ((ABL & 2) != 0) return;
    h8 t0h, t0l;
    if constexpr ((ABL & 16) != 0) {
      t0h = *reinterpret_cast<const h8*>(smem + vb[0] + sub * 32 * ROWB);
      t0l = *reinterpret_cast<const h8*>(smem + vb[0] + sub * 32 * ROWB + ARRB);
    }
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const h8 thi = (ABL & 16) ? t0h : *reinterpret_cast<const h8*>(smem + vb[kk] + sub * 32 * ROWB);
      const h8 tlo = (ABL & 16) ? t0l : *reinterpret_cast<const h8*>(smem + vb[kk] + sub * 32 * ROWB + ARRB);
      // k-step 0 starts both chains from an inline-constant zero accumulator
      ahh = __builtin_amdgcn_mfma_f32_32x32x16_f16(thi, qhi[kk], kk == 0 ? f32x16{} : ahh, 0, 0, 0);
      ax = __builtin_amdgcn_mfma_f32_32x32x16_f16(thi, qlo[kk], kk == 0 ? f32x16{} : ax, 0, 0, 0);
      ax = __builtin_amdgcn_mfma_f32_32x32x16_f16(tlo, qhi[kk], ax, 0, 0, 0);
    }
  };
  // this lane's 16 target norms of sub-tile `sub` (MFMA row layout: 8 (rr >> 2) + 4 half + (rr & 3))
  auto load_nb = [&](int nbuf, int sub, float (&nb)[16]) {
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const float4 v = *reinterpret_cast<const float4*>(sNb + nbuf * kTT2 + 32 * sub + 8 * g4 + 4 * half);
      nb[4 * g4 + 0] = v.x; nb[4 * g4 + 1] = v.y; nb[4 * g4 + 2] = v.z; nb[4 * g4 + 3] = v.w;
    }
  };
  float b1 = INFINITY, b2 = INFINITY;
  float thr_w = 3.0e38f;  // wave-merged running threshold of the previous stage (finite:
                          // padding targets, d~ = +inf, are never admitted)
  // d~ = na + nb - 2 a.b with a.b = (ahh + ax 2^-11) 2^-16: two fmas by exact powers of two
  // (each rounding is covered by E's 4e-6 (na + nb) term); padding targets
  // have norm2 = +inf: d~ = +inf.  Bit rr of mm for d~ <= min(b2~ + 2E, thr_w).
  // The sub-tile's two smallest d~ by a tournament (pairs (min, max), then merges
  // m = min(ma, mb), s = min3(max(ma, mb), sa, sb)): the same multiset top-2 as an element-by-
  // element update, at a dependency depth of 9 instead of 32; merged into the running
  // (b1, b2) the same way.  The admission mask is built only when some lane's smallest d~
  // passes the threshold (after the first stages, most sub-tiles admit nothing).
  auto epi = [&](const f32x16& ahh, const f32x16& ax, const float (&nb)[16], float (&d)[16], uint32_t& mm) {
    if constexpr ((ABL & 1) != 0) {
      asm volatile("" ::"v"(ahh), "v"(ax));  // keep the MFMAs
      return;
    }
#pragma unroll
    for (int rr = 0; rr < 16; ++rr)
      d[rr] = __builtin_fmaf(ax[rr], -1.4901161193847656e-08f /* -2^-26 */,
                             __builtin_fmaf(ahh[rr], -3.0517578125e-05f /* -2^-15 */, na + nb[rr]));
    float m[8], sc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      m[i] = fminf(d[2 * i], d[2 * i + 1]);
      sc[i] = fmaxf(d[2 * i], d[2 * i + 1]);
    }
#pragma unroll
    for (int w = 4; w >= 1; w >>= 1)
#pragma unroll
      for (int i = 0; i < w; ++i) {
        const float mm0 = fminf(m[i], m[i + w]);
        sc[i] = fminf(fmaxf(m[i], m[i + w]), fminf(sc[i], sc[i + w]));
        m[i] = mm0;
      }
    const float tm = m[0];
    b2 = fminf(fmaxf(b1, tm), fminf(b2, sc[0]));
    b1 = fminf(b1, tm);
    // the row's b2~ so far over both halves (every lane's b2 and b1 >= its half's final ones)
    const float ob1 = other_half(b1), ob2 = other_half(b2);
    const float t = fminf(fminf(fmaxf(b1, ob1), fminf(b2, ob2)) + E2, thr_w);
    if ((ABL & 4) == 0 && __any(tm <= t)) {
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) mm |= (d[rr] <= t) ? (1u << rr) : 0u;
    }
  };
  // MFMA / VALU interleave of one software-pipelined region: the three MFMAs of a k-step
  // with the epilogue's vector instructions in their gaps
  auto interleave = [&]() {
    // fragment reads run two k-steps ahead of the MFMAs that consume them, so no MFMA
    // waits on an LDS read issued just before it
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);  // DS read: k-steps 0 and 1
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // VALU
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if (kk < 6) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read: k-step kk + 2
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
    }
  };
  // the region's epilogue results are needed here: keeps the compiler from sinking the
  // epilogue past the stage barrier, out of the region it interleaves with
  auto pin = [](float x1, float x2, uint32_t mm) { asm volatile("" ::"v"(x1), "v"(x2), "v"(mm)); };
  // admitted elements of one sub-tile (bit rr of mm, targets jb + 8 (rr >> 2) + 4 half +
  // (rr & 3)) -> the row's global list as (index | d~ rounded down to bf16 << 16).  When
  // any lane of the wave admits, the lane's 16 d~ go to the wave's LDS area (no dynamic
  // register indexing into d) and each admitted one is read back by index.  Layout
  // [pair rr / 2][lane] of float2: the 8-B stores cover all 32 banks per 16-lane group and a
  // read of element rr hits bank 2 lane + (rr & 1) (mod 32), so lanes reading different rr
  // conflict at most 2-way (a lane-major [lane][16] row put 4 lanes on the same banks)
  float2* const my_d2 = reinterpret_cast<float2*>(sDb) + wid * 8 * 64 + lane;
  auto append = [&](uint32_t mm, const float (&d)[16], int jb) {
    if constexpr (H3) {  // no LDS staging: d[rr] by a 4-level v_bfi_b32 select tree
      if (live) {
        for (; mm; mm &= mm - 1, ++cnt) {
          const int rr = __builtin_ctz(mm);
          uint32_t a8[8], a4[4], a2[2];
          const uint32_t m0 = lane_bit_mask(rr, 0), m1 = lane_bit_mask(rr, 1), m2 = lane_bit_mask(rr, 2),
                         m3 = lane_bit_mask(rr, 3);
#pragma unroll
          for (int i = 0; i < 8; ++i) a8[i] = bfi(m0, __float_as_uint(d[2 * i + 1]), __float_as_uint(d[2 * i]));
#pragma unroll
          for (int i = 0; i < 4; ++i) a4[i] = bfi(m1, a8[2 * i + 1], a8[2 * i]);
#pragma unroll
          for (int i = 0; i < 2; ++i) a2[i] = bfi(m2, a4[2 * i + 1], a4[2 * i]);
          const float dr = __uint_as_float(bfi(m3, a2[1], a2[0]));
          if (cnt < kHalfCap)
            my_list[cnt] = (uint32_t)(jb + 4 * half + (rr & 3) + 8 * (rr >> 2)) | ((uint32_t)bf16_down(dr) << 16);
        }
      }
    } else if (__any(mm != 0u)) {  // wave-uniform: skip when no lane admits
#pragma unroll
      for (int q = 0; q < 8; ++q) my_d2[64 * q] = make_float2(d[2 * q], d[2 * q + 1]);
      if (live && mm) {
        for (; mm; mm &= mm - 1, ++cnt) {
          const int rr = __builtin_ctz(mm);
          const float dr = reinterpret_cast<const float*>(my_d2 + 64 * (rr >> 1))[rr & 1];
          if (cnt < kHalfCap)
            my_list[cnt] = (uint32_t)(jb + 4 * half + (rr & 3) + 8 * (rr >> 2)) | ((uint32_t)bf16_down(dr) << 16);
        }
      }
    }
  };

  // prologue: stages 0 and 1 (DMA) / stage 0 (registers); "stage -1"'s norms are +inf, so
  // the carried sub-tile's first epilogue is a no-op
  if constexpr (DMA) {
    // the query fragments are in registers before the first DMA is issued: hipcc's wait for
    // them would otherwise be a vmcnt(0) that drains the prologue's prefetch too
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) asm volatile("" ::"v"(qhi[kk]), "v"(qlo[kk]));
    asm volatile("" ::"v"(E2), "v"(na));
    if constexpr (H3) {
      issue_part3(0, 0, 0, 0);
      issue_part3(0, 0, 0, 1);
    } else {
      issue_stage(0, 0, 0);
      issue_stage(min(1, nst - 1), 1, 1);
    }
    if (wid_u == 0) sNb[(NNB - 1) * kTT2 + lane] = INFINITY;
  } else {
    load_stage(0);
    const float nrm_t0 = (tid < kTT2) ? nrm_t[tid] : 0.0f;
    store_stage(0);
    if (tid < kTT2) {
      sNb[tid] = nrm_t0;
      sNb[(NNB - 1) * kTT2 + tid] = INFINITY;
    }
  }
  // accumulators: set A = sub-tile 0 of a stage, set B = sub-tile 1 (carried into the next
  // iteration's first region); alternating sets instead of copies
  f32x16 hA = {}, xA = {}, hB = {}, xB = {};
  int nbc = 0;                   // norm buffer of stage st (st % NNB)
  int buf = 0;                   // stage buffer of stage st (st % NBUF)
  if constexpr (STAMP) {
    if (lane == 0) {
      s_stamp[(wid * (kStampSt + 1) + kStampSt) * 4 + 0] = __builtin_amdgcn_s_memtime();
      s_stamp[(wid * (kStampSt + 1) + kStampSt) * 4 + 1] = __builtin_amdgcn_s_memrealtime();
      s_stamp[(wid * (kStampSt + 1) + kStampSt) * 4 + 3] = (uint64_t)p | ((uint64_t)nst << 32);
    }
  }
  if constexpr (H3) {
    // two buffers: stage st + 1 goes into stage st - 1's buffer (every wave is past it: the
    // barrier), half of its pieces in each sub-tile region
    for (int st = 0; st < nst; ++st) {
      stage_barrier();
      stamp(st, 0);
      const int nbp = nbc == 0 ? NNB - 1 : nbc - 1, nbn = nbc == NNB - 1 ? 0 : nbc + 1;
      const bool more = st + 1 < nst;
      int vb[8];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) vb[kk] = frag[kk] + buf * BUFB;
      {
        float nb[16], d[16];
        uint32_t mm = 0;
        if (more) issue_part3(st + 1, buf ^ 1, nbn, 0);
        load_nb(nbp, 1, nb);
        mfma_sub(vb, 0, hA, xA);
        epi(hB, xB, nb, d, mm);
        interleave();
        pin(b1, b2, mm);
        append(mm, d, (st - 1) * kTT2 + 32);
      }
      stamp(st, 1);
      {
        float nb[16], d[16];
        uint32_t mm = 0;
        if (more) issue_part3(st + 1, buf ^ 1, nbn, 1);
        load_nb(nbc, 0, nb);
        mfma_sub(vb, 1, hB, xB);
        epi(hA, xA, nb, d, mm);
        interleave();
        pin(b1, b2, mm);
        append(mm, d, st * kTT2);
      }
      stamp(st, 2);
      {
        const float ob1 = other_half(b1), ob2 = other_half(b2);
        thr_w = fminf(fminf(fmaxf(b1, ob1), fminf(b2, ob2)) + E2, thr_w);
      }
      stamp(st, 3);
      nbc = nbn;
      buf ^= 1;
    }
  } else {
  for (int st = 0; st < nst; ++st) {
    // stage st is visible, and every wave is done with stage st - 1 (DMA: st - 1's buffer
    // takes stage st + 2 at the end of this iteration; registers: stage st + 1): one barrier
    stage_barrier();
    stamp(st, 0);
    const int nbp = nbc == 0 ? NNB - 1 : nbc - 1, nbn = nbc == NNB - 1 ? 0 : nbc + 1;
    float nrm_next = 0.0f;
    if constexpr (!DMA) {  // next stage's rows (the last stage re-reads itself: branch-free body)
      const int sn = min(st + 1, nst - 1);
      load_stage(sn);
      nrm_next = nrm_t[sn * kTT2 + (tid & (kTT2 - 1))];
    }
    int vb[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) vb[kk] = frag[kk] + buf * BUFB;
    {
      float nb[16], d[16];
      uint32_t mm = 0;
      load_nb(nbp, 1, nb);
      mfma_sub(vb, 0, hA, xA);
      epi(hB, xB, nb, d, mm);
      interleave();
      pin(b1, b2, mm);
      append(mm, d, (st - 1) * kTT2 + 32);
    }
    stamp(st, 1);
    {
      float nb[16], d[16];
      uint32_t mm = 0;
      load_nb(nbc, 0, nb);
      mfma_sub(vb, 1, hB, xB);
      epi(hA, xA, nb, d, mm);
      interleave();
      pin(b1, b2, mm);
      append(mm, d, st * kTT2);
    }
    stamp(st, 2);
    {  // the wave-merged running threshold for the next stage (both halves of a row)
      const float ob1 = other_half(b1), ob2 = other_half(b2);
      thr_w = fminf(fminf(fmaxf(b1, ob1), fminf(b2, ob2)) + E2, thr_w);
    }
    if constexpr (DMA) {
      // stage st + 2 into stage st - 1's buffer, after this iteration's appends in issue
      // order (the counted wait above leaves exactly these in flight)
      const int b2i = buf == 0 ? 2 : buf - 1;
      const int n2i = nbn == NNB - 1 ? 0 : nbn + 1;
      issue_stage(min(st + 2, nst - 1), b2i, n2i);
    } else {
      store_stage(buf ^ 1);
      if (tid < kTT2) sNb[nbn * kTT2 + tid] = nrm_next;
    }
    stamp(st, 3);
    nbc = nbn;
    buf = buf == NBUF - 1 ? 0 : buf + 1;
  }
  }  // !H3
  {
    uint32_t mm = 0;  // the last stage's sub-tile 1 (its norms: stage nst - 1)
    float nb[16], d[16];
    load_nb(nbc == 0 ? NNB - 1 : nbc - 1, 1, nb);
    epi(hB, xB, nb, d, mm);
    append(mm, d, (nst - 1) * kTT2 + 32);
  }
  if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA in flight at exit
  if constexpr (STAMP) {
    if (tid == 0 && blockIdx.x < kStampAll) {
      g_match_wg[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
      g_match_wg[blockIdx.x][3] = (uint64_t)p | ((uint64_t)row0 << 32);
    }
    if (lane == 0) s_stamp[(wid * (kStampSt + 1) + kStampSt) * 4 + 2] = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x < kStampWg) {
      __builtin_amdgcn_s_waitcnt(0xc07f);  // the stamps in LDS (lgkmcnt 0)
      const uint64_t* src = s_stamp + wid * (kStampSt + 1) * 4;
      uint64_t* dst = &g_match_stamps[blockIdx.x][wid][0][0];
      for (int i = lane; i < (kStampSt + 1) * 4; i += 64) dst[i] = src[i];
    }
  }
  // the row's final window threshold (both halves merged): the re-rank drops the admitted
  // targets above it (their stored d~ is rounded down, so no window member is dropped)
  const float ob1 = other_half(b1), ob2 = other_half(b2);
  const float thr_final = fminf(fminf(fmaxf(b1, ob1), fminf(b2, ob2)) + E2, thr_w);
  const int ocnt = other_half(cnt);
  if (live && half == 0) {
    cand_thr[(int64_t)p * max_rows + qi] = thr_final;
    cand_n[(int64_t)p * max_rows + qi] = cnt | (ocnt << 16);  // n2 < 2^16 (kMaxMatchRows)
    if (cnt > kHalfCap || ocnt > kHalfCap) {  // a list overflowed: exact over every target instead
      const int k = atomicAdd(ovf_count, 1);
      ovf_list[k] = make_int2(p, qi);
    }
  }
}

// Exact re-rank of the row's final window: the admitted targets whose stored d~ (rounded
// down) is within the row's final threshold, compacted by a ballot into LDS, then the
// reference's float32 distance (numpy's pairwise order) of each: one wavefront per query
// row, eight lanes per candidate — lane l of a group accumulates numpy's accumulator
// r[l] = sum_i (a[8 i + l] - b[8 i + l])^2 in i order (32-B coalesced reads per group),
// and the groups' partial sums combine as ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7))
// by xor shuffles (IEEE addition is commutative, so the shuffle pairing is bitwise the
// reference's).  Per group a running (distance, index) top-2, merged over the 8 groups ->
// nndr and the ratio test.
__global__ void __launch_bounds__(256) k_match_rerank(const float* __restrict__ desc,
                                                      const int32_t* __restrict__ count, int64_t cap,
                                                      const int32_t* __restrict__ pairs, int P, float ratio,
                                                      int max_rows, const uint32_t* __restrict__ cand,
                                                      const int32_t* __restrict__ cand_n,
                                                      const float* __restrict__ cand_thr,
                                                      RowBest* __restrict__ rows_out) {
  __shared__ uint16_t sJ[4][kCandCap];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int grp = lane >> 3, l8 = lane & 7;
  const int64_t w = (int64_t)blockIdx.x * 4 + wv;  // (pair, row)
  const int p = (int)(w / max_rows), row = (int)(w % max_rows);
  if (p >= P) return;
  const int i1 = pairs[2 * p], i2 = pairs[2 * p + 1];
  const int n1 = count[i1], n2 = count[i2];
  if (row >= n1 || n2 < 1) return;
  const int cw = cand_n[w];
  const int c0 = cw & 0xffff, c1 = cw >> 16;  // the two half-lists' lengths
  if (c0 > kHalfCap || c1 > kHalfCap) return;  // k_match_overflow's row
  const float thr = cand_thr[w];
  const uint32_t* list = cand + w * kCandCap;
  const float* A = desc + ((int64_t)i1 * cap + row) * 128;
  const float* Bd = desc + (int64_t)i2 * cap * 128;
  float a[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = A[8 * i + l8];
  int nk = 0;  // window members, compacted into sJ[wv] in list order
  static_assert(kHalfCap % 64 == 0, "whole wavefront passes per half-list");
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int ch = h ? c1 : c0;
    for (int b0 = 0; b0 < ch; b0 += 64) {
      const int idx = b0 + lane;
      const bool in = idx < ch;
      const uint32_t e = in ? list[h * kHalfCap + idx] : 0u;
      const bool keep = in && __uint_as_float(e & 0xffff0000u) <= thr;
      const uint64_t bal = __ballot(keep);
      if (keep) sJ[wv][nk + __popcll(bal & ((1ull << lane) - 1ull))] = (uint16_t)(e & 0xffffu);
      nk += __popcll(bal);
    }
  }
  __builtin_amdgcn_wave_barrier();
  float e1 = INFINITY, e2 = INFINITY;
  int j1 = 0x7fffffff;
  for (int s0 = 0; s0 < nk; s0 += 8) {
    const int s = s0 + grp;
    const bool ok = s < nk;
    const int j = ok ? (int)sJ[wv][s] : 0;
    const float* b = Bd + (int64_t)j * 128;
    float r = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float dd = a[i] - b[8 * i + l8];
      const float sq = dd * dd;
      r = (i == 0) ? sq : r + sq;
    }
    r = r + __shfl_xor(r, 1);  // t01, t23, t45, t67
    r = r + __shfl_xor(r, 2);  // u0 = t01 + t23, u1 = t45 + t67
    r = r + __shfl_xor(r, 4);  // u0 + u1
    if (ok) {
      if (r < e1 || (r == e1 && j < j1)) { e2 = e1; e1 = r; j1 = j; }
      else if (r < e2) e2 = r;
    }
  }
#pragma unroll
  for (int off = 8; off <= 32; off <<= 1) {
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
    rows_out[w] = rb;
  }
}

// As k_match_rerank with two (pair, row) items per wavefront, one per half-wave: half h of
// wave w takes item 2 w + h, four candidates per step (eight lanes each, the same numpy
// pairwise order), the top-2 merged over the half's four groups.  Half the wavefronts for the
// same latency chain per item (count, list, ballot, candidate rows).
__global__ void __launch_bounds__(256) k_match_rerank2(const float* __restrict__ desc,
                                                       const int32_t* __restrict__ count, int64_t cap,
                                                       const int32_t* __restrict__ pairs, int P, float ratio,
                                                       int max_rows, const uint32_t* __restrict__ cand,
                                                       const int32_t* __restrict__ cand_n,
                                                       const float* __restrict__ cand_thr,
                                                       RowBest* __restrict__ rows_out) {
  __shared__ uint16_t sJ[4][2][kCandCap];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, hf = lane >> 5, hl = lane & 31;
  const int grp = hl >> 3, l8 = lane & 7;
  const int64_t w = ((int64_t)blockIdx.x * 4 + wv) * 2 + hf;  // (pair, row) of this half-wave
  const int p = (int)(w / max_rows), row = (int)(w % max_rows);
  bool ok = p < P;
  int i1 = 0, i2 = 0, n1 = 0, n2 = 0;
  if (ok) {
    i1 = pairs[2 * p];
    i2 = pairs[2 * p + 1];
    n1 = count[i1];
    n2 = count[i2];
    ok = row < n1 && n2 >= 1;
  }
  int c0 = 0, c1 = 0;
  float thr = 0.0f;
  if (ok) {
    const int cw = cand_n[w];
    c0 = cw & 0xffff;
    c1 = cw >> 16;
    ok = c0 <= kHalfCap && c1 <= kHalfCap;  // else k_match_overflow's row
    thr = cand_thr[w];
  }
  const uint32_t* list = cand + w * kCandCap;
  const float* A = desc + ((int64_t)i1 * cap + row) * 128;
  const float* Bd = desc + (int64_t)i2 * cap * 128;
  float a[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = ok ? A[8 * i + l8] : 0.0f;
  int nk = 0;  // window members of this half's item, compacted into sJ[wv][hf] in list order
  const uint64_t hmask = hf ? 0xFFFFFFFF00000000ull : 0x00000000FFFFFFFFull;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int ch = ok ? (h ? c1 : c0) : 0;
    const int chmax = max(ch, __shfl_xor(ch, 32));  // both halves walk the longer list
    for (int b0 = 0; b0 < chmax; b0 += 32) {
      const int idx = b0 + hl;
      const bool in = idx < ch;
      const uint32_t e = in ? list[h * kHalfCap + idx] : 0u;
      const bool keep = in && __uint_as_float(e & 0xffff0000u) <= thr;
      const uint64_t bal = __ballot(keep) & hmask;
      const uint64_t below = bal & ((1ull << lane) - 1ull);
      if (keep) sJ[wv][hf][nk + __popcll(below)] = (uint16_t)(e & 0xffffu);
      nk += __popcll(bal);
    }
  }
  __builtin_amdgcn_wave_barrier();
  float e1 = INFINITY, e2 = INFINITY;
  int j1 = 0x7fffffff;
  const int nkmax = max(nk, __shfl_xor(nk, 32));
  for (int s0 = 0; s0 < nkmax; s0 += 4) {
    const int sidx = s0 + grp;
    const bool okc = sidx < nk;
    // j = 0 for the group's idle lanes: a valid row (of image 0 for an idle item), whose
    // distance is computed and never used, so the loads need no lane masks
    const int j = okc ? (int)sJ[wv][hf][sidx] : 0;
    const float* b = Bd + (int64_t)j * 128;
    float r = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float dd = a[i] - b[8 * i + l8];
      const float sq = dd * dd;
      r = (i == 0) ? sq : r + sq;
    }
    r = r + __shfl_xor(r, 1);  // t01, t23, t45, t67
    r = r + __shfl_xor(r, 2);  // u0 = t01 + t23, u1 = t45 + t67
    r = r + __shfl_xor(r, 4);  // u0 + u1
    if (okc) {
      if (r < e1 || (r == e1 && j < j1)) { e2 = e1; e1 = r; j1 = j; }
      else if (r < e2) e2 = r;
    }
  }
#pragma unroll
  for (int off = 8; off <= 16; off <<= 1) {
    const float o1 = __shfl_xor(e1, off), o2 = __shfl_xor(e2, off);
    const int oj = __shfl_xor(j1, off);
    top2_merge(e1, j1, e2, o1, oj, o2);
  }
  if (hl == 0 && ok) {
    RowBest rb;
    rb.col = -1;
    rb.nndr = 0.0f;
    const float d1 = sqrtf(e1), d2 = sqrtf(e2);
    if (d2 > 0.0f) {
      const float nndr = d1 / d2;
      if (nndr <= ratio) { rb.col = j1; rb.nndr = nndr; }
    }
    rows_out[w] = rb;
  }
}

// Exact re-rank, eight (pair, row) items per wavefront (A/B variant, kRerank8MaxPairs):
// for launches of few pairs k_match_rerank's wave per row leaves most lanes idle and pays
// three dependent memory latencies per row with few waves to hide them:
//   1. the eight rows' counts and final thresholds (lanes 0-7), their list entries (the
//      eight 512-B lists are contiguous: 16 coalesced loads per lane) and their query rows
//      (into LDS) are fetched together;
//   2. the entries whose stored d~ (rounded down) lies within the row's final threshold
//      are compacted by ballots into the wave's LDS list, in row order;
//   3. eight lanes per candidate compute the reference's float32 distance (numpy's
//      pairwise order: lane l accumulates r[l] = sum_i (a[8 i + l] - b[8 i + l])^2 in i
//      order, and the group combines ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) by
//      xor shuffles — IEEE addition is commutative, so the pairing is bitwise numpy's);
//   4. lane r scans row r's contiguous range of distances for the (distance, index)
//      top-2 -> nndr and the ratio test.
constexpr int kRrRows = 8;             // (pair, row) items per wavefront
// launches of up to this many pairs take k_match_rerank8 (default 0: off).  Alone, a
// 31-pair match call measured 0.291 ms with it against 0.382 (tools/bench_match.py), but
// inside bench.py's pipeline the match stage measured 0.253 vs 0.222 ms and the headline
// 29.7k vs 30.9k img/s, so the wave-per-row kernel is the default; SFMFEAT_RERANK8_MAX=N
// switches it on for A/B timing
constexpr int kRerank8MaxPairs = 0;
__global__ void __launch_bounds__(256) k_match_rerank8(const float* __restrict__ desc,
                                                      const int32_t* __restrict__ count, int64_t cap,
                                                      const int32_t* __restrict__ pairs, int P, float ratio,
                                                      int max_rows, const uint32_t* __restrict__ cand,
                                                      const int32_t* __restrict__ cand_n,
                                                      const float* __restrict__ cand_thr,
                                                      RowBest* __restrict__ rows_out) {
  __shared__ __attribute__((aligned(16))) float sA[4][kRrRows][128];  // query rows
  __shared__ uint16_t sL[4][kRrRows * kCandCap];  // window members (target index), row order
  __shared__ float sDist[4][kRrRows * kCandCap];
  __shared__ int sBeg[4][kRrRows + 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int grp = lane >> 3, l8 = lane & 7;
  const int64_t total = (int64_t)P * max_rows;
  const int64_t w0 = ((int64_t)blockIdx.x * 4 + wv) * kRrRows;  // first (pair, row) item
  if (w0 >= total) return;
  // 1. per-row state on lanes 0..7, then broadcast by shuffles
  int c_l = 0, ok_l = 0, i1_l = 0, i2_l = 0, row_l = 0, p_l = 0;
  float thr_l = 0.0f;
  if (lane < kRrRows) {
    const int64_t w = w0 + lane;
    if (w < total) {
      p_l = (int)(w / max_rows);
      row_l = (int)(w % max_rows);
      i1_l = pairs[2 * p_l];
      i2_l = pairs[2 * p_l + 1];
      const int n1 = count[i1_l], n2 = count[i2_l];
      if (row_l < n1 && n2 >= 1) {
        c_l = cand_n[w];  // half-list lengths, low / high 16 bits
        thr_l = cand_thr[w];
        ok_l = ((c_l & 0xffff) <= kHalfCap && (c_l >> 16) <= kHalfCap) ? 1 : 0;  // else k_match_overflow's row
      }
    }
    if (!ok_l) c_l = 0;
  }
  // query rows of the eight items -> LDS (row r: 128 floats; 16 per lane)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = lane * 4 + 256 * q;  // float index in [0, 1024)
    const int r = e >> 7, k = e & 127;
    const int ir = __shfl(i1_l, r), rr = __shfl(row_l, r), okr = __shfl(ok_l, r);
    float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (okr) v = *reinterpret_cast<const float4*>(desc + ((int64_t)ir * cap + rr) * 128 + k);
    *reinterpret_cast<float4*>(&sA[wv][r][k]) = v;
  }
  // 2. list entries of the eight rows (contiguous), filtered and compacted in row order
  const uint32_t* lists = cand + w0 * kCandCap;
  int nk = 0;
#pragma unroll 4
  for (int sidx = 0; sidx < kRrRows * kCandCap / 64; ++sidx) {
    const int e = sidx * 64 + lane;
    const int r = e / kCandCap, pos = e % kCandCap;  // r is wave-uniform per sidx
    const int cr = __shfl(c_l, r);
    const float tr = __shfl(thr_l, r);
    const int crh = pos < kHalfCap ? (cr & 0xffff) : (cr >> 16);
    const bool valid = (pos & (kHalfCap - 1)) < crh && w0 + r < total;
    const uint32_t ent = valid ? lists[e] : 0u;
    const bool keep = valid && __uint_as_float(ent & 0xffff0000u) <= tr;
    const uint64_t bal = __ballot(keep);
    if (pos == 0 && lane == (sidx * 64) % 64 && (e % kCandCap) == 0) sBeg[wv][r] = nk;  // row start
    if (keep) sL[wv][nk + __popcll(bal & ((1ull << lane) - 1ull))] = (uint16_t)(ent & 0xffffu);
    nk += __popcll(bal);
  }
  if (lane == 0) sBeg[wv][kRrRows] = nk;
  __builtin_amdgcn_wave_barrier();
  // 3. exact distances, eight candidates per iteration
  for (int s0 = 0; s0 < nk; s0 += 8) {
    const int s = s0 + grp;
    const bool ok = s < nk;
    const int j = ok ? (int)sL[wv][s] : 0;
    int r = 0;  // the entry's row: ranges [sBeg[r], sBeg[r + 1]) are in row order
#pragma unroll
    for (int k = 1; k < kRrRows; ++k) r += (s >= sBeg[wv][k]) ? 1 : 0;
    const int i2 = __shfl(i2_l, r);
    const float* b = desc + ((int64_t)i2 * cap + j) * 128;
    const float* a = &sA[wv][r][0];
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float dd = a[8 * i + l8] - (ok ? b[8 * i + l8] : a[8 * i + l8]);
      const float sq = dd * dd;
      acc = (i == 0) ? sq : acc + sq;
    }
    acc = acc + __shfl_xor(acc, 1);  // t01, t23, t45, t67
    acc = acc + __shfl_xor(acc, 2);  // u0 = t01 + t23, u1 = t45 + t67
    acc = acc + __shfl_xor(acc, 4);  // u0 + u1
    if (ok && l8 == 0) sDist[wv][s] = acc;
  }
  __builtin_amdgcn_wave_barrier();
  // 4. lane r: row r's top-2 over its contiguous range
  if (lane < kRrRows && ok_l) {
    float e1 = INFINITY, e2 = INFINITY;
    int j1 = 0x7fffffff;
    const int beg = sBeg[wv][lane], end = lane + 1 < kRrRows ? sBeg[wv][lane + 1] : nk;
    for (int s = beg; s < end; ++s) {
      const float dd = sDist[wv][s];
      const int j = (int)sL[wv][s];
      if (dd < e1 || (dd == e1 && j < j1)) { e2 = e1; e1 = dd; j1 = j; }
      else if (dd < e2) e2 = dd;
    }
    RowBest rb;
    rb.col = -1;
    rb.nndr = 0.0f;
    const float d1 = sqrtf(e1), d2 = sqrtf(e2);
    if (d2 > 0.0f) {
      const float nndr = d1 / d2;
      if (nndr <= ratio) { rb.col = j1; rb.nndr = nndr; }
    }
    rows_out[w0 + lane] = rb;
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

size_t match_units_words(int P, int max_rows) {  // for the smallest block (the half-CU form's)
  return 1 + (size_t)P * ((max_rows + sweep_rows(3) - 1) / sweep_rows(3));
}

size_t match_pmax_bytes(int64_t capP) { return (size_t)(capP / kPrepRows) * sizeof(float2); }

void launch_match_prep(const float* desc, const int32_t* count, int nimg, int64_t cap, int64_t capP,
                       _Float16* hi, _Float16* lo, float* norm2, float* rnorm, void* pmax, hipStream_t st) {
  hipLaunchKernelGGL(k_match_prep, dim3((unsigned)(capP / kPrepRows), nimg), dim3(256), 0, st, desc, count, cap,
                     capP, hi, lo, norm2, rnorm, static_cast<float2*>(pmax));
}

void launch_match_mfma(const float* desc, const int32_t* count, int64_t cap, int64_t capP,
                       const _Float16* hi, const _Float16* lo, const float* norm2, const float* rnorm,
                       const void* pmax, const int32_t* pairs, int P, float ratio,
                       RowBest* rows, int max_rows, uint32_t* cand, int32_t* cand_n, float* cand_thr,
                       int* ovf_count, int2* ovf_list, int32_t* units, hipStream_t st) {
  // the half-CU form (STAGE 3) by default since round 5: 38.55k vs 37.91k img/s (six
  // interleaved runs each, one box; 38.51k vs 37.90k over four on another);
  // SFMFEAT_MATCH_STAGE=1 / reg: the one-workgroup-per-CU LDS-DMA / register-staged sweep (A/B)
  static const int stage = [] {
    const char* e = getenv("SFMFEAT_MATCH_STAGE");
    return (e && e[0] == 'r') ? 0 : (e && e[0] == '1') ? 1 : 3;
  }();
  static const int rr8_max = [] {  // SFMFEAT_RERANK8_MAX: pair-count switch (A/B timing)
    const char* e = SFM_DIAG_ENV("SFMFEAT_RERANK8_MAX");
    return e ? atoi(e) : kRerank8MaxPairs;
  }();
  static const bool use_units = [] {  // SFMFEAT_MATCH_UNITS=0: the per-pair XCD mapping (A/B)
    const char* e = SFM_DIAG_ENV("SFMFEAT_MATCH_UNITS");
    return !(e && e[0] == '0');
  }();
  const int qbr = stage == 3 ? sweep_rows(3) : kQB;
  const int qb = (max_rows + qbr - 1) / qbr;
  const dim3 grid((unsigned)(8 * ((P + 7) / 8) * qb));
  if (!use_units) units = nullptr;
  if (units) hipLaunchKernelGGL(k_match_units, dim3(1), dim3(1024), 0, st, count, pairs, P, max_rows, qbr, units);
  // ovf_count is zero here: set once at allocation, re-zeroed by k_match_compact
#define SFM_SWEEP(A, ABL)                                                                             \
  hipLaunchKernelGGL((k_match_mfma<A, ABL>), grid, dim3(64 * sweep_waves(A)), 0, st, count, capP, hi, lo,  \
                     norm2, rnorm,                                                                         \
                     static_cast<const float2*>(pmax), pairs, P, max_rows, cand, cand_n, cand_thr, ovf_count, \
                     ovf_list, units)
  static const int abl = [] {  // timing ablations: diagnostic build only (SFM_ABLATION_ENV)
    const char* e = SFM_ABLATION_ENV("SFMFEAT_MATCH_ABL");
    return e ? atoi(e) : 0;
  }();
#ifdef SFM_ABLATIONS
  switch (abl) {
    case 1: SFM_SWEEP(1, 1); break;
    case 2: SFM_SWEEP(1, 2); break;
    case 3: SFM_SWEEP(1, 3); break;
    case 4: SFM_SWEEP(1, 4); break;
    case 6: SFM_SWEEP(1, 6); break;
    case 16: SFM_SWEEP(1, 16); break;
    case 17: SFM_SWEEP(1, 17); break;
    case 32: SFM_SWEEP(1, 32); break;
    default: if (stage == 0) SFM_SWEEP(0, 0); else if (stage == 3) SFM_SWEEP(3, 0); else SFM_SWEEP(1, 0);
  }
#else
  (void)abl;
  if (stage == 0)
    SFM_SWEEP(0, 0);
  else if (stage == 3)
    SFM_SWEEP(3, 0);
  else
    SFM_SWEEP(1, 0);
#endif
#undef SFM_SWEEP
  // two (pair, row) items per wavefront above the eight-item kernel's range (round 4: match
  // stage 0.229 -> 0.223 ms/step at configs[1]); SFMFEAT_RERANK2=0: one item per wavefront (A/B)
  static const int rr2 = [] {
    const char* e = getenv("SFMFEAT_RERANK2");
    return e ? atoi(e) : 1;
  }();
  if (rr2 && P > rr8_max)
    hipLaunchKernelGGL(k_match_rerank2, dim3((unsigned)(((int64_t)P * max_rows + 7) / 8)), dim3(256), 0, st, desc,
                       count, cap, pairs, P, ratio, max_rows, cand, cand_n, cand_thr, rows);
  else if (P <= rr8_max)
    hipLaunchKernelGGL(k_match_rerank8, dim3((unsigned)(((int64_t)P * max_rows + 4 * kRrRows - 1) / (4 * kRrRows))),
                       dim3(256), 0, st, desc, count, cap, pairs, P, ratio, max_rows, cand, cand_n, cand_thr, rows);
  else
    hipLaunchKernelGGL(k_match_rerank, dim3((unsigned)(((int64_t)P * max_rows + 3) / 4)), dim3(256), 0, st, desc,
                       count, cap, pairs, P, ratio, max_rows, cand, cand_n, cand_thr, rows);
  // the overflow list's length stays on the device: a fixed grid strides over it
  hipLaunchKernelGGL(k_match_overflow, dim3(256), dim3(256), 0, st, desc, count, cap, pairs, ratio, rows, max_rows,
                     ovf_count, ovf_list);
}

// the sweep's clock stamps of its last SFMFEAT_MATCH_ABL=32 launch (diagnostic build): u64
// [kStampWg][kWaves][kStampSt + 1][4], then [kStampAll][4]; returns the slots copied, -1 in
// the shipped build
int64_t match_stamps_copy(uint64_t* out, int64_t cap) {
#ifdef SFM_ABLATIONS
  const int64_t n1 = (int64_t)sizeof(g_match_stamps) / 8, n = n1 + (int64_t)sizeof(g_match_wg) / 8;
  if (cap < n) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_match_stamps), sizeof(g_match_stamps)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out + n1, HIP_SYMBOL(g_match_wg), sizeof(g_match_wg)) != hipSuccess) return -1;
  return n;
#else
  (void)out;
  (void)cap;
  return -1;
#endif
}

}  // namespace sfm
