// harris.hip — fused Harris response (NaiveSIFT._find_harris_interest_points,
// NaiveSIFT.py:59-74): Sobel gradients -> Ix^2, Iy^2, IxIy -> three 2-D Gaussian
// window sums -> R = det - alpha * trace^2, plus the first radix digit histogram of R
// for the exact median (NaiveSIFT.py:91).
//
// One workgroup walks 64 x 64 output tiles of one plane (see k_harris).  The
// 2-D window is the reference's full KS x KS correlation (not separable: a separable sum
// would round differently and move keypoints), accumulated per pixel as an
// fma chain in row-major tap order (OpenCV FilterVec_32f's v_muladd chain; DESIGN.md
// §Numerics).
// VALU-bound by design.
#include <stdlib.h>

#include <algorithm>
#include <utility>

#include "kernels.h"

namespace sfm {

// static_for<N>(f): f(std::integral_constant<int, 0>{}) ... f(<N-1>{}), fully expanded
// (the window loop body is too large for the unroll pragma, and its taps must be
// compile-time indices to stay in SGPRs)
template <int... I, class F>
__device__ __forceinline__ void static_for_impl(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(std::make_integer_sequence<int, N>{}, f);
}

constexpr int kHT = 64;   // output tile columns (rows: HarrisShape::TH, 64 or 32)
// SFM_HARRIS_COUNT_INTERIOR (instruction counting only, tools/isa_phases.py --interior; never
// run): every tile takes the interior-tile code path, so the static count of the tile loop is
// the per-tile-wave count of the tiles that lie inside the image (all but the border tiles)
#ifdef SFM_HARRIS_COUNT_INTERIOR
#define SFM_INTERIOR(cond) true
#else
#define SFM_INTERIOR(cond) (cond)
#endif
// levels with at most this many 64 x 64 tiles per resident workgroup take the 64 x 32 form
// (SFMFEAT_HARRIS_SMALL overrides; 0 = never)
constexpr int kHarrisSmallTiles = 4;
// 1: the 7 x 7 window's default form keeps product planes in LDS (form 3; SFMFEAT_HARRIS_PP)
constexpr int kHarrisProductPlanes = 0;
// 1: the 7 x 7 window's large levels sum their windows on MFMA (form 4; SFMFEAT_HARRIS_MF,
// 2 = every level)
constexpr int kHarrisMfma = 0;

typedef float f32x2 __attribute__((ext_vector_type(2)));
// the window's tap pairs, read through the constant address space: wave-uniform scalar loads
// (s_load_dwordx*) into SGPRs that the packed fmas take as an operand — no LDS reads and no
// VGPRs for the 49 taps (round 5 read them as LDS broadcasts: 8 ds_read_b128 per gradient row
// per thread into 32 VGPRs)
typedef __attribute__((address_space(4))) const f32x2 cf32x2;

// acc = (k.x, k.y) * (v[H], v[H]) + acc : one v_pk_fma_f32 (two IEEE fmas, each bitwise
// fmaf) with the product value broadcast to both halves by op_sel — no register shuffles.
//
// gfx950 hazard (tools/pk_mfma_hazard.hip, profiles/r04_pk_mfma_hazard.txt): a v_pk_fma_f32
// whose LOW result reads src1's HIGH half (op_sel:[0,1,0]) returns wrong low results in lanes
// 48-63 while an MFMA of another wave runs on the same SIMD.  The high-half broadcast is
// therefore taken on src0 (op_sel:[1,0,0], product value first: a*b == b*a, so each half is
// still bitwise fmaf(k, v, acc)); the low-half broadcast (op_sel_hi:[1,0,1]) is unaffected.
// SFM_HARRIS_SRC1_HI (diagnostics builds only) restores the affected form.
template <int H>
__device__ __forceinline__ void pk_fma_bcast(f32x2& acc, f32x2 k, f32x2 v) {
#if defined(SFM_HARRIS_NATIVE_PK)  // diagnostics builds only (tools/coresidency_repro.hip)
  const float b = v[H];
  acc = __builtin_elementwise_fma(k, f32x2{b, b}, acc);
  return;
#elif defined(SFM_HARRIS_SCALAR_FMA)
  acc.x = __builtin_fmaf(k.x, v[H], acc.x);
  acc.y = __builtin_fmaf(k.y, v[H], acc.y);
  return;
#endif
  // k (the tap pair) is wave-uniform and lives in an SGPR pair (one scalar operand: the
  // constant-bus limit)
  if constexpr (H == 0)
    asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(acc) : "s"(k), "v"(v));
#ifdef SFM_HARRIS_SRC1_HI
  else
    asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "s"(k), "v"(v));
#else
  else
    asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(v), "s"(k));
#endif
}

// One workgroup (2 per CU; see HarrisShape) walks 64 x 64 output tiles of one plane.
// LDS holds the image tile (+ Sobel and window halo) and the two gradient planes Ix, Iy of
// the tile + window halo.  Each thread owns 4 columns x 4 rows: for every LDS gradient row
// it forms the three products Ix^2, Iy^2, IxIy in registers (v_pk_mul_f32; the same IEEE
// products the reference's elementwise multiplies give) and feeds them to all 4 output
// rows' window sums, as two row pairs of packed fmas.  LDS traffic per window fma is ~5x
// below a one-plane-per-product, 2-row layout, which left the kernel LDS-bound.
//
// VEC (W % 4 == 0): the image tile is fetched as 16-B loads (its left edge sits XA columns
// left of the tile, XA = round_up(GA + 1, 4), so every float4 is either wholly inside the
// image or wholly outside); otherwise scalar loads.  Both variants are prefetched into
// registers one tile ahead.
//
// ABL (timing builds only): 0 = full kernel, 1 = no digit histogram, 2 = window sums over
// the first tap row only, 3 = full kernel + per-workgroup timestamps into g_harris_stamps,
// 4 = no workgroup barriers in the tile loop (LDS races: results wrong; the barriers' cost).
// ABL = 3 diagnostics: per workgroup kStampSlots u64 = {start, end, cu id, tiles, end of
// each tile ...} (s_memrealtime, 100 MHz)
constexpr int kStampSlots = 48;
__device__ uint64_t* g_harris_stamps;
__device__ int64_t g_harris_stamps_cap;  // u64 slots behind g_harris_stamps (workgroups beyond it skip)

// NPAIR: output row pairs per thread.  2: 256 threads x (4 columns x 4 rows), 2 waves per
// SIMD at up to 256 VGPRs.  1: 512 threads x (4 columns x 2 rows), 4 waves per SIMD at up to
// 128 VGPRs (the window's packed fmas issue faster at 4 waves per SIMD, DESIGN_LOG.md §B), at
// the price of each gradient row's products being formed by twice as many threads.
// F (the workgroup form):
//   0: 256 threads x (4 columns x 4 rows), 64 x 64 tiles, 2 workgroups per CU (2 waves per
//      SIMD at up to 256 VGPRs) — the default;
//   1: 512 threads x (4 x 2), 64 x 64 tiles, 2 per CU (4 waves per SIMD at 128 VGPRs);
//   2: 256 threads x (4 x 2), 64 x 32 tiles, 3 per CU (3 waves per SIMD at 168 VGPRs): the
//      small levels, whose 64 x 64 tiles would give each resident workgroup only a few
//      tiles to walk one after another;
//   3: as 0, but the Sobel phase forms the three products once per pixel and LDS holds
//      product planes Ix^2, Iy^2, IxIy (the image tile aliased into them) instead of the two
//      gradient planes, so the window phase reads products instead of re-forming them for
//      every row it feeds (each gradient row's products were formed by 2.5 threads).
//   4: the window sums on the matrix pipe (v_mfma_f32_4x4x1_16b_f32, see "MFMA window"
//      below): 256 threads, 64 x 64 tiles, 2 workgroups per CU; wave w owns tile columns
//      16w .. 16w+15 and lane l tile row l.
//   5: as 0, with S_xy on the matrix pipe beside the VALU's S_xx and S_yy: the lanes of each
//      4-lane MFMA block share their 4 columns and hold 4 different row groups (rq from lane
//      bits 0-1 and 5, tq from bits 2-4), so an MFMA accumulator per output row o puts
//      pixel (4rq + o, 4tq + i) in register i of the thread that owns it in form 0, and the
//      B operand is the IxIy product that thread already formed for its VALU work.
template <int F>
struct HarrisShape {
  static constexpr bool PP = F == 3;                     // product planes in LDS
  static constexpr bool MF = F == 4;                     // window sums on MFMA
  static constexpr bool HY = F == 5;                     // S_xy on MFMA, S_xx / S_yy on VALU
  static constexpr int NPAIR = (F == 0 || F == 3 || F == 4 || F == 5) ? 2 : 1;  // output row pairs per thread
  static constexpr int NT = F == 1 ? 512 : 256;          // threads per workgroup
  static constexpr int RPT = 2 * NPAIR;                  // output rows per thread
  static constexpr int TH = RPT * 4 * (NT / 64);         // tile rows (tile columns: kHT)
  static constexpr int WPC = F == 2 ? 3 : 2;             // workgroups per CU
  static constexpr int WPE = WPC * NT / 256;             // waves per SIMD
};

// MFMA window (form 4).  v_mfma_f32_4x4x1_16b_f32 is 16 independent 4 x 4 outer products
// per instruction, D[lane 4b+j][reg i] += A[lane 4b+i] * B[lane 4b+j], and its result is
// bitwise a k-ordered fmaf chain (tools/mfma_f32_probe.hip, profiles/r04_mfma_f32_probe.txt:
// 0 of 256 results differ over chains of 1 .. 4096 steps).  A horizontal window row is a
// banded (Toeplitz) product: for a 4-column strip at tile columns x .. x+3, step s = 0 ..
// KS+2 takes gradient column x + s (B: the product at that column in the lane's row) and the
// tap g[dy][s - i] for output column x + i (A: 0 outside the band).  Each output pixel then
// sees its taps in row-major order with zero taps in between, and fmaf(0, p, acc) == acc
// for finite p and acc != -0 (acc starts at +0 and a sum of finite values never rounds to
// -0), so the chain is the reference's.  7 of every 10 MACs are taps at KS = 7.
template <int KS>
struct MfWin {
  static constexpr int NS = KS + 3;              // steps per tap row (4 columns + KS - 1)
  static constexpr int NC = 12 + NS;             // gradient columns a wave reads per row (4 strips)
  static constexpr int NB4 = (NC + 3) / 4;       // b128 LDS reads per row per plane
  // row stride: >= the tile's gradient columns and the last wave's reads, stride/4 odd
  // (ds_read_b128 lane groups of 16 rows then hit 16 distinct 16-B slots)
  static constexpr int stride() {
    int s = kHT + KS - 1;
    if (s < 48 + 4 * NB4) s = 48 + 4 * NB4;
    s = (s + 3) / 4 * 4;
    if (((s / 4) & 1) == 0) s += 4;
    return s;
  }
};

template <int KS, bool VEC, int ABL = 0, int F = 0>
__global__ void __launch_bounds__(HarrisShape<F>::NT, HarrisShape<F>::WPE) k_harris(HarrisLevels lvs, const float* __restrict__ gk, float alpha) {
  constexpr int NT = HarrisShape<F>::NT, RPT = HarrisShape<F>::RPT, NPAIR = HarrisShape<F>::NPAIR;
  constexpr int TH = HarrisShape<F>::TH;
  constexpr bool PP = HarrisShape<F>::PP;
  constexpr bool MF = HarrisShape<F>::MF;
  constexpr bool HY = HarrisShape<F>::HY;
  static_assert(!MF || (TH == 64 && NT == 256), "MFMA form: 4 waves x 64 rows");
  // this workgroup's level (one launch may hold several pyramid levels: the small levels'
  // tiles share a launch instead of each paying a launch and a tail)
  int li = 0;
#pragma unroll
  for (int k = 1; k < kHarrisMaxLevels; ++k) li += (k < lvs.n && (int)blockIdx.x >= lvs.l[k].wg0) ? 1 : 0;
  const float* __restrict__ lvl = lvs.l[li].lvl;
  float* __restrict__ Rout = lvs.l[li].R;
  uint32_t* __restrict__ hist_g = lvs.l[li].hist;
  const int H = lvs.l[li].H, W = lvs.l[li].W, tiles_x = lvs.l[li].tiles_x, ntiles = lvs.l[li].ntiles;
  const SelectScan scan = lvs.l[li].scan;
  const int wgx = (int)blockIdx.x - lvs.l[li].wg0, nwg = lvs.l[li].nwg;  // workgroups of this level's plane
  constexpr int GA = KS / 2;
  constexpr int PH = TH + KS - 1;           // gradient rows of a tile (window halo)
  constexpr int NV = 4 + KS - 1;            // gradient values per row per thread
  constexpr int NV4 = (NV + 3) / 4;         // b128 LDS loads per row per plane
  constexpr int NVP = 4 * NV4;
  constexpr int NP2 = (NV + 1) / 2;         // product pairs per row
  // a 16-lane group of a ds_read_b128 holds 8 column groups x 2 row groups (RPT rows apart):
  // RPT * stride / 4 == 8 (mod 16) 16-B chunks keeps the chunks 8*rq + tq (mod 16) distinct,
  // i.e. stride == 8 (mod 32) floats for RPT 4 and == 16 (mod 32) for RPT 2
  constexpr int PWP = MF ? MfWin<KS>::stride()
                    : HY ? ((kHT + KS - 1 <= 76 && 60 + NVP <= 76) ? 76 : ((60 + NVP <= 108) ? 108 : 140))
                    : RPT == 4 ? ((kHT + KS - 1 <= 72 && 60 + NVP <= 72) ? 72 : ((60 + NVP <= 104) ? 104 : 136))
                               : ((kHT + KS - 1 <= 80 && 60 + NVP <= 80) ? 80 : ((60 + NVP <= 112) ? 112 : 144));
  static_assert(PWP >= kHT + KS - 1 && (MF || 60 + NVP <= PWP), "harris LDS row stride");
  constexpr int NS = PWP / 4;               // 4-wide gradient strips per row
  constexpr int XA = (GA + 1 + 3) / 4 * 4;  // image tile margin left of the output tile
  constexpr int SH = XA - GA - 1;           // image column of gradient column 0, minus 1
  constexpr int NR4 = (SH + 6 + 3) / 4;     // float4 reads per Sobel strip row
  constexpr int IH = PH + 2;                // image tile rows (Sobel halo)
  constexpr int IWP = PWP + 4 * (NR4 - 1);  // covers every strip's reads
  constexpr int IW4 = IWP / 4;
  constexpr int NIMG = VEC ? (IH * IW4 + NT - 1) / NT : (IH * IWP + NT - 1) / NT;
  static_assert(NIMG <= 64, "prefetch mask");
  // gradient planes (or, PP, product planes) and the image tile; PP aliases the image tile
  // into the product planes (the tile is dead once the Sobel pass has read it)
  constexpr int NPL = PP ? 3 : 2;
  static_assert(!PP || IH * IWP <= NPL * PH * PWP, "image tile alias");
  __shared__ __attribute__((aligned(16))) float s_pl[NPL * PH * PWP + (PP ? 0 : IH * IWP)];
  float (*const s_g)[PH][PWP] = reinterpret_cast<float (*)[PH][PWP]>(s_pl);
  float (*const s_img)[IWP] = reinterpret_cast<float (*)[IWP]>(s_pl + (PP ? 0 : NPL * PH * PWP));
  // digit-1 histogram, flushed once per workgroup: two copies (even / odd lanes) where the LDS
  // budget of WPC workgroups per CU allows, halving the same-address serialisation of one
  // wave's LDS adds; the second copy is shifted by 16 words, half of the 32 banks a ds_add_u32
  // lane group spans, so a bucket's two copies never share a bank (round 6: a 32-word shift
  // put them on the same bank; L0 alone 397 -> 390 us, profiles/r06_harris_hist_variants.txt)
  constexpr int kHistCopy = kMedBins1 + 16;
  constexpr int kLdsRest = 4 * (NPL * PH * PWP + (PP ? 0 : IH * IWP)) + 1024;
  constexpr int NHC = kLdsRest + 8 * kHistCopy <= 163840 / HarrisShape<F>::WPC ? 2 : 1;
  __shared__ uint32_t s_hist[NHC * kHistCopy];
  __shared__ uint32_t s_last, s_red[10];

  const int tid = threadIdx.x;
  const int b = blockIdx.y;
  // kernel-active span (bench.py's roofline timing; rocprofv3's kernel duration minus the
  // dispatch latency): one atomic per workgroup at its start and at its exit
  if (lvs.span != nullptr && tid == 0) atomicMin(lvs.span, (unsigned long long)wall_clock64());
  auto span_end = [&]() {
    if (lvs.span != nullptr && tid == 0) atomicMax(lvs.span + 1, (unsigned long long)wall_clock64());
  };
  uint64_t* stamp = nullptr;
  int nst = 0;
  if constexpr (ABL == 3) {
    const int64_t s0 = ((int64_t)b * gridDim.x + blockIdx.x) * kStampSlots;
    stamp = s0 + kStampSlots <= g_harris_stamps_cap ? g_harris_stamps + s0 : nullptr;
    if (tid == 0 && stamp) {
      stamp[0] = wall_clock64();
      stamp[2] = (uint64_t)__smid();
    }
  }
  const float* img = lvl + (int64_t)b * H * W;
  float* Rp = Rout + (int64_t)b * H * W;
  for (int i = tid; i < NHC * kHistCopy; i += NT) s_hist[i] = 0u;
  const int lane = tid & 63, wv = tid >> 6;
  uint32_t* const s_hc = s_hist + (NHC == 2 ? (lane & 1) * kHistCopy : 0);
  // MFMA window: the banded tap operand A(dy, s), lane 4b+i: g[dy][s - i] (0 off the band).
  // Every block of an A operand holds the same taps, so the instruction's A broadcast
  // (cbsz 4: block abid's A to all 16 blocks; tools/mfma_f32_probe.hip) lets one VGPR carry
  // 16 steps: step k = dy * NS + s sits in block k % 16 of tapV[k / 16]
  constexpr int MNS = (MF || HY) ? MfWin<KS>::NS : 1;
  constexpr int NTAPV = (MF || HY) ? (KS * MNS + 15) / 16 : 1;
  float tapV[NTAPV];
  if constexpr (MF || HY) {
#pragma unroll
    for (int v = 0; v < NTAPV; ++v) {
      const int k = 16 * v + (lane >> 2), dy = k / MNS, t = k % MNS - (lane & 3);
      const bool on = k < KS * MNS && t >= 0 && t < KS;
      tapV[v] = on ? gk[on ? dy * KS + t : 0] : 0.0f;
    }
  }
  // columns 4tq .. 4tq+3, rows RPT*rq .. RPT*rq+RPT-1 (HY: a 4-lane block shares tq)
  const int tq = HY ? (((lane >> 2) & 7) | ((wv & 1) << 3)) : ((lane & 7) | ((wv & 1) << 3));
  const int rq = HY ? ((lane & 3) | (((lane >> 5) & 1) << 2) | ((wv >> 1) << 3))
                    : (((lane >> 3) & 7) | ((wv >> 1) << 3));

  // image tile of `tile` -> registers (zero outside the image = BORDER_CONSTANT)
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  f32x4 t4[VEC ? NIMG : 1];
  float t1[VEC ? 1 : NIMG];
  uint64_t okmask = 0;
  // the interior form's element offsets inside the tile window (row * W + column), fixed per
  // thread: a tile whose window lies wholly inside the image loads from one scalar base plus
  // these, with no per-element bounds (the image-tile copy below stores it unmasked too)
  int eoff[VEC ? NIMG : 1];
  if constexpr (VEC) {
#pragma unroll
    for (int k = 0; k < NIMG; ++k) {
      const int e = tid + NT * k, iy = e / IW4;
      eoff[k] = e < IH * IW4 ? iy * W + 4 * (e - iy * IW4) : 0;
    }
  }
  auto prefetch = [&](int tile) {
    const int gx0 = (tile % tiles_x) * kHT - XA;
    const int gy0 = (tile / tiles_x) * TH - GA - 1;
    okmask = 0;
    if (VEC && SFM_INTERIOR(gx0 >= 0 && gx0 + IWP <= W && gy0 >= 0 && gy0 + IH <= H)) {
      const float* tb = img + (int64_t)gy0 * W + gx0;
#pragma unroll
      for (int k = 0; k < NIMG; ++k) t4[VEC ? k : 0] = *reinterpret_cast<const f32x4*>(tb + (VEC ? eoff[k] : 0));
      return;
    }
    if constexpr (VEC) {
#pragma unroll
      for (int k = 0; k < NIMG; ++k) {
        const int e = tid + NT * k;
        const int iy = e / IW4, gx = gx0 + 4 * (e - iy * IW4), gy = gy0 + iy;
        const bool ok = e < IH * IW4 && gy >= 0 && gy < H && gx >= 0 && gx < W;
        const int64_t off = ok ? (int64_t)gy * W + gx : 0;
        t4[k] = *reinterpret_cast<const f32x4*>(img + off);
        okmask |= ok ? (1ull << k) : 0ull;
      }
    } else {
#pragma unroll
      for (int k = 0; k < NIMG; ++k) {
        const int e = tid + NT * k;
        const int iy = e / IWP, gx = gx0 + (e - iy * IWP), gy = gy0 + iy;
        const bool ok = e < IH * IWP && gy >= 0 && gy < H && gx >= 0 && gx < W;
        t1[k] = img[ok ? (int64_t)gy * W + gx : 0];
        okmask |= ok ? (1ull << k) : 0ull;
      }
    }
  };
  if (wgx < ntiles) prefetch(wgx);
  if (lvs.stagger && (blockIdx.x & 1))  // A/B: offset co-resident workgroups' phases
    for (int i = 0; i < lvs.stagger; ++i) __builtin_amdgcn_s_sleep(127);
  const int tmax = (ntiles + nwg - 1) / nwg;  // tiles of the busiest workgroup
  for (int tile = wgx; tile < ntiles; tile += nwg) {
    if (lvs.prio) {
      // the two workgroups resident on a CU share its SIMDs; the arbiter favours the older
      // waves, so one runs ahead and the other finishes alone.  A workgroup with more tiles
      // left issues at a higher priority, which keeps the two level.
      const int left = (ntiles - tile + nwg - 1) / nwg;
      if (4 * left > 3 * tmax) __builtin_amdgcn_s_setprio(3);
      else if (2 * left > tmax) __builtin_amdgcn_s_setprio(2);
      else if (4 * left > tmax) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
    const int tx0 = (tile % tiles_x) * kHT;
    const int ty0 = (tile / tiles_x) * TH;
    // tap pairs (harris_taps_build): pair (d, j) = (g[d][j], g[d-1][j]) for d = 0..KS, a
    // missing tap row 0.  The pointer is laundered once per tile so the compiler re-issues the
    // scalar loads per gradient row instead of hoisting all (KS+1) x KS pairs into SGPRs
    const cf32x2* tp = (const cf32x2*)(gk + kHarrisPairOff);
    asm volatile("" : "+s"(tp));
    if constexpr (ABL != 4) __syncthreads();  // the previous tile's LDS reads are done
    // 0. the prefetched image tile -> LDS, then start fetching the next tile (a tile whose
    //    whole image window lies inside the image stores its loads unmasked)
    const bool img_in = SFM_INTERIOR(tx0 - XA >= 0 && tx0 - XA + IWP <= W && ty0 - GA - 1 >= 0 && ty0 - GA - 1 + IH <= H);
    if (VEC && img_in) {
#pragma unroll
      for (int k = 0; k < NIMG; ++k) {
        const int e = tid + NT * k;
        if (e < IH * IW4) reinterpret_cast<f32x4*>(&s_img[0][0])[e] = t4[VEC ? k : 0];
      }
    } else {
#pragma unroll
      for (int k = 0; k < NIMG; ++k) {
        const bool ok = (okmask >> k) & 1ull;
        if constexpr (VEC) {
          const int e = tid + NT * k;
          if (e < IH * IW4)
            reinterpret_cast<f32x4*>(&s_img[0][0])[e] = ok ? t4[k] : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        } else {
          const int e = tid + NT * k;
          if (e < IH * IWP) (&s_img[0][0])[e] = ok ? t1[k] : 0.0f;
        }
      }
    }
    if constexpr (ABL != 4) __syncthreads();
    // (PP: after the product pass, so the prefetch registers are not live beside the
    // strips' gradients)
    if (!PP && tile + nwg < ntiles) prefetch(tile + nwg);
    // 1. gradients (NaiveSIFT.py:201-213: fma chain over the non-zero Sobel taps in
    //    row-major order from +0; k*p is exact for these taps) for 4-wide strips; outside
    //    the image the gradients are 0, so their products (:61-63) are the zero border of
    //    the window sums (:67-69)
    //    Packed over column pairs (q, q+1) when the strip's image reads are pair-aligned
    //    (each half an IEEE fma, as the scalar chain); interior tiles skip the masking.
    constexpr int NSI = (PH * NS + NT - 1) / NT;  // strips per thread (PP: held in registers)
    float4 GXs[PP ? NSI : 1], GYs[PP ? NSI : 1];
    auto sobel = [&](auto maskedc) {
      constexpr bool MASKED = decltype(maskedc)::value;
#pragma unroll
      for (int it = 0; it < (PP ? NSI : 1); ++it)
      for (int sidx = tid + it * NT; sidx < PH * NS; sidx += (PP ? PH * NS : NT)) {
        const int py = sidx / NS, px0 = (sidx - py * NS) * 4;
        f32x2 w[3][2 * NR4];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
          const float4* row = reinterpret_cast<const float4*>(&s_img[py + dy][px0]);
#pragma unroll
          for (int c4 = 0; c4 < NR4; ++c4) {
            const float4 v = row[c4];
            w[dy][2 * c4] = f32x2{v.x, v.y};
            w[dy][2 * c4 + 1] = f32x2{v.z, v.w};
          }
        }
        auto val = [&](int dy, int c) { return w[dy][c >> 1][c & 1]; };
        float gxq[4], gyq[4];
        if constexpr ((SH & 1) == 0) {
          const f32x2 m1 = {-1.0f, -1.0f}, p1 = {1.0f, 1.0f}, m2 = {-2.0f, -2.0f}, p2 = {2.0f, 2.0f};
#pragma unroll
          for (int h = 0; h < 2; ++h) {  // columns (2h, 2h+1)
            const int c = (2 * h + SH) >> 1;  // pair index of column 2h + SH
            f32x2 ix = {0.0f, 0.0f}, iy = {0.0f, 0.0f};
            // the (c+1) pair straddles pairs: (w[c].y, w[c+1].x) is read as columns
            // q+1; build it only for iy's centre taps
            const f32x2 mid0 = f32x2{w[0][c].y, w[0][c + 1].x};
            const f32x2 mid2 = f32x2{w[2][c].y, w[2][c + 1].x};
            ix = __builtin_elementwise_fma(m1, w[0][c], ix);
            ix = __builtin_elementwise_fma(p1, w[0][c + 1], ix);
            ix = __builtin_elementwise_fma(m2, w[1][c], ix);
            ix = __builtin_elementwise_fma(p2, w[1][c + 1], ix);
            ix = __builtin_elementwise_fma(m1, w[2][c], ix);
            ix = __builtin_elementwise_fma(p1, w[2][c + 1], ix);
            iy = __builtin_elementwise_fma(m1, w[0][c], iy);
            iy = __builtin_elementwise_fma(m2, mid0, iy);
            iy = __builtin_elementwise_fma(m1, w[0][c + 1], iy);
            iy = __builtin_elementwise_fma(p1, w[2][c], iy);
            iy = __builtin_elementwise_fma(p2, mid2, iy);
            iy = __builtin_elementwise_fma(p1, w[2][c + 1], iy);
            gxq[2 * h] = ix.x;
            gxq[2 * h + 1] = ix.y;
            gyq[2 * h] = iy.x;
            gyq[2 * h + 1] = iy.y;
          }
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c = q + SH;
            float ix = 0.0f;
            ix = __builtin_fmaf(-1.0f, val(0, c), ix);
            ix = __builtin_fmaf(1.0f, val(0, c + 2), ix);
            ix = __builtin_fmaf(-2.0f, val(1, c), ix);
            ix = __builtin_fmaf(2.0f, val(1, c + 2), ix);
            ix = __builtin_fmaf(-1.0f, val(2, c), ix);
            ix = __builtin_fmaf(1.0f, val(2, c + 2), ix);
            float iy = 0.0f;
            iy = __builtin_fmaf(-1.0f, val(0, c), iy);
            iy = __builtin_fmaf(-2.0f, val(0, c + 1), iy);
            iy = __builtin_fmaf(-1.0f, val(0, c + 2), iy);
            iy = __builtin_fmaf(1.0f, val(2, c), iy);
            iy = __builtin_fmaf(2.0f, val(2, c + 1), iy);
            iy = __builtin_fmaf(1.0f, val(2, c + 2), iy);
            gxq[q] = ix;
            gyq[q] = iy;
          }
        }
        if constexpr (MASKED) {
          const int gy = ty0 - GA + py;
          const bool rowin = gy >= 0 && gy < H;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int gx = tx0 - GA + px0 + q;
            const bool inside = rowin && gx >= 0 && gx < W;
            gxq[q] = inside ? gxq[q] : 0.0f;
            gyq[q] = inside ? gyq[q] : 0.0f;
          }
        }
        if constexpr (PP) {
          GXs[it] = make_float4(gxq[0], gxq[1], gxq[2], gxq[3]);
          GYs[it] = make_float4(gyq[0], gyq[1], gyq[2], gyq[3]);
        } else {
          *reinterpret_cast<float4*>(&s_g[0][py][px0]) = make_float4(gxq[0], gxq[1], gxq[2], gxq[3]);
          *reinterpret_cast<float4*>(&s_g[1][py][px0]) = make_float4(gyq[0], gyq[1], gyq[2], gyq[3]);
        }
      }
    };
    // every gradient position of the tile (incl. the unused stride padding) in the image
    const bool grad_in = SFM_INTERIOR(tx0 - GA >= 0 && tx0 - GA + PWP <= W && ty0 - GA >= 0 && ty0 - GA + PH <= H);
    if (grad_in) sobel(std::false_type{});
    else sobel(std::true_type{});
    if constexpr (ABL != 4) __syncthreads();
    if constexpr (F == 0) {
      // fused pyramid: the tile's 8 x 8 blocks of this level -> the next three exact 2x levels
      // (pyramid.hip k_down2x3's arithmetic, so the levels are bit-identical), one block per
      // lane of the first wave, read from the image tile in LDS instead of from HBM again.
      // After the Sobel barrier, so the other waves start their windows meanwhile (form 0
      // keeps the image tile intact until the next tile's copy)
      float* const d1 = lvs.l[li].down[0];
#ifdef SFM_HARRIS_COUNT_NO_DOWN  // instruction counting only (tools/isa_phases.py --interior)
      if (false) {
#else
      if (d1 != nullptr && tid < 64) {
#endif
        const int bx = tid & 7, by = tid >> 3;
        const int gy = ty0 + 8 * by, gx = tx0 + 8 * bx;
        if (gy < H && gx < W) {
          float a[8][8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float4 lo = *reinterpret_cast<const float4*>(&s_img[GA + 1 + 8 * by + i][XA + 8 * bx]);
            const float4 hi = *reinterpret_cast<const float4*>(&s_img[GA + 1 + 8 * by + i][XA + 8 * bx + 4]);
            a[i][0] = lo.x; a[i][1] = lo.y; a[i][2] = lo.z; a[i][3] = lo.w;
            a[i][4] = hi.x; a[i][5] = hi.y; a[i][6] = hi.z; a[i][7] = hi.w;
          }
          down2x3_block(a, d1, lvs.l[li].down[1], lvs.l[li].down[2], b, H, W, gy >> 3, gx >> 3);
        }
      }
    }
    if constexpr (PP) {
      // the image tile is dead: the three products of every gradient (NaiveSIFT.py:61-63, the
      // same IEEE products the window phase formed) into their planes
#pragma unroll
      for (int it = 0; it < NSI; ++it) {
        const int sidx = tid + it * NT;
        if (sidx < PH * NS) {
          const int py = sidx / NS, px0 = (sidx - py * NS) * 4;
          const f32x2 x0 = {GXs[it].x, GXs[it].y}, x1 = {GXs[it].z, GXs[it].w};
          const f32x2 y0 = {GYs[it].x, GYs[it].y}, y1 = {GYs[it].z, GYs[it].w};
          const f32x2 a0 = x0 * x0, a1 = x1 * x1, b0 = y0 * y0, b1 = y1 * y1, c0 = x0 * y0, c1 = x1 * y1;
          *reinterpret_cast<float4*>(&s_g[0][py][px0]) = make_float4(a0.x, a0.y, a1.x, a1.y);
          *reinterpret_cast<float4*>(&s_g[1][py][px0]) = make_float4(b0.x, b0.y, b1.x, b1.y);
          *reinterpret_cast<float4*>(&s_g[2][py][px0]) = make_float4(c0.x, c0.y, c1.x, c1.y);
        }
      }
      __syncthreads();
      if (tile + nwg < ntiles) prefetch(tile + nwg);
    }

    if constexpr (MF) {
      // 2'. window sums on the matrix pipe (see MfWin): lane l = tile row l, wave w = tile
      //     columns 16w .. 16w+15 as 4 strips q of 4 columns; acc[q][pl][i] = column
      //     16w + 4q + i.  Per tap row dy the lane reads its gradient row l + dy (columns
      //     16w .. 16w + NC - 1), forms the three products of each column once (the same IEEE
      //     products as :61-63) and feeds every strip whose band covers that column.
      using MW = MfWin<KS>;
      typedef float f32x4 __attribute__((ext_vector_type(4)));
      f32x4 macc[4][3];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) macc[q][pl] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      // gradient rows are read one tap row ahead (two register buffers)
      float X[2][4 * MW::NB4], Y[2][4 * MW::NB4];
      auto load_row = [&](int dy, float (&x)[4 * MW::NB4], float (&y)[4 * MW::NB4]) {
        const float4* rx = reinterpret_cast<const float4*>(&s_g[0][lane + dy][16 * wv]);
        const float4* ry = reinterpret_cast<const float4*>(&s_g[1][lane + dy][16 * wv]);
#pragma unroll
        for (int c4 = 0; c4 < MW::NB4; ++c4) {
          const float4 a = rx[c4], c = ry[c4];
          x[4 * c4] = a.x, x[4 * c4 + 1] = a.y, x[4 * c4 + 2] = a.z, x[4 * c4 + 3] = a.w;
          y[4 * c4] = c.x, y[4 * c4 + 1] = c.y, y[4 * c4 + 2] = c.z, y[4 * c4 + 3] = c.w;
        }
      };
      load_row(0, X[0], Y[0]);
      constexpr int NDY = (ABL == 2) ? 1 : KS;
      static_for<NDY>([&](auto dyc) {
        constexpr int dy = decltype(dyc)::value, cb = dy & 1;
        if constexpr (dy + 1 < NDY) load_row(dy + 1, X[cb ^ 1], Y[cb ^ 1]);
        // the row's products, once per column
        float pxx[MW::NC], pyy[MW::NC], pxy[MW::NC];
#pragma unroll
        for (int c = 0; c < MW::NC; ++c) {
          const float xv = X[cb][c], yv = Y[cb][c];
          pxx[c] = xv * xv, pyy[c] = yv * yv, pxy[c] = xv * yv;
        }
        // step-major: every step feeds all 12 accumulators (4 strips x 3 planes), so an
        // accumulator's next MFMA is 12 instructions behind its last
        static_for<MW::NS>([&](auto sc) {
          constexpr int s = decltype(sc)::value, k = dy * MW::NS + s;
          const float tv = tapV[k / 16];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            macc[q][0] = __builtin_amdgcn_mfma_f32_4x4x1f32(tv, pxx[4 * q + s], macc[q][0], 4, k % 16, 0);
            macc[q][1] = __builtin_amdgcn_mfma_f32_4x4x1f32(tv, pyy[4 * q + s], macc[q][1], 4, k % 16, 0);
            macc[q][2] = __builtin_amdgcn_mfma_f32_4x4x1f32(tv, pxy[4 * q + s], macc[q][2], 4, k % 16, 0);
          }
        });
      });
      // 3'. R (:71-74) per pixel, the digit-1 histogram, R stored as 16-B row segments
      const int gy = ty0 + lane;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int gx0 = tx0 + 16 * wv + 4 * q;
        float Rq[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float sxx = macc[q][0][i], syy = macc[q][1][i], sxy = macc[q][2][i];
          const float t1v = sxx * syy;
          const float t2v = sxy * sxy;
          const float det = t1v - t2v;
          const float tr = sxx + syy;
          const float tr2 = tr * tr;
          const float at = alpha * tr2;
          Rq[i] = det - at;
          if (ABL != 1) atomicAdd(&s_hc[fkey(Rq[i]) >> (32 - kMedBits1)], (gy < H && gx0 + i < W) ? 1u : 0u);
        }
        if (gy < H) {
          float* dst = Rp + (int64_t)gy * W + gx0;
          if (VEC) {
            if (gx0 < W) *reinterpret_cast<float4*>(dst) = make_float4(Rq[0], Rq[1], Rq[2], Rq[3]);
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (gx0 + i < W) dst[i] = Rq[i];
          }
        }
      }
    } else {
    // 2. window sums (:67-69): per pixel an fma chain over the KS x KS taps in row-major
    //    order.  acc[p][pl][q] = (row 4rq+2p, row 4rq+2p+1) at column 4tq+q; gradient row
    //    4rq+r feeds tap row r-2p of the pair's first row and r-2p-1 of its second: packed
    //    fmas where both are taps, a scalar fma on one half at the pair's first/last row.
    f32x2 acc[NPAIR][3][4];
#pragma unroll
    for (int p = 0; p < NPAIR; ++p)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[p][pl][q] = f32x2{0.0f, 0.0f};
    // HY: S_xy of output row RPT*rq + o in MFMA accumulator o (register i = column 4tq + i)
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    f32x4 macc2[HY ? 4 : 1];
#pragma unroll
    for (int o = 0; o < (HY ? 4 : 1); ++o) macc2[o] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    constexpr int NR = (ABL == 2) ? 1 : KS + 2 * NPAIR - 1;  // gradient rows feeding this thread
    static_for<NR>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      f32x2 P[3][NP2];
      if constexpr (PP) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          const float4* rp = reinterpret_cast<const float4*>(&s_g[pl][RPT * rq + r][4 * tq]);
#pragma unroll
          for (int c4 = 0; c4 < NV4; ++c4) {
            const float4 a = rp[c4];
            if (2 * c4 < NP2) P[pl][2 * c4] = f32x2{a.x, a.y};
            if (2 * c4 + 1 < NP2) P[pl][2 * c4 + 1] = f32x2{a.z, a.w};
          }
        }
      } else {
        const float4* rx = reinterpret_cast<const float4*>(&s_g[0][RPT * rq + r][4 * tq]);
        const float4* ry = reinterpret_cast<const float4*>(&s_g[1][RPT * rq + r][4 * tq]);
        f32x2 X[NVP / 2], Y[NVP / 2];
#pragma unroll
        for (int c4 = 0; c4 < NV4; ++c4) {
          const float4 a = rx[c4], c = ry[c4];
          X[2 * c4] = f32x2{a.x, a.y};
          X[2 * c4 + 1] = f32x2{a.z, a.w};
          Y[2 * c4] = f32x2{c.x, c.y};
          Y[2 * c4 + 1] = f32x2{c.z, c.w};
        }
#pragma unroll
        for (int m = 0; m < NP2; ++m) {
          P[0][m] = X[m] * X[m];
          P[1][m] = Y[m] * Y[m];
          P[2][m] = X[m] * Y[m];
        }
      }
      f32x2 T[NPAIR][KS];
      asm volatile("" : "+s"(tp));  // this row's pairs are loaded here, not hoisted with every row's
#pragma unroll
      for (int p = 0; p < NPAIR; ++p) {
        const int d = r - 2 * p;  // tap rows (d, d - 1) of the pair's two output rows
        if (d >= 0 && d <= KS) {
#pragma unroll
          for (int j = 0; j < KS; ++j) T[p][j] = tp[d * KS + j];
        }
      }
#pragma unroll
      for (int p = 0; p < NPAIR; ++p) {
        const int i0 = r - 2 * p, i1 = r - 2 * p - 1;  // tap rows of the pair's two rows
        const bool v0 = i0 >= 0 && i0 < KS && (ABL != 2 || i0 == 0);
        const bool v1 = i1 >= 0 && i1 < KS && ABL != 2;
        if (!v0 && !v1) continue;  // (a compile-time condition)
#pragma unroll
        for (int pl = 0; pl < (HY ? 2 : 3); ++pl)
#pragma unroll
          for (int j = 0; j < KS; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int m = q + j;
              if (v0 && v1) {
                if (m & 1) pk_fma_bcast<1>(acc[p][pl][q], T[p][j], P[pl][m >> 1]);
                else pk_fma_bcast<0>(acc[p][pl][q], T[p][j], P[pl][m >> 1]);
              } else if (v0) {
                acc[p][pl][q].x = __builtin_fmaf(T[p][j].x, P[pl][m >> 1][m & 1], acc[p][pl][q].x);
              } else {
                acc[p][pl][q].y = __builtin_fmaf(T[p][j].y, P[pl][m >> 1][m & 1], acc[p][pl][q].y);
              }
            }
      }
      if constexpr (HY) {
        // S_xy: gradient row r is tap row r - o of output row o; step s takes column 4tq + s
        // (the thread's own IxIy product) with the banded taps (MfWin)
        static_for<RPT>([&](auto oc) {
          constexpr int o = decltype(oc)::value, dy = r - o;
          if constexpr (dy >= 0 && dy < KS && (ABL != 2 || dy == 0)) {
            static_for<MNS>([&](auto sc) {
              constexpr int st = decltype(sc)::value, k = dy * MNS + st;
              macc2[o] = __builtin_amdgcn_mfma_f32_4x4x1f32(tapV[k / 16], P[2][st >> 1][st & 1], macc2[o], 4, k % 16, 0);
            });
          }
        });
      }
    });
    // 3. R = det - alpha * trace^2 (:71-74), digit-1 histogram of R, R stored as 16-B
    //    row segments (a wave writes 8 rows x 128 contiguous bytes per store); a tile wholly
    //    inside the plane counts and stores without per-pixel bounds
    auto epilogue = [&](auto fullc) {
      constexpr bool FULL = decltype(fullc)::value;
      // R of both rows of each accumulator pair at once: the same IEEE operations as the
      // per-pixel form (t1 = sxx*syy, t2 = sxy*sxy, det = t1 - t2, tr = sxx + syy, tr2 =
      // tr*tr, at = alpha*tr2, R = det - at), as plain v_pk_mul / v_pk_add (no op_sel)
      f32x2 Rpk[NPAIR][4];
      const f32x2 al2 = {alpha, alpha};
#pragma unroll
      for (int p = 0; p < NPAIR; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x2 sxx = acc[p][0][q], syy = acc[p][1][q];
          const f32x2 sxy = HY ? f32x2{macc2[HY ? 2 * p : 0][q], macc2[HY ? 2 * p + 1 : 0][q]} : acc[p][2][q];
          const f32x2 t1v = sxx * syy;
          const f32x2 t2v = sxy * sxy;
          const f32x2 det = t1v - t2v;
          const f32x2 tr = sxx + syy;
          const f32x2 tr2 = tr * tr;
          const f32x2 at = al2 * tr2;
          Rpk[p][q] = det - at;
        }
#pragma unroll
      for (int o = 0; o < RPT; ++o) {
        const int gy = ty0 + RPT * rq + o;
        const int gx0 = tx0 + 4 * tq;
        float Rq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          Rq[q] = Rpk[o >> 1][q][o & 1];
          if (ABL != 1)
            atomicAdd(&s_hc[fkey_nz(Rq[q]) >> (32 - kMedBits1)], (FULL || (gy < H && gx0 + q < W)) ? 1u : 0u);
        }
        if (FULL || gy < H) {
          float* dst = Rp + (int64_t)gy * W + gx0;
          if (VEC) {
            if (FULL || gx0 < W) *reinterpret_cast<float4*>(dst) = make_float4(Rq[0], Rq[1], Rq[2], Rq[3]);
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (FULL || gx0 + q < W) dst[q] = Rq[q];
          }
        }
      }
    };
    if (SFM_INTERIOR(ty0 + TH <= H && tx0 + kHT <= W)) epilogue(std::true_type{});
    else epilogue(std::false_type{});
    }  // !MF
    if constexpr (ABL == 3) {
      if (tid == 0 && stamp && nst < kStampSlots - 4) stamp[4 + nst] = wall_clock64();
      ++nst;
    }
  }  // tile loop
  if constexpr (ABL == 3) {
    if (tid == 0 && stamp) {
      stamp[1] = wall_clock64();
      stamp[3] = (uint64_t)nst;
    }
  }
  __syncthreads();
  uint32_t* hg = hist_g + (int64_t)b * kMedBins1;
  for (int i = tid; i < kMedBins1; i += NT) {
    uint32_t c = s_hist[i] + (NHC == 2 ? s_hist[kHistCopy + i] : 0u);
    if (c) atomicAdd(&hg[i], c);
  }
  if (scan.state == nullptr) {
    span_end();
    return;
  }
  // The last workgroup of this plane to finish runs the select scan.  The
  // flushes are device-scope atomics, performed at the memory side: waiting for their
  // acknowledgement (vmcnt) orders them before the arrival count without the L2
  // write-back a __threadfence() costs; the scan reads the histogram with agent-scope
  // atomic loads.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) s_last = atomicAdd(&scan.done[(int64_t)b * kCounterStride], 1ull) == (unsigned long long)(nwg - 1) ? 1u : 0u;
  __syncthreads();
  if (!s_last) {
    span_end();
    return;
  }
  select_scan_plane(hg, scan.state + b, scan.list_count + (int64_t)b * kCounterStride, (int64_t)H * W,
                    scan.vmin, scan.force_exact, s_red);
  span_end();
}

// Workgroups per plane for a group of levels: a common tile budget per workgroup
// T = ceil(sum of tiles / slots per plane), each level gets ceil(tiles / T) workgroups, so
// every workgroup walks at most T tiles (`slots` resident over the batch; each loops over
// tiles so the digit histogram is flushed once per workgroup instead of once per tile)
static int harris_plan(HarrisLevels& g, int B, int slots) {
  const int per_plane = std::max(1, slots / std::max(B, 1));
  int total = 0;
  for (int k = 0; k < g.n; ++k) total += g.l[k].ntiles;
  const int T = std::max(1, (total + per_plane - 1) / per_plane);
  int wg = 0;
  for (int k = 0; k < g.n; ++k) {
    g.l[k].wg0 = wg;
    g.l[k].nwg = std::max(1, std::min(g.l[k].ntiles, (g.l[k].ntiles + T - 1) / T));
    wg += g.l[k].nwg;
  }
  return wg;
}

size_t harris_taps_floats(int ks) { return (size_t)kHarrisPairOff + 2 * (size_t)(ks + 1) * ks; }

void harris_taps_build(const float* g, int ks, float* out) {
  for (size_t i = 0; i < harris_taps_floats(ks); ++i) out[i] = 0.0f;
  for (int i = 0; i < ks * ks; ++i) out[i] = g[i];
  float* tp = out + kHarrisPairOff;
  for (int d = 0; d <= ks; ++d)
    for (int j = 0; j < ks; ++j) {
      tp[2 * (d * ks + j)] = d < ks ? g[d * ks + j] : 0.0f;
      tp[2 * (d * ks + j) + 1] = d >= 1 ? g[(d - 1) * ks + j] : 0.0f;
    }
}

static int env_int(const char* name, int dflt) {  // product switch (tests/test_gpu_switches.py)
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
static int diag_int(const char* name, int dflt) {  // diagnostic build only (SFM_DIAG_ENV)
  const char* e = SFM_DIAG_ENV(name);
  return e ? atoi(e) : dflt;
}

template <int KS, int ABL, int F>
static void launch_form(HarrisLevels g, int B, const float* gk, float alpha, hipStream_t st) {
  using S = HarrisShape<F>;
  // Resident-workgroup budget of the default form (SFMFEAT_HARRIS_SLOTS overrides).  Batches
  // of >= 16 planes take 448 = 14 workgroups per plane at 32 planes, which leaves 64 CUs
  // with one Harris workgroup instead of two for the other batch in flight: measured 33.4k
  // -> 34.8-35.5k img/s on the headline (13 per plane: 33.0k, 15: 32.5k, 16: 33.4k, 18:
  // 34.2-34.6k; DESIGN_LOG.md §B); at 8 planes of 4K 448 cost 6 % and 480 (60 per plane)
  // measured best (6.15-6.17k against 5.98-6.00k img/s at 512, 5.95k at 576, 5.87k at 640).
  static const int slots_env = env_int("SFMFEAT_HARRIS_SLOTS", 0);
  // SFMFEAT_HARRIS_SLOTS_UPPER=n (A/B): the budget of levels above the first (fewer than
  // 200 64 x 64 tiles per plane)
  static const int slots_up = diag_int("SFMFEAT_HARRIS_SLOTS_UPPER", 0);
  int slots2 = slots_env > 0 ? slots_env : (B >= 16 ? 448 : 480);
  if (slots_up > 0 && g.n == 1 && ((g.l[0].W + kHT - 1) / kHT) * ((g.l[0].H + kHT - 1) / kHT) < 200) slots2 = slots_up;
  bool vec = true;
  for (int k = 0; k < g.n; ++k) {
    g.l[k].tiles_x = (g.l[k].W + kHT - 1) / kHT;
    g.l[k].ntiles = g.l[k].tiles_x * ((g.l[k].H + S::TH - 1) / S::TH);
    vec = vec && (g.l[k].W & 3) == 0;
  }
  const int nwg = harris_plan(g, B, slots2 * S::WPC / 2);
  if (vec)
    hipLaunchKernelGGL((k_harris<KS, true, ABL, F>), dim3(nwg, B), dim3(S::NT), 0, st, g, gk, alpha);
  else
    hipLaunchKernelGGL((k_harris<KS, false, ABL, F>), dim3(nwg, B), dim3(S::NT), 0, st, g, gk, alpha);
}

template <int KS, int ABL = 0>
static void launch_ks(HarrisLevels g, int B, const float* gk, float alpha, hipStream_t st) {
  // SFMFEAT_HARRIS_PRIO=1: tile-balancing issue priority (A/B)
  static const int prio = diag_int("SFMFEAT_HARRIS_PRIO", 0);
  // SFMFEAT_HARRIS_NPAIR=1: the four-wave form for every level (A/B)
  static const int npair = diag_int("SFMFEAT_HARRIS_NPAIR", 2);
  // SFMFEAT_HARRIS_SMALL=t: levels whose 64 x 64 tiles number at most t per resident
  // workgroup (over the batch) take the 64 x 32 form (0: never)
  static const int small = diag_int("SFMFEAT_HARRIS_SMALL", kHarrisSmallTiles);
  g.prio = prio;
  // SFMFEAT_HARRIS_STAGGER=n: odd workgroups sleep n x 8k cycles before their first tile (A/B)
  static const int stagger = diag_int("SFMFEAT_HARRIS_STAGGER", 0);
  g.stagger = stagger;
  // SFMFEAT_HARRIS_PP=1: product planes in LDS (form 3) instead of gradient planes (A/B)
  static const int pp = diag_int("SFMFEAT_HARRIS_PP", kHarrisProductPlanes);
  // SFMFEAT_HARRIS_MF=1: window sums on the matrix pipe (form 4) for the levels that take
  // form 0; 2: for every level; 3 / 4: S_xy on MFMA beside the VALU (form 5), form-0 levels
  // / every level
  static const int mf = diag_int("SFMFEAT_HARRIS_MF", kHarrisMfma);
  if constexpr (KS == 7) {  // the alternative forms are built for the 7 x 7 window only
    // the fused pyramid (levels with down[0] set) is validated in form 0 only
    bool fused = false;
    for (int k = 0; k < g.n; ++k) fused = fused || g.l[k].down[0] != nullptr;
    if (fused) return launch_form<KS, ABL, 0>(g, B, gk, alpha, st);
#ifdef SFM_ABLATIONS  // the forms measured slower (1, 3, 4, 5): diagnostic build only
    if (npair == 1) return launch_form<KS, ABL, 1>(g, B, gk, alpha, st);
    if (mf == 2) return launch_form<KS, ABL, 4>(g, B, gk, alpha, st);
    if (mf == 4) return launch_form<KS, ABL, 5>(g, B, gk, alpha, st);
#else
    (void)npair;
    (void)pp;
    (void)mf;
#endif
    bool sm = small > 0;
    for (int k = 0; k < g.n; ++k) {
      const int64_t t64 = (int64_t)((g.l[k].W + kHT - 1) / kHT) * ((g.l[k].H + kHT - 1) / kHT) * B;
      sm = sm && t64 <= (int64_t)small * 512;
    }
    if (sm) return launch_form<KS, ABL, 2>(g, B, gk, alpha, st);
#ifdef SFM_ABLATIONS
    if (pp == 1) return launch_form<KS, ABL, 3>(g, B, gk, alpha, st);
    if (mf == 1) return launch_form<KS, ABL, 4>(g, B, gk, alpha, st);
    if (mf == 3) return launch_form<KS, ABL, 5>(g, B, gk, alpha, st);
#endif
  }
  launch_form<KS, ABL, 0>(g, B, gk, alpha, st);
}

void launch_harris_levels(const HarrisLevels& g, int B, const float* d_gauss, int ks, float alpha, hipStream_t st) {
  switch (ks) {
    case 1: launch_ks<1>(g, B, d_gauss, alpha, st); break;
    case 2: launch_ks<2>(g, B, d_gauss, alpha, st); break;
    case 3: launch_ks<3>(g, B, d_gauss, alpha, st); break;
    case 4: launch_ks<4>(g, B, d_gauss, alpha, st); break;
    case 5: launch_ks<5>(g, B, d_gauss, alpha, st); break;
    case 6: launch_ks<6>(g, B, d_gauss, alpha, st); break;
    case 7: {
      // SFMFEAT_HARRIS_ABL=1|2: timing ablations inside the pipeline (results are wrong)
      static const int abl = [] {
        const char* e = SFM_ABLATION_ENV("SFMFEAT_HARRIS_ABL");
        return e ? atoi(e) : 0;
      }();
      if (abl == 1) launch_ks<7, 1>(g, B, d_gauss, alpha, st);
      else if (abl == 2) launch_ks<7, 2>(g, B, d_gauss, alpha, st);
      else launch_ks<7>(g, B, d_gauss, alpha, st);
      break;
    }
    case 8: launch_ks<8>(g, B, d_gauss, alpha, st); break;
    case 9: launch_ks<9>(g, B, d_gauss, alpha, st); break;
    case 11: launch_ks<11>(g, B, d_gauss, alpha, st); break;
    case 13: launch_ks<13>(g, B, d_gauss, alpha, st); break;
    case 15: launch_ks<15>(g, B, d_gauss, alpha, st); break;
    default: break;  // rejected at context creation
  }
}

void launch_harris(const float* lvl, float* R, uint32_t* hist, int B, int H, int W,
                   const float* d_gauss, int ks, float alpha, SelectScan scan, hipStream_t st) {
  HarrisLevels g{};
  g.n = 1;
  g.l[0].lvl = lvl;
  g.l[0].R = R;
  g.l[0].hist = hist;
  g.l[0].H = H;
  g.l[0].W = W;
  g.l[0].scan = scan;
  launch_harris_levels(g, B, d_gauss, ks, alpha, st);
}

// Ablation timing (diagnostics): KS = 7 only, returns the mean launch time in ms.
float time_harris_ablation(int abl, const float* lvl, float* R, uint32_t* hist, int B, int H, int W,
                           const float* gk, float alpha, int iters, uint64_t* stamps, int64_t stamps_cap) {
  if (abl == 3) {
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_harris_stamps), &stamps, sizeof(stamps));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_harris_stamps_cap), &stamps_cap, sizeof(stamps_cap));
  }
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  HarrisLevels g{};
  g.n = 1;
  g.l[0].lvl = lvl;
  g.l[0].R = R;
  g.l[0].hist = hist;
  g.l[0].H = H;
  g.l[0].W = W;
  g.l[0].scan = SelectScan{nullptr, nullptr, nullptr, 0, 0};
  auto run = [&]() {
    switch (abl) {
      case 1: launch_ks<7, 1>(g, B, gk, alpha, 0); break;
      case 2: launch_ks<7, 2>(g, B, gk, alpha, 0); break;
      case 3: launch_ks<7, 3>(g, B, gk, alpha, 0); break;
      case 4: launch_ks<7, 4>(g, B, gk, alpha, 0); break;
      default: launch_ks<7, 0>(g, B, gk, alpha, 0); break;
    }
  };
  run();
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < iters; ++i) run();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms / iters;
}

}  // namespace sfm
