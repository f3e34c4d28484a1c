// nms.hip — max-pool NMS + threshold + candidate compaction (NaiveSIFT.py:77-97):
//   R_maxpool[r,c] = max of R over the ksize x ksize window clipped to the image (:85-88)
//   R_maxpool[R < median] = 0                                                    (:92)
//   candidate  <=> R == R_maxpool                                                (:95)
// i.e. (R >= med && R == window max) || (R < med && R == 0).  Candidates are appended
// per plane as 64-bit keys ~fkey(R) << 32 | raster index, so ascending key order is the
// reference's confidence-descending order with ties broken by raster index.
//
// Two predicates (kernels.h, MedianState):
//   mode 0 (certified planes): key(R) >= tnms && R == window max — a few percent of the
//          pixels pass the threshold, and only those test their window;
//   mode 1 (fallback planes):  the exact predicate above with the exact median.
// "R == window max" is tested as "no cell of the clipped window is larger"; out-of-image
// cells hold -inf and never win.
//
// k_nms_tile (ksize <= 9): persistent workgroups walk contiguous row-major runs of 64 x 64
// tiles of one plane; the tile + halo (72-float rows, 16-B aligned) is loaded with 16-B
// loads into registers one tile ahead, then staged through LDS.  HBM-bound: ~1.03 reads
// of R (the column halo's lines are the neighbour tiles', fetched by the same workgroup).
// k_nms_generic (larger ksize): separable window max on an LDS tile.
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "kernels.h"

namespace sfm {

constexpr int kNT_W = 64;
constexpr int kNT_H = 32;          // k_nms_generic tile height
constexpr int kTT_H = 64;          // k_nms_tile tile height (more bytes in flight per workgroup)
constexpr int kNmsBlocksPerPlane = 64;

template <int KH, int MODE, bool VEC>  // VEC: W % 4 == 0 (16-B aligned rows and planes)
__global__ void __launch_bounds__(256) k_nms_tile(const float* __restrict__ R,
                                                  const MedianState* __restrict__ st,
                                                  uint64_t* __restrict__ cand,
                                                  unsigned long long* __restrict__ cand_count, int H,
                                                  int W, int tiles_x, int ntiles) {
  static_assert(KH <= 4, "72-float rows hold a 4-column halo");
  constexpr int LW = 72;                // tile columns tx0-4 .. tx0+67
  constexpr int LW4 = LW / 4;
  constexpr int LH = kTT_H + 2 * KH;
  constexpr int NV4 = LH * LW4;
  constexpr int PER = (NV4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float s_t[LH][LW];
  __shared__ uint32_t s_wsum[4];
  __shared__ unsigned long long s_base;
  const int tid = threadIdx.x;
  const int b = blockIdx.y;
  const bool fb = st[b].fallback != 0;
  if (MODE == 0 ? fb : !fb) return;
  const uint32_t tnms = st[b].tnms;
  const float med = st[b].median;
  const int64_t n = (int64_t)H * W;
  const float* Rp = R + (int64_t)b * n;

  // loads are unconditional (clamped addresses) and masked afterwards, so all of them are
  // in flight together — a branch around a load makes the compiler wait on it in place
  // (and masked only when stored to LDS, one tile later, so nothing waits on them early)
  float4 t[PER];
  uint32_t okm = 0;  // VEC: bit k = slot k inside the image; !VEC: 4 bits per slot
  auto prefetch = [&](int tile) {
    const int x0 = (tile % tiles_x) * kNT_W - 4;
    const int y0 = (tile / tiles_x) * kTT_H - KH;
    okm = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = min(tid + 256 * k, NV4 - 1);
      const int row = e / LW4, c4 = e - row * LW4;
      const int gy = y0 + row, gx = x0 + 4 * c4;
      const bool rowok = gy >= 0 && gy < H;
      const float* rp = Rp + (int64_t)min(max(gy, 0), H - 1) * W;
      if (VEC) {
        t[k] = *reinterpret_cast<const float4*>(rp + min(max(gx, 0), W - 4));
        okm |= (rowok && gx >= 0 && gx < W) ? (1u << k) : 0u;  // W % 4 == 0: all in or all out
      } else {
        float q[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int x = gx + j;
          q[j] = rp[min(max(x, 0), W - 1)];
          okm |= (rowok && x >= 0 && x < W) ? (1u << (4 * k + j)) : 0u;
        }
        t[k] = make_float4(q[0], q[1], q[2], q[3]);
      }
    }
  };
  static_assert(VEC ? PER <= 32 : PER <= 8, "prefetch mask bits");

  const int c0 = (tid & 7) * 8;    // 8 output columns, rows tid >> 3 and (tid >> 3) + 32
  // one workgroup per band of tile rows, walking its tiles left to right: a tile's column
  // halo lies in the 128-B lines of its neighbours, which this workgroup fetches next (or
  // just did) through the same L2 instead of another XCD's — the strided assignment of
  // adjacent tiles to different workgroups fetched those lines twice
  const int t_lo = (int)((int64_t)ntiles * blockIdx.x / gridDim.x);
  const int t_hi = (int)((int64_t)ntiles * (blockIdx.x + 1) / gridDim.x);
  if (t_lo < t_hi) prefetch(t_lo);
  for (int tile = t_lo; tile < t_hi; ++tile) {
    const int tx0 = (tile % tiles_x) * kNT_W;
    const int ty0 = (tile / tiles_x) * kTT_H;
    __syncthreads();  // previous tile's LDS reads done
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = tid + 256 * k;
      float4 v = t[k];
      if (VEC) {
        if (!((okm >> k) & 1u)) v = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
      } else {
        v.x = ((okm >> (4 * k)) & 1u) ? v.x : -INFINITY;
        v.y = ((okm >> (4 * k + 1)) & 1u) ? v.y : -INFINITY;
        v.z = ((okm >> (4 * k + 2)) & 1u) ? v.z : -INFINITY;
        v.w = ((okm >> (4 * k + 3)) & 1u) ? v.w : -INFINITY;
      }
      if (e < NV4) reinterpret_cast<float4*>(&s_t[0][0])[e] = v;
    }
    __syncthreads();
    if (tile + 1 < t_hi) prefetch(tile + 1);
    uint32_t flags = 0;
    float vals[16];
    // pixel q of this thread: KH == 1 -> 4 x 4 block (rows 4rg + q/4, columns 4cg + q%4);
    // otherwise 8 columns x rows tid/8 and tid/8 + 32
    const int cg = tid & 15, rg = tid >> 4;
    auto pix_r = [&](int q) { return KH == 1 ? 4 * rg + (q >> 2) : (tid >> 3) + 32 * (q >> 3); };
    auto pix_c = [&](int q) { return KH == 1 ? 4 * cg + (q & 3) : c0 + (q & 7); };
    if constexpr (KH == 1) {
      // separable 3 x 3 max from 16-B LDS reads (a 16-lane group reads 16 distinct
      // chunks of one row): per input row the horizontal max3 of the 4 columns, then the
      // vertical max3; max is exact, so v == max <=> no cell of the window is larger
      float hm[6][4], ctr[4][4];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const float* row = &s_t[4 * rg + i][4 * cg];
        const float4 a = *reinterpret_cast<const float4*>(row);
        const float4 bq = *reinterpret_cast<const float4*>(row + 4);
        const float cx = row[8];
        const float x[6] = {a.w, bq.x, bq.y, bq.z, bq.w, cx};
#pragma unroll
        for (int e = 0; e < 4; ++e) hm[i][e] = fmaxf(fmaxf(x[e], x[e + 1]), x[e + 2]);
        if (i >= 1 && i <= 4) {
          ctr[i - 1][0] = bq.x; ctr[i - 1][1] = bq.y; ctr[i - 1][2] = bq.z; ctr[i - 1][3] = bq.w;
        }
      }
#pragma unroll
      for (int o = 0; o < 4; ++o)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int q = 4 * o + e;
          const float v = ctr[o][e];
          vals[q] = v;
          const float m = fmaxf(fmaxf(hm[o][e], hm[o + 1][e]), hm[o + 2][e]);
          const bool inside = ty0 + 4 * rg + o < H && tx0 + 4 * cg + e < W;
          bool pred;
          if (MODE == 0) pred = fkey(v) >= tnms && v == m;
          else pred = (v < med) ? (v == 0.0f) : (v == m);  // R_maxpool[R < median] = 0 (:92)
          flags |= (inside && pred) ? (1u << q) : 0u;
        }
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int r = pix_r(q), c = pix_c(q);
        const float v = s_t[r + KH][4 + c];
        vals[q] = v;
        const bool inside = ty0 + r < H && tx0 + c < W;
        bool pred = false;
        if (inside && (MODE == 1 || fkey(v) >= tnms)) {
          if (MODE == 1 && v < med) {
            pred = (v == 0.0f);  // R_maxpool[R < median] = 0 (:92)
          } else {
            bool ismax = true;
#pragma unroll
            for (int dy = -KH; dy <= KH; ++dy)
#pragma unroll
              for (int dx = -KH; dx <= KH; ++dx) ismax &= !(s_t[r + KH + dy][4 + c + dx] > v);
            pred = ismax;
          }
        }
        flags |= pred ? (1u << q) : 0u;
      }
    }
    if (__syncthreads_or(flags != 0)) {
      const int64_t slot = block_append(&cand_count[(int64_t)b * kCounterStride], (uint32_t)__popc(flags),
                                        s_wsum, &s_base);
      uint64_t* out = cand + (int64_t)b * n + slot;
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (flags & (1u << q)) {
          const int r = pix_r(q), c = pix_c(q);
          *out++ = ((uint64_t)(~fkey(vals[q])) << 32) | (uint32_t)((ty0 + r) * W + tx0 + c);
        }
    }
  }
}

// k_nms_stream (ksize 3, certified planes, W % 4 == 0): the streaming form of mode 0.
// Thread t of a plane owns one 16-B column group c4 = t % C4 of strip s = t / C4 (SH rows),
// so a wavefront reads 1 KB of contiguous row per load and every row of R is read once
// (plus the strip's two halo rows).  All SH + 2 rows are loaded up front (16-B loads, one
// per row), the horizontal max3 takes its outer columns from the neighbouring lanes
// (__shfl_up/__shfl_down; the wave's edge lanes load them), then the vertical max3 and the
// predicate.  No LDS staging: the tiled kernel's per-tile barriers and LDS round trip
// paced it at ~21 % of HBM (DESIGN_LOG.md §B).  Candidates are appended with one atomic per
// workgroup; their order is irrelevant (k_topk orders them by key).
template <int SH, int NT>
__global__ void __launch_bounds__(NT) k_nms_stream(const float* __restrict__ R,
                                                    const MedianState* __restrict__ st,
                                                    uint64_t* __restrict__ cand,
                                                    unsigned long long* __restrict__ cand_count, int H,
                                                    int W, int nstrips, int dry) {
  constexpr int NR = SH + 2;
  static_assert(4 * SH <= 64, "flags hold 4 bits per output row");
  const int b = blockIdx.y;
  if (st[b].fallback != 0) return;  // whole workgroup: fallback planes take the exact path
  const uint32_t tnms = st[b].tnms;
  const int64_t n = (int64_t)H * W;
  const float* Rp = R + (int64_t)b * n;
  const int C4 = W >> 2;
  const int lane = threadIdx.x & 63;
  // persistent workgroups (the grid may be capped, SFMFEAT_NMS_STREAM_WG): virtual block vb
  // covers groups [vb * NT, vb * NT + NT); every thread of a workgroup runs the same vb's
  __shared__ uint32_t s_wsum[NT / 64];
  __shared__ unsigned long long s_base;
  const int64_t nvb = ((int64_t)C4 * nstrips + NT - 1) / NT;
  for (int64_t vb = blockIdx.x; vb < nvb; vb += gridDim.x) {
    const int64_t gid = vb * NT + threadIdx.x;
    const bool active = gid < (int64_t)C4 * nstrips;
    const int g = active ? (int)gid : C4 * nstrips - 1;  // inactive lanes mirror the last group
    const int s = g / C4, c4 = g - s * C4;
    const int y0 = s * SH - 1;  // buffer row j is image row y0 + j
    const float* colp = Rp + 4 * c4;

    float4 v[NR];
  #pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int gy = min(max(y0 + j, 0), H - 1);
      v[j] = *reinterpret_cast<const float4*>(colp + (int64_t)gy * W);
    }
    // the wave's edge lanes fetch the column beyond their group (the neighbour lane's value
    // is in another wavefront); the same 128-B lines are being read by that wavefront
    float edge[NR];
    const bool need_l = lane == 0 && c4 > 0, need_r = lane == 63 && c4 < C4 - 1;
  #pragma unroll
    for (int j = 0; j < NR; ++j) edge[j] = -INFINITY;
    if (need_l || need_r) {
      const int off = need_l ? -1 : 4;
  #pragma unroll
      for (int j = 0; j < NR; ++j) {
        const int gy = min(max(y0 + j, 0), H - 1);
        edge[j] = colp[(int64_t)gy * W + off];
      }
    }

    // rolling horizontal maxima: hm[j % 3] holds buffer row j; output row i = buffer row
    // i + 1 is decided once buffer row i + 2 is in
    float hm[3][4];
    uint64_t flags = 0;
  #pragma unroll
    for (int j = 0; j < NR; ++j) {
      const bool rowok = y0 + j >= 0 && y0 + j < H;
      if (!rowok) v[j] = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
      const float up = __shfl_up(v[j].w, 1);    // lane - 1's last column
      const float dn = __shfl_down(v[j].x, 1);  // lane + 1's first column
      float l = c4 == 0 ? -INFINITY : (lane == 0 ? edge[j] : up);
      float r = c4 == C4 - 1 ? -INFINITY : (lane == 63 ? edge[j] : dn);
      if (!rowok) l = r = -INFINITY;
      float* h = hm[j % 3];
      h[0] = fmaxf(fmaxf(l, v[j].x), v[j].y);
      h[1] = fmaxf(fmaxf(v[j].x, v[j].y), v[j].z);
      h[2] = fmaxf(fmaxf(v[j].y, v[j].z), v[j].w);
      h[3] = fmaxf(fmaxf(v[j].z, v[j].w), r);
      if (j >= 2) {
        const int i = j - 2;
        const float c[4] = {v[i + 1].x, v[i + 1].y, v[i + 1].z, v[i + 1].w};
        const bool inside = active && !dry && y0 + 1 + i < H;
  #pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float m = fmaxf(fmaxf(hm[0][e], hm[1][e]), hm[2][e]);
          const bool pred = inside && fkey(c[e]) >= tnms && c[e] == m;
          flags |= pred ? (1ull << (4 * i + e)) : 0ull;
        }
      }
    }

    // one atomic per workgroup (device-scope atomics on the per-plane counters, not the
    // bytes, paced the per-wavefront form: a candidate-free pass over R took 58 us at L0
    // against 93 us with the appends)
    if (!__syncthreads_or(flags != 0)) continue;
    const int64_t slot = block_append(&cand_count[(int64_t)b * kCounterStride], (uint32_t)__popcll(flags),
                                      s_wsum, &s_base);
    if (flags == 0) continue;
    uint64_t* out = cand + (int64_t)b * n + slot;
    // the few candidates re-read their value (an L2 hit) instead of keeping the strip's
    // rows live across the append: 156 -> fewer VGPRs, more workgroups per CU in flight
    while (flags) {
      const int bit = __builtin_ctzll(flags);
      flags &= flags - 1;
      const uint32_t idx = (uint32_t)((y0 + 1 + (bit >> 2)) * W + 4 * c4 + (bit & 3));
      *out++ = ((uint64_t)(~fkey(Rp[idx])) << 32) | idx;
    }
  }
}

// k_nms_band (the default certified 3x3 form since round 4): as k_nms_stream, but each
// thread walks NB strips of 8 rows down its column group, carrying the last two rows' values
// and horizontal maxima from one strip to the next in registers, so every row of R is read
// once per band instead of 10 / 8 times (the strips' halo rows: PMC traffic 1.36x the
// algorithmic bytes).  Candidates of the whole band are appended with one
// atomic per workgroup (flag words: 32 bits per strip).
template <int NB, int NT>
__global__ void __launch_bounds__(NT) k_nms_band(const float* __restrict__ R, const MedianState* __restrict__ st,
                                                  uint64_t* __restrict__ cand,
                                                  unsigned long long* __restrict__ cand_count, int H, int W,
                                                  int nbands) {
  constexpr int SH = 8;
  static_assert(NB >= 1 && NB <= 4, "two 64-bit flag words");
  const int b = blockIdx.y;
  if (st[b].fallback != 0) return;  // whole workgroup: fallback planes take the exact path
  const uint32_t tnms = st[b].tnms;
  // fkey(v) >= tnms as one float compare v >= T: fkey is a monotone bijection between the
  // non-NaN floats (-0 folded onto +0, as IEEE compares them) and the keys 0x007FFFFF ..
  // 0xFF800000, so T = fkey_inv(tnms) inside that range, -inf below it (every value passes)
  // and NaN above it (none does)
  const float T = tnms <= 0x007FFFFFu ? -INFINITY : tnms > 0xFF800000u ? __uint_as_float(0x7FC00000u) : fkey_inv(tnms);
  const int64_t n = (int64_t)H * W;
  const float* Rp = R + (int64_t)b * n;
  const int C4 = W >> 2;
  const int lane = threadIdx.x & 63;
  __shared__ uint32_t s_wsum[NT / 64];
  __shared__ unsigned long long s_base;
  const int64_t groups = (int64_t)C4 * nbands;
  const int64_t nvb = (groups + NT - 1) / NT;
  for (int64_t vb = blockIdx.x; vb < nvb; vb += gridDim.x) {
    const int64_t gid = vb * NT + threadIdx.x;
    const bool active = gid < groups;
    const int g = active ? (int)gid : (int)(groups - 1);  // inactive lanes mirror the last group
    const int band = g / C4, c4 = g - band * C4;
    const int ytop = band * NB * SH;  // first output row of the band
    const float* colp = Rp + 4 * c4;
    const bool need_l = lane == 0 && c4 > 0, need_r = lane == 63 && c4 < C4 - 1;
    const int eoff = need_l ? -1 : 4;
    // one image row of this column group: its 4 values (-inf outside the image) and the
    // horizontal max3 of each column (outer neighbours from the adjacent lanes / the edge load)
    // (rowok is a compile-time true for bands whose every row lies inside the image)
    auto hrow = [&](const float4& v0, float e, bool rowok, float4& v, float (&h)[4]) {
      v = rowok ? v0 : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
      // lane - 1's v.w and lane + 1's v.x by DPP wave_shr:1 / wave_shl:1 (no LDS round trip;
      // lane 0's up and lane 63's dn are never used: they take e or -inf)
      const float up = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v.w), 0x138, 0xF, 0xF, false));
      const float dn = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v.x), 0x130, 0xF, 0xF, false));
      float l = c4 == 0 ? -INFINITY : (lane == 0 ? e : up);
      float r = c4 == C4 - 1 ? -INFINITY : (lane == 63 ? e : dn);
      if (!rowok) l = r = -INFINITY;
      h[0] = fmaxf(fmaxf(l, v.x), v.y);
      h[1] = fmaxf(fmaxf(v.x, v.y), v.z);
      h[2] = fmaxf(fmaxf(v.y, v.z), v.w);
      h[3] = fmaxf(fmaxf(v.z, v.w), r);
    };
    auto load = [&](int y, float4& v, float& e) {
      const int gy = min(max(y, 0), H - 1);
      v = *reinterpret_cast<const float4*>(colp + (int64_t)gy * W);
      e = (need_l || need_r) ? colp[(int64_t)gy * W + eoff] : -INFINITY;
    };
    uint64_t flags0 = 0ull, flags1 = 0ull;
    // IN: every image row the band reads (ytop - 1 .. ytop + NB * SH) lies inside the image,
    // so no row needs its -inf fill and every output row is inside
    auto band_body = [&](auto inc) {
    constexpr bool IN = decltype(inc)::value;
    // carried rows: a = row y - 1, c = row y (values and horizontal maxima)
    float4 va, vc;
    float ha[4], hc[4];
    {
      float4 r0, r1;
      float e0, e1;
      load(ytop - 1, r0, e0);
      load(ytop, r1, e1);
      hrow(r0, e0, IN || (ytop - 1 >= 0 && ytop - 1 < H), va, ha);
      hrow(r1, e1, IN || ytop < H, vc, hc);
    }
#pragma unroll 1
    for (int sb = 0; sb < NB; ++sb) {  // not unrolled: one strip's registers at a time
      const int y0 = ytop + sb * SH;  // output rows y0 .. y0 + 7 need image rows up to y0 + 8
      float4 raw[SH];
      float er[SH];
      uint32_t strip = 0;  // 4 bits per output row of this strip
#pragma unroll
      for (int j = 0; j < SH; ++j) load(y0 + 1 + j, raw[j], er[j]);  // every load in flight
#pragma unroll
      for (int j = 0; j < SH; ++j) {
        float4 vn;
        float hn[4];
        const int yn = y0 + 1 + j;
        hrow(raw[j], er[j], IN || yn < H, vn, hn);
        // output row y = yn - 1: centre vc, window rows a (y - 1), c (y), n (y + 1)
        const int y = yn - 1;
        const bool inside = active && (IN || y < H);
        const float cv[4] = {vc.x, vc.y, vc.z, vc.w};
        uint32_t fr = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float m = fmaxf(fmaxf(ha[e], hc[e]), hn[e]);
          const bool pred = inside && cv[e] >= T && cv[e] == m;
          fr |= pred ? (1u << (4 * j + e)) : 0u;
        }
        strip |= fr;
        va = vc;
        vc = vn;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ha[e] = hc[e];
          hc[e] = hn[e];
        }
      }
      const uint64_t sw = (uint64_t)strip << (32 * (sb & 1));
      if (sb < 2) flags0 |= sw;
      else flags1 |= sw;
    }
    };
    if (ytop >= 1 && ytop + NB * SH <= H - 1) band_body(std::true_type{});
    else band_body(std::false_type{});
    const uint64_t flags[2] = {flags0, flags1};
    const uint32_t nf = (uint32_t)(__popcll(flags[0]) + __popcll(flags[1]));
    if (!__syncthreads_or(nf != 0)) continue;
    const int64_t slot = block_append(&cand_count[(int64_t)b * kCounterStride], nf, s_wsum, &s_base);
    if (nf == 0) continue;
    uint64_t* out = cand + (int64_t)b * n + slot;
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      uint64_t f = flags[w];
      while (f) {  // the few candidates re-read their value (an L2 hit)
        const int bit = __builtin_ctzll(f);
        f &= f - 1;
        const int sb = 2 * w + (bit >> 5), j = (bit & 31) >> 2;
        const uint32_t idx = (uint32_t)((ytop + sb * SH + j) * W + 4 * c4 + (bit & 3));
        *out++ = ((uint64_t)(~fkey(Rp[idx])) << 32) | idx;
      }
    }
  }
}

constexpr int kStreamSH = 8;
constexpr int kBandStrips = 4;  // strips of 8 rows per k_nms_band thread (SFMFEAT_NMS_BAND=0: k_nms_stream)

static bool nms_tile_forced() {  // SFMFEAT_NMS_TILE=1: the tiled kernel for mode 0 too (A/B)
  static const bool f = [] {
    const char* e = getenv("SFMFEAT_NMS_TILE");
    return e && atoi(e) != 0;
  }();
  return f;
}

constexpr int kRowsPerThread = kNT_H / 4;  // 256 threads = 64 columns x 4 row groups

template <int KH>  // LDS sized for half-width KH (SFM_NMS_MAX_HALF); kh <= KH at run time
__global__ void __launch_bounds__(256) k_nms_generic(const float* __restrict__ R,
                                                     const MedianState* __restrict__ st,
                                                     uint64_t* __restrict__ cand,
                                                     unsigned long long* __restrict__ cand_count, int H,
                                                     int W, int kh, int tiles_x, int ntiles, int mode) {
  __shared__ float s_r[kNT_H + 2 * KH][kNT_W + 2 * KH];
  __shared__ float s_m[kNT_H + 2 * KH][kNT_W];
  __shared__ uint32_t s_wsum[4];
  __shared__ unsigned long long s_base;
  const int tid = threadIdx.x;
  const int b = blockIdx.y;
  const bool fb = st[b].fallback != 0;
  if (mode == 0 ? fb : !fb) return;
  const uint32_t tnms = st[b].tnms;
  const float med = st[b].median;
  const int64_t n = (int64_t)H * W;
  const float* Rp = R + (int64_t)b * n;
  const int TWh = kNT_W + 2 * kh, THh = kNT_H + 2 * kh;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int tx0 = (tile % tiles_x) * kNT_W;
    const int ty0 = (tile / tiles_x) * kNT_H;
    __syncthreads();
    for (int idx = tid; idx < THh * TWh; idx += 256) {
      int iy = idx / TWh, ix = idx - iy * TWh;
      int gy = ty0 - kh + iy, gx = tx0 - kh + ix;
      float v = -INFINITY;  // outside the image: never the (clipped) window max
      if (gy >= 0 && gy < H && gx >= 0 && gx < W) v = Rp[(int64_t)gy * W + gx];
      s_r[iy][ix] = v;
    }
    __syncthreads();
    for (int idx = tid; idx < THh * kNT_W; idx += 256) {
      int iy = idx / kNT_W, ix = idx - iy * kNT_W;
      float m = s_r[iy][ix];
      for (int d = 1; d <= 2 * kh; ++d) m = fmaxf(m, s_r[iy][ix + d]);
      s_m[iy][ix] = m;
    }
    __syncthreads();
    const int c = tid & 63;
    const int rg = tid >> 6;
    uint32_t flags = 0;
#pragma unroll
    for (int q = 0; q < kRowsPerThread; ++q) {
      const int r = rg * kRowsPerThread + q;
      const int gy = ty0 + r, gx = tx0 + c;
      if (gy < H && gx < W) {
        float m = s_m[r][c];
        for (int d = 1; d <= 2 * kh; ++d) m = fmaxf(m, s_m[r + d][c]);
        const float v = s_r[r + kh][c + kh];
        const bool pred = mode == 0 ? (fkey(v) >= tnms && v == m) : ((v < med) ? (v == 0.0f) : (v == m));
        flags |= pred ? (1u << q) : 0u;
      }
    }
    const int64_t slot = block_append(&cand_count[(int64_t)b * kCounterStride], (uint32_t)__popc(flags),
                                      s_wsum, &s_base);
    uint64_t* out = cand + (int64_t)b * n + slot;
#pragma unroll
    for (int q = 0; q < kRowsPerThread; ++q) {
      if (flags & (1u << q)) {
        const int r = rg * kRowsPerThread + q;
        const int gy = ty0 + r, gx = tx0 + c;
        const float v = s_r[r + kh][c + kh];
        *out++ = ((uint64_t)(~fkey(v)) << 32) | (uint32_t)(gy * W + gx);
      }
    }
  }
}

template <int KH>
static void launch_tile(const float* R, const MedianState* state, uint64_t* cand, unsigned long long* cnt,
                        int B, int H, int W, int tiles_x, int mode, hipStream_t st, int force_tile) {
  const bool vec = (W & 3) == 0;
  if (KH == 1 && mode == 0 && vec && !force_tile && !nms_tile_forced()) {
    // SFMFEAT_NMS_SH=8: 8-row strips (A/B); SFMFEAT_NMS_DRY=1: a candidate-free read pass
    // of R ahead of the real one (timing only: how fast R reads once Harris's writes drained)
    static const int sh = [] { const char* e = SFM_DIAG_ENV("SFMFEAT_NMS_SH"); return e ? atoi(e) : kStreamSH; }();
    static const bool dry = [] { const char* e = SFM_ABLATION_ENV("SFMFEAT_NMS_DRY"); return e && atoi(e) != 0; }();
    static const int band = [] { const char* e = SFM_DIAG_ENV("SFMFEAT_NMS_BAND"); return e ? atoi(e) : kBandStrips; }();
    if (band >= 1 && band <= 4 && !dry) {
      const int rows = 8 * band;
      const int nbands = (H + rows - 1) / rows;
      const int64_t nvb = ((int64_t)(W >> 2) * nbands + 255) / 256;
      dim3 grid((unsigned)nvb, B);
      switch (band) {
        case 1: hipLaunchKernelGGL((k_nms_band<1, 256>), grid, dim3(256), 0, st, R, state, cand, cnt, H, W, nbands); break;
        case 2: hipLaunchKernelGGL((k_nms_band<2, 256>), grid, dim3(256), 0, st, R, state, cand, cnt, H, W, nbands); break;
        case 3: hipLaunchKernelGGL((k_nms_band<3, 256>), grid, dim3(256), 0, st, R, state, cand, cnt, H, W, nbands); break;
        default: hipLaunchKernelGGL((k_nms_band<4, 256>), grid, dim3(256), 0, st, R, state, cand, cnt, H, W, nbands); break;
      }
      return;
    }
    const int SHr = (sh == 4 || sh == 16) ? sh : kStreamSH;
    const int NTr = 256;
    const int nstrips = (H + SHr - 1) / SHr;
    const int64_t threads = (int64_t)(W >> 2) * nstrips;
    static const int wg = [] { const char* e = SFM_DIAG_ENV("SFMFEAT_NMS_STREAM_WG"); return e ? atoi(e) : 0; }();
    const int64_t nvb = (threads + NTr - 1) / NTr;
    // SFMFEAT_NMS_STREAM_WG=n: at most n workgroups per launch over all planes (persistent)
    dim3 grid((unsigned)(wg > 0 ? std::min<int64_t>(nvb, std::max(1, wg / std::max(B, 1))) : nvb), B);
    for (int pass = dry ? 0 : 1; pass < 2; ++pass) {
#define SFM_NMS_STREAM(S, T)                                                                                 \
  if (SHr == S && NTr == T)                                                                                  \
    hipLaunchKernelGGL((k_nms_stream<S, T>), grid, dim3(T), 0, st, R, state, cand, cnt, H, W, nstrips, pass == 0);
      SFM_NMS_STREAM(4, 256) SFM_NMS_STREAM(8, 256) SFM_NMS_STREAM(16, 256)
#undef SFM_NMS_STREAM
    }
    return;
  }
  const int ntiles = tiles_x * ((H + kTT_H - 1) / kTT_H);
  // contiguous row-major tile ranges per workgroup (enough workgroups to keep the bytes in
  // flight: each holds one tile of prefetch)
  static const int slots = [] {  // SFMFEAT_NMS_SLOTS: workgroups per launch over all planes (A/B)
    const char* e = SFM_DIAG_ENV("SFMFEAT_NMS_SLOTS");
    return e ? atoi(e) : 0;
  }();
  const int per_plane = slots > 0 ? std::max(1, slots / std::max(B, 1)) : kNmsBlocksPerPlane;
  dim3 grid(std::min(ntiles, per_plane), B);
  if (mode == 0 && vec)
    hipLaunchKernelGGL((k_nms_tile<KH, 0, true>), grid, dim3(256), 0, st, R, state, cand, cnt, H, W, tiles_x, ntiles);
  else if (mode == 0)
    hipLaunchKernelGGL((k_nms_tile<KH, 0, false>), grid, dim3(256), 0, st, R, state, cand, cnt, H, W, tiles_x, ntiles);
  else if (vec)
    hipLaunchKernelGGL((k_nms_tile<KH, 1, true>), grid, dim3(256), 0, st, R, state, cand, cnt, H, W, tiles_x, ntiles);
  else
    hipLaunchKernelGGL((k_nms_tile<KH, 1, false>), grid, dim3(256), 0, st, R, state, cand, cnt, H, W, tiles_x, ntiles);
}

void launch_nms(const float* R, const MedianState* state, uint64_t* cand,
                unsigned long long* cand_count, int B, int H, int W, int ksize, int mode, hipStream_t st,
                int force_tile) {
  const int kh = ksize / 2;
  const int tiles_x = (W + kNT_W - 1) / kNT_W;
  const int tiles_y = (H + kNT_H - 1) / kNT_H;
  const int ntiles = tiles_x * tiles_y;
  switch (kh) {
    case 0: launch_tile<0>(R, state, cand, cand_count, B, H, W, tiles_x, mode, st, force_tile); break;
    case 1: launch_tile<1>(R, state, cand, cand_count, B, H, W, tiles_x, mode, st, force_tile); break;
    case 2: launch_tile<2>(R, state, cand, cand_count, B, H, W, tiles_x, mode, st, force_tile); break;
    case 3: launch_tile<3>(R, state, cand, cand_count, B, H, W, tiles_x, mode, st, force_tile); break;
    case 4: launch_tile<4>(R, state, cand, cand_count, B, H, W, tiles_x, mode, st, force_tile); break;
    default: {
      dim3 grid(std::min(ntiles, kNmsBlocksPerPlane), B);
      hipLaunchKernelGGL(k_nms_generic<SFM_NMS_MAX_HALF>, grid, dim3(256), 0, st, R, state, cand, cand_count, H, W,
                         kh, tiles_x, ntiles, mode);
      break;
    }
  }
}

}  // namespace sfm
