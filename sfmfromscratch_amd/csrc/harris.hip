// harris.hip — fused Harris response (NaiveSIFT._find_harris_interest_points,
// NaiveSIFT.py:59-74): Sobel gradients -> Ix^2, Iy^2, IxIy -> three 2-D Gaussian
// window sums -> R = det - alpha * trace^2, plus the first radix digit histogram of R
// for the exact median (NaiveSIFT.py:91).
//
// One workgroup (256 threads, 4 waves) walks 64 x 32 output tiles of one plane.  The three
// product planes of a tile (+ window halo) live in LDS; each thread accumulates 4 pixels x
// 2 rows with packed fp32 fmas (v_pk_fma_f32: the two rows' taps as one SGPR pair, the LDS
// value broadcast).  The 2-D window is the
// reference's full KS x KS correlation (not separable: a separable sum would round
// differently and move keypoints), accumulated per pixel as an fma chain
// in row-major tap order (OpenCV FilterVec_32f's v_muladd chain).
// VALU-bound by design.
#include <algorithm>

#include "kernels.h"

namespace sfm {

constexpr int kHT_W = 64;   // output tile width  (16 thread columns x 4 pixels)
constexpr int kHT_H = 32;   // output tile height (16 thread row pairs x 2 rows)

typedef float f32x2 __attribute__((ext_vector_type(2)));

// acc = (k.x, k.y) * (v[H], v[H]) + acc : one v_pk_fma_f32 (two IEEE fmas, each bitwise
// fmaf) with the LDS value broadcast to both halves by op_sel — no register shuffles.
template <int H>
__device__ __forceinline__ void pk_fma_bcast(f32x2& acc, f32x2 k, f32x2 v) {
  if constexpr (H == 0)
    asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(acc) : "s"(k), "v"(v));
  else
    asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "s"(k), "v"(v));
}

// ABL (ablation, timing builds only): 0 = full kernel, 1 = no digit histogram,
// 2 = no window sums, 3 = no Sobel/products (image copied into the product planes),
// 4 = image load + R store only, 5 = R store only
template <int KS, int ABL = 0>
__global__ void __launch_bounds__(256) k_harris(const float* __restrict__ lvl, float* __restrict__ Rout,
                                                uint32_t* __restrict__ hist_g, int H, int W,
                                                int tiles_x, int ntiles,
                                                const float* __restrict__ gk, float alpha,
                                                SelectScan scan) {
  constexpr int GA = KS / 2;
  constexpr int PW = kHT_W + KS - 1;        // product tile width
  constexpr int PH = kHT_H + KS - 1;        // product tile height
  // product row stride S == 8 (mod 32) floats: with lane = 4*rp + (tq & 3) every 16-lane
  // group of a ds_read_b128 ({0-3,12-15,20-27}, ...) covers 4 row pairs x 4 column
  // groups, whose 16-B chunks 4*rp + tq (mod 16) are all distinct -> conflict-free
  constexpr int PWP = (PW <= 72) ? 72 : (PW <= 104 ? 104 : 136);
  constexpr int NV = 4 + KS - 1;            // window values per row per plane
  constexpr int NV4 = (NV + 3) / 4;         // b128 loads per row per plane
  constexpr int NVP = 4 * NV4;
  static_assert(PWP >= PW && 60 + NVP <= PWP, "harris LDS row stride");
  constexpr int NS = PWP / 4;               // 4-wide product strips per product row
  constexpr int IH = PH + 2;                // image tile (Sobel halo)
  constexpr int IWP = PWP + 4;              // covers every strip's 8-float read
  constexpr int NIMG = (IH * IWP + 255) / 256;
  constexpr int SRW = kHT_W + 4;            // R staging row stride (in the image tile)
  static_assert(IH * IWP >= kHT_H * SRW, "R staging fits in the image tile");
  static_assert(NIMG <= 32, "prefetch mask");
  __shared__ __attribute__((aligned(16))) float s_prod[3][PH][PWP];
  __shared__ __attribute__((aligned(16))) float s_img[IH][IWP];
  __shared__ uint32_t s_hist[kMedBins1];  // digit-1 histogram, flushed once per workgroup
  __shared__ uint32_t s_last, s_red[8];

  const int tid = threadIdx.x;
  const int b = blockIdx.y;
  const float* img = lvl + (int64_t)b * H * W;
  for (int i = tid; i < kMedBins1; i += 256) s_hist[i] = 0u;
  const int lane = tid & 63;
  const int rp = lane >> 2;                      // row pair: output rows 2rp, 2rp+1
  const int tq = ((tid >> 6) << 2) | (lane & 3); // pixel columns 4tq .. 4tq+3
  // image tile loads for `tile` into registers (clamped, always-valid addresses; zero
  // outside the image = BORDER_CONSTANT).  Issued one tile ahead so their latency hides
  // under the previous tile's window sums.
  float t[NIMG];
  uint32_t okmask = 0;
  auto prefetch = [&](int tile) {
    const int px0 = (tile % tiles_x) * kHT_W - GA - 1;
    const int py0 = (tile / tiles_x) * kHT_H - GA - 1;
    okmask = 0;
#pragma unroll
    for (int k = 0; k < NIMG; ++k) {
      const int idx = tid + 256 * k;
      const int iy = idx / IWP, ix = idx - iy * IWP;
      const int gy = py0 + iy, gx = px0 + ix;
      const int yc = min(max(gy, 0), H - 1), xc = min(max(gx, 0), W - 1);
      t[k] = img[(int64_t)yc * W + xc];
      okmask |= (idx < IH * IWP && gy >= 0 && gy < H && gx >= 0 && gx < W) ? (1u << k) : 0u;
    }
  };
  if (ABL != 5 && blockIdx.x < ntiles) prefetch(blockIdx.x);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int tx0 = (tile % tiles_x) * kHT_W;
    const int ty0 = (tile / tiles_x) * kHT_H;
    __syncthreads();  // previous tile's LDS reads are done
    // 0. the prefetched image tile -> LDS
#pragma unroll
    for (int k = 0; k < NIMG; ++k) {
      const int idx = tid + 256 * k;
      if (idx < IH * IWP) (&s_img[0][0])[idx] = (okmask >> k) & 1u ? t[k] : 0.0f;
    }
    __syncthreads();
    // 1. gradients (NaiveSIFT.py:201-213: fma chain over the non-zero Sobel taps in
    //    row-major order from +0; k*p is exact for these taps) and products Ix^2, Iy^2,
    //    IxIy (:61-63) for 4-wide strips; consecutive lanes fill consecutive 16-B chunks
    //    (row stride == strip count * 4), outside the image -> 0
    for (int sidx = tid; sidx < PH * NS; sidx += 256) {
      if (ABL >= 4) break;
      const int py = sidx / NS, px0 = (sidx - py * NS) * 4;
      if (ABL == 3) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          *reinterpret_cast<float4*>(&s_prod[pl][py][px0]) =
              *reinterpret_cast<const float4*>(&s_img[py + 1][px0]);
        continue;
      }
      float w[3][8];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const float4* row = reinterpret_cast<const float4*>(&s_img[py + dy][px0]);
#pragma unroll
        for (int c4 = 0; c4 < 2; ++c4) {
          const float4 v = row[c4];
          w[dy][4 * c4 + 0] = v.x;
          w[dy][4 * c4 + 1] = v.y;
          w[dy][4 * c4 + 2] = v.z;
          w[dy][4 * c4 + 3] = v.w;
        }
      }
      const int gy = ty0 - GA + py;
      const bool rowin = gy >= 0 && gy < H;
      float pxx[4], pyy[4], pxy[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int gx = tx0 - GA + px0 + q;
        float ix = 0.0f;
        ix = __builtin_fmaf(-1.0f, w[0][q], ix);
        ix = __builtin_fmaf(1.0f, w[0][q + 2], ix);
        ix = __builtin_fmaf(-2.0f, w[1][q], ix);
        ix = __builtin_fmaf(2.0f, w[1][q + 2], ix);
        ix = __builtin_fmaf(-1.0f, w[2][q], ix);
        ix = __builtin_fmaf(1.0f, w[2][q + 2], ix);
        float iy = 0.0f;
        iy = __builtin_fmaf(-1.0f, w[0][q], iy);
        iy = __builtin_fmaf(-2.0f, w[0][q + 1], iy);
        iy = __builtin_fmaf(-1.0f, w[0][q + 2], iy);
        iy = __builtin_fmaf(1.0f, w[2][q], iy);
        iy = __builtin_fmaf(2.0f, w[2][q + 1], iy);
        iy = __builtin_fmaf(1.0f, w[2][q + 2], iy);
        const bool inside = rowin && gx >= 0 && gx < W;
        pxx[q] = inside ? ix * ix : 0.0f;
        pyy[q] = inside ? iy * iy : 0.0f;
        pxy[q] = inside ? ix * iy : 0.0f;
      }
      *reinterpret_cast<float4*>(&s_prod[0][py][px0]) = make_float4(pxx[0], pxx[1], pxx[2], pxx[3]);
      *reinterpret_cast<float4*>(&s_prod[1][py][px0]) = make_float4(pyy[0], pyy[1], pyy[2], pyy[3]);
      *reinterpret_cast<float4*>(&s_prod[2][py][px0]) = make_float4(pxy[0], pxy[1], pxy[2], pxy[3]);
    }
    __syncthreads();

    if (ABL != 5 && tile + (int)gridDim.x < ntiles) prefetch(tile + gridDim.x);
    // 2. window sums (:67-69): per pixel an fma chain over the KS x KS taps in row-major
    //    order.  acc[pl][q] = (row 2rp, row 2rp+1) at column 4tq+q; LDS row 2rp+i feeds
    //    tap row i of the first and tap row i-1 of the second, so rows 1..KS-1 are packed
    //    fmas and the first / last rows are scalar fmas on one half.
    f32x2 acc[3][4];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[pl][q] = f32x2{0.0f, 0.0f};
    auto load_row = [&](int pl, int i, f32x2 (&v)[NVP / 2]) {
      const float4* row = reinterpret_cast<const float4*>(&s_prod[pl][2 * rp + i][4 * tq]);
#pragma unroll
      for (int c4 = 0; c4 < NV4; ++c4) {
        const float4 t4 = row[c4];
        v[2 * c4] = f32x2{t4.x, t4.y};
        v[2 * c4 + 1] = f32x2{t4.z, t4.w};
      }
    };
    constexpr int NWR = (ABL == 2) ? 1 : (ABL >= 4 ? 0 : KS);  // tap rows
    constexpr int NWC = (ABL == 2) ? 1 : KS;                    // taps per row
    if constexpr (NWR > 0) {
      // LDS row 0: tap row 0 of the first row only
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        f32x2 v[NVP / 2];
        load_row(pl, 0, v);
#pragma unroll
        for (int j = 0; j < NWC; ++j) {
          const float kk = gk[j];
#pragma unroll
          for (int q = 0; q < 4; ++q)
            acc[pl][q].x = __builtin_fmaf(kk, v[(q + j) >> 1][(q + j) & 1], acc[pl][q].x);
        }
      }
#pragma unroll 1
      for (int i = 1; i < NWR; ++i) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          f32x2 v[NVP / 2];
          load_row(pl, i, v);
#pragma unroll
          for (int j = 0; j < NWC; ++j) {
            const f32x2 k2 = f32x2{gk[i * KS + j], gk[(i - 1) * KS + j]};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              if (((q + j) & 1) == 0)
                pk_fma_bcast<0>(acc[pl][q], k2, v[(q + j) >> 1]);
              else
                pk_fma_bcast<1>(acc[pl][q], k2, v[(q + j) >> 1]);
            }
          }
        }
      }
      // LDS row NWR: tap row NWR-1 of the second row only
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        f32x2 v[NVP / 2];
        load_row(pl, NWR, v);
#pragma unroll
        for (int j = 0; j < NWC; ++j) {
          const float kk = gk[(NWR - 1) * KS + j];
#pragma unroll
          for (int q = 0; q < 4; ++q)
            acc[pl][q].y = __builtin_fmaf(kk, v[(q + j) >> 1][(q + j) & 1], acc[pl][q].y);
        }
      }
    }
    // 3. R = det - alpha * trace^2 (:71-74), digit-1 histogram of R; R goes through LDS
    //    (the image tile's space, dead after step 1) so the global store is coalesced rows
    float* sR = &s_img[0][0];  // [kHT_H][SRW]
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int rr = 2 * rp + h;
      const int gy = ty0 + rr;
      float Rq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int gx = tx0 + 4 * tq + q;
        const float sxx = acc[0][q][h], syy = acc[1][q][h], sxy = acc[2][q][h];
        const float t1 = sxx * syy;
        const float t2 = sxy * sxy;
        const float det = t1 - t2;
        const float tr = sxx + syy;
        const float tr2 = tr * tr;
        const float at = alpha * tr2;
        const float Rv = det - at;
        Rq[q] = Rv;
        if (ABL != 1 && gy < H && gx < W) atomicAdd(&s_hist[fkey(Rv) >> (32 - kMedBits1)], 1u);
      }
      *reinterpret_cast<float4*>(&sR[rr * SRW + 4 * tq]) = make_float4(Rq[0], Rq[1], Rq[2], Rq[3]);
    }
    __syncthreads();
    float* Rp = Rout + (int64_t)b * H * W;
    if ((W & 3) == 0 && tx0 + kHT_W <= W) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int e = tid + 256 * k;            // 512 float4 = 32 rows x 16
        const int rr = e >> 4, c4 = (e & 15) * 4;
        if (ty0 + rr < H)
          *reinterpret_cast<float4*>(Rp + (int64_t)(ty0 + rr) * W + tx0 + c4) =
              *reinterpret_cast<const float4*>(&sR[rr * SRW + c4]);
      }
    } else {
      for (int e = tid; e < kHT_H * kHT_W; e += 256) {
        const int rr = e / kHT_W, cc = e - rr * kHT_W;
        if (ty0 + rr < H && tx0 + cc < W) Rp[(int64_t)(ty0 + rr) * W + tx0 + cc] = sR[rr * SRW + cc];
      }
    }
  }  // tile loop
  __syncthreads();
  uint32_t* hg = hist_g + (int64_t)b * kMedBins1;
  for (int i = tid; i < kMedBins1; i += 256) {
    uint32_t c = s_hist[i];
    if (c) atomicAdd(&hg[i], c);
  }
  if (scan.state == nullptr) return;
  // The last workgroup of this plane to finish runs the select scan.  The
  // flushes are device-scope atomics, performed at the memory side: waiting for their
  // acknowledgement (vmcnt) orders them before the arrival count without the L2
  // write-back a __threadfence() costs; the scan reads the histogram with agent-scope
  // atomic loads.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) s_last = atomicAdd(&scan.done[(int64_t)b * kCounterStride], 1ull) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (!s_last) return;
  select_scan_plane(hg, scan.state + b, scan.list_count + (int64_t)b * kCounterStride, (int64_t)H * W,
                    scan.vmin, scan.force_exact, s_red);
}

template <int KS, int ABL = 0>
static void launch_ks(const float* lvl, float* R, uint32_t* hist, int B, int H, int W,
                      const float* gk, float alpha, SelectScan scan, hipStream_t st) {
  int tiles_x = (W + kHT_W - 1) / kHT_W;
  int tiles_y = (H + kHT_H - 1) / kHT_H;
  int ntiles = tiles_x * tiles_y;
  // ~4 resident workgroups per CU over the whole batch; each loops over tiles so the
  // digit histogram is flushed once per workgroup instead of once per tile
  int per_plane = std::max(1, std::min(ntiles, 768 / std::max(B, 1)));
  hipLaunchKernelGGL((k_harris<KS, ABL>), dim3(per_plane, B), dim3(256), 0, st, lvl, R, hist, H, W,
                     tiles_x, ntiles, gk, alpha, scan);
}

void launch_harris(const float* lvl, float* R, uint32_t* hist, int B, int H, int W,
                   const float* d_gauss, int ks, float alpha, SelectScan scan, hipStream_t st) {
  switch (ks) {
    case 1: launch_ks<1>(lvl, R, hist, B, H, W, d_gauss, alpha, scan, st); break;
    case 2: launch_ks<2>(lvl, R, hist, B, H, W, d_gauss, alpha, scan, st); break;
    case 3: launch_ks<3>(lvl, R, hist, B, H, W, d_gauss, alpha, scan, st); break;
    case 4: launch_ks<4>(lvl, R, hist, B, H, W, d_gauss, alpha, scan, st); break;
    case 5: launch_ks<5>(lvl, R, hist, B, H, W, d_gauss, alpha, scan, st); break;
    case 6: launch_ks<6>(lvl, R, hist, B, H, W, d_gauss, alpha, scan, st); break;
    case 7: launch_ks<7>(lvl, R, hist, B, H, W, d_gauss, alpha, scan, st); break;
    case 8: launch_ks<8>(lvl, R, hist, B, H, W, d_gauss, alpha, scan, st); break;
    case 9: launch_ks<9>(lvl, R, hist, B, H, W, d_gauss, alpha, scan, st); break;
    case 11: launch_ks<11>(lvl, R, hist, B, H, W, d_gauss, alpha, scan, st); break;
    case 13: launch_ks<13>(lvl, R, hist, B, H, W, d_gauss, alpha, scan, st); break;
    case 15: launch_ks<15>(lvl, R, hist, B, H, W, d_gauss, alpha, scan, st); break;
    default: break;  // rejected at context creation
  }
}

// Ablation timing (diagnostics): KS = 7 only, returns the mean launch time in ms.
float time_harris_ablation(int abl, const float* lvl, float* R, uint32_t* hist, int B, int H, int W,
                           const float* gk, float alpha, int iters) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const SelectScan none{nullptr, nullptr, nullptr, 0, 0};
  auto run = [&]() {
    switch (abl) {
      case 1: launch_ks<7, 1>(lvl, R, hist, B, H, W, gk, alpha, none, 0); break;
      case 2: launch_ks<7, 2>(lvl, R, hist, B, H, W, gk, alpha, none, 0); break;
      case 3: launch_ks<7, 3>(lvl, R, hist, B, H, W, gk, alpha, none, 0); break;
      case 4: launch_ks<7, 4>(lvl, R, hist, B, H, W, gk, alpha, none, 0); break;
      case 5: launch_ks<7, 5>(lvl, R, hist, B, H, W, gk, alpha, none, 0); break;
      default: launch_ks<7, 0>(lvl, R, hist, B, H, W, gk, alpha, none, 0); break;
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
