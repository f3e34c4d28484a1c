// match.hip — brute-force L2 nearest neighbour + Lowe ratio test
// (NNRatioFeatureMatcher.match_features_ratio_test, NNRatioFeatureMatcher.py:8-60).
//
// Exact restatement of the reference's float32 arithmetic (SURVEY.md §8.1 'distance'):
//   d^2(i,j) = numpy pairwise sum of (a-b)**2 over 128 dims with 8 accumulators:
//              r[j] = sq[j]; r[j] += sq[8i+j] (i = 1..15); ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))
//   dist = sqrt(d^2) (f32), nearest / second nearest by (distance, index),
//   nndr = d1 / d2 if d2 > 0, accept if nndr <= float32(ratio), output sorted by
//   (nndr, row).
// sqrt is monotone, so the two nearest are tracked on d^2 and rooted once per row.
//
// k_match_rows: one 256-thread workgroup = 64 query rows x all target columns, column
// tiles of 64 staged in LDS from a k-major (transposed) copy of the descriptor table so
// both LDS fills and the 4x4 register-tile reads are contiguous.  VALU-bound: 383
// separately rounded f32 ops per pair.
#include "kernels.h"

namespace sfm {

constexpr int kMR = 64;  // query rows per workgroup
constexpr int kMC = 64;  // target columns per LDS tile

// descT[img][k][capP] = desc[img][row][k] (zero padded rows up to capP)
__global__ void __launch_bounds__(256) k_transpose_desc(const float* __restrict__ desc,
                                                        const int32_t* __restrict__ count,
                                                        int64_t cap, int64_t capP,
                                                        float* __restrict__ descT) {
  __shared__ float s_t[64][129];
  const int img = blockIdx.y;
  const int r0 = blockIdx.x * 64;
  const int n = count[img];
  const float* src = desc + (int64_t)img * cap * 128;
  for (int idx = threadIdx.x; idx < 64 * 128; idx += 256) {
    int r = idx >> 7, k = idx & 127;
    s_t[r][k] = (r0 + r < n) ? src[(int64_t)(r0 + r) * 128 + k] : 0.0f;
  }
  __syncthreads();
  float* dst = descT + (int64_t)img * 128 * capP;
  for (int idx = threadIdx.x; idx < 64 * 128; idx += 256) {
    int k = idx >> 6, r = idx & 63;
    dst[(int64_t)k * capP + r0 + r] = s_t[r][k];
  }
}

SFM_DEV void best_update(float s, int col, float& b1, int& j1, float& b2) {
  if (s < b1 || (s == b1 && col < j1)) {
    b2 = b1;
    b1 = s;
    j1 = col;
  } else if (s < b2) {
    b2 = s;
  }
}

__global__ void __launch_bounds__(256) k_match_rows(const float* __restrict__ descT,
                                                    const int32_t* __restrict__ count, int64_t capP,
                                                    const int32_t* __restrict__ pairs, float ratio,
                                                    RowBest* __restrict__ rows_out, int max_rows) {
  __shared__ __attribute__((aligned(16))) float sA[128][kMR];
  __shared__ __attribute__((aligned(16))) float sB[128][kMC];
  const int p = blockIdx.y;
  const int tid = threadIdx.x;
  const int i1 = pairs[2 * p], i2 = pairs[2 * p + 1];
  const int n1 = count[i1], n2 = count[i2];
  const int row0 = blockIdx.x * kMR;
  if (row0 >= n1) return;
  const float* At = descT + (int64_t)i1 * 128 * capP;
  const float* Bt = descT + (int64_t)i2 * 128 * capP;
  for (int idx = tid; idx < 128 * (kMR / 4); idx += 256) {
    int k = idx / (kMR / 4), c4 = idx % (kMR / 4);
    *reinterpret_cast<float4*>(&sA[k][4 * c4]) =
        *reinterpret_cast<const float4*>(At + (int64_t)k * capP + row0 + 4 * c4);
  }
  const int tr = tid >> 4;   // rows 4*tr .. 4*tr+3
  const int tc = tid & 15;   // cols 4*tc .. 4*tc+3
  float b1[4], b2[4];
  int j1[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) { b1[q] = INFINITY; b2[q] = INFINITY; j1[q] = 0x7fffffff; }

  for (int col0 = 0; col0 < n2; col0 += kMC) {
    __syncthreads();
    for (int idx = tid; idx < 128 * (kMC / 4); idx += 256) {
      int k = idx / (kMC / 4), c4 = idx % (kMC / 4);
      *reinterpret_cast<float4*>(&sB[k][4 * c4]) =
          *reinterpret_cast<const float4*>(Bt + (int64_t)k * capP + col0 + 4 * c4);
    }
    __syncthreads();
    // per pair: u0 = (r0+r1) + (r2+r3), u1 = (r4+r5) + (r6+r7), tot = u0 + u1, where
    // r_j = sum over i of sq[8i+j] in i order; slots are produced two at a time.
    float ua[4][4], ub[4][4];
#pragma unroll 1
    for (int jp = 0; jp < 4; ++jp) {
      float re[4][4], ro[4][4];
#pragma unroll
      for (int odd = 0; odd < 2; ++odd) {
#pragma unroll 4
        for (int ii = 0; ii < 16; ++ii) {
          const int k = 8 * ii + 2 * jp + odd;
          float4 a = *reinterpret_cast<const float4*>(&sA[k][4 * tr]);
          float4 bv = *reinterpret_cast<const float4*>(&sB[k][4 * tc]);
          float av[4] = {a.x, a.y, a.z, a.w};
          float bw[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
          for (int ri = 0; ri < 4; ++ri)
#pragma unroll
            for (int ci = 0; ci < 4; ++ci) {
              float d = av[ri] - bw[ci];
              float sq = d * d;
              float& acc = odd ? ro[ri][ci] : re[ri][ci];
              if (ii == 0) acc = sq;
              else acc = acc + sq;
            }
        }
      }
#pragma unroll
      for (int ri = 0; ri < 4; ++ri)
#pragma unroll
        for (int ci = 0; ci < 4; ++ci) {
          const float t = re[ri][ci] + ro[ri][ci];   // t01 / t23 / t45 / t67
          if (jp == 0) ua[ri][ci] = t;
          else if (jp == 1) ua[ri][ci] = ua[ri][ci] + t;
          else if (jp == 2) ub[ri][ci] = t;
          else ub[ri][ci] = ub[ri][ci] + t;
        }
    }
    float tot[4][4];
#pragma unroll
    for (int ri = 0; ri < 4; ++ri)
#pragma unroll
      for (int ci = 0; ci < 4; ++ci) tot[ri][ci] = ua[ri][ci] + ub[ri][ci];
#pragma unroll
    for (int ci = 0; ci < 4; ++ci) {
      const int col = col0 + 4 * tc + ci;
      if (col < n2) {
#pragma unroll
        for (int ri = 0; ri < 4; ++ri) best_update(tot[ri][ci], col, b1[ri], j1[ri], b2[ri]);
      }
    }
  }
  // reduce over the 16 lanes sharing the same rows
#pragma unroll
  for (int ri = 0; ri < 4; ++ri) {
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) {
      float ob1 = __shfl_xor(b1[ri], off, 16);
      float ob2 = __shfl_xor(b2[ri], off, 16);
      int oj1 = __shfl_xor(j1[ri], off, 16);
      if (ob1 < b1[ri] || (ob1 == b1[ri] && oj1 < j1[ri])) {
        b2[ri] = fminf(b1[ri], ob2);
        b1[ri] = ob1;
        j1[ri] = oj1;
      } else {
        b2[ri] = fminf(b2[ri], ob1);
      }
    }
  }
  if (tc == 0) {
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int row = row0 + 4 * tr + ri;
      if (row < n1) {
        RowBest rb;
        rb.col = -1;
        rb.nndr = 0.0f;
        float d1 = sqrtf(b1[ri]), d2 = sqrtf(b2[ri]);
        if (d2 > 0.0f) {
          float nndr = d1 / d2;
          if (nndr <= ratio) { rb.col = j1[ri]; rb.nndr = nndr; }
        }
        rows_out[(int64_t)p * max_rows + row] = rb;
      }
    }
  }
}

__global__ void __launch_bounds__(1024) k_match_compact(const RowBest* __restrict__ rows,
                                                        const int32_t* __restrict__ count,
                                                        const int32_t* __restrict__ pairs,
                                                        int max_rows, int64_t cap,
                                                        int32_t* __restrict__ matches,
                                                        float* __restrict__ conf,
                                                        int32_t* __restrict__ nmatch,
                                                        int* __restrict__ reset_counter) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
  // the MFMA matcher's overflow counter, read by k_match_overflow just before this kernel:
  // zeroed here for the next call (no separate memset launch on the stream)
  if (reset_counter != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *reset_counter = 0;
  uint64_t* s_k = reinterpret_cast<uint64_t*>(s_raw);
  __shared__ uint32_t s_n;
  const int p = blockIdx.x;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int n1 = count[pairs[2 * p]], n2 = count[pairs[2 * p + 1]];
  if (n1 >= 1 && n2 < 2) {  // the reference raises IndexError (:42)
    if (tid == 0) nmatch[p] = -1;
    return;
  }
  if (tid == 0) s_n = 0u;
  __syncthreads();
  const RowBest* rp = rows + (int64_t)p * max_rows;
  for (int r = tid; r < n1; r += nt) {
    RowBest rb = rp[r];
    if (rb.col >= 0) s_k[atomicAdd(&s_n, 1u)] = ((uint64_t)fbits(rb.nndr) << 32) | (uint32_t)r;
  }
  __syncthreads();
  const int m = (int)s_n;
  sort_keys_u64(s_k, m);  // (nndr, row): distinct keys
  for (int i = tid; i < m; i += nt) {
    uint64_t key = s_k[i];
    int r = (int)(uint32_t)key;
    int64_t o = (int64_t)p * cap + i;
    matches[2 * o] = r;
    matches[2 * o + 1] = rp[r].col;
    conf[o] = ffrom((uint32_t)(key >> 32));
  }
  if (tid == 0) nmatch[p] = m;
}

void launch_transpose_desc(const float* desc, const int32_t* count, int nimg, int64_t cap,
                           int64_t capP, float* descT, hipStream_t st) {
  hipLaunchKernelGGL(k_transpose_desc, dim3((unsigned)(capP / 64), nimg), dim3(256), 0, st, desc, count,
                     cap, capP, descT);
}

size_t match_compact_lds(int max_rows) {
  int P = 1;
  while (P < max_rows) P <<= 1;
  return (size_t)P * 8;
}

void init_match_attributes(int max_rows) {
  (void)hipFuncSetAttribute((const void*)k_match_compact, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)match_compact_lds(max_rows));
}

void launch_match_rows(const float* descT, const int32_t* count, int64_t capP, const int32_t* pairs,
                       int P, float ratio, RowBest* rows, int max_rows, hipStream_t st) {
  hipLaunchKernelGGL(k_match_rows, dim3((max_rows + kMR - 1) / kMR, P), dim3(256), 0, st, descT, count,
                     capP, pairs, ratio, rows, max_rows);
}

void launch_match_compact(const RowBest* rows, const int32_t* count, const int32_t* pairs, int P,
                          int max_rows, int64_t cap, int32_t* matches, float* conf, int32_t* nmatch,
                          int* reset_counter, hipStream_t st) {
  hipLaunchKernelGGL(k_match_compact, dim3(P), dim3(1024), match_compact_lds(max_rows), st, rows, count,
                     pairs, max_rows, cap, matches, conf, nmatch, reset_counter);
}

}  // namespace sfm
