// mfma_f32_probe.hip — the f32-input MFMA forms a Harris window could run on (gfx950):
//   1. lane maps of v_mfma_f32_4x4x1_16b_f32 (A, B, D), from exact integer data;
//   2. numerics: a K=1 chain of N steps against a host fmaf chain, bit for bit (random
//      signs, zeros in B, subnormal-range products, C = +0 start);
//   3. issue rate (shader cycles per instruction per wave) of 4x4x1_16b, 16x16x1_4b,
//      16x16x4 with 1 and 2 waves per SIMD;
//   4. co-issue: 4 waves of MFMA and 4 waves of v_pk_fma_f32 in one 512-thread workgroup,
//      each group's cycles alone and together.
// Output: one text report on stdout.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>
#include <utility>
#include <vector>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// 1. one MFMA, C = 0, A and B from the host: D (4 regs per lane)
__global__ void k_layout(const float* A, const float* B, float* D) {
  const int l = threadIdx.x;
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(A[l], B[l], c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = c[r];
}

// 1b. A broadcast: cbsz = 4 (one block's A to all 16), abid = k
template <int K>
__global__ void k_layout_bcast(const float* A, const float* B, float* D) {
  const int l = threadIdx.x;
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(A[l], B[l], c, 4, K, 0);
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = c[r];
}

// 2. N chained steps: D = mfma(A[s], B[s], D), D0 = +0
__global__ void k_chain(const float* A, const float* B, float* D, int N) {
  const int l = threadIdx.x;
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < N; ++s) c = __builtin_amdgcn_mfma_f32_4x4x1f32(A[s * 64 + l], B[s * 64 + l], c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = c[r];
}

// 3. rate: NACC independent accumulators, ITER rounds; per-wave cycles via s_memtime
template <int FORM, int NACC>
__global__ void k_rate(float* out, long long* cyc, int iters) {
  const int l = threadIdx.x & 63;
  float a = 1.0f + l * 1e-3f, b = 0.5f - l * 1e-4f;
  f32x4 acc4[NACC];
  for (int i = 0; i < NACC; ++i) acc4[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      if constexpr (FORM == 0) acc4[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc4[i], 0, 0, 0);
      if constexpr (FORM == 1) acc4[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc4[i], 0, 0, 0);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc4[i][0] + acc4[i][1] + acc4[i][2] + acc4[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (l == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

// 4. co-issue: waves < nm run MFMA (4x4x1, 8 accumulators), the others v_pk_fma_f32 chains
__global__ void __launch_bounds__(512) k_coissue(float* out, long long* cyc, int iters_m, int iters_v, int nm) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float a = 1.0f + l * 1e-3f, b = 0.5f - l * 1e-4f;
  float s = 0.f;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (w < nm) {
    f32x4 acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters_m; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[i], 0, 0, 0);
    }
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][3];
  } else {
    f32x2 acc[8];
    const f32x2 k = {a, b}, v = {b, a};
    for (int i = 0; i < 8; ++i) acc[i] = f32x2{0.f, 0.f};
    for (int it = 0; it < iters_v; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(k), "v"(v));
    }
    for (int i = 0; i < 8; ++i) s += acc[i].x + acc[i].y;
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (l == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

template <int... I, class F>
__device__ __forceinline__ void sfor_impl(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(std::make_integer_sequence<int, N>{}, f);
}

// 5. the Harris window's inner loop in isolation: per "row" 22 columns, 4 strips x 3 planes
// x 10 steps = 120 MFMAs on 12 accumulators.  V: 0 = MFMA only (B constant), 1 = + cbsz/abid
// tap broadcast, 2 = + v_mul products per column (registers), 3 = + LDS row reads (b128)
template <int V, int PARTNER = 0>
__global__ void __launch_bounds__(512) k_win(float* out, long long* cyc, int rows) {
  __shared__ float s_g[2][72][76];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 2 * 72 * 76; i += blockDim.x) (&s_g[0][0][0])[i] = 1.0f + 1e-3f * (i % 97);
  __syncthreads();
  if (w >= 4) {  // partner waves: scalar v_fma_f32 chains (PARTNER iterations of 16 fmas)
    float a[16];
    for (int i = 0; i < 16; ++i) a[i] = 1e-3f * (i + l);
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < PARTNER; ++r)
#pragma unroll
      for (int i = 0; i < 16; ++i) a[i] = __builtin_fmaf(a[i], 0.999f, 1e-4f);
    const long long t1 = __builtin_amdgcn_s_memtime();
    float sum = 0.f;
    for (int i = 0; i < 16; ++i) sum += a[i];
    out[blockIdx.x * 512 + threadIdx.x] = sum;
    if (l == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
    return;
  }
  float tapV[5];
  for (int v = 0; v < 5; ++v) tapV[v] = 0.01f * (v + 1) + 1e-4f * l;
  f32x4 acc[4][3];
  for (int q = 0; q < 4; ++q)
    for (int p = 0; p < 3; ++p) acc[q][p] = f32x4{0.f, 0.f, 0.f, 0.f};
  float X[24], Y[24];
  for (int c = 0; c < 24; ++c) X[c] = 1.0f + c * 1e-3f + l * 1e-5f, Y[c] = 0.5f + c * 1e-3f;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < rows; ++r) {
    if constexpr (V >= 3) {
      const float4* rx = reinterpret_cast<const float4*>(&s_g[0][(l + r) % 8 + l][16 * w]);
      const float4* ry = reinterpret_cast<const float4*>(&s_g[1][(l + r) % 8 + l][16 * w]);
#pragma unroll
      for (int c4 = 0; c4 < 6; ++c4) {
        const float4 a = rx[c4], b = ry[c4];
        X[4 * c4] = a.x, X[4 * c4 + 1] = a.y, X[4 * c4 + 2] = a.z, X[4 * c4 + 3] = a.w;
        Y[4 * c4] = b.x, Y[4 * c4 + 1] = b.y, Y[4 * c4 + 2] = b.z, Y[4 * c4 + 3] = b.w;
      }
    }
    float pxx[22], pyy[22], pxy[22];
#pragma unroll
    for (int c = 0; c < 22; ++c) {
      if constexpr (V >= 2) pxx[c] = X[c] * X[c], pyy[c] = Y[c] * Y[c], pxy[c] = X[c] * Y[c];
      else pxx[c] = X[c], pyy[c] = Y[c], pxy[c] = X[0];
    }
    sfor<10>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if constexpr (V >= 1) {
          acc[q][0] = __builtin_amdgcn_mfma_f32_4x4x1f32(tapV[s / 4], pxx[4 * q + s], acc[q][0], 4, s % 4, 0);
          acc[q][1] = __builtin_amdgcn_mfma_f32_4x4x1f32(tapV[s / 4], pyy[4 * q + s], acc[q][1], 4, s % 4, 0);
          acc[q][2] = __builtin_amdgcn_mfma_f32_4x4x1f32(tapV[s / 4], pxy[4 * q + s], acc[q][2], 4, s % 4, 0);
        } else {
          acc[q][0] = __builtin_amdgcn_mfma_f32_4x4x1f32(tapV[s / 4], pxx[4 * q + s], acc[q][0], 0, 0, 0);
          acc[q][1] = __builtin_amdgcn_mfma_f32_4x4x1f32(tapV[s / 4], pyy[4 * q + s], acc[q][1], 0, 0, 0);
          acc[q][2] = __builtin_amdgcn_mfma_f32_4x4x1f32(tapV[s / 4], pxy[4 * q + s], acc[q][2], 0, 0, 0);
        }
      }
    });
    if constexpr (V < 3) {  // keep the row data live and changing without memory
#pragma unroll
      for (int c = 0; c < 24; ++c) X[c] = __builtin_amdgcn_fmed3f(X[c], Y[c], 2.0f);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float sum = 0.f;
  for (int q = 0; q < 4; ++q)
    for (int p = 0; p < 3; ++p) sum += acc[q][p][0] + acc[q][p][3];
  out[blockIdx.x * 512 + threadIdx.x] = sum;
  if (l == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

static unsigned long long rng = 88172645463325252ull;
static unsigned rnd() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (unsigned)(rng >> 11);
}
static float rndf() {
  // mixed magnitudes, signs, exact zeros, subnormal-range values
  unsigned r = rnd();
  switch (r % 8) {
    case 0: return 0.0f;
    case 1: return ldexpf((float)(int)(rnd() % 2000000) - 1e6f, -150 + (int)(rnd() % 20));
    default: return ((float)(int)(rnd() & 0xffffff) - 8388608.0f) * ldexpf(1.0f, -(int)(rnd() % 40));
  }
}

int main() {
  // 1. layout
  std::vector<float> hA(64), hB(64), hD(256), hD2(256);
  float *dA, *dB, *dD;
  CK(hipMalloc(&dA, 64 * 4096 * 4));
  CK(hipMalloc(&dB, 64 * 4096 * 4));
  CK(hipMalloc(&dD, 256 * 4));
  for (int l = 0; l < 64; ++l) {
    hA[l] = (float)(l + 1);
    hB[l] = 1.0f;
  }
  CK(hipMemcpy(dA, hA.data(), 256, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB.data(), 256, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  CK(hipMemcpy(hD.data(), dD, 1024, hipMemcpyDeviceToHost));
  for (int l = 0; l < 64; ++l) {
    hA[l] = 1.0f;
    hB[l] = (float)(l + 1);
  }
  CK(hipMemcpy(dA, hA.data(), 256, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB.data(), 256, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  CK(hipMemcpy(hD2.data(), dD, 1024, hipMemcpyDeviceToHost));
  printf("== 1. v_mfma_f32_4x4x1_16b_f32 lane map: D[lane][reg] = A[lane a] * B[lane b]\n");
  int ok_map = 1;
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int r = 0; r < 4; ++r) {
      const int la = (int)hD[l * 4 + r] - 1, lb = (int)hD2[l * 4 + r] - 1;
      printf(" r%d=(a%2d,b%2d)", r, la, lb);
      // expected: block = l/4, D row i = reg, column j = l%4: A lane 4*block + r, B lane l
      ok_map &= (la == 4 * (l / 4) + r) && (lb == l);
    }
    printf("\n");
  }
  printf("map D[lane 4b+j][reg i] = A[lane 4b+i] * B[lane 4b+j]: %s\n", ok_map ? "yes" : "NO");
  // broadcast: A = lane + 1, B = 1 -> D = (A lane) + 1
  for (int l = 0; l < 64; ++l) {
    hA[l] = (float)(l + 1);
    hB[l] = 1.0f;
  }
  CK(hipMemcpy(dA, hA.data(), 256, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB.data(), 256, hipMemcpyHostToDevice));
  int ok_b = 1;
  auto bc = [&](auto kc) {
    constexpr int K = decltype(kc)::value;
    hipLaunchKernelGGL(k_layout_bcast<K>, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    CK(hipMemcpy(hD.data(), dD, 1024, hipMemcpyDeviceToHost));
    int ok = 1;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) ok &= ((int)hD[l * 4 + r] - 1 == 4 * K + r);
    printf("cbsz 4 abid %2d: D[lane][reg i] = A[lane 4*abid + i] for every lane: %s (lane 0: %g %g %g %g, lane 63: %g %g %g %g)\n", K,
           ok ? "yes" : "NO", hD[0], hD[1], hD[2], hD[3], hD[252], hD[253], hD[254], hD[255]);
    ok_b &= ok;
  };
  bc(std::integral_constant<int, 0>{});
  bc(std::integral_constant<int, 1>{});
  bc(std::integral_constant<int, 7>{});
  bc(std::integral_constant<int, 15>{});
  printf("A broadcast (cbsz 4): %s\n", ok_b ? "yes" : "NO");

  // 2. numerics: chains of N steps vs host fmaf
  const int N = 4096;
  std::vector<float> cA(64 * N), cB(64 * N), cD(256);
  for (int i = 0; i < 64 * N; ++i) {
    cA[i] = rndf();
    cB[i] = (rnd() % 4 == 0) ? 0.0f : rndf();
  }
  CK(hipMemcpy(dA, cA.data(), 64 * N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, cB.data(), 64 * N * 4, hipMemcpyHostToDevice));
  int bad = 0, negz = 0;
  for (int n : {1, 2, 7, 49, 70, 4096}) {
    hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, dA, dB, dD, n);
    CK(hipMemcpy(cD.data(), dD, 1024, hipMemcpyDeviceToHost));
    int badn = 0;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) {
        const int la = 4 * (l / 4) + r, lb = l;
        float acc = 0.0f;
        for (int s = 0; s < n; ++s) acc = fmaf(cA[s * 64 + la], cB[s * 64 + lb], acc);
        unsigned u1, u2;
        memcpy(&u1, &acc, 4);
        memcpy(&u2, &cD[l * 4 + r], 4);
        if (u1 != u2) {
          if (badn < 4) printf("  n=%d lane %d reg %d: host %a (%08x) mfma %a (%08x)\n", n, l, r, acc, u1, cD[l * 4 + r], u2);
          ++badn;
        }
        negz += (u2 == 0x80000000u);
      }
    printf("== 2. chain of %4d K=1 steps: %d of 256 results differ from the host fmaf chain\n", n, badn);
    bad += badn;
  }
  printf("numerics: %s (results equal to -0: %d)\n", bad ? "DIFFER" : "bitwise fmaf chain", negz);

  // 3. rate
  float* dout;
  long long* dcyc;
  CK(hipMalloc(&dout, 256 * 1024 * 4));
  CK(hipMalloc(&dcyc, 256 * 16 * 8));
  std::vector<long long> cyc(256 * 16);
  auto report = [&](const char* name, int nwaves, double per) {
    CK(hipMemcpy(cyc.data(), dcyc, nwaves * 8, hipMemcpyDeviceToHost));
    double s = 0, mx = 0;
    for (int i = 0; i < nwaves; ++i) {
      s += (double)cyc[i];
      mx = fmax(mx, (double)cyc[i]);
    }
    // s_memtime counts at the 100 MHz reference on some parts: report raw and per-op
    printf("%-44s mean %.0f max %.0f ticks per wave, %.3f ticks per instruction\n", name, s / nwaves, mx, s / nwaves / per);
  };
  const int it = 4096;
  for (int wpc : {4, 8}) {  // waves per CU: 1 or 2 per SIMD
    hipLaunchKernelGGL((k_rate<0, 8>), dim3(256), dim3(64 * wpc), 0, 0, dout, dcyc, it);
    CK(hipDeviceSynchronize());
    char nm[80];
    snprintf(nm, sizeof nm, "3. 4x4x1_16b, 8 acc, %d waves/SIMD", wpc / 4);
    report(nm, 256 * wpc, it * 8.0);
    hipLaunchKernelGGL((k_rate<1, 8>), dim3(256), dim3(64 * wpc), 0, 0, dout, dcyc, it);
    CK(hipDeviceSynchronize());
    snprintf(nm, sizeof nm, "3. 16x16x4, 8 acc, %d waves/SIMD", wpc / 4);
    report(nm, 256 * wpc, it * 8.0);
  }
  // wall-clock rate over the whole chip for 4x4x1 (events)
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int form = 0; form < 2; ++form) {
    const int blocks = 256 * 4, threads = 256;
    CK(hipEventRecord(e0));
    if (form == 0) hipLaunchKernelGGL((k_rate<0, 8>), dim3(blocks), dim3(threads), 0, 0, dout, dcyc, it);
    else hipLaunchKernelGGL((k_rate<1, 8>), dim3(blocks), dim3(threads), 0, 0, dout, dcyc, it);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double macs = (double)blocks * (threads / 64) * it * 8 * (form == 0 ? 256.0 : 1024.0);
    printf("3. %s chip-wide: %.3f ms, %.1f TFLOP/s\n", form == 0 ? "4x4x1_16b" : "16x16x4 ", ms, 2 * macs / ms / 1e9);
  }

  // 4. co-issue (one 512-thread workgroup per CU; waves 0-3 MFMA, 4-7 packed VALU)
  const int im = 2048, iv = 4096;
  for (int mode = 0; mode < 3; ++mode) {
    // mode 0: MFMA waves only (nm = 8 -> all MFMA? no: run 4 MFMA waves + 4 idle VALU waves with 0 iters)
    const int ivv = mode == 0 ? 0 : iv, imm = mode == 1 ? 0 : im;
    hipLaunchKernelGGL(k_coissue, dim3(256), dim3(512), 0, 0, dout, dcyc, imm, ivv, 4);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(cyc.data(), dcyc, 256 * 8 * 8, hipMemcpyDeviceToHost));
    double sm = 0, sv = 0;
    for (int b = 0; b < 256; ++b)
      for (int w = 0; w < 8; ++w) (w < 4 ? sm : sv) += (double)cyc[b * 8 + w];
    printf("4. co-issue %s: MFMA waves %.0f ticks (%d x 8 MFMA), VALU waves %.0f ticks (%d x 8 v_pk_fma_f32)\n",
           mode == 0 ? "MFMA alone" : mode == 1 ? "VALU alone" : "both      ", sm / 1024, imm, sv / 1024, ivv);
  }
  // 5. window loop in isolation: (a) 2 workgroups of 4 MFMA waves per CU (2 MFMA waves per
  // SIMD), (b) 1 per CU (1 MFMA wave per SIMD), (c) 1 per CU + 4 scalar-VALU partner waves
  CK(hipMalloc(&dout, 1024 * 512 * 4));
  CK(hipFree(dcyc));
  CK(hipMalloc(&dcyc, 1024 * 8 * 8));
  cyc.resize(1024 * 8);
  auto win = [&](const char* name, auto kern, int blocks, int threads, int rows) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, dout, dcyc, rows);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemcpy(cyc.data(), dcyc, blocks * 8 * 8, hipMemcpyDeviceToHost));
    double sc = 0, sp = 0;
    int np = 0;
    for (int b = 0; b < blocks; ++b)
      for (int w = 0; w < 8; ++w) {
        if (w < 4) sc += (double)cyc[b * 8 + w];
        else if (threads > 256) sp += (double)cyc[b * 8 + w], ++np;
      }
    const double mf = (double)rows * 120;
    const double per_simd = mf * blocks * 4 / 1024;
    printf("5. %-44s %.3f ms, %.2f ticks per MFMA per MFMA wave, %.2f ns per MFMA per SIMD; partner %.0f ticks\n", name, ms,
           sc / (blocks * 4) / mf, ms * 1e6 / per_simd, np ? sp / np : 0.0);
  };
  win("V=0 MFMA only, 2 MFMA waves/SIMD", k_win<0>, 512, 256, 512);
  win("V=3 LDS+products, 2 MFMA waves/SIMD", k_win<3>, 512, 256, 512);
  win("V=0 MFMA only, 1 MFMA wave/SIMD", k_win<0>, 256, 256, 1024);
  win("V=3 LDS+products, 1 MFMA wave/SIMD", k_win<3>, 256, 256, 1024);
  win("V=3, 1 MFMA wave/SIMD + idle partner", k_win<3, 0>, 256, 512, 1024);
  win("V=3, 1 MFMA wave/SIMD + scalar-fma partner", k_win<3, 4096>, 256, 512, 1024);
  win("partner alone (V=3 rows 0)", k_win<3, 4096>, 256, 512, 0);
  return bad ? 1 : 0;
}
