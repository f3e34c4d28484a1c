// Diagnostic: issue rate of v_mfma_f32_32x32x16_f16 on gfx950 in the matcher sweep's shape —
// per k-step three MFMAs (hi.hi into one accumulator, hi.lo + lo.hi into another) — at 1 and 2
// waves per SIMD, with the target fragments (a) in registers, (b) read from LDS one k-step
// ahead (two ds_read_b128 per k-step, as k_match_mfma does).  Prints cycles per MFMA per SIMD.
// With rnd = 1 every operand is a pseudo-random f16 of descriptor-like magnitude (full mantissa
// toggling) instead of the few repeated values of rnd = 0: the matcher's operands are random.
// Usage: mfma_rate [iters] [rnd]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ inline _Float16 rnd_h(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return (_Float16)(0.25f + (float)(x & 0xffffff) * (1.0f / 16777216.0f) * 63.0f);  // [0.25, 63.25)
}

template <int MODE>
__global__ void __launch_bounds__(256) k_rate(float* out, int iters, unsigned long long* cyc, int rnd) {
  __shared__ __attribute__((aligned(16))) _Float16 s_t[2][64 * 136];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 2 * 64 * 136; i += 256)
    (&s_t[0][0])[i] = rnd ? rnd_h(i * 2654435761u + 17) : (_Float16)(0.001f * (i & 63));
  __syncthreads();
  h8 q[8], t[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    q[k] = h8{(_Float16)(0.01f * k), 1, 2, 3, 4, 5, 6, (_Float16)lane};
    t[k] = h8{(_Float16)(0.02f * k), 2, 1, 3, 5, 4, 6, (_Float16)lane};
    if (rnd)
      for (int e = 0; e < 8; ++e) {
        q[k][e] = rnd_h((lane * 64 + k * 8 + e) * 40503u + blockIdx.x);
        t[k][e] = rnd_h((lane * 64 + k * 8 + e) * 9973u + 7 * blockIdx.x + 1);
      }
  }
  f32x16 a = {}, x = {};
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        a = __builtin_amdgcn_mfma_f32_32x32x16_f16(t[k], q[k], a, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_32x32x16_f16(t[k], q[(k + 1) & 7], x, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_32x32x16_f16(t[(k + 3) & 7], q[k], x, 0, 0, 0);
      }
    } else {
      const _Float16* base = &s_t[it & 1][(lane & 31) * 136 + 8 * (lane >> 5)];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const h8 thi = *reinterpret_cast<const h8*>(base + 16 * k);
        const h8 tlo = *reinterpret_cast<const h8*>(base + 16 * k + 64 * 136 / 2);
        a = __builtin_amdgcn_mfma_f32_32x32x16_f16(thi, q[k], a, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_32x32x16_f16(thi, q[(k + 1) & 7], x, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_32x32x16_f16(tlo, q[k], x, 0, 0, 0);
      }
    }
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += a[i] + x[i];
  if (s == 1.2345f) out[0] = s;
  if (lane == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = c1 - c0;
}

static int g_rnd = 0;
template <int MODE>
static void launch(dim3 grid, float* out, int iters, unsigned long long* cyc) {
  hipLaunchKernelGGL(k_rate<MODE>, grid, dim3(256), 0, 0, out, iters, cyc, g_rnd);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  g_rnd = argc > 2 ? atoi(argv[2]) : 0;
  printf("operands: %s\n", g_rnd ? "pseudo-random f16" : "repeated values");
  float* out;
  (void)hipMalloc(&out, 4);
  unsigned long long* cyc;
  (void)hipMalloc(&cyc, 8 * 65536);
  static unsigned long long hc[65536];
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const char* names[2] = {"32x32x16 f16, operands in VGPRs", "32x32x16 f16, A from LDS"};
  void (*fns[2])(dim3, float*, int, unsigned long long*) = {launch<0>, launch<1>};
  for (int mode = 0; mode < 2; ++mode)
    for (int wps = 1; wps <= 2; ++wps) {
      dim3 grid(cus * wps);
      fns[mode](grid, out, iters, cyc);
      (void)hipDeviceSynchronize();
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0, 0);
      fns[mode](grid, out, iters, cyc);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      (void)hipMemcpy(hc, cyc, 8 * 4 * grid.x, hipMemcpyDeviceToHost);
      double mc = 0;
      for (unsigned w = 0; w < 4 * grid.x; ++w) mc = hc[w] > mc ? hc[w] : mc;
      const double mhz = mc / (ms * 1e-3) / 1e6;
      const double mfma = (double)iters * 24 * wps;  // per SIMD
      printf("%-34s waves/SIMD %d: %.3f ms at %.0f MHz -> %.1f cycles per MFMA per SIMD, %.0f TFLOP/s (f16)\n",
             names[mode], wps, ms, mhz, ms * 1e-3 * mhz * 1e6 / mfma,
             mfma * cus * 4 * 32768.0 / (ms * 1e-3) / 1e12);
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
    }
  return 0;
}
