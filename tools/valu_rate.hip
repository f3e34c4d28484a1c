// Diagnostic: VALU issue rate of v_pk_fma_f32 (op_sel broadcast, as k_harris uses it) and
// v_fmac_f32 on gfx950 at 1 / 2 / 3 / 4 waves per SIMD.  Each wave runs ITERS x 16
// independent instructions (16 accumulators); the time of the launch gives cycles per
// instruction per SIMD.  Usage: valu_rate [iters]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ void __launch_bounds__(256) k_rate(float* out, int iters, float s, unsigned long long* cyc) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  f32x2 a[16];
  float b[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    a[i] = f32x2{s * i, s + i};
    b[i] = s * (i + 1);
  }
  f32x2 k = {s, s * 0.5f};
  f32x2 v = {s * 3.0f, s * 0.25f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if constexpr (MODE == 0)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(a[i]) : "v"(k), "v"(v));
      else if constexpr (MODE == 1)
        asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(b[i]) : "v"(k.x), "v"(v.y));
      else
        asm volatile("v_pk_mul_f32 %0, %1, %2" : "+v"(a[i]) : "v"(k), "v"(v));
    }
  }
  float acc = 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc += a[i].x + a[i].y + b[i];
  if (acc == 1.2345f) out[0] = acc;
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  float* out;
  hipMalloc(&out, 4);
  unsigned long long* cyc;
  hipMalloc(&cyc, 8 * 4096);
  unsigned long long hc[4096];
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const double clk = p.clockRate * 1e3;  // Hz (max)
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[3] = {"v_pk_fma_f32 (op_sel bcast)", "v_fmac_f32", "v_pk_mul_f32"};
  for (int mode = 0; mode < 3; ++mode)
    for (int wps = 1; wps <= 4; ++wps) {
      // one 256-thread workgroup = one wave per SIMD of a CU
      dim3 grid(cus * wps);
      auto launch = [&]() {
        if (mode == 0) hipLaunchKernelGGL(k_rate<0>, grid, dim3(256), 0, 0, out, iters, 1.0f, cyc);
        else if (mode == 1) hipLaunchKernelGGL(k_rate<1>, grid, dim3(256), 0, 0, out, iters, 1.0f, cyc);
        else hipLaunchKernelGGL(k_rate<2>, grid, dim3(256), 0, 0, out, iters, 1.0f, cyc);
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(e0, 0);
      launch();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double insts_per_simd = (double)iters * 16 * wps;
      hipMemcpy(hc, cyc, 8 * grid.x, hipMemcpyDeviceToHost);
      double mc = 0;
      for (unsigned i = 0; i < grid.x; ++i) mc = hc[i] > mc ? hc[i] : mc;
      printf("%-28s waves/SIMD %d: %.3f ms, %.2f cyc/instr/SIMD (s_memtime, max over WGs), clock %.0f MHz\n",
             names[mode], wps, ms, mc / insts_per_simd, mc / (ms * 1e-3) / 1e6);
    }
  return 0;
}
