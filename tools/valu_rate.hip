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
  float kv[16];
  f32x2 pv[8];
#pragma unroll
  for (int i = 0; i < 16; ++i) kv[i] = s * (0.5f + i);
#pragma unroll
  for (int i = 0; i < 8; ++i) pv[i] = f32x2{s * i, s - i};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if constexpr (MODE == 0)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(a[i]) : "v"(k), "v"(v));
      else if constexpr (MODE == 1)
        asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(b[i]) : "v"(k.x), "v"(v.y));
      else if constexpr (MODE == 2)
        asm volatile("v_pk_mul_f32 %0, %1, %2" : "+v"(a[i]) : "v"(k), "v"(v));
      else if constexpr (MODE == 3)  // distinct operands per instruction
        asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(b[i]) : "v"(kv[i]), "v"(kv[(i + 5) & 15]));
      else  // pk_fma, distinct operands
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(a[i]) : "v"(pv[i & 7]), "v"(pv[(i + 3) & 7]));
    }
  }
  float acc = 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc += a[i].x + a[i].y + b[i];
  if (acc == 1.2345f) out[0] = acc;
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  // HW_ID: wave slot [3:0], SIMD [5:4], CU [11:8], SH [12], SE [15:13] (gfx9 layout)
  const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
  if ((threadIdx.x & 63) == 0) {
    cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6))] = c1 - c0;
    cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6)) + 1] = hw;
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  float* out;
  hipMalloc(&out, 4);
  unsigned long long* cyc;
  hipMalloc(&cyc, 8 * 65536);
  static unsigned long long hc[65536];
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const double clk = p.clockRate * 1e3;  // Hz (max)
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[5] = {"v_pk_fma_f32 (op_sel bcast)", "v_fmac_f32", "v_pk_mul_f32", "v_fmac_f32 (distinct ops)",
                          "v_pk_fma_f32 (distinct ops)"};
  for (int mode = 0; mode < 5; ++mode)
    for (int wps = 1; wps <= 4; ++wps) {
      // one 256-thread workgroup = one wave per SIMD of a CU
      dim3 grid(cus * wps);
      auto launch = [&]() {
        if (mode == 0) hipLaunchKernelGGL(k_rate<0>, grid, dim3(256), 0, 0, out, iters, 1.0f, cyc);
        else if (mode == 1) hipLaunchKernelGGL(k_rate<1>, grid, dim3(256), 0, 0, out, iters, 1.0f, cyc);
        else if (mode == 2) hipLaunchKernelGGL(k_rate<2>, grid, dim3(256), 0, 0, out, iters, 1.0f, cyc);
        else if (mode == 3) hipLaunchKernelGGL(k_rate<3>, grid, dim3(256), 0, 0, out, iters, 1.0f, cyc);
        else hipLaunchKernelGGL(k_rate<4>, grid, dim3(256), 0, 0, out, iters, 1.0f, cyc);
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
      hipMemcpy(hc, cyc, 8 * 2 * 4 * grid.x, hipMemcpyDeviceToHost);
      double mc = 0;
      // waves per (SE, SH, CU, SIMD) slot
      static int occ[1 << 16];
      for (int i = 0; i < (1 << 16); ++i) occ[i] = 0;
      int maxocc = 0;
      for (unsigned w = 0; w < 4 * grid.x; ++w) {
        mc = hc[2 * w] > mc ? hc[2 * w] : mc;
        const unsigned hw = (unsigned)hc[2 * w + 1];
        const unsigned key = (hw >> 4) & 0xfff3u;  // SIMD, CU, SH, SE (drop pipe bits 7:6)
        maxocc = ++occ[key] > maxocc ? occ[key] : maxocc;
      }
      (void)insts_per_simd;
      printf("%-28s WGs/CU %d: %.3f ms, max waves on one SIMD %d, %.2f cyc per instruction per SIMD at that occupancy, clock %.0f MHz\n",
             names[mode], wps, ms, maxocc, mc / ((double)iters * 16 * maxocc), mc / (ms * 1e-3) / 1e6);
    }
  return 0;
}
