// pk_mfma_hazard.hip — which packed-FP32 VALU instructions give different results while an
// MFMA from another wave runs on the same SIMD (gfx950)?  The minimal form of the
// co-residency finding (tools/coresidency_repro.hip, DESIGN.md §7 "Co-residency").
//
// k_ops<OP>: 256-thread workgroups; every lane runs 8 independent register chains of one
// instruction form (inline asm, so the instruction is exactly the one named) and stores its
// 16 floats.  Run alone, then right after a registers-only MFMA co-runner (one 256-thread
// workgroup per CU, v_mfma_f32_32x32x16_f16 back to back) was launched on another stream;
// the outputs are compared bit for bit, by lane (0-63) and half (.x / .y).
//
// OP: 0 v_pk_fma_f32 op_sel_hi:[1,0,1] (src1's low half broadcast: Harris's window form)
//     1 v_pk_fma_f32 op_sel:[0,1,0] op_sel_hi:[1,1,1] (src1's high half broadcast)
//     2 v_pk_fma_f32 (no op_sel)
//     3 v_pk_mul_f32
//     4 v_pk_add_f32
//     5 v_fma_f32 pairs (scalar control)
//     6 v_pk_fma_f32 op_sel:[1,0,0] op_sel_hi:[1,1,1] (src0's high half broadcast)
//     7 v_pk_fma_f32 op_sel:[0,1,0] op_sel_hi:[1,0,1] (src1's halves swapped)
//     8 v_pk_mul_f32 op_sel:[0,1] op_sel_hi:[1,1] (src1's high half broadcast)
//     9 v_pk_add_f32 op_sel:[0,1] op_sel_hi:[1,1] (src1's high half broadcast)
//    10 v_pk_mul_f32 op_sel_hi:[1,0] (src1's low half broadcast)
//    11 v_pk_fma_f32 op_sel:[0,0,1] op_sel_hi:[1,1,1] (src2's high half broadcast)
//    12 v_pk_mov_b32 op_sel:[1,0] (src0's high half into the low result), then v_pk_add_f32
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int OP>
__device__ __forceinline__ void step(f32x2& a, f32x2 k, f32x2 v) {
  if constexpr (OP == 0) asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(a) : "v"(k), "v"(v));
  if constexpr (OP == 1)
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "+v"(a) : "v"(k), "v"(v));
  if constexpr (OP == 2) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(k), "v"(v));
  if constexpr (OP == 3) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a) : "v"(k));
  if constexpr (OP == 4) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a) : "v"(v));
  if constexpr (OP == 6)
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(a) : "v"(v), "v"(k));
  if constexpr (OP == 7)
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,0,1]" : "+v"(a) : "v"(k), "v"(v));
  if constexpr (OP == 8) asm volatile("v_pk_mul_f32 %0, %0, %1 op_sel:[0,1] op_sel_hi:[1,1]" : "+v"(a) : "v"(k));
  if constexpr (OP == 9) asm volatile("v_pk_add_f32 %0, %0, %1 op_sel:[0,1] op_sel_hi:[1,1]" : "+v"(a) : "v"(v));
  if constexpr (OP == 10) asm volatile("v_pk_mul_f32 %0, %0, %1 op_sel_hi:[1,0]" : "+v"(a) : "v"(k));
  if constexpr (OP == 11) {
    f32x2 t = a;
    asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,1] op_sel_hi:[1,1,1]" : "=v"(a) : "v"(k), "v"(v), "v"(t));
    a.x = a.x * 0.5f;  // keep the chain bounded
  }
  if constexpr (OP == 12) {
    f32x2 t;
    asm volatile("v_pk_mov_b32 %0, %1, %1 op_sel:[1,0]" : "=v"(t) : "v"(a));
    asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(a) : "v"(t), "v"(v));
  }
  if constexpr (OP == 5) {
    asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a.x) : "v"(k.x), "v"(v.x));
    asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a.y) : "v"(k.y), "v"(v.y));
  }
}

template <int OP>
__global__ void __launch_bounds__(256) k_ops(int iters, float* out) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  f32x2 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f32x2{1e-3f * (t % 977) + i, 2e-3f * (t % 613) - i};
  // products stay near 1 (mul), sums grow slowly (add: +1e-7 per step), fmas converge
  const bool mul = OP == 3 || OP == 8 || OP == 10, add = OP == 4 || OP == 9 || OP == 12;
  const f32x2 k = mul ? f32x2{0.9999999f, 1.0000001f} : f32x2{0.5f, 0.25f};
  const f32x2 v = add ? f32x2{1e-7f, -1e-7f} : f32x2{0.75f, 1.5f};
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) step<OP>(acc[i], k, v);
  for (int i = 0; i < 8; ++i) {
    out[(size_t)t * 16 + 2 * i] = acc[i].x;
    out[(size_t)t * 16 + 2 * i + 1] = acc[i].y;
  }
}

__global__ void __launch_bounds__(256) k_co_mfma(int iters, float* sink) {
  f16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (_Float16)(0.001f * (threadIdx.x + i));
    b[i] = (_Float16)(0.002f * (threadIdx.x - i));
  }
  f32x16 acc = {};
  for (int it = 0; it < iters; ++it) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  float s = 0.0f;
  for (int i = 0; i < 16; ++i) s += acc[i];
  if (s == 1234.5678f && threadIdx.x == 1000) sink[0] = s;  // never
}

template <int OP>
void launch_ops(int nwg, int iters, float* out, hipStream_t st) {
  hipLaunchKernelGGL(k_ops<OP>, dim3(nwg), dim3(256), 0, st, iters, out);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  const int co_iters = argc > 2 ? atoi(argv[2]) : 20000;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int nwg = ncu * 4;  // ops workgroups: 4 per CU beside one co-runner workgroup
  const size_t n = (size_t)nwg * 256 * 16;
  float *d_ref, *d_out, *d_sink;
  CK(hipMalloc(&d_ref, n * 4));
  CK(hipMalloc(&d_out, n * 4));
  CK(hipMalloc(&d_sink, 64));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  constexpr int NOPS = 13;
  const char* names[NOPS] = {"v_pk_fma_f32 op_sel_hi:[1,0,1]", "v_pk_fma_f32 op_sel:[0,1,0]", "v_pk_fma_f32",
                             "v_pk_mul_f32", "v_pk_add_f32", "v_fma_f32 (scalar)",
                             "v_pk_fma_f32 op_sel:[1,0,0]", "v_pk_fma_f32 op_sel:[0,1,0] hi:[1,0,1]",
                             "v_pk_mul_f32 op_sel:[0,1]", "v_pk_add_f32 op_sel:[0,1]",
                             "v_pk_mul_f32 op_sel_hi:[1,0]", "v_pk_fma_f32 op_sel:[0,0,1]",
                             "v_pk_mov_b32 op_sel:[1,0] + v_pk_add_f32"};
  void (*launch[NOPS])(int, int, float*, hipStream_t) = {
      launch_ops<0>, launch_ops<1>, launch_ops<2>, launch_ops<3>, launch_ops<4>, launch_ops<5>,
      launch_ops<6>, launch_ops<7>, launch_ops<8>, launch_ops<9>, launch_ops<10>, launch_ops<11>,
      launch_ops<12>};
  std::vector<float> ref(n), got(n);
  printf("pk_mfma_hazard: %d ops workgroups x 256 threads x %d iterations x 8 chains; co-runner %d x 256 "
         "threads, %d MFMAs each\n", nwg, iters, ncu, co_iters);
  const int op0 = argc > 3 ? atoi(argv[3]) : 0;
  for (int op = op0; op < NOPS; ++op) {
    launch[op](nwg, iters, d_ref, s1);
    CK(hipStreamSynchronize(s1));
    CK(hipMemcpy(ref.data(), d_ref, n * 4, hipMemcpyDeviceToHost));
    for (int co = 0; co < 2; ++co) {
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemset(d_out, 0xff, n * 4));
        CK(hipDeviceSynchronize());
        if (co) hipLaunchKernelGGL(k_co_mfma, dim3(ncu), dim3(256), 0, s2, co_iters, d_sink);
        launch[op](nwg, iters, d_out, s1);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), d_out, n * 4, hipMemcpyDeviceToHost));
        long long bad = 0, lane_bad[64] = {0}, half_bad[2] = {0};
        for (size_t i = 0; i < n; ++i) {
          if (*reinterpret_cast<uint32_t*>(&ref[i]) != *reinterpret_cast<uint32_t*>(&got[i])) {
            ++bad;
            ++lane_bad[(i / 16) % 64];
            ++half_bad[i % 2];
          }
        }
        printf("  %-40s %s rep %d: %lld of %zu results differ (.x %lld, .y %lld)", names[op],
               co ? "beside MFMA" : "alone      ", rep, bad, n, half_bad[0], half_bad[1]);
        if (bad) {
          printf("; lanes:");
          for (int l = 0; l < 64; ++l)
            if (lane_bad[l]) printf(" %d", l);
        }
        printf("\n");
      }
    }
  }
  return 0;
}
