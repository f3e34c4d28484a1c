// coresidency_repro.hip — minimal reproducer for the round-3 Harris co-residency finding
// (DESIGN.md §7 "Co-residency"): does k_harris produce different R maps when another
// kernel's waves share its CUs?
//
// Harris (the product kernel, compiled from sfmfromscratch_amd/csrc/harris.hip; built twice
// by tools/Makefile: window fmas as inline-asm v_pk_fma_f32, as the compiler's own packed
// fmas (-DSFM_HARRIS_NATIVE_PK) and as scalar v_fma_f32 (-DSFM_HARRIS_SCALAR_FMA)) runs on stream 1 over 32 synthetic 1080p planes, right after
// a co-runner was launched on stream 2 with one 256-thread workgroup per CU (one wave per
// SIMD, few VGPRs), so that every CU can hold one Harris workgroup beside it.  Each R map is
// compared bit for bit with the R map of the same launch run alone.
//
// Co-runners (no global writes; a never-taken branch keeps their results live):
//   none   control: Harris alone again
//   mfma   v_mfma_f32_32x32x16_f16 chain, registers only, 4 KB of dynamic LDS allocated and
//          never touched
//   mfmal  the same MFMA chain plus ds_write/ds_read traffic in its own 4 KB of LDS
//   valu   v_fma_f32 chain (VALU only)
//
// Output: per co-runner and repetition the number of differing R values and, over all
// repetitions, where they fall (plane, tile, row and column inside the 64 x 64 tile, the
// column within a thread's 4-column group, the row within its 4-row group).
#include "../sfmfromscratch_amd/csrc/harris.hip"

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <string>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void __launch_bounds__(256) k_co_mfma(int iters, int lds_traffic, float* sink) {
  extern __shared__ float s_dyn[];
  f16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (_Float16)(0.001f * (threadIdx.x + i));
    b[i] = (_Float16)(0.002f * (threadIdx.x - i));
  }
  f32x16 acc = {};
  for (int it = 0; it < iters; ++it) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    if (lds_traffic) {
      s_dyn[threadIdx.x * 4 + (it & 3)] = acc[it & 15];
      a[0] = (_Float16)s_dyn[(threadIdx.x ^ 1) * 4 + (it & 3)];
    }
  }
  float s = 0.0f;
  for (int i = 0; i < 16; ++i) s += acc[i];
  if (s == 1234.5678f && threadIdx.x == 1000) sink[0] = s;  // never (256 threads)
}

__global__ void __launch_bounds__(256) k_co_valu(int iters, float* sink) {
  float x0 = threadIdx.x * 1e-3f, x1 = x0 + 1.0f, x2 = x0 + 2.0f, x3 = x0 + 3.0f;
  for (int it = 0; it < iters; ++it) {
    x0 = fmaf(x0, 0.999f, 0.5f);
    x1 = fmaf(x1, 0.999f, 0.5f);
    x2 = fmaf(x2, 0.999f, 0.5f);
    x3 = fmaf(x3, 0.999f, 0.5f);
  }
  const float s = x0 + x1 + x2 + x3;
  if (s == 1234.5678f && threadIdx.x == 1000) sink[0] = s;
}

// mismatch records: (index, ref bits, got bits) for the first `cap`
__global__ void k_compare(const float* __restrict__ ref, const float* __restrict__ got, int64_t n,
                          unsigned long long* count, long long* rec, int cap) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t a = __float_as_uint(ref[i]), b = __float_as_uint(got[i]);
    if (a != b) {
      const unsigned long long k = atomicAdd(count, 1ull);
      if (k < (unsigned long long)cap) {
        rec[3 * k] = i;
        rec[3 * k + 1] = a;
        rec[3 * k + 2] = b;
      }
    }
  }
}

int main(int argc, char** argv) {
  const int B = 32, H = 1080, W = 1920, KS = 7;
  const int reps = argc > 1 ? atoi(argv[1]) : 4;
  const int iters = argc > 2 ? atoi(argv[2]) : 40000;
  std::vector<std::string> kinds;
  for (int i = 3; i < argc; ++i) kinds.push_back(argv[i]);
  if (kinds.empty()) kinds = {"none", "mfma", "mfmal", "valu", "none"};
#if defined(SFM_HARRIS_NATIVE_PK)
  const char* variant = "native packed fma";
#elif defined(SFM_HARRIS_SCALAR_FMA)
  const char* variant = "scalar v_fma_f32 window sums";
#elif defined(SFM_HARRIS_SRC1_HI)
  const char* variant = "inline-asm v_pk_fma_f32, high-half broadcast on src1 (op_sel:[0,1,0], round 3)";
#else
  const char* variant = "inline-asm v_pk_fma_f32, high-half broadcast on src0 (op_sel:[1,0,0])";
#endif
  const int64_t n = (int64_t)B * H * W;
  float *d_img, *d_ref, *d_R, *d_g, *d_sink;
  uint32_t* d_hist;
  unsigned long long* d_cnt;
  long long* d_rec;
  const int cap = 1 << 16;
  CK(hipMalloc(&d_img, n * 4));
  CK(hipMalloc(&d_ref, n * 4));
  CK(hipMalloc(&d_R, n * 4));
  CK(hipMalloc(&d_g, 4 * KS * KS));
  CK(hipMalloc(&d_sink, 64));
  CK(hipMalloc(&d_hist, (size_t)B * 4 * sfm::kMedBins1));
  CK(hipMalloc(&d_cnt, 8));
  CK(hipMalloc(&d_rec, (size_t)cap * 3 * 8));
  {
    std::vector<float> h(n);
    uint32_t x = 12345u;
    for (int64_t i = 0; i < n; ++i) {  // textured: a smooth pattern plus LCG noise
      x = x * 1664525u + 1013904223u;
      const int64_t p = i % ((int64_t)H * W);
      const int yy = (int)(p / W), xx = (int)(p % W);
      h[i] = 0.5f + 0.25f * sinf(0.05f * xx + 0.031f * yy) + (float)(x >> 24) / 1024.0f;
    }
    CK(hipMemcpy(d_img, h.data(), n * 4, hipMemcpyHostToDevice));
    double g[KS * KS], tot = 0.0;
    for (int i = 0; i < KS; ++i)
      for (int j = 0; j < KS; ++j) {
        const double ax = i - KS / 2, ay = j - KS / 2;
        g[i * KS + j] = exp(-(ax * ax + ay * ay) / (2.0 * 36.0));
        tot += g[i * KS + j];
      }
    float gf[KS * KS];
    for (int i = 0; i < KS * KS; ++i) gf[i] = (float)(g[i] / tot);
    CK(hipMemcpy(d_g, gf, sizeof(gf), hipMemcpyHostToDevice));
  }
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t h0, h1, c0, c1;
  CK(hipEventCreate(&h0));
  CK(hipEventCreate(&h1));
  CK(hipEventCreate(&c0));
  CK(hipEventCreate(&c1));
  const sfm::SelectScan noscan{nullptr, nullptr, nullptr, 0, 0};
  auto harris = [&](float* R) {
    CK(hipMemsetAsync(d_hist, 0, (size_t)B * 4 * sfm::kMedBins1, s1));
    sfm::launch_harris(d_img, R, d_hist, B, H, W, d_g, KS, 0.05f, noscan, s1);
  };
  harris(d_ref);
  CK(hipStreamSynchronize(s1));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  printf("coresidency_repro: Harris (%s) 7x7, %d x %dx%d planes; co-runner %d workgroups x 256 threads, "
         "%d iterations\n", variant, B, H, W, ncu, iters);
  std::vector<long long> rec((size_t)cap * 3);
  int total_bad = 0;
  for (const std::string& kind : kinds) {
    std::map<std::string, std::map<long long, long long>> hist;
    long long kind_bad = 0;
    for (int r = 0; r < reps; ++r) {
      CK(hipMemsetAsync(d_R, 0xff, n * 4, s1));
      CK(hipMemsetAsync(d_cnt, 0, 8, s1));
      CK(hipStreamSynchronize(s1));
      CK(hipEventRecord(c0, s2));
      if (kind == "mfma" || kind == "mfmal")
        hipLaunchKernelGGL(k_co_mfma, dim3(ncu), dim3(256), 4096, s2, iters, kind == "mfmal" ? 1 : 0, d_sink);
      else if (kind == "valu")
        hipLaunchKernelGGL(k_co_valu, dim3(ncu), dim3(256), 0, s2, iters * 8, d_sink);
      CK(hipEventRecord(c1, s2));
      CK(hipEventRecord(h0, s1));
      harris(d_R);
      CK(hipEventRecord(h1, s1));
      CK(hipStreamSynchronize(s1));
      CK(hipStreamSynchronize(s2));
      float hm = 0, cm = 0, off = 0;
      CK(hipEventElapsedTime(&hm, h0, h1));
      CK(hipEventElapsedTime(&cm, c0, c1));
      CK(hipEventElapsedTime(&off, c0, h0));
      hipLaunchKernelGGL(k_compare, dim3(2048), dim3(256), 0, s1, d_ref, d_R, n, d_cnt, d_rec, cap);
      unsigned long long bad = 0;
      CK(hipMemcpyAsync(&bad, d_cnt, 8, hipMemcpyDeviceToHost, s1));
      CK(hipStreamSynchronize(s1));
      printf("  %-6s rep %d: harris %.3f ms, co-runner %.3f ms (harris start +%.3f ms): %llu of %lld R values differ\n",
             kind.c_str(), r, hm, cm, off, bad, (long long)n);
      kind_bad += (long long)bad;
      const int nr = (int)std::min<unsigned long long>(bad, (unsigned long long)cap);
      if (nr) {
        CK(hipMemcpy(rec.data(), d_rec, (size_t)nr * 3 * 8, hipMemcpyDeviceToHost));
        for (int k = 0; k < nr; ++k) {
          const long long i = rec[3 * k];
          const long long b = i / ((long long)H * W), p = i % ((long long)H * W);
          const long long y = p / W, x = p % W;
          hist["plane"][b]++;
          hist["tile_row(y%64)"][y % 64]++;
          hist["tile_col(x%64)"][x % 64]++;
          hist["thread_col(x%4)"][x % 4]++;
          hist["thread_row(y%4)"][y % 4]++;
          hist["tile"][(y / 64) * ((W + 63) / 64) + x / 64]++;
          const uint32_t a = (uint32_t)rec[3 * k + 1], g = (uint32_t)rec[3 * k + 2];
          hist["xor_bit_top"][31 - __builtin_clz(a ^ g)]++;
        }
        if (r == 0)
          for (int k = 0; k < std::min(nr, 8); ++k) {
            float fa, fg;
            uint32_t a = (uint32_t)rec[3 * k + 1], g = (uint32_t)rec[3 * k + 2];
            memcpy(&fa, &a, 4);
            memcpy(&fg, &g, 4);
            const long long i = rec[3 * k];
            printf("    e.g. plane %lld y %lld x %lld: alone %.9g (0x%08x), beside co-runner %.9g (0x%08x)\n",
                   i / ((long long)H * W), (i % ((long long)H * W)) / W, i % W, fa, a, fg, g);
          }
      }
    }
    printf("  %-6s total: %lld differing R values over %d launches\n", kind.c_str(), kind_bad, reps);
    for (auto& h : hist) {
      printf("    %s:", h.first.c_str());
      int shown = 0;
      for (auto& e : h.second) {
        if (shown++ >= 40) {
          printf(" ...");
          break;
        }
        printf(" %lld:%lld", e.first, e.second);
      }
      printf("\n");
    }
    total_bad += kind_bad ? 1 : 0;
  }
  printf("co-runners with differences: %d\n", total_bad);
  return 0;
}
