// Diagnostic: are the LDS allocations of workgroups of two kernels running concurrently (on
// two streams) on one CU isolated from each other?  Kernel A (LDS size SA, like k_harris)
// fills its LDS with a per-workgroup pattern and re-checks it ITERS times; kernel B (LDS size
// SB, like k_match_mfma) keeps overwriting its own LDS (in bounds) with +inf.  A counts the
// words it finds changed.  Usage: lds_isolation [SA_bytes SB_bytes iters]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void __launch_bounds__(256) k_a(unsigned* bad, int words, int iters) {
  extern __shared__ unsigned s[];
  const unsigned pat = 0x12340000u ^ (blockIdx.x * 2654435761u);
  for (int i = threadIdx.x; i < words; i += 256) s[i] = pat + i;
  __syncthreads();
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    for (int i = threadIdx.x; i < words; i += 256) nb += (s[i] != pat + i) ? 1u : 0u;
    __syncthreads();
  }
  if (nb) atomicAdd(bad, nb);
}

__global__ void __launch_bounds__(256) k_b(unsigned* sink, int words, int iters) {
  extern __shared__ unsigned s[];
  unsigned acc = 0;
  for (int it = 0; it < iters; ++it) {
    for (int i = threadIdx.x * 4; i + 3 < words; i += 1024)
      *reinterpret_cast<uint4*>(&s[i]) = make_uint4(0x7f800000u, 0x7f800000u, 0x7f800000u, 0x7f800000u + it);
    __syncthreads();
    acc += s[(threadIdx.x * 7 + it) % words];
    __syncthreads();
  }
  if (acc == 0x12345u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const int SA = argc > 1 ? atoi(argv[1]) : 73472;
  const int SB = argc > 2 ? atoi(argv[2]) : 51712;
  const int iters = argc > 3 ? atoi(argv[3]) : 4000;
  const int nb = argc > 4 ? atoi(argv[4]) : 256;
  hipFuncSetAttribute((const void*)k_a, hipFuncAttributeMaxDynamicSharedMemorySize, SA);
  hipFuncSetAttribute((const void*)k_b, hipFuncAttributeMaxDynamicSharedMemorySize, SB);
  unsigned *bad, *sink;
  hipMalloc(&bad, 4);
  hipMalloc(&sink, 4);
  hipStream_t s1, s2;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  for (int mode = 0; mode < 2; ++mode) {  // 0: A alone, 1: A with B concurrently
    hipMemset(bad, 0, 4);
    hipDeviceSynchronize();
    for (int rep = 0; rep < 4; ++rep) {
      // B first with one workgroup per CU (long), so A's workgroups land beside B's
      if (mode) hipLaunchKernelGGL(k_b, dim3(nb), dim3(256), SB, s2, sink, SB / 4, iters * 4);
      hipLaunchKernelGGL(k_a, dim3(512), dim3(256), SA, s1, bad, SA / 4, iters);
    }
    hipError_t e = hipDeviceSynchronize();
    unsigned h = 0;
    hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost);
    printf("SA %d SB %d mode %s: %s, changed LDS words seen by A: %u\n", SA, SB, mode ? "A+B" : "A alone",
           hipGetErrorString(e), h);
  }
  return 0;
}
