// Diagnostic: does the VGPR bank (register number mod 4) of the operands change the issue
// rate of v_fmac_f32 / v_pk_fma_f32 on gfx950?  Each variant runs 2 workgroups of 256
// threads per CU (2 waves per SIMD), ITERS x 16 independent instructions per wave with
// explicitly numbered registers; prints cycles per instruction per SIMD (s_memtime).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
#define CLOB "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", \
  "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", \
  "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", \
  "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", \
  "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103"

// dst v(40 + 4i) (bank 0, pairs (0,1)); sources named per variant
#define F_A(i) "v_fmac_f32 v" #i "_" "\n"
template <int MODE>
__global__ void __launch_bounds__(256) k_bank(int iters, unsigned long long* cyc) {
  asm volatile(
      "v_mov_b32 v1, 1.0\n v_mov_b32 v2, 0.5\n v_mov_b32 v3, 0.25\n v_mov_b32 v4, 2.0\n v_mov_b32 v5, 1.5\n"
      "v_mov_b32 v6, 0.75\n v_mov_b32 v7, 3.0\n v_mov_b32 v8, 1.25\n v_mov_b32 v9, 0.125\n v_mov_b32 v10, 1.0\n"
      "v_mov_b32 v11, 1.0\n v_mov_b32 v12, 1.0\n v_mov_b32 v13, 1.0\n v_mov_b32 v14, 1.0\n v_mov_b32 v15, 1.0\n" ::
          : CLOB);
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {  // fmac: dst bank 0, src0 bank 1, src1 bank 2 (conflict-free)
#define X(i) "v_fmac_f32 v" #i "0, v1, v2\n"
      asm volatile(
          "v_fmac_f32 v40, v1, v2\n v_fmac_f32 v44, v1, v2\n v_fmac_f32 v48, v1, v2\n v_fmac_f32 v52, v1, v2\n"
          "v_fmac_f32 v56, v1, v2\n v_fmac_f32 v60, v1, v2\n v_fmac_f32 v64, v1, v2\n v_fmac_f32 v68, v1, v2\n"
          "v_fmac_f32 v72, v1, v2\n v_fmac_f32 v76, v1, v2\n v_fmac_f32 v80, v1, v2\n v_fmac_f32 v84, v1, v2\n"
          "v_fmac_f32 v88, v1, v2\n v_fmac_f32 v92, v1, v2\n v_fmac_f32 v96, v1, v2\n v_fmac_f32 v100, v1, v2\n" ::
              : CLOB);
#undef X
    } else if constexpr (MODE == 1) {  // fmac: all three operands bank 0
      asm volatile(
          "v_fmac_f32 v40, v4, v8\n v_fmac_f32 v44, v4, v8\n v_fmac_f32 v48, v4, v8\n v_fmac_f32 v52, v4, v8\n"
          "v_fmac_f32 v56, v4, v8\n v_fmac_f32 v60, v4, v8\n v_fmac_f32 v64, v4, v8\n v_fmac_f32 v68, v4, v8\n"
          "v_fmac_f32 v72, v4, v8\n v_fmac_f32 v76, v4, v8\n v_fmac_f32 v80, v4, v8\n v_fmac_f32 v84, v4, v8\n"
          "v_fmac_f32 v88, v4, v8\n v_fmac_f32 v92, v4, v8\n v_fmac_f32 v96, v4, v8\n v_fmac_f32 v100, v4, v8\n" ::
              : CLOB);
    } else if constexpr (MODE == 2) {  // fmac: src0 bank 0 (= dst), src1 bank 1
      asm volatile(
          "v_fmac_f32 v40, v4, v1\n v_fmac_f32 v44, v4, v1\n v_fmac_f32 v48, v4, v1\n v_fmac_f32 v52, v4, v1\n"
          "v_fmac_f32 v56, v4, v1\n v_fmac_f32 v60, v4, v1\n v_fmac_f32 v64, v4, v1\n v_fmac_f32 v68, v4, v1\n"
          "v_fmac_f32 v72, v4, v1\n v_fmac_f32 v76, v4, v1\n v_fmac_f32 v80, v4, v1\n v_fmac_f32 v84, v4, v1\n"
          "v_fmac_f32 v88, v4, v1\n v_fmac_f32 v92, v4, v1\n v_fmac_f32 v96, v4, v1\n v_fmac_f32 v100, v4, v1\n" ::
              : CLOB);
    } else if constexpr (MODE == 3) {  // pk_fma: acc (0,1), src0 (2,3), src1 (2,3)
      asm volatile(
          "v_pk_fma_f32 v[40:41], v[2:3], v[6:7], v[40:41]\n v_pk_fma_f32 v[44:45], v[2:3], v[6:7], v[44:45]\n"
          "v_pk_fma_f32 v[48:49], v[2:3], v[6:7], v[48:49]\n v_pk_fma_f32 v[52:53], v[2:3], v[6:7], v[52:53]\n"
          "v_pk_fma_f32 v[56:57], v[2:3], v[6:7], v[56:57]\n v_pk_fma_f32 v[60:61], v[2:3], v[6:7], v[60:61]\n"
          "v_pk_fma_f32 v[64:65], v[2:3], v[6:7], v[64:65]\n v_pk_fma_f32 v[68:69], v[2:3], v[6:7], v[68:69]\n"
          "v_pk_fma_f32 v[72:73], v[2:3], v[6:7], v[72:73]\n v_pk_fma_f32 v[76:77], v[2:3], v[6:7], v[76:77]\n"
          "v_pk_fma_f32 v[80:81], v[2:3], v[6:7], v[80:81]\n v_pk_fma_f32 v[84:85], v[2:3], v[6:7], v[84:85]\n"
          "v_pk_fma_f32 v[88:89], v[2:3], v[6:7], v[88:89]\n v_pk_fma_f32 v[92:93], v[2:3], v[6:7], v[92:93]\n"
          "v_pk_fma_f32 v[96:97], v[2:3], v[6:7], v[96:97]\n v_pk_fma_f32 v[100:101], v[2:3], v[6:7], v[100:101]\n" ::
              : CLOB);
    } else if constexpr (MODE == 4) {  // pk_fma: acc (0,1), src0 (2,3), src1 (0,1)
      asm volatile(
          "v_pk_fma_f32 v[40:41], v[2:3], v[4:5], v[40:41]\n v_pk_fma_f32 v[44:45], v[2:3], v[4:5], v[44:45]\n"
          "v_pk_fma_f32 v[48:49], v[2:3], v[4:5], v[48:49]\n v_pk_fma_f32 v[52:53], v[2:3], v[4:5], v[52:53]\n"
          "v_pk_fma_f32 v[56:57], v[2:3], v[4:5], v[56:57]\n v_pk_fma_f32 v[60:61], v[2:3], v[4:5], v[60:61]\n"
          "v_pk_fma_f32 v[64:65], v[2:3], v[4:5], v[64:65]\n v_pk_fma_f32 v[68:69], v[2:3], v[4:5], v[68:69]\n"
          "v_pk_fma_f32 v[72:73], v[2:3], v[4:5], v[72:73]\n v_pk_fma_f32 v[76:77], v[2:3], v[4:5], v[76:77]\n"
          "v_pk_fma_f32 v[80:81], v[2:3], v[4:5], v[80:81]\n v_pk_fma_f32 v[84:85], v[2:3], v[4:5], v[84:85]\n"
          "v_pk_fma_f32 v[88:89], v[2:3], v[4:5], v[88:89]\n v_pk_fma_f32 v[92:93], v[2:3], v[4:5], v[92:93]\n"
          "v_pk_fma_f32 v[96:97], v[2:3], v[4:5], v[96:97]\n v_pk_fma_f32 v[100:101], v[2:3], v[4:5], v[100:101]\n" ::
              : CLOB);
    } else if constexpr (MODE == 5) {  // pk_fma op_sel broadcast of src1's lo (v6, bank 2): acc (0,1), src0 (2,3)
      asm volatile(
          "v_pk_fma_f32 v[40:41], v[2:3], v[6:7], v[40:41] op_sel_hi:[1,0,1]\n v_pk_fma_f32 v[44:45], v[2:3], v[6:7], v[44:45] op_sel_hi:[1,0,1]\n"
          "v_pk_fma_f32 v[48:49], v[2:3], v[6:7], v[48:49] op_sel_hi:[1,0,1]\n v_pk_fma_f32 v[52:53], v[2:3], v[6:7], v[52:53] op_sel_hi:[1,0,1]\n"
          "v_pk_fma_f32 v[56:57], v[2:3], v[6:7], v[56:57] op_sel_hi:[1,0,1]\n v_pk_fma_f32 v[60:61], v[2:3], v[6:7], v[60:61] op_sel_hi:[1,0,1]\n"
          "v_pk_fma_f32 v[64:65], v[2:3], v[6:7], v[64:65] op_sel_hi:[1,0,1]\n v_pk_fma_f32 v[68:69], v[2:3], v[6:7], v[68:69] op_sel_hi:[1,0,1]\n"
          "v_pk_fma_f32 v[72:73], v[2:3], v[6:7], v[72:73] op_sel_hi:[1,0,1]\n v_pk_fma_f32 v[76:77], v[2:3], v[6:7], v[76:77] op_sel_hi:[1,0,1]\n"
          "v_pk_fma_f32 v[80:81], v[2:3], v[6:7], v[80:81] op_sel_hi:[1,0,1]\n v_pk_fma_f32 v[84:85], v[2:3], v[6:7], v[84:85] op_sel_hi:[1,0,1]\n"
          "v_pk_fma_f32 v[88:89], v[2:3], v[6:7], v[88:89] op_sel_hi:[1,0,1]\n v_pk_fma_f32 v[92:93], v[2:3], v[6:7], v[92:93] op_sel_hi:[1,0,1]\n"
          "v_pk_fma_f32 v[96:97], v[2:3], v[6:7], v[96:97] op_sel_hi:[1,0,1]\n v_pk_fma_f32 v[100:101], v[2:3], v[6:7], v[100:101] op_sel_hi:[1,0,1]\n" ::
              : CLOB);
    } else if constexpr (MODE == 6) {  // pk_fma, src0 an SGPR pair (taps in SGPRs), src1 (2,3), acc (0,1)
      asm volatile(
          "s_mov_b32 s90, 1.0\n s_mov_b32 s91, 0.5\n"
          "v_pk_fma_f32 v[40:41], s[90:91], v[6:7], v[40:41]\n v_pk_fma_f32 v[44:45], s[90:91], v[6:7], v[44:45]\n"
          "v_pk_fma_f32 v[48:49], s[90:91], v[6:7], v[48:49]\n v_pk_fma_f32 v[52:53], s[90:91], v[6:7], v[52:53]\n"
          "v_pk_fma_f32 v[56:57], s[90:91], v[6:7], v[56:57]\n v_pk_fma_f32 v[60:61], s[90:91], v[6:7], v[60:61]\n"
          "v_pk_fma_f32 v[64:65], s[90:91], v[6:7], v[64:65]\n v_pk_fma_f32 v[68:69], s[90:91], v[6:7], v[68:69]\n"
          "v_pk_fma_f32 v[72:73], s[90:91], v[6:7], v[72:73]\n v_pk_fma_f32 v[76:77], s[90:91], v[6:7], v[76:77]\n"
          "v_pk_fma_f32 v[80:81], s[90:91], v[6:7], v[80:81]\n v_pk_fma_f32 v[84:85], s[90:91], v[6:7], v[84:85]\n"
          "v_pk_fma_f32 v[88:89], s[90:91], v[6:7], v[88:89]\n v_pk_fma_f32 v[92:93], s[90:91], v[6:7], v[92:93]\n"
          "v_pk_fma_f32 v[96:97], s[90:91], v[6:7], v[96:97]\n v_pk_fma_f32 v[100:101], s[90:91], v[6:7], v[100:101]\n" ::
              : CLOB, "s90", "s91");
    } else {  // fmac with an SGPR tap: v_fmac_f32 vD, sT, vP (dst bank 0, P bank 1)
      asm volatile(
          "s_mov_b32 s90, 1.0\n"
          "v_fmac_f32 v40, s90, v1\n v_fmac_f32 v44, s90, v1\n v_fmac_f32 v48, s90, v1\n v_fmac_f32 v52, s90, v1\n"
          "v_fmac_f32 v56, s90, v1\n v_fmac_f32 v60, s90, v1\n v_fmac_f32 v64, s90, v1\n v_fmac_f32 v68, s90, v1\n"
          "v_fmac_f32 v72, s90, v1\n v_fmac_f32 v76, s90, v1\n v_fmac_f32 v80, s90, v1\n v_fmac_f32 v84, s90, v1\n"
          "v_fmac_f32 v88, s90, v1\n v_fmac_f32 v92, s90, v1\n v_fmac_f32 v96, s90, v1\n v_fmac_f32 v100, s90, v1\n" ::
              : CLOB, "s90");
    }
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = c1 - c0;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  unsigned long long* cyc;
  hipMalloc(&cyc, 8 * 8 * cus * 4);
  static unsigned long long hc[1 << 16];
  const char* names[8] = {"fmac dst b0 src b1,b2", "fmac all bank 0", "fmac src0=b0 src1=b1",
                          "pk_fma acc(0,1) s0(2,3) s1(2,3)", "pk_fma acc(0,1) s0(2,3) s1(0,1)",
                          "pk_fma bcast s1 lo(b2) s0(2,3)", "pk_fma s0 SGPR pair s1(2,3)", "fmac s0 SGPR s1 b1"};
  for (int mode = 0; mode < 8; ++mode)
    for (int wgs = 2; wgs <= 4; wgs += 2) {
      dim3 grid(cus * wgs);
      auto go = [&]() {
        switch (mode) {
          case 0: hipLaunchKernelGGL(k_bank<0>, grid, dim3(256), 0, 0, iters, cyc); break;
          case 1: hipLaunchKernelGGL(k_bank<1>, grid, dim3(256), 0, 0, iters, cyc); break;
          case 2: hipLaunchKernelGGL(k_bank<2>, grid, dim3(256), 0, 0, iters, cyc); break;
          case 3: hipLaunchKernelGGL(k_bank<3>, grid, dim3(256), 0, 0, iters, cyc); break;
          case 4: hipLaunchKernelGGL(k_bank<4>, grid, dim3(256), 0, 0, iters, cyc); break;
          case 5: hipLaunchKernelGGL(k_bank<5>, grid, dim3(256), 0, 0, iters, cyc); break;
          case 6: hipLaunchKernelGGL(k_bank<6>, grid, dim3(256), 0, 0, iters, cyc); break;
          default: hipLaunchKernelGGL(k_bank<7>, grid, dim3(256), 0, 0, iters, cyc); break;
        }
      };
      go();
      hipDeviceSynchronize();
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0, 0);
      go();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(hc, cyc, 8 * 4 * grid.x, hipMemcpyDeviceToHost);
      double mc = 0;
      for (unsigned w = 0; w < 4 * grid.x; ++w) mc = hc[w] > mc ? hc[w] : mc;
      // waves per SIMD = wgs (4-wave workgroups spread over the 4 SIMDs)
      printf("%-34s waves/SIMD %d: %.3f ms, %.2f cyc per instruction per SIMD, clock %.0f MHz\n", names[mode], wgs,
             ms, mc / ((double)iters * 16 * wgs), mc / (ms * 1e-3) / 1e6);
    }
  return 0;
}
