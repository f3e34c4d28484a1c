// debug.hip — diagnostic entry points of the C-ABI (declared in include/sfmfeat.h under
// "diagnostics").  They expose intermediate stages of the same kernels the pipeline runs
// so the parity tests can localise a mismatch (device atan2, the Harris R map, the exact
// median and the candidate count).  Not used by the throughput path.
#include <string.h>

#include <vector>

#include "../../include/sfmfeat.h"
#include "kernels.h"

using namespace sfm;

namespace sfm {

__global__ void k_debug_atan2(const float* __restrict__ y, const float* __restrict__ x,
                              float* __restrict__ out, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = svml_atan2f(y[i], x[i]);
}

// Exchange emulation (bench.py --emulate-exchange): a grid-stride 16-B copy run by exactly
// gridDim.x persistent workgroups, the shape of a collective's kernel (one workgroup per
// channel), so its CU residency and HBM traffic compete with extraction the way an all-gather
// of the same bytes would on the GPU that receives them.
__global__ void __launch_bounds__(256) k_copy_wg(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t n16,
                                                 const uint8_t* __restrict__ src_b, uint8_t* __restrict__ dst_b,
                                                 int64_t tail) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
  if (blockIdx.x == 0 && threadIdx.x < tail) dst_b[threadIdx.x] = src_b[threadIdx.x];
}

}  // namespace sfm

extern "C" {

int32_t sfm_debug_atan2(int32_t device, const float* y, const float* x, float* out, int64_t n) {
  if (n <= 0) return SFM_OK;
  if (hipSetDevice(device) != hipSuccess) return SFM_EDEVICE;
  float *dy = nullptr, *dx = nullptr, *dout = nullptr;
  size_t bytes = (size_t)n * 4;
  if (hipMalloc(&dy, bytes) || hipMalloc(&dx, bytes) || hipMalloc(&dout, bytes)) return SFM_EDEVICE;
  int32_t rc = SFM_OK;
  if (hipMemcpy(dy, y, bytes, hipMemcpyHostToDevice) || hipMemcpy(dx, x, bytes, hipMemcpyHostToDevice)) {
    rc = SFM_EDEVICE;
  } else {
    hipLaunchKernelGGL(k_debug_atan2, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, dy, dx, dout, n);
    if (hipDeviceSynchronize() || hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost)) rc = SFM_EDEVICE;
  }
  (void)hipFree(dy);
  (void)hipFree(dx);
  (void)hipFree(dout);
  return rc;
}

// Harris R map, exact median and candidate count of ONE level-0 plane with the
// context's parameters (NaiveSIFT.py:59-97).
int32_t sfm_debug_harris(int32_t device, const float* gauss, int32_t gs, double alpha, int32_t ksize,
                         const float* img, int32_t H, int32_t W, float* R_out, float* median_out,
                         int64_t* ncand_out) {
  if (H < 1 || W < 1 || gs < 1 || gs > SFM_MAX_GAUSS) return SFM_EINVAL;
  if (hipSetDevice(device) != hipSuccess) return SFM_EDEVICE;
  int64_t n = (int64_t)H * W;
  float *d_img = nullptr, *d_R = nullptr, *d_g = nullptr;
  uint32_t *d_hist = nullptr, *d_list = nullptr;
  MedianState* d_med = nullptr;
  unsigned long long* d_cnt = nullptr;
  uint64_t* d_cand = nullptr;
  int32_t rc = SFM_OK;
  std::vector<float> taps(harris_taps_floats(gs));
  harris_taps_build(gauss, gs, taps.data());
  if (hipMalloc(&d_img, n * 4) || hipMalloc(&d_R, n * 4) || hipMalloc(&d_g, 4 * taps.size()) ||
      hipMalloc(&d_hist, 4 * kMedBins1) || hipMalloc(&d_list, n * 4) || hipMalloc(&d_med, sizeof(MedianState)) ||
      hipMalloc(&d_cnt, 16 * kCounterStride) || hipMalloc(&d_cand, n * 8)) {
    rc = SFM_EDEVICE;
  } else {
    (void)hipMemcpy(d_img, img, n * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_g, taps.data(), 4 * taps.size(), hipMemcpyHostToDevice);
    (void)hipMemset(d_hist, 0, 4 * kMedBins1);
    (void)hipMemset(d_cnt, 0, 16 * kCounterStride);
    launch_harris(d_img, d_R, d_hist, 1, H, W, d_g, gs, (float)alpha, SelectScan{nullptr, nullptr, nullptr, 0, 0},
                  0);
    launch_select_scan(d_hist, d_med, d_cnt, 1, H, W, 0, /*force_exact=*/1, 0);
    launch_median_exact(d_R, d_med, d_list, d_cnt, 1, H, W, 0);
    launch_nms(d_R, d_med, d_cand, d_cnt + kCounterStride, 1, H, W, ksize, 1, 0);
    MedianState ms;
    unsigned long long cnt[2 * kCounterStride];
    if (hipDeviceSynchronize() || hipMemcpy(R_out, d_R, n * 4, hipMemcpyDeviceToHost) ||
        hipMemcpy(&ms, d_med, sizeof(ms), hipMemcpyDeviceToHost) ||
        hipMemcpy(cnt, d_cnt, sizeof(cnt), hipMemcpyDeviceToHost)) {
      rc = SFM_EDEVICE;
    } else {
      *median_out = ms.median;
      *ncand_out = (int64_t)cnt[kCounterStride];
    }
  }
  void* bufs[] = {d_img, d_R, d_g, d_hist, d_list, d_med, d_cnt, d_cand};
  for (void* b : bufs) (void)hipFree(b);
  return rc;
}

// Certified-mode NMS (the predicate of NaiveSIFT.py:77-95 restricted to keys >= tnms, §5)
// on B host planes with per-plane thresholds tnms[B]: the candidate keys of plane b land in
// keys_out[b * H * W ...] (unordered), their number in counts_out[b].  tile = 1 runs the
// tiled kernel where the streaming one would run, so the tests can hold both to one oracle.
int32_t sfm_debug_nms(int32_t device, const float* R, int32_t B, int32_t H, int32_t W, int32_t ksize,
                      const uint32_t* tnms, int32_t tile, uint64_t* keys_out, int64_t* counts_out) {
  if (B < 1 || H < 1 || W < 1 || ksize < 1 || (ksize & 1) == 0 || ksize / 2 > SFM_NMS_MAX_HALF) return SFM_EINVAL;
  if (hipSetDevice(device) != hipSuccess) return SFM_EDEVICE;
  const int64_t n = (int64_t)H * W, tot = n * B;
  float* d_R = nullptr;
  MedianState* d_med = nullptr;
  unsigned long long* d_cnt = nullptr;
  uint64_t* d_cand = nullptr;
  int32_t rc = SFM_OK;
  if (hipMalloc(&d_R, tot * 4) || hipMalloc(&d_med, sizeof(MedianState) * B) ||
      hipMalloc(&d_cnt, 8 * (size_t)B * kCounterStride) || hipMalloc(&d_cand, tot * 8)) {
    rc = SFM_EDEVICE;
  } else {
    std::vector<MedianState> ms(B);
    memset(ms.data(), 0, sizeof(MedianState) * B);
    for (int b = 0; b < B; ++b) ms[b].tnms = tnms[b];  // fallback = 0: certified planes
    (void)hipMemcpy(d_R, R, tot * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_med, ms.data(), sizeof(MedianState) * B, hipMemcpyHostToDevice);
    (void)hipMemset(d_cnt, 0, 8 * (size_t)B * kCounterStride);
    launch_nms(d_R, d_med, d_cand, d_cnt, B, H, W, ksize, 0, 0, tile);
    std::vector<unsigned long long> cnt((size_t)B * kCounterStride);
    if (hipDeviceSynchronize() || hipMemcpy(cnt.data(), d_cnt, 8 * cnt.size(), hipMemcpyDeviceToHost) ||
        hipMemcpy(keys_out, d_cand, tot * 8, hipMemcpyDeviceToHost)) {
      rc = SFM_EDEVICE;
    } else {
      for (int b = 0; b < B; ++b) counts_out[b] = (int64_t)cnt[(size_t)b * kCounterStride];
    }
  }
  void* bufs[] = {d_R, d_med, d_cnt, d_cand};
  for (void* b : bufs) (void)hipFree(b);
  return rc;
}

// Mean time (ms) of one k_harris<7> launch over B x H x W synthetic planes for ablation
// variant `abl` (0 full, 1 no histogram, 2 no window sums, 3 no Sobel/products).
float sfm_debug_time_harris(int32_t device, int32_t abl, int32_t B, int32_t H, int32_t W, int32_t iters) {
  return sfm_debug_harris_stamps(device, abl, B, H, W, iters, nullptr, 0);
}

// As sfm_debug_time_harris; abl = 3 also copies the last launch's per-workgroup timestamps
// (48 u64 per workgroup, workgroup (x, plane) at (plane * grid_x + x) * 48) into `out`.
float sfm_debug_harris_stamps(int32_t device, int32_t abl, int32_t B, int32_t H, int32_t W, int32_t iters,
                              uint64_t* out, int64_t cap) {
  if (hipSetDevice(device) != hipSuccess) return -1.0f;
  uint64_t* d_st = nullptr;
  if (abl == 3) {
    if (cap <= 0 || hipMalloc(&d_st, (size_t)cap * 8) != hipSuccess) return -1.0f;
    (void)hipMemset(d_st, 0, (size_t)cap * 8);
  }
  int64_t n = (int64_t)B * H * W;
  float *d_img = nullptr, *d_R = nullptr, *d_g = nullptr;
  uint32_t* d_hist = nullptr;
  if (hipMalloc(&d_img, n * 4) || hipMalloc(&d_R, n * 4) || hipMalloc(&d_g, 4 * harris_taps_floats(7)) ||
      hipMalloc(&d_hist, (size_t)B * 4 * kMedBins1))
    return -1.0f;
  std::vector<float> h(n);
  uint32_t x = 12345u;
  for (int64_t i = 0; i < n; ++i) {
    x = x * 1664525u + 1013904223u;
    h[i] = (float)(x >> 24) / 255.0f;
  }
  float g0[49];
  for (int i = 0; i < 49; ++i) g0[i] = 1.0f / 49.0f;
  std::vector<float> g(harris_taps_floats(7));
  harris_taps_build(g0, 7, g.data());
  (void)hipMemcpy(d_img, h.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_g, g.data(), 4 * g.size(), hipMemcpyHostToDevice);
  (void)hipMemset(d_hist, 0, (size_t)B * 4 * kMedBins1);
  // the kernel skips the stamps of workgroups whose slots lie beyond cap (the grid is
  // chosen inside the launcher, so the caller cannot size cap exactly)
  float ms = time_harris_ablation(abl, d_img, d_R, d_hist, B, H, W, d_g, 0.05f, iters, d_st, d_st ? cap : 0);
  if (d_st) {
    (void)hipMemcpy(out, d_st, (size_t)cap * 8, hipMemcpyDeviceToHost);
    (void)hipFree(d_st);
  }
  void* bufs[] = {d_img, d_R, d_g, d_hist};
  for (void* b : bufs) (void)hipFree(b);
  return ms;
}

int32_t sfm_copy_wg(void* dst, const void* src, int64_t bytes, int32_t workgroups, void* stream) {
  if (bytes < 0 || workgroups < 1 || (bytes > 0 && (!dst || !src))) return SFM_EINVAL;
  if ((((uintptr_t)dst) | ((uintptr_t)src)) & 15) return SFM_EINVAL;
  if (bytes == 0) return SFM_OK;
  const int64_t n16 = bytes / 16, tail = bytes - 16 * n16;
  hipLaunchKernelGGL(k_copy_wg, dim3((unsigned)workgroups), dim3(256), 0, (hipStream_t)stream,
                     (const uint4*)src, (uint4*)dst, n16, (const uint8_t*)src + 16 * n16, (uint8_t*)dst + 16 * n16,
                     tail);
  return hipGetLastError() == hipSuccess ? SFM_OK : SFM_EDEVICE;
}

// The matcher sweep's per-wave clock stamps (diagnostic build, SFMFEAT_MATCH_ABL=32).
int64_t sfm_debug_match_stamps(uint64_t* out, int64_t cap) { return sfm::match_stamps_copy(out, cap); }

}  // extern "C"
