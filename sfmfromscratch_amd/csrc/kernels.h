// kernels.h — launcher declarations and the per-plane bookkeeping shared between the
// host orchestration (sfmfeat.cpp) and the gfx950 kernels.
//
// A "plane" is one pyramid level of one image.  All B planes of a level are stored
// contiguously ([B][h][w]) and are processed by one launch per stage.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "common.h"

namespace sfm {

#define SFM_NMS_MAX_HALF 15                 // ksize <= 31

constexpr int kHistBits = 12;               // first radix digit of the median select
constexpr int kHistBins = 1 << kHistBits;   // 4096: generic LDS histogram for <= 12-bit digits
constexpr int kMedBits1 = 11;               // median digit 1 (histogrammed inside Harris)
constexpr int kMedBins1 = 1 << kMedBits1;   // 2048 (digits 2 / 3 are 11 / 10 bits)
constexpr int kTopkLdsCap = 8192;           // max keys sorted in LDS by the top-k kernel
constexpr int kMaxMatchRows = 16384;        // max keypoints per image for the matcher sort
constexpr int kMatchCandCap = 256;          // admitted targets per query row (MFMA matcher lists)
constexpr int kCounterStride = 32;          // u64 per per-plane atomic counter (own 256-B line)
// the sweep's work units (k_match_units) encode pair | block << kMatchUnitPairBits: one
// matcher sub-launch takes at most 2^kMatchUnitPairBits pairs (match_impl clamps)
constexpr int kMatchUnitPairBits = 20;

// The matcher's per-descriptor operands (match_mfma.hip): split-f16 copies hi = f16(v * 2^8),
// lo = f16((v * 2^8 - hi) * 2^11), the squared norm float(sum v^2 in double) and the norm,
// [img][capP] rows (capP = cap rounded up to 128; padding rows: norm2 = +inf, hi = lo = 0),
// and per 16-row block the maxima of (norm2, norm) over the valid rows.  k_match_prep writes
// them from a slot table; an extraction with fused operands (sfm_ctx_set_fused_prep) has the
// descriptor kernel write them for every row it produces.
constexpr float kMatchScale = 256.0f;   // operand pre-scale (2^8)
constexpr float kMatchLoScale = 2048.0f;  // lo part scale (2^11)
constexpr int kPrepRows = 16;           // rows per (norm2, norm) maxima block
struct MatchOperands {
  _Float16* hi;    // nullptr: not written
  _Float16* lo;
  float* norm2;
  float* rnorm;
  float2* pmax;    // [img][capP / kPrepRows], zeroed by the extraction before its levels
  int64_t capP;
};

// Per-plane state of the keypoint selection (NaiveSIFT.py:90-120).
//
// Certified select (default): the reference keeps R == window max && R >= median, then the
// k largest.  NMS collects the window maxima with key >= tnms (a volume threshold: about
// vmin pixels lie above it).  If at least k were found and the k-th largest has key >=
// tcert (the first key above the median's digit-1 bucket), all of the top k are >= the
// median and every reference candidate outranking the k-th was found: the top k equal
// the reference's whatever the exact median is — so the median is only bounded, from the
// Harris histogram.  Other planes (and forced exact mode) set `fallback` and run the
// exact path: np.median by radix select, then the full NMS predicate.
struct MedianState {
  uint32_t bucket[2];   // digit-1 (top 11 bits) bucket holding rank k1 / k2
  uint32_t rank[2];     // residual rank inside that bucket
  uint32_t odd;         // H*W odd -> median is element k1 alone
  float median;         // exact median (fallback planes only)
  uint32_t tnms;        // certified select: candidate threshold key
  uint32_t tcert;       // certified select: the k-th key must reach this
  uint32_t fallback;    // 1: this plane takes the exact path
  // higher candidate thresholds (>= tnms): the buckets holding the 3 vmin / 8-th and
  // vmin / 2-th largest values.  k_select first tries the candidates at or above them (a
  // subset of about 2k-4k at vmin = 128 k, sorted whole), the full list when they are too few.
  uint32_t tsub[2];
};

// Buckets from 2^126 up (and inf / NaN) never certify: (lo + hi) / 2 could overflow.
constexpr uint32_t kHugeBucket = 0x7F4u;

// Per-plane select scan (median.hip k_med_scan; fused into the Harris kernel's last
// workgroup of each plane): from the digit-1 histogram, the buckets holding the two
// middle ranks (exact-median state) and the certified-select thresholds.  Needs 256 or
// 512 threads (8 bins each for the first 256, one prefix pass for all five ranks); s_red
// holds 10 u32.
// `hist` is read with agent-scope atomic loads so a fused caller sees every workgroup's
// flush (L2 is per XCD); the 8 loads per thread are issued together.
SFM_DEV void select_scan_plane(const uint32_t* hist, MedianState* st, unsigned long long* list_count,
                               int64_t n, int64_t vmin, int force_exact, uint32_t* s_red) {
  static_assert(kMedBins1 == 256 * 8, "select scan: 8 bins per thread");
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool act = tid < 256;  // a 512-thread caller: the upper half holds no bins
  uint32_t v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
    v[j] = act ? __hip_atomic_load(hist + 8 * tid + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
  uint32_t local = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) local += v[j];
  uint32_t x = local;  // inclusive scan within the wave
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_red[wid] = x;
  __syncthreads();
  uint32_t wbase = 0;
  for (int w = 0; w < wid; ++w) wbase += s_red[w];
  const uint32_t excl = wbase + x - local;  // values in bins below this thread's first bin
  __syncthreads();
  const uint32_t k1 = (n % 2 == 1) ? (uint32_t)(n / 2) : (uint32_t)(n / 2 - 1);
  const uint32_t k2 = (uint32_t)(n / 2);
  const uint32_t kv = n > vmin ? (uint32_t)(n - vmin) : 0u;  // vmin-th largest value
  const int64_t vs0 = 3 * vmin / 8, vs1 = vmin / 2;          // the subset thresholds' ranks
  const uint32_t ks0 = n > vs0 ? (uint32_t)(n - vs0) : 0u, ks1 = n > vs1 ? (uint32_t)(n - vs1) : 0u;
  const uint32_t ranks[5] = {k1, k2, kv, ks0, ks1};
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const uint32_t r = ranks[q];
    if (r >= excl && r < excl + local) {  // exactly one thread owns each rank
      uint32_t c = excl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (r >= c && r < c + v[j]) {
          s_red[2 * q] = (uint32_t)(8 * tid + j);
          s_red[2 * q + 1] = r - c;  // residual rank inside the bucket
        }
        c += v[j];
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    const uint32_t b1 = s_red[0], r1 = s_red[1], b2 = s_red[2], r2 = s_red[3];
    // candidate threshold: the bucket holding the vmin-th largest value (so >= vmin values
    // lie at or above it), at least the median's lower bucket b1 (nothing below certifies)
    const uint32_t tb = max(n > vmin ? s_red[4] : 0u, b1);
    const bool certifiable = !force_exact && b2 < kHugeBucket;
    st->tnms = tb << (32 - kMedBits1);
    st->tsub[0] = max(n > vs0 ? s_red[6] : 0u, tb) << (32 - kMedBits1);
    st->tsub[1] = max(n > vs1 ? s_red[8] : 0u, tb) << (32 - kMedBits1);
    st->tcert = certifiable ? (b2 + 1) << (32 - kMedBits1) : 0xffffffffu;
    st->fallback = certifiable ? 0u : 1u;
    st->bucket[0] = b1;
    st->bucket[1] = b2;
    st->rank[0] = r1;
    st->rank[1] = r2;
    st->odd = (uint32_t)(n % 2);
    *list_count = 0ull;
  }
}

// Resolve one rank within bucket `bk` (the key's top 11 bits) from a collected list of keys
// (exact median, digits 2 and 3; every thread of the block calls it).
SFM_DEV uint32_t select_in_list(const uint32_t* lp, int64_t m, uint32_t bk, uint32_t rank,
                                uint32_t* s_h, uint32_t* s_scan, uint32_t* s_out) {
  const int tid = threadIdx.x, nt = blockDim.x;
  // digit 2: bits [20:10]
  for (int i = tid; i < kHistBins; i += nt) s_h[i] = 0u;
  __syncthreads();
  for (int64_t i = tid; i < m; i += nt) {
    uint32_t k = lp[i];
    if ((k >> 21) == bk) atomicAdd(&s_h[(k >> 10) & 0x7ffu], 1u);
  }
  __syncthreads();
  find_bin(s_h, kHistBins, rank, s_scan, s_out);
  uint32_t d2 = s_out[0];
  rank -= s_out[1];
  uint32_t pre = (bk << 11) | d2;  // top 22 bits
  __syncthreads();
  // digit 3: bits [9:0] (histogram padded to 4096 bins for find_bin)
  for (int i = tid; i < kHistBins; i += nt) s_h[i] = 0u;
  __syncthreads();
  for (int64_t i = tid; i < m; i += nt) {
    uint32_t k = lp[i];
    if ((k >> 10) == pre) atomicAdd(&s_h[k & 0x3ffu], 1u);
  }
  __syncthreads();
  find_bin(s_h, kHistBins, rank, s_scan, s_out);
  uint32_t d3 = s_out[0];
  __syncthreads();
  return (pre << 10) | d3;
}

// Arguments of the select scan fused into the Harris launch (state == nullptr: not fused).
struct SelectScan {
  MedianState* state;                  // [B]
  unsigned long long* list_count;      // [B], stride kCounterStride
  unsigned long long* done;            // [B], stride kCounterStride: workgroup arrivals (zeroed)
  int64_t vmin;
  int force_exact;
};

// Per-plane keypoint list produced by the top-k kernel (level coordinates).
struct KpList {
  int32_t* x;      // [planes][kcap]
  int32_t* y;
  float* conf;
  int32_t* count;  // [planes]
};

// pyramid.hip
void launch_u8_to_f32(const uint8_t* src, float* dst, int64_t n, hipStream_t st);

// ransac.hip: CameraPose.find_inliers (SFM.py:126-160) for P correspondence sets
// pts [P][nmax][4] int32 (x1, y1, x2, y2), sample indices idx (+ idx_off[p]) [iters][8].
void ransac_sample_indices(int n, int iters, uint32_t seed, int32_t* out);
void launch_ransac(const int32_t* pts, const int32_t* npts, int nmax, int P, const int32_t* idx,
                   const int32_t* idx_off, int iters, double thr, double* Fs, int32_t* counts, int32_t* out_pts,
                   int32_t* out_n, int32_t* out_iter, hipStream_t st);

// ingest.hip: PIL BICUBIC resize of [B][H][W][3] u8 RGB to H2 x W2 + /255 + _rgb2gray
// (Runner.py:33-46) -> [B][H2][W2] float32; tmp holds [B][H][W2][3] u8.  Tables from
// build_resample_table (host, Pillow's double-precision taps in 22-bit fixed point).
int build_resample_table(int in, int out, std::vector<int32_t>& tab);
bool ingest_rows_tables(const std::vector<int32_t>& tab_h, int ks_h, int W, int W2, int ks,
                        std::vector<int32_t>& colmap, std::vector<int32_t>& sets);
int ingest_rows_ks(int ks_h, int ks_v);
void launch_ingest_rgb(const uint8_t* rgb, uint8_t* tmp, float* gray, const int32_t* tab_h, int ks_h,
                       const int32_t* tab_v, int ks_v, const int32_t* colmap, const int32_t* sets, int nsets,
                       int B, int H, int W, int H2, int W2, hipStream_t st);
// levels l+1..l+3 of exact 2x steps in one pass; false (nothing launched) when the sizes or
// alignments do not allow it
// z0 / z1 (optional, 16-B aligned, multiples of 16 B): buffers the launch zeroes on the side
bool launch_down2x3(const float* src, int sh, int sw, float* d1, float* d2, float* d3, int B, hipStream_t st,
                    void* z0 = nullptr, size_t z0_bytes = 0, void* z1 = nullptr, size_t z1_bytes = 0);
void launch_resize(const float* src, int sh, int sw, float* dst, int dh, int dw, int B,
                   hipStream_t st);

// harris.hip: R map + first median digit histogram (hist zeroed by the caller); with
// scan.state set, the last workgroup of each plane also runs select_scan_plane.
void launch_harris(const float* lvl, float* R, uint32_t* hist, int B, int H, int W,
                   const float* d_gauss, int ks, float alpha, SelectScan scan, hipStream_t st);
// Several pyramid levels of a batch in one Harris launch (workgroups partitioned by
// level; tiles_x / ntiles / wg0 / nwg are filled in by the launcher)
constexpr int kHarrisMaxLevels = 4;
struct HarrisLevels {
  struct Level {
    const float* lvl;
    float* R;
    uint32_t* hist;
    int H, W, tiles_x, ntiles, wg0, nwg;
    SelectScan scan;
    // fused pyramid (64 x 64 tiles, H and W multiples of 8): the three exact 2x levels below
    // this one, written from the image tile in LDS (nullptr: none)
    float* down[3];
  } l[kHarrisMaxLevels];
  int n;
  int prio;  // 1: waves raise their issue priority with the tiles they have left (A/B)
  int stagger;  // n > 0: odd workgroups sleep n x 8k cycles before their first tile (A/B)
  // kernel-active span of this launch (sfm_profile_spans; nullptr: off): {earliest workgroup
  // start, latest workgroup end} on the device's constant-rate realtime clock, folded in with
  // one atomic min / max per workgroup (the slot starts at {~0, 0})
  unsigned long long* span;
};
void launch_harris_levels(const HarrisLevels& g, int B, const float* d_gauss, int ks, float alpha,
                          hipStream_t st);
// The Harris launches' tap buffer (d_gauss above): the ks x ks Gaussian taps (row-major) at 0,
// then from float kHarrisPairOff the window's tap pairs (g[d][j], g[d-1][j]) for d = 0..ks,
// j < ks (a missing tap row is 0), which the kernel reads as wave-uniform scalar loads.
constexpr int kHarrisPairOff = 256;
size_t harris_taps_floats(int ks);
void harris_taps_build(const float* g, int ks, float* out);

int64_t match_stamps_copy(uint64_t* out, int64_t cap);
// words of the sweep's work-unit list (k_match_units) for P pairs of up to max_rows rows
size_t match_units_words(int P, int max_rows);
float time_harris_ablation(int abl, const float* lvl, float* R, uint32_t* hist, int B, int H, int W,
                           const float* gk, float alpha, int iters, uint64_t* stamps = nullptr,
                           int64_t stamps_cap = 0);

// median.hip.  launch_select_scan: median buckets + certified threshold per plane
// (vmin = pixels required at or above the threshold).  launch_median_exact: the exact
// median of the planes flagged `fallback`.
void launch_select_scan(const uint32_t* hist, MedianState* state, unsigned long long* list_count, int B,
                        int H, int W, int64_t vmin, int force_exact, hipStream_t st);
void launch_median_exact(const float* R, MedianState* state, uint32_t* list, unsigned long long* list_count,
                         int B, int H, int W, hipStream_t st);

// nms.hip: candidates as 64-bit keys (~fkey(conf) << 32 | raster index), appended per
// plane.  mode 0 (certified planes): R == window max && key(R) >= tnms; mode 1 (fallback
// planes): the exact predicate (R == window max, or R == 0 below the median).
// force_tile: the tiled kernel for the certified 3x3 case too (parity test of both forms)
void launch_nms(const float* R, const MedianState* state, uint64_t* cand,
                unsigned long long* cand_count, int B, int H, int W, int ksize, int mode, hipStream_t st,
                int force_tile = 0);

// select.hip: keypoint selection of one level, one workgroup per plane: top-k by (conf
// desc, index asc) of the certified NMS candidates + edge filter (NaiveSIFT.py:99-120);
// planes that do not certify (or are flagged fallback already) run the exact path in the
// same workgroup: exact median into state.median (medlist: n u32 per plane), the full NMS
// predicate into cand (n u64 per plane), then the same top-k.  scratch: n u64 per plane.
void init_topk_attributes();
void init_describe_attributes(size_t max_lds);
// the quad describe kernel's bin-edge key tables on the current device (once per device)
void init_describe_quad_tables();
size_t describe_lds_bytes(int fw, int rotate);
void launch_select(const float* R, uint64_t* cand, const unsigned long long* cand_count, uint32_t* medlist,
                   uint64_t* scratch, KpList kp, int kcap, int k, int B, int H, int W, int ksize, int half_window,
                   MedianState* state, hipStream_t st);
// Several levels' selections in one launch (B workgroups per level, level-major); each
// level brings its own medlist / scratch regions (they must not overlap).
constexpr int kSelectMaxLevels = 4;
struct SelectLevels {
  struct Level {
    const float* R;
    uint64_t* cand;
    const unsigned long long* cand_count;
    uint32_t* medlist;
    uint64_t* scratch;
    KpList kp;
    MedianState* state;
    int H, W, hw;
  } l[kSelectMaxLevels];
  int n;
};
void launch_select_levels(const SelectLevels& g, int kcap, int k, int B, int ksize, hipStream_t st);

// describe_q.hip: four keypoints per wavefront for window widths 2..22 (false: not handled)
// out_count (the last level's launch): also write each slot's keypoint count
bool launch_describe_quad(const float* lvl, int B, int H, int W, int fw, int rotate, KpList kp, int kcap,
                          const int32_t* level_counts_all, int level, double scale, int32_t* out_xy,
                          float* out_desc, float* out_conf, int64_t out_cap, int32_t* out_count, int L,
                          const MatchOperands& mo, hipStream_t st);
// describe.hip: descriptors of one level written into the output slot table; returns true when
// the launch also wrote the slot counts (out_count set and the quad kernel took the level),
// otherwise the caller runs launch_finalize_counts
// mo.hi set: the quad kernel also writes the matcher operands of every row (and, in the last
// level's launch, the padding rows); *operands_written reports whether it did (the
// one-wavefront kernel of widths above 22 does not)
bool launch_describe(const float* lvl, int B, int H, int W, int fw, int rotate, KpList kp,
                     int kcap, const int32_t* level_counts_all, int level, int L, double scale,
                     int32_t* out_xy, float* out_desc, float* out_conf, int64_t out_cap,
                     int32_t* out_count, const MatchOperands& mo, bool* operands_written, hipStream_t st);
void launch_finalize_counts(const int32_t* level_counts_all, int B, int L, int32_t* out_count,
                            hipStream_t st);

// match.hip
struct RowBest {
  int32_t col;   // -1: rejected
  float nndr;
};
void launch_transpose_desc(const float* desc, const int32_t* count, int nimg, int64_t cap,
                           int64_t capP, float* descT, hipStream_t st);
void launch_match_rows(const float* descT, const int32_t* count, int64_t capP, const int32_t* pairs,
                       int P, float ratio, RowBest* rows, int max_rows, hipStream_t st);
void launch_match_compact(const RowBest* rows, const int32_t* count, const int32_t* pairs, int P,
                          int max_rows, int64_t cap, int32_t* matches, float* conf, int32_t* nmatch,
                          int* reset_counter, hipStream_t st);
void init_match_attributes(int max_rows);
// match_mfma.hip: exact matching with the split-fp16 MFMA prefilter
// pmax: per-16-row-block maxima of (norm2, norm) per image, match_pmax_bytes(capP) per image
size_t match_pmax_bytes(int64_t capP);
void launch_match_prep(const float* desc, const int32_t* count, int nimg, int64_t cap, int64_t capP,
                       _Float16* hi, _Float16* lo, float* norm2, float* rnorm, void* pmax, hipStream_t st);
void launch_match_mfma(const float* desc, const int32_t* count, int64_t cap, int64_t capP,
                       const _Float16* hi, const _Float16* lo, const float* norm2, const float* rnorm,
                       const void* pmax, const int32_t* pairs, int P, float ratio,
                       RowBest* rows, int max_rows, uint32_t* cand, int32_t* cand_n, float* cand_thr,
                       int* ovf_count, int2* ovf_list, int32_t* units, hipStream_t st);

}  // namespace sfm
