// sfmfeat_api.hip — the C-ABI (include/sfmfeat.h): contexts, device workspace and the
// per-batch launch sequence of the detect + describe + match stage.
//
// Launch sequence for a batch of B same-size images (one stream, no host sync inside):
//   pyramid (L-1 resize launches)
//   per level: harris(+digit histogram) -> median (scan, collect, final) -> nms/candidates
//              -> top-k + edge filter
//   per level: descriptors into the caller's slot table; finalize counts
// Matching: transpose slot table -> row kernel (exact pairwise distances, best/second)
//           -> per-pair compaction + (nndr, row) sort.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sfmfeat.h"
#include "kernels.h"

using namespace sfm;

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct Level {
  int h, w, fw;
  double scale;
};

// slots beyond an extraction's batch the fused matcher operand buffers are sized for (a match
// of the batch's table with a few extra slots then needs no reallocation)
constexpr int kFusedPrepSpare = 8;

}  // namespace

// Lane gate (sfm_gate_*): the contexts of batches in flight share one; each extraction's
// pyramid starts after the previous gated extraction's level-0 Harris launch has finished
// (SFMFEAT_GATE_LEVEL moves the release point), so the two batches' largest VALU launches
// alternate instead of competing for the CUs.
struct sfm_gate {
  int device = 0;
  hipEvent_t ev = nullptr;  // release point of the last gated extraction (timing disabled)
  bool armed = false;       // ev has been recorded
};

struct sfm_ctx {
  int device = 0;
  sfm_gate* gate = nullptr;
  sfm_params p;
  hipStream_t stream = nullptr;
  // extraction fork/join: keypoint selection + description of level l run on `aux` while
  // the caller's stream computes Harris + NMS of level l + 1 (events ev[0..SFM_MAX_LEVELS])
  hipStream_t aux = nullptr;
  hipEvent_t ev[SFM_MAX_LEVELS + 3] = {};
  std::string err;
  int L = 1;
  int kcap = 0;       // per-level keypoint capacity = int(k / L) (ScaleRotInvSIFT.py:90)
  int64_t cap = 0;    // per-image capacity = L * kcap
  float gauss[SFM_MAX_GAUSS * SFM_MAX_GAUSS];
  DevBuf d_gauss, d_img0, d_lvl, d_R, d_hist, d_med, d_medlist, d_counts, d_cand, d_scratch,
      d_kpx, d_kpy, d_kpc, d_lc, d_xy, d_desc, d_conf, d_count, d_u8;
  DevBuf m_desc, m_count, m_pairs, m_descT, m_rows, m_matches, m_conf, m_nmatch;
  DevBuf m_hi, m_lo, m_norm2, m_rnorm, m_imgmax, m_ovf, m_ovfc, m_cand, m_candn, m_candt, m_units;
  // ingest (sfm_ingest_rgb*): resample tables for the cached (W -> W2, H -> H2) and the
  // RGB temp of the horizontal pass; host staging for the host-pointer variant
  DevBuf i_tab_h, i_tab_v, i_tmp, i_rgb, i_gray;
  int i_w = -1, i_w2 = -1, i_h = -1, i_h2 = -1, i_ksh = 0, i_ksv = 0;
  std::vector<int32_t> i_th, i_tv;  // host copies of the tables
  // RANSAC (sfm_ransac_*): sample-index streams cached per (n, iterations), device buffers
  std::vector<std::pair<std::pair<int, int>, std::vector<int32_t>>> r_cache;
  DevBuf r_idx, r_off, r_F, r_counts, r_pts, r_npts, r_out, r_on, r_oit;
  DevBuf i_colmap, i_sets;          // row path (k_rows_h): column map + tap sets
  int i_nsets = 0;
  bool i_rows = false;
  // the table the matcher operands were last prepped for (sfm_match_prep_dev): a prepped
  // match call on any other table is SFM_ESTATE
  const float* prep_desc = nullptr;
  const int32_t* prep_count = nullptr;
  int prep_nimg = -1;
  int64_t prep_cap = -1;
  // fused matcher operands (sfm_ctx_set_fused_prep): the last extraction on this context wrote
  // the operands of slots [0, fp_B) of the table (fp_desc, fp_count, fp_cap) itself
  bool fused_prep = false;
  const float* fp_desc = nullptr;
  const int32_t* fp_count = nullptr;
  int64_t fp_cap = -1;
  int fp_B = 0;
  bool match_direct = false;  // SFMFEAT_MATCH_DIRECT=1: all-pairs exact VALU kernel (A/B checks)
  bool exact_select = false;
  bool serial = false;        // SFMFEAT_SERIAL=1: no aux-stream overlap (diagnostic timings)
  int prio = 0;               // stream priority of both context streams (sfm_ctx_set_priority)
  // SFMFEAT_MATCH_BUDGET_MB: matcher per-pair workspace bound (4 GB: 1,575 pairs of 2,500 rows per
  // sub-launch at 256 admitted targets per row, configs[2]'s 4,096-pair calls in three)
  size_t match_budget = (size_t)4096 << 20;
  int last_B = 0;             // planes per level of the last extraction
  int last_H = 0, last_W = 0;
  // stage profiling (sfm_profile_*): HIP events bracketing each stage's launches
  bool prof = false;
  uint32_t prof_mask = ~0u;  // stages bracketed while profiling (sfm_profile_stages)
  int64_t extractions = 0;  // extract_impl calls (SFMFEAT_SKIP leaves the first one whole)
  int64_t match_calls = 0;  // match sub-launches (likewise)
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> prof_pending;
  std::vector<hipEvent_t> prof_pool;
  double prof_ms[SFM_PROF_STAGES] = {0};
  int64_t prof_launches[SFM_PROF_STAGES] = {0};
  // kernel-active spans of the Harris launches (sfm_profile_spans): span_cap slots of
  // {start, end} realtime ticks, the next free slot, each slot's first pyramid level
  DevBuf d_spans;
  int64_t span_cap = 0, span_n = 0, span_dropped = 0;
  std::vector<int32_t> span_level;
};

namespace {

hipEvent_t prof_event(sfm_ctx* c) {
  if (!c->prof_pool.empty()) {
    hipEvent_t e = c->prof_pool.back();
    c->prof_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

// RAII bracket: records a start event now and a stop event at scope exit (when enabled).
struct StageScope {
  sfm_ctx* c;
  int stage;
  hipStream_t st;
  hipEvent_t a = nullptr, b = nullptr;
  StageScope(sfm_ctx* c_, int stage_, hipStream_t st_) : c(c_), stage(stage_), st(st_) {
    if (c->prof && ((c->prof_mask >> stage) & 1u)) {
      a = prof_event(c);
      b = prof_event(c);
      (void)hipEventRecord(a, st);
    }
  }
  ~StageScope() {
    if (a) {
      (void)hipEventRecord(b, st);
      c->prof_pending.push_back({stage, {a, b}});
    }
  }
};

int set_err(sfm_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIPCHK(ctx, expr)                                                              \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return set_err(ctx, SFM_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

int ensure(sfm_ctx* c, DevBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.bytes >= bytes) return SFM_OK;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  HIPCHK(c, hipMalloc(&b.p, bytes));
  b.bytes = bytes;
  return SFM_OK;
}

// the stream of the host-pointer calls, created on first use
int host_stream(sfm_ctx* c, hipStream_t* out) {
  if (!c->stream) HIPCHK(c, hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, c->prio));
  *out = c->stream;
  return SFM_OK;
}

template <class T>
T* as(DevBuf& b) {
  return reinterpret_cast<T*>(b.p);
}

void free_buf(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

// NaiveSIFT._generate_gaussian_kernel (NaiveSIFT.py:175-199) evaluated natively in double
// (numpy's linspace/exp/sum order); the Python wrapper passes numpy's own taps instead.
void gaussian_taps(int ks, double sigma, float* out) {
  double ax[SFM_MAX_GAUSS], k[SFM_MAX_GAUSS * SFM_MAX_GAUSS];
  int m = ks / 2;
  if (ks == 1) {
    ax[0] = (double)-m;
  } else {
    double step = ((double)m - (double)-m) / (double)(ks - 1);
    for (int i = 0; i < ks; ++i) ax[i] = (double)i * step + (double)-m;
    ax[ks - 1] = (double)m;
  }
  const double PI = 3.141592653589793;
  double c = 1.0 / (2.0 * PI * (sigma * sigma));
  double den = 2.0 * (sigma * sigma);
  for (int i = 0; i < ks; ++i)
    for (int j = 0; j < ks; ++j) k[i * ks + j] = c * exp(-((ax[i] * ax[i]) + (ax[j] * ax[j])) / den);
  int n = ks * ks;
  double total = 0.0;
  if (n < 8) {
    for (int i = 0; i < n; ++i) total += k[i];
  } else {
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = k[j];
    int i;
    for (i = 8; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += k[i + j];
    total = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) total += k[i];
  }
  for (int i = 0; i < n; ++i) out[i] = (float)(k[i] / total);
}

bool gauss_size_supported(int ks) {
  return (ks >= 1 && ks <= 9) || ks == 11 || ks == 13 || ks == 15;
}

int geometry(const sfm_params* p, int H, int W, std::vector<Level>& lv) {
  int L = p->mode == SFM_MODE_NAIVE ? 1 : p->pyramid_level;
  if (L < 1 || L > SFM_MAX_LEVELS) return SFM_EINVAL;
  lv.resize(L);
  int h = H, w = W;
  for (int l = 0; l < L; ++l) {
    if (l > 0) {
      h = (int)((double)h / p->pyramid_scale_factor);  // int(h / s) (ScaleRotInvSIFT.py:114)
      w = (int)((double)w / p->pyramid_scale_factor);
    }
    if (h <= 0 || w <= 0) return SFM_EINVAL;
    double scale = p->mode == SFM_MODE_NAIVE ? 1.0 : pow(p->pyramid_scale_factor, (double)l);
    int fw = p->mode == SFM_MODE_NAIVE ? p->feature_width : (int)((double)p->feature_width / scale);
    if (p->mode != SFM_MODE_NAIVE && fw < 3) fw = 3;  // min_feature_width (:92,:96)
    lv[l] = Level{h, w, fw, scale};
  }
  return SFM_OK;
}

int reserve_impl(sfm_ctx* c, int B, int H, int W) {
  std::vector<Level> lv;
  if (geometry(&c->p, H, W, lv) != SFM_OK)
    return set_err(c, SFM_EINVAL, "image too small for the pyramid");
  int64_t A0 = (int64_t)H * W, Arest = 0;
  for (int l = 1; l < c->L; ++l) Arest += (int64_t)lv[l].h * lv[l].w;
  int rc;
  if ((rc = ensure(c, c->d_img0, (size_t)B * A0 * 4))) return rc;
  if ((rc = ensure(c, c->d_lvl, (size_t)B * Arest * 4))) return rc;
  if ((rc = ensure(c, c->d_R, (size_t)B * (A0 + Arest) * 4))) return rc;       // one R map per level
  if ((rc = ensure(c, c->d_hist, (size_t)c->L * B * kMedBins1 * 4))) return rc;
  if ((rc = ensure(c, c->d_med, (size_t)c->L * B * sizeof(MedianState)))) return rc;
  // keypoint-selection scratch (tie lists) and exact-median lists: the aux stream's levels
  // share region [0, B*A0); the caller stream's levels each own a region starting at B*A0,
  // packed by level (extract_impl); SFMFEAT_SERIAL puts every level's region from 0.
  // B * (A0 + A0 + Arest) covers both layouts at any pyramid_scale_factor.
  const size_t sel_slots = (size_t)B * (2 * A0 + Arest);
  if ((rc = ensure(c, c->d_medlist, sel_slots * 4))) return rc;
  if ((rc = ensure(c, c->d_counts, (size_t)4 * c->L * B * 8 * kCounterStride))) return rc;
  if ((rc = ensure(c, c->d_cand, (size_t)B * (A0 + Arest) * 8))) return rc;    // candidates per level
  if ((rc = ensure(c, c->d_scratch, sel_slots * 8))) return rc;
  size_t nk = (size_t)c->L * B * (size_t)std::max(c->kcap, 1);
  if ((rc = ensure(c, c->d_kpx, nk * 4))) return rc;
  if ((rc = ensure(c, c->d_kpy, nk * 4))) return rc;
  if ((rc = ensure(c, c->d_kpc, nk * 4))) return rc;
  if ((rc = ensure(c, c->d_lc, (size_t)c->L * B * 4))) return rc;
  return SFM_OK;
}

// SFMFEAT_SKIP=mask (timing bounds only, results wrong by design): stages whose launches are
// left out from a context's second extraction on (the first fills every buffer the skipped
// stages' consumers read) — 1 keypoint selection, 2 descriptors, 8 match sweep + re-rank,
// 16 Harris of the levels above 0
int skip_mask() {
  static const int m = [] {
    const char* e = SFM_ABLATION_ENV("SFMFEAT_SKIP");
    return e ? atoi(e) : 0;
  }();
  return m;
}

// The matcher operand buffers hold `nimg` slots of capP rows (no reallocation: false when they
// are smaller, i.e. a prep of that many slots would reallocate them and lose their contents).
bool match_operands_fit(const sfm_ctx* c, int nimg, int64_t capP) {
  return c->m_hi.bytes >= (size_t)nimg * capP * 128 * 2 && c->m_imgmax.bytes >= (size_t)nimg * match_pmax_bytes(capP);
}

int match_operands_reserve(sfm_ctx* c, int nimg, int64_t capP) {
  int rc;
  if ((rc = ensure(c, c->m_hi, (size_t)nimg * capP * 128 * 2))) return rc;
  if ((rc = ensure(c, c->m_lo, (size_t)nimg * capP * 128 * 2))) return rc;
  if ((rc = ensure(c, c->m_norm2, (size_t)nimg * capP * 4))) return rc;
  if ((rc = ensure(c, c->m_rnorm, (size_t)nimg * capP * 4))) return rc;
  if ((rc = ensure(c, c->m_imgmax, (size_t)nimg * match_pmax_bytes(capP)))) return rc;
  return SFM_OK;
}

int extract_impl(sfm_ctx* c, const float* imgs, int B, int H, int W, int32_t* xy, float* desc,
                 float* conf, int32_t* count, int64_t cap, hipStream_t st) {
  if (B < 1 || H < 1 || W < 1) return set_err(c, SFM_EINVAL, "empty batch or image");
  if (cap < c->cap) return set_err(c, SFM_ERANGE, "slot capacity below L * int(k / L)");
  std::vector<Level> lv;
  if (geometry(&c->p, H, W, lv) != SFM_OK)
    return set_err(c, SFM_EINVAL, "image too small for the pyramid");
  int rc = reserve_impl(c, B, H, W);
  if (rc) return rc;
  const int L = c->L;
  const int skip = c->extractions++ > 0 ? skip_mask() : 0;
  if (c->gate && c->gate->armed) HIPCHK(c, hipStreamWaitEvent(st, c->gate->ev, 0));
  c->last_B = B;
  c->last_H = H;
  c->last_W = W;
  // pyramid
  std::vector<const float*> lvl(L);
  lvl[0] = imgs;
  // the first three-level pyramid pass also zeroes the histograms and append counters
  const size_t hist_bytes = (size_t)L * B * kMedBins1 * 4, count_bytes = (size_t)4 * L * B * 8 * kCounterStride;
  static const bool fill_launches = [] {  // SFMFEAT_FILL_LAUNCHES=1: separate fills (A/B)
    const char* e = SFM_DIAG_ENV("SFMFEAT_FILL_LAUNCHES");
    return e && atoi(e) != 0;
  }();
  bool zeroed = fill_launches;
  // Levels 1-3 exact 2x below level 0 (H, W multiples of 8): the level-0 Harris launch writes
  // them from its image tiles in LDS (level 0 is read from HBM once; round 4: 35.6k -> 37.3k
  // img/s at configs[1]), levels >= 4 follow that launch, and the histograms / counters take
  // the fill launches instead of k_down2x3's side job.  SFMFEAT_PYR_FUSED=0: k_down2x3 (A/B).
  static const bool pyr_fused_env = [] {
    const char* e = getenv("SFMFEAT_PYR_FUSED");
    return !e || atoi(e) != 0;
  }();
  const bool pyr_fused = pyr_fused_env && L >= 4 && H % 8 == 0 && W % 8 == 0 && lv[1].h * 2 == H &&
                         lv[1].w * 2 == W && lv[2].h * 4 == H && lv[2].w * 4 == W && lv[3].h * 8 == H &&
                         lv[3].w * 8 == W;
  // levels [from, L) from their predecessors: three exact 2x levels from one read of their
  // source where the sizes allow, else one resize per level
  auto pyramid_from = [&](int from) {
    for (int l = from; l < L;) {
      // three exact 2x levels from one read of their source where the sizes allow
      const auto& s = lv[l - 1];
      const bool x2 = l + 2 < L && lv[l].h * 2 == s.h && lv[l].w * 2 == s.w && lv[l + 1].h * 4 == s.h &&
                      lv[l + 1].w * 4 == s.w && lv[l + 2].h * 8 == s.h && lv[l + 2].w * 8 == s.w;
      if (x2 && launch_down2x3(lvl[l - 1], s.h, s.w, const_cast<float*>(lvl[l]), const_cast<float*>(lvl[l + 1]),
                               const_cast<float*>(lvl[l + 2]), B, st, zeroed ? nullptr : c->d_hist.p, hist_bytes,
                               zeroed ? nullptr : c->d_counts.p, count_bytes)) {
        zeroed = true;
        l += 3;
        continue;
      }
      launch_resize(lvl[l - 1], s.h, s.w, const_cast<float*>(lvl[l]), lv[l].h, lv[l].w, B, st);
      ++l;
    }
  };
  {
    StageScope sc(c, SFM_PROF_PYRAMID, st);
    int64_t off = 0;
    for (int l = 1; l < L; ++l) {
      float* dst = as<float>(c->d_lvl) + off;
      lvl[l] = dst;
      off += (int64_t)B * lv[l].h * lv[l].w;
    }
    if (!pyr_fused) pyramid_from(1);
  }
  // fused matcher operands: buffers for the B slots (plus spare slots, so a match of the table
  // with a few extra slots, e.g. BatchPipeline's halo slot, does not reallocate them), their
  // per-block maxima zeroed ahead of the descriptor launches' atomic maxima
  MatchOperands mo{nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  c->fp_desc = nullptr;  // (a failed or non-fused extraction leaves no fused slots)
  c->fp_B = 0;
  if (c->fused_prep && !c->match_direct) {
    const int64_t capP = (cap + 127) / 128 * 128;
    if (!match_operands_fit(c, B + kFusedPrepSpare, capP) &&
        (rc = match_operands_reserve(c, B + kFusedPrepSpare, capP)))
      return rc;
    mo = MatchOperands{as<_Float16>(c->m_hi), as<_Float16>(c->m_lo), as<float>(c->m_norm2), as<float>(c->m_rnorm),
                       as<float2>(c->m_imgmax), capP};
    HIPCHK(c, hipMemsetAsync(c->m_imgmax.p, 0, (size_t)B * match_pmax_bytes(capP), st));
  }
  bool fused_ok = mo.hi != nullptr;
  if (!zeroed || fill_launches) {
    HIPCHK(c, hipMemsetAsync(c->d_hist.p, 0, hist_bytes, st));
    HIPCHK(c, hipMemsetAsync(c->d_counts.p, 0, count_bytes, st));
    // the fused pyramid's later k_down2x3 (pyramid_from(4), after level 0's Harris) must not
    // zero them again: level 0's histogram and counters are live by then
    zeroed = true;
  }
  unsigned long long* medcnt = as<unsigned long long>(c->d_counts);
  unsigned long long* candcnt = medcnt + (size_t)L * B * kCounterStride;    // certified NMS
  unsigned long long* candcnt2 = candcnt + (size_t)L * B * kCounterStride;  // fallback NMS
  unsigned long long* donecnt = candcnt2 + (size_t)L * B * kCounterStride;  // Harris arrivals
  const float alpha = (float)c->p.alpha;  // NEP 50: the python float becomes float32
  // certified select: at least max(65536, 128 k) pixels at or above the threshold
  const int64_t vmin = std::max<int64_t>(65536, (int64_t)128 * c->kcap);
  // Fork/join over two streams.  The caller's stream runs Harris (+ fused select scan) and
  // the certified NMS of every level; the keypoint selection (top-k, the exact path for
  // the planes flagged `fallback`) and the descriptors of the two largest levels run on
  // `aux`, overlapping the later levels' Harris; the small levels' selection and
  // descriptors run on the caller's stream once its Harris work is done.  Descriptors of
  // level l need the keypoint counts of levels < l (slot offsets): ev[L + 2 + l].
  // serial (SFMFEAT_SERIAL=1 or sfm_ctx_set_serial): one stream, no fork/join at all
  const int L_aux = c->serial ? 0 : std::min(L, 2);
  hipStream_t ax = nullptr;
  if (L_aux > 0) {
    if (!c->aux) HIPCHK(c, hipStreamCreateWithPriority(&c->aux, hipStreamNonBlocking, c->prio));  // on first use
    ax = c->aux;
    HIPCHK(c, hipEventRecord(c->ev[L], st));
    HIPCHK(c, hipStreamWaitEvent(ax, c->ev[L], 0));
  }
  const int rotate = c->p.mode == SFM_MODE_NAIVE ? 0 : 1;
  struct LevelBufs {
    float* R;
    uint64_t* cand;
    MedianState* med;
    KpList kp;
    size_t co;
    bool exact;
  };
  // levels of fewer than 128 x kcap pixels (the certified select's vmin) skip certification:
  // they hardly ever certify (4K level 3 never did), and the attempt costs a certified NMS
  // pass and a top-k before the exact path (configs[4] 8.85k -> 9.02k img/s with 128 against
  // 64; 1080p takes the same levels either way).  SFMFEAT_EXACT_PX=n: n x kcap (A/B)
  static const int exact_px = [] {
    const char* e = getenv("SFMFEAT_EXACT_PX");
    return e ? atoi(e) : 128;
  }();
  std::vector<LevelBufs> lb(L);
  int64_t plane_off = 0;  // element offset of level l's planes in the per-level R / candidates
  for (int l = 0; l < L; ++l) {
    const int h = lv[l].h, w = lv[l].w;
    LevelBufs& e = lb[l];
    e.co = (size_t)l * B * kCounterStride;
    e.R = as<float>(c->d_R) + plane_off;
    e.cand = as<uint64_t>(c->d_cand) + plane_off;
    plane_off += (int64_t)B * h * w;
    e.med = as<MedianState>(c->d_med) + (size_t)l * B;
    const size_t ko = (size_t)l * B * std::max(c->kcap, 1);
    e.kp.x = as<int32_t>(c->d_kpx) + ko;
    e.kp.y = as<int32_t>(c->d_kpy) + ko;
    e.kp.conf = as<float>(c->d_kpc) + ko;
    e.kp.count = as<int32_t>(c->d_lc) + (size_t)l * B;
    // levels too small to certify go straight to the exact path (a size-only decision: no
    // host synchronisation)
    e.exact = c->exact_select || (int64_t)h * w < (int64_t)exact_px * c->kcap;
  }
  auto select_level = [&](int l, hipStream_t s) {  // top-k, exact path in the same launch
    const LevelBufs& e = lb[l];
    StageScope sc(c, SFM_PROF_TOPK, s);
    // the scratch regions of this level's stream (the aux stream's levels and the caller
    // stream's levels select concurrently)
    const int64_t so = l < L_aux ? 0 : (int64_t)B * H * W;
    if (skip & 1) return;
    launch_select(e.R, e.cand, candcnt + e.co, as<uint32_t>(c->d_medlist) + so, as<uint64_t>(c->d_scratch) + so, e.kp,
                  std::max(c->kcap, 1), c->kcap, B, lv[l].h, lv[l].w, c->p.ksize, lv[l].fw / 2, e.med, s);
  };
  bool counted = false;  // the last level's describe launch wrote the slot counts
  auto describe_level = [&](int l, hipStream_t s) {
    StageScope sc(c, SFM_PROF_DESCRIBE, s);
    if ((skip & 2) && l != L - 1) {
      fused_ok = false;
      return;
    }
    bool ow = false;
    const bool r = launch_describe(lvl[l], B, lv[l].h, lv[l].w, lv[l].fw, rotate, lb[l].kp, c->kcap,
                                   as<int32_t>(c->d_lc), l, L, lv[l].scale, xy, desc, conf, cap,
                                   l == L - 1 ? count : nullptr, mo, &ow, s);
    if (l == L - 1) counted = r;
    fused_ok = fused_ok && ow;
  };
  // Harris launches: one per level, unless SFMFEAT_HARRIS_GROUP=g (g >= 1): levels >= g then
  // share launches (up to kHarrisMaxLevels each).  Off by default: grouping L1-L3 or L2-L3 cut
  // the Harris stage time by ~2% but the pipeline lost more overlap than that (DESIGN_LOG.md §B).
  static const int group_from = [] {
    const char* e = SFM_DIAG_ENV("SFMFEAT_HARRIS_GROUP");
    return e ? atoi(e) : 0;
  }();
  // the lane gate's release point: after the Harris launch of level gate_level (default 0:
  // the next gated extraction's pyramid and level-0 Harris follow this one's level-0 Harris;
  // SFMFEAT_GATE_LEVEL=-1: after every level's Harris and NMS)
  static const int gate_level = [] {
    const char* e = SFM_DIAG_ENV("SFMFEAT_GATE_LEVEL");
    return e ? atoi(e) : 0;
  }();
  bool gate_released = false;
  auto release_gate = [&]() -> int {
    if (c->gate && !gate_released) {
      HIPCHK(c, hipEventRecord(c->gate->ev, st));
      c->gate->armed = true;
      gate_released = true;
    }
    return SFM_OK;
  };
  for (int l0 = 0; l0 < L;) {
    int l1 = l0 + 1;
    if (group_from > 0 && l0 >= group_from) l1 = std::min(L, l0 + kHarrisMaxLevels);
    {
      StageScope sc(c, SFM_PROF_HARRIS, st);
      HarrisLevels g{};
      g.n = l1 - l0;
      for (int l = l0; l < l1; ++l) {
        const LevelBufs& e = lb[l];
        HarrisLevels::Level& q = g.l[l - l0];
        q.lvl = lvl[l];
        q.R = e.R;
        q.hist = as<uint32_t>(c->d_hist) + (size_t)l * B * kMedBins1;
        q.H = lv[l].h;
        q.W = lv[l].w;
        q.scan = SelectScan{e.med, medcnt + e.co, donecnt + e.co, vmin, e.exact ? 1 : 0};
        q.down[0] = q.down[1] = q.down[2] = nullptr;
        if (pyr_fused && l == 0) {
          q.down[0] = const_cast<float*>(lvl[1]);
          q.down[1] = const_cast<float*>(lvl[2]);
          q.down[2] = const_cast<float*>(lvl[3]);
        }
      }
      if (c->span_cap > 0) {
        if (c->span_n < c->span_cap) {
          g.span = as<unsigned long long>(c->d_spans) + 2 * c->span_n++;
          c->span_level.push_back(l0);
        } else {
          ++c->span_dropped;
        }
      }
      if (!(l0 > 0 && (skip & 16))) launch_harris_levels(g, B, as<float>(c->d_gauss), c->p.gaussian_size, alpha, st);
    }
    if (pyr_fused && l0 == 0 && L > 4) {
      StageScope sc(c, SFM_PROF_PYRAMID, st);
      pyramid_from(4);
    }
    if (gate_level >= l0 && gate_level < l1 && (rc = release_gate())) return rc;
    for (int l = l0; l < l1; ++l) {
      const LevelBufs& e = lb[l];
      if (!e.exact) {
        StageScope sc(c, SFM_PROF_NMS, st);
        launch_nms(e.R, e.med, e.cand, candcnt + e.co, B, lv[l].h, lv[l].w, c->p.ksize, 0, st);
      }
      if (l < L_aux) {
        // SFMFEAT_SELECT_CALLER=1 (A/B): the level's selection on the caller's stream ahead of
        // the next level's Harris, only its descriptors on aux
        static const bool sel_caller = [] {
          const char* e = SFM_DIAG_ENV("SFMFEAT_SELECT_CALLER");
          return e && atoi(e) == 1;
        }();
        if (sel_caller) select_level(l, st);
        HIPCHK(c, hipEventRecord(c->ev[l], st));
        HIPCHK(c, hipStreamWaitEvent(ax, c->ev[l], 0));
        if (!sel_caller) select_level(l, ax);
        if (l == L_aux - 1) HIPCHK(c, hipEventRecord(c->ev[L + 2], ax));  // counts of the aux levels known
        describe_level(l, ax);
      }
    }
    l0 = l1;
  }
  if ((rc = release_gate())) return rc;  // (SFMFEAT_GATE_LEVEL=-1, or fewer levels)
  // the caller stream's levels: one selection launch for all of them (each level its own
  // scratch regions inside the stream's half), unless SFMFEAT_SELECT_MERGE=0
  static const bool merge_select = [] {
    const char* e = SFM_DIAG_ENV("SFMFEAT_SELECT_MERGE");
    return !(e && atoi(e) == 0);
  }();
  if (merge_select && L - L_aux > 1 && L - L_aux <= kSelectMaxLevels) {
    StageScope sc(c, SFM_PROF_TOPK, st);
    SelectLevels g{};
    g.n = L - L_aux;
    int64_t so = L_aux > 0 ? (int64_t)B * H * W : 0;
    for (int l = L_aux; l < L; ++l) {
      const LevelBufs& e = lb[l];
      g.l[l - L_aux] = SelectLevels::Level{e.R, e.cand, candcnt + e.co, as<uint32_t>(c->d_medlist) + so,
                                           as<uint64_t>(c->d_scratch) + so, e.kp, e.med, lv[l].h, lv[l].w,
                                           lv[l].fw / 2};
      so += (int64_t)B * lv[l].h * lv[l].w;
    }
    if (!(skip & 1)) launch_select_levels(g, std::max(c->kcap, 1), c->kcap, B, c->p.ksize, st);
  } else {
    for (int l = L_aux; l < L; ++l) select_level(l, st);
  }
  if (L_aux > 0 && L > L_aux) HIPCHK(c, hipStreamWaitEvent(st, c->ev[L + 2], 0));
  for (int l = L_aux; l < L; ++l) describe_level(l, st);
  if (L_aux > 0) {  // join: the caller's stream waits for the aux work
    HIPCHK(c, hipEventRecord(c->ev[L + 1], ax));
    HIPCHK(c, hipStreamWaitEvent(st, c->ev[L + 1], 0));
  }
  if (!counted) launch_finalize_counts(as<int32_t>(c->d_lc), B, L, count, st);
  HIPCHK(c, hipGetLastError());
  if (fused_ok && counted) {  // every level's descriptors (and the padding rows) carry operands
    c->fp_desc = desc;
    c->fp_count = count;
    c->fp_cap = cap;
    c->fp_B = B;
  }
  return SFM_OK;
}

// Matcher operands for slots [lo, lo + n) of a table of nimg slots (buffers sized for
// the whole table; the kernels index slots relative to the offset base pointers).
int match_prep_range(sfm_ctx* c, const float* desc, const int32_t* count, int nimg, int64_t cap, int lo, int n,
                     hipStream_t st) {
  if (cap < 1 || cap > kMaxMatchRows)
    return set_err(c, SFM_EINVAL, "match capacity must be in [1, 16384]");
  if (lo < 0 || n < 0 || lo + n > nimg) return set_err(c, SFM_EINVAL, "prep slot range outside the table");
  int rc;
  const float* d0 = desc + (int64_t)lo * cap * 128;
  c->prep_desc = desc;
  c->prep_count = count;
  c->prep_nimg = nimg;
  c->prep_cap = cap;
  if (c->match_direct) {
    const int64_t capP = (cap + 63) / 64 * 64;
    if ((rc = ensure(c, c->m_descT, (size_t)nimg * 128 * capP * 4))) return rc;
    if (n == 0) return SFM_OK;
    StageScope sc(c, SFM_PROF_MATCH_PREP, st);
    launch_transpose_desc(d0, count + lo, n, cap, capP, as<float>(c->m_descT) + (int64_t)lo * 128 * capP, st);
  } else {
    const int64_t capP = (cap + 127) / 128 * 128;
    if ((rc = match_operands_reserve(c, nimg, capP))) return rc;
    if (n == 0) return SFM_OK;
    StageScope sc(c, SFM_PROF_MATCH_PREP, st);
    const int64_t o = (int64_t)lo * capP;
    launch_match_prep(d0, count + lo, n, cap, capP, as<_Float16>(c->m_hi) + o * 128, as<_Float16>(c->m_lo) + o * 128,
                      as<float>(c->m_norm2) + o, as<float>(c->m_rnorm) + o,
                      as<char>(c->m_imgmax) + (size_t)lo * match_pmax_bytes(capP), st);
  }
  HIPCHK(c, hipGetLastError());
  return SFM_OK;
}

int match_impl(sfm_ctx* c, const float* desc, const int32_t* count, int nimg, int64_t cap,
               const int32_t* pairs, int P, float ratio, int32_t* matches, float* conf,
               int32_t* nmatch, hipStream_t st, bool prep = true) {
  if (P <= 0) return SFM_OK;
  if (cap < 1 || cap > kMaxMatchRows)
    return set_err(c, SFM_EINVAL, "match capacity must be in [1, 16384]");
  int rc;
  if (prep) {
    // slots the last extraction on this context wrote with their operands (fused prep) keep
    // them; only the rest of the table is prepped (none in BatchPipeline's own tables)
    int lo = 0;
    if (!c->match_direct && c->fp_desc == desc && c->fp_count == count && c->fp_cap == cap && c->fp_B <= nimg &&
        match_operands_fit(c, nimg, (cap + 127) / 128 * 128))
      lo = c->fp_B;
    if ((rc = match_prep_range(c, desc, count, nimg, cap, lo, nimg - lo, st))) return rc;
  } else {  // operands from earlier sfm_match_prep_dev calls on this same table
    // (which slots the device-resident pairs touch, and whether their descriptors changed
    // since, cannot be checked without a host sync: that part is the caller's contract)
    if (c->prep_desc != desc || c->prep_count != count || c->prep_nimg != nimg || c->prep_cap != cap)
      return set_err(c, SFM_ESTATE, "sfm_match_pairs_prepped_dev: this table was not the last one prepped "
                                    "(sfm_match_prep_dev) on this context");
  }
  // Per-pair workspace (row results, overflow list and, for the MFMA sweep, kMatchCandCap
  // admitted targets per query row: 512 B per row) is bounded: large P runs as consecutive
  // sub-launches over a fixed budget (SFMFEAT_MATCH_BUDGET_MB, default 2048) instead of one
  // allocation that grows with P * cap.
  const size_t budget = c->match_budget;
  const size_t per_pair = (size_t)cap * (sizeof(RowBest) + sizeof(int2) + (c->match_direct ? 0 : kMatchCandCap * 4 + 8));
  // (at most 2^kMatchUnitPairBits pairs per sub-launch: the sweep's work units hold the pair
  // index in that many bits, so a small capacity under a large budget cannot wrap it)
  const int Pmax = (int)std::max<size_t>(
      1, std::min<size_t>(std::min<size_t>((size_t)P, budget / per_pair), (size_t)1 << kMatchUnitPairBits));
  if ((rc = ensure(c, c->m_rows, (size_t)Pmax * cap * sizeof(RowBest)))) return rc;
  if ((rc = ensure(c, c->m_ovf, (size_t)Pmax * cap * sizeof(int2)))) return rc;
  if (c->m_ovfc.bytes == 0) {  // the overflow counter starts at zero; k_match_compact re-zeroes it
    if ((rc = ensure(c, c->m_ovfc, 16))) return rc;
    HIPCHK(c, hipMemsetAsync(c->m_ovfc.p, 0, 16, st));
  }
  if (!c->match_direct) {  // admitted-target lists of the MFMA sweep (kMatchCandCap per row)
    if ((rc = ensure(c, c->m_cand, (size_t)Pmax * cap * kMatchCandCap * 4))) return rc;
    if ((rc = ensure(c, c->m_candn, (size_t)Pmax * cap * 4))) return rc;
    if ((rc = ensure(c, c->m_candt, (size_t)Pmax * cap * 4))) return rc;
    if ((rc = ensure(c, c->m_units, match_units_words(Pmax, (int)cap) * 4))) return rc;
  }
  for (int p0 = 0; p0 < P; p0 += Pmax, ++c->match_calls) {
    const int Pn = std::min(Pmax, P - p0);
    const int32_t* pr = pairs + 2 * (int64_t)p0;
    if (c->match_direct) {
      const int64_t capP = (cap + 63) / 64 * 64;
      StageScope sc(c, SFM_PROF_MATCH, st);
      launch_match_rows(as<float>(c->m_descT), count, capP, pr, Pn, ratio, as<RowBest>(c->m_rows), (int)cap, st);
    } else {
      const int64_t capP = (cap + 127) / 128 * 128;
      StageScope sc(c, SFM_PROF_MATCH, st);
      if (!(c->match_calls > 0 && (skip_mask() & 8))) launch_match_mfma(desc, count, cap, capP, as<_Float16>(c->m_hi), as<_Float16>(c->m_lo), as<float>(c->m_norm2),
                        as<float>(c->m_rnorm), c->m_imgmax.p, pr, Pn, ratio, as<RowBest>(c->m_rows),
                        (int)cap, as<uint32_t>(c->m_cand), as<int32_t>(c->m_candn), as<float>(c->m_candt),
                        as<int>(c->m_ovfc), as<int2>(c->m_ovf), as<int32_t>(c->m_units), st);
    }
    {
      StageScope sc(c, SFM_PROF_MATCH_POST, st);
      launch_match_compact(as<RowBest>(c->m_rows), count, pr, Pn, (int)cap, cap, matches + (int64_t)p0 * cap * 2,
                           conf + (int64_t)p0 * cap, nmatch + p0, c->match_direct ? nullptr : as<int>(c->m_ovfc), st);
    }
  }
  HIPCHK(c, hipGetLastError());
  return SFM_OK;
}

}  // namespace

extern "C" {

void sfm_params_default(sfm_params* p, int32_t mode) {
  memset(p, 0, sizeof(*p));
  p->mode = mode;
  p->num_interest_points = 2500;  // FeatureExtractor.py:11
  p->ksize = 7;                   // NaiveSIFT.py:35
  p->gaussian_size = 7;           // :36
  p->sigma = 5.0;                 // :37
  p->alpha = 0.05;                // :38
  p->feature_width = 16;          // :39
  p->pyramid_level = mode == SFM_MODE_NAIVE ? 1 : 4;  // ScaleRotInvSIFT.py:12
  p->pyramid_scale_factor = 2.0;                      // :13
  p->gauss_kernel_set = 0;
}

int32_t sfm_abi_version(void) { return 1; }

int32_t sfm_build_flags(void) {
#ifdef SFM_ABLATIONS
  return SFM_BUILD_ABLATIONS;
#else
  return 0;
#endif
}

int64_t sfm_keypoint_capacity(const sfm_params* p) {
  if (!p) return 0;
  if (p->mode == SFM_MODE_NAIVE) return p->num_interest_points > 0 ? p->num_interest_points : 0;
  int L = p->pyramid_level;
  if (L < 1) return 0;
  int64_t k = (int64_t)((double)p->num_interest_points / (double)L);
  return k > 0 ? (int64_t)L * k : 0;
}

int32_t sfm_pyramid_dims(const sfm_params* p, int32_t H, int32_t W, int32_t* dims) {
  if (!p || !dims) return SFM_EINVAL;
  std::vector<Level> lv;
  if (geometry(p, H, W, lv) != SFM_OK) return SFM_EINVAL;
  for (size_t l = 0; l < lv.size(); ++l) {
    dims[2 * l] = lv[l].h;
    dims[2 * l + 1] = lv[l].w;
  }
  return SFM_OK;
}

int32_t sfm_ctx_create(int32_t device, const sfm_params* p, sfm_ctx** out) {
  if (!p || !out) return SFM_EINVAL;
  *out = nullptr;
  if (p->mode != SFM_MODE_SCALEROT && p->mode != SFM_MODE_NAIVE) return SFM_EINVAL;
  if (!gauss_size_supported(p->gaussian_size)) return SFM_EINVAL;
  if (p->ksize < 0 || p->ksize / 2 > SFM_NMS_MAX_HALF) return SFM_EINVAL;
  if (p->feature_width < 0 || p->feature_width > SFM_MAX_FW) return SFM_EINVAL;
  if (p->mode == SFM_MODE_SCALEROT && (p->pyramid_level < 1 || p->pyramid_level > SFM_MAX_LEVELS))
    return SFM_EINVAL;
  if (p->mode == SFM_MODE_SCALEROT && !(p->pyramid_scale_factor > 0.0)) return SFM_EINVAL;
  sfm_ctx* c = new sfm_ctx();
  c->device = device;
  c->p = *p;
  c->L = p->mode == SFM_MODE_NAIVE ? 1 : p->pyramid_level;
  if (c->p.mode == SFM_MODE_NAIVE) c->p.pyramid_level = 1;
  int64_t k = p->mode == SFM_MODE_NAIVE ? p->num_interest_points
                                        : (int64_t)((double)p->num_interest_points / (double)c->L);
  if (k < 0) k = 0;
  if (k > kTopkLdsCap || (int64_t)c->L * k > kMaxMatchRows) {
    delete c;
    return SFM_EINVAL;
  }
  c->kcap = (int)k;
  {
    const char* e = getenv("SFMFEAT_MATCH_DIRECT");
    c->match_direct = e && e[0] == '1';
    const char* se = getenv("SFMFEAT_SELECT");
    c->exact_select = se && strcmp(se, "exact") == 0;
    const char* sr = getenv("SFMFEAT_SERIAL");
    c->serial = sr && sr[0] == '1';
    const char* mb = getenv("SFMFEAT_MATCH_BUDGET_MB");
    if (mb && atoi(mb) > 0) c->match_budget = (size_t)atoi(mb) << 20;
  }
  c->cap = (int64_t)c->L * k;
  int gs = p->gaussian_size;
  if (p->gauss_kernel_set) memcpy(c->gauss, p->gauss_kernel, sizeof(float) * gs * gs);
  else gaussian_taps(gs, p->sigma, c->gauss);
  // Both streams are created on first use: the context's own stream (host-pointer calls,
  // sfm_ctx_stream) and the aux stream (non-serial extractions).  The HIP runtime maps streams
  // onto GPU_MAX_HW_QUEUES hardware queues (4 by default) and streams beyond that share one,
  // which serialises them; a context that only carries work on the streams it needs keeps
  // the caller's stream layout under the caller's control (pipeline.BatchPipeline).
  bool ok = hipSetDevice(device) == hipSuccess;
  {  // SFMFEAT_EAGER_HOST_STREAM=1 (A/B): the round-3 stream layout (both made here)
    const char* e = SFM_DIAG_ENV("SFMFEAT_EAGER_HOST_STREAM");
    if (ok && e && atoi(e) == 1)
      ok = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
           hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) == hipSuccess;
  }
  for (hipEvent_t& e : c->ev) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->aux) (void)hipStreamDestroy(c->aux);
    for (hipEvent_t e : c->ev)
      if (e) (void)hipEventDestroy(e);
    delete c;
    return SFM_EDEVICE;
  }
  std::vector<float> taps(harris_taps_floats(gs));
  harris_taps_build(c->gauss, gs, taps.data());
  if (ensure(c, c->d_gauss, sizeof(float) * taps.size()) ||
      hipMemcpy(c->d_gauss.p, taps.data(), sizeof(float) * taps.size(), hipMemcpyHostToDevice) != hipSuccess) {
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->aux) (void)hipStreamDestroy(c->aux);
    for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
    delete c;
    return SFM_EDEVICE;
  }
  init_topk_attributes();
  init_describe_attributes(describe_lds_bytes(SFM_MAX_FW, 1));
  init_describe_quad_tables();
  init_match_attributes(kMaxMatchRows);
  *out = c;
  return SFM_OK;
}

int32_t sfm_ctx_destroy(sfm_ctx* c) {
  if (!c) return SFM_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  DevBuf* bufs[] = {&c->d_gauss, &c->d_img0, &c->d_lvl, &c->d_R, &c->d_hist, &c->d_med, &c->d_medlist,
                    &c->d_counts, &c->d_cand, &c->d_scratch, &c->d_kpx, &c->d_kpy, &c->d_kpc, &c->d_lc,
                    &c->d_xy, &c->d_desc, &c->d_conf, &c->d_count, &c->d_u8, &c->m_desc, &c->m_count, &c->m_pairs,
                    &c->m_descT, &c->m_rows, &c->m_matches, &c->m_conf, &c->m_nmatch,
                    &c->m_hi, &c->m_lo, &c->m_norm2, &c->m_rnorm, &c->m_imgmax, &c->m_ovf, &c->m_ovfc, &c->m_cand, &c->m_candn, &c->m_candt, &c->m_units,
                    &c->i_tab_h, &c->i_tab_v, &c->i_tmp, &c->i_rgb, &c->i_gray, &c->i_colmap, &c->i_sets,
                    &c->r_idx, &c->r_off, &c->r_F, &c->r_counts, &c->r_pts, &c->r_npts, &c->r_out, &c->r_on,
                    &c->r_oit, &c->d_spans};
  for (DevBuf* b : bufs) free_buf(*b);
  for (auto& e : c->prof_pending) {
    (void)hipEventDestroy(e.second.first);
    (void)hipEventDestroy(e.second.second);
  }
  for (hipEvent_t e : c->prof_pool) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->aux) (void)hipStreamDestroy(c->aux);
  for (hipEvent_t e : c->ev)
    if (e) (void)hipEventDestroy(e);
  delete c;
  return SFM_OK;
}

const char* sfm_last_error(const sfm_ctx* c) { return c ? c->err.c_str() : "null context"; }

int32_t sfm_reserve(sfm_ctx* c, int32_t B, int32_t H, int32_t W) {
  if (!c || B < 1 || H < 1 || W < 1) return SFM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  return reserve_impl(c, B, H, W);
}

int32_t sfm_extract_batch_dev(sfm_ctx* c, const float* imgs, int32_t B, int32_t H, int32_t W,
                              int32_t* xy, float* desc, int32_t* count, int64_t cap, void* stream) {
  if (!c || !imgs || !xy || !desc || !count) return SFM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;  // exactly the caller's stream (NULL = null stream)
  return extract_impl(c, imgs, B, H, W, xy, desc, nullptr, count, cap, st);
}

int32_t sfm_extract_batch_u8_dev(sfm_ctx* c, const uint8_t* imgs, int32_t B, int32_t H, int32_t W,
                                 int32_t* xy, float* desc, int32_t* count, int64_t cap, void* stream) {
  if (!c || !imgs || !xy || !desc || !count || B < 1 || H < 1 || W < 1) return SFM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;  // exactly the caller's stream (NULL = null stream)
  int rc = reserve_impl(c, B, H, W);
  if (rc) return rc;
  launch_u8_to_f32(imgs, as<float>(c->d_img0), (int64_t)B * H * W, st);
  return extract_impl(c, as<float>(c->d_img0), B, H, W, xy, desc, nullptr, count, cap, st);
}

int32_t sfm_resize_dims(int32_t H, int32_t W, double scale, int32_t* H2, int32_t* W2) {
  if (!H2 || !W2 || H < 1 || W < 1 || !(scale > 0.0)) return SFM_EINVAL;
  const double h = (double)H * scale, w = (double)W * scale;  // int(shape * scale_factor)
  if (h < 1.0 || w < 1.0 || h > 65535.0 || w > 65535.0) return SFM_EINVAL;
  *H2 = (int32_t)h;
  *W2 = (int32_t)w;
  return SFM_OK;
}

namespace {
int ingest_impl(sfm_ctx* c, const uint8_t* rgb, int B, int H, int W, int H2, int W2, float* gray,
                hipStream_t st) {
  int rc;
  const bool newh = c->i_w != W || c->i_w2 != W2, newv = c->i_h != H || c->i_h2 != H2;
  if (newh) {
    c->i_ksh = build_resample_table(W, W2, c->i_th);
    if ((rc = ensure(c, c->i_tab_h, c->i_th.size() * 4))) return rc;
    HIPCHK(c, hipMemcpy(c->i_tab_h.p, c->i_th.data(), c->i_th.size() * 4, hipMemcpyHostToDevice));
    c->i_w = W;
    c->i_w2 = W2;
  }
  if (newv) {
    c->i_ksv = build_resample_table(H, H2, c->i_tv);
    if ((rc = ensure(c, c->i_tab_v, c->i_tv.size() * 4))) return rc;
    HIPCHK(c, hipMemcpy(c->i_tab_v.p, c->i_tv.data(), c->i_tv.size() * 4, hipMemcpyHostToDevice));
    c->i_h = H;
    c->i_h2 = H2;
  }
  if (newh || newv) {
    std::vector<int32_t> cm, sets;
    const int ks = ingest_rows_ks(c->i_ksh, c->i_ksv);
    c->i_rows = ks && ingest_rows_tables(c->i_th, c->i_ksh, W, W2, ks, cm, sets);
    if (c->i_rows) {
      if ((rc = ensure(c, c->i_colmap, cm.size() * 4))) return rc;
      if ((rc = ensure(c, c->i_sets, sets.size() * 4))) return rc;
      HIPCHK(c, hipMemcpy(c->i_colmap.p, cm.data(), cm.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(c, hipMemcpy(c->i_sets.p, sets.data(), sets.size() * 4, hipMemcpyHostToDevice));
      c->i_nsets = (int)(sets.size() / ks);
    }
  }
  if ((rc = ensure(c, c->i_tmp, (size_t)B * H * W2 * 3 + 16))) return rc;
  launch_ingest_rgb(rgb, as<uint8_t>(c->i_tmp), gray, as<int32_t>(c->i_tab_h), c->i_ksh, as<int32_t>(c->i_tab_v),
                    c->i_ksv, c->i_rows ? as<int32_t>(c->i_colmap) : nullptr, as<int32_t>(c->i_sets), c->i_nsets,
                    B, H, W, H2, W2, st);
  HIPCHK(c, hipGetLastError());
  return SFM_OK;
}
}  // namespace

int32_t sfm_ingest_rgb_dev(sfm_ctx* c, const uint8_t* rgb, int32_t B, int32_t H, int32_t W, int32_t H2,
                           int32_t W2, float* gray, void* stream) {
  if (!c || !rgb || !gray || B < 1 || H < 1 || W < 1 || H2 < 1 || W2 < 1 || H2 > 65535 || W2 > 65535)
    return SFM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  return ingest_impl(c, rgb, B, H, W, H2, W2, gray, (hipStream_t)stream);
}

int32_t sfm_ingest_rgb(sfm_ctx* c, const uint8_t* rgb, int32_t H, int32_t W, int32_t H2, int32_t W2,
                       float* gray) {
  if (!c || !rgb || !gray || H < 1 || W < 1 || H2 < 1 || W2 < 1 || H2 > 65535 || W2 > 65535)
    return SFM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = ensure(c, c->i_rgb, (size_t)H * W * 3))) return rc;
  if ((rc = ensure(c, c->i_gray, (size_t)H2 * W2 * 4))) return rc;
  hipStream_t st;
  if ((rc = host_stream(c, &st))) return rc;
  HIPCHK(c, hipMemcpyAsync(c->i_rgb.p, rgb, (size_t)H * W * 3, hipMemcpyHostToDevice, st));
  if ((rc = ingest_impl(c, as<uint8_t>(c->i_rgb), 1, H, W, H2, W2, as<float>(c->i_gray), st))) return rc;
  HIPCHK(c, hipMemcpyAsync(gray, c->i_gray.p, (size_t)H2 * W2 * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  return SFM_OK;
}

int32_t sfm_ransac_sample_indices(int32_t n, int32_t iters, uint32_t seed, int32_t* out) {
  if (n < 8 || iters < 0 || !out) return SFM_EINVAL;
  ransac_sample_indices(n, iters, seed, out);
  return SFM_OK;
}

namespace {
constexpr size_t kRansacCacheCap = 256;  // cached (n, iterations) streams per context (~190 KB each)

const std::vector<int32_t>* ransac_cached(sfm_ctx* c, int n, int iters) {
  for (auto& e : c->r_cache)
    if (e.first.first == n && e.first.second == iters) return &e.second;
  return nullptr;
}

// Replays the sample streams of every size in `ns` not cached yet, the sizes spread over
// host threads (each walks the shared raw MT19937 words on its own), and caches them.
void ransac_prefetch_streams(sfm_ctx* c, const std::vector<int>& ns, int iters) {
  std::vector<int> todo;
  for (int n : ns)
    if (!ransac_cached(c, n, iters)) todo.push_back(n);
  if (todo.empty()) return;
  std::vector<std::vector<int32_t>> out(todo.size());
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (size_t i; (i = next.fetch_add(1)) < todo.size();) {
      out[i].resize((size_t)iters * 8);
      ransac_sample_indices(todo[i], iters, 5u, out[i].data());  // np.random.seed(5), SFM.py:133
    }
  };
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const size_t nt = std::min<size_t>(todo.size(), hw);
  std::vector<std::thread> pool;
  for (size_t t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  for (size_t i = 0; i < todo.size(); ++i) c->r_cache.push_back({{todo[i], iters}, std::move(out[i])});
  // trim: the oldest streams this call does not use go first
  for (auto it = c->r_cache.begin(); c->r_cache.size() > kRansacCacheCap && it != c->r_cache.end();) {
    if (it->first.second != iters || std::find(ns.begin(), ns.end(), it->first.first) == ns.end())
      it = c->r_cache.erase(it);
    else
      ++it;
  }
}

int ransac_impl(sfm_ctx* c, const int32_t* pts, const int32_t* npts_dev, const int32_t* npts_host, int P, int nmax,
                int iters, double thr, int32_t* out_pts, int32_t* out_n, int32_t* out_iter, hipStream_t st) {
  // sample streams (host replay of numpy's RandomState; identical for equal n)
  {
    std::vector<int> ns;
    for (int p = 0; p < P; ++p) {
      const int n = npts_host[p];
      if (n > nmax) return set_err(c, SFM_EINVAL, "correspondence count above nmax");
      if (n >= 8 && std::find(ns.begin(), ns.end(), n) == ns.end()) ns.push_back(n);
    }
    ransac_prefetch_streams(c, ns, iters);
  }
  std::vector<int32_t> all, off(P, 0);
  std::vector<int> seen_n;
  std::vector<int32_t> seen_off;
  for (int p = 0; p < P; ++p) {
    const int n = npts_host[p];
    if (n < 8 || n > nmax) {
      if (n > nmax) return set_err(c, SFM_EINVAL, "correspondence count above nmax");
      continue;
    }
    int k = -1;
    for (size_t i = 0; i < seen_n.size(); ++i)
      if (seen_n[i] == n) k = (int)i;
    if (k < 0) {
      const std::vector<int32_t>& s = *ransac_cached(c, n, iters);
      seen_n.push_back(n);
      seen_off.push_back((int32_t)all.size());
      all.insert(all.end(), s.begin(), s.end());
      k = (int)seen_n.size() - 1;
    }
    off[p] = seen_off[k];
  }
  if (all.empty()) all.assign(8, 0);
  int rc;
  if ((rc = ensure(c, c->r_idx, all.size() * 4))) return rc;
  if ((rc = ensure(c, c->r_off, (size_t)P * 4))) return rc;
  if ((rc = ensure(c, c->r_F, (size_t)P * std::max(iters, 1) * 9 * 8))) return rc;
  if ((rc = ensure(c, c->r_counts, (size_t)P * std::max(iters, 1) * 4))) return rc;
  HIPCHK(c, hipMemcpyAsync(c->r_idx.p, all.data(), all.size() * 4, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(c->r_off.p, off.data(), (size_t)P * 4, hipMemcpyHostToDevice, st));
  // iters == 0 still launches the select kernel: it writes every pair's empty / None result
  launch_ransac(pts, npts_dev, nmax, P, as<int32_t>(c->r_idx), as<int32_t>(c->r_off), iters, thr, as<double>(c->r_F),
                as<int32_t>(c->r_counts), out_pts, out_n, out_iter, st);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(st));  // the host index buffers above are stack-owned
  return SFM_OK;
}
}  // namespace

int32_t sfm_ransac_find_inliers_dev(sfm_ctx* c, const int32_t* pts, const int32_t* npts, const int32_t* npts_host,
                                    int32_t P, int32_t nmax, int32_t iters, double threshold, int32_t* out_pts,
                                    int32_t* out_n, int32_t* out_iter, void* stream) {
  if (!c || !pts || !npts || !npts_host || !out_pts || !out_n || !out_iter || P < 1 || nmax < 1 || iters < 0)
    return SFM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  return ransac_impl(c, pts, npts, npts_host, P, nmax, iters, threshold, out_pts, out_n, out_iter,
                     (hipStream_t)stream);
}

int32_t sfm_ransac_find_inliers(sfm_ctx* c, const int64_t* p1, const int64_t* p2, int64_t n, int32_t iters,
                                double threshold, int64_t* in1, int64_t* in2, int64_t* n_out, int32_t* best_iter) {
  if (!c || !n_out || n < 0 || iters < 0 || (n > 0 && (!p1 || !p2))) return SFM_EINVAL;
  if (n > INT32_MAX / 4) return set_err(c, SFM_EINVAL, "too many correspondences");
  HIPCHK(c, hipSetDevice(c->device));
  *n_out = -1;
  if (n < 8) return SFM_OK;  // the reference returns (None, None, None, None)
  const int nmax = (int)n;
  std::vector<int32_t> h((size_t)nmax * 4);
  for (int64_t i = 0; i < n; ++i) {
    h[4 * i + 0] = (int32_t)p1[2 * i];
    h[4 * i + 1] = (int32_t)p1[2 * i + 1];
    h[4 * i + 2] = (int32_t)p2[2 * i];
    h[4 * i + 3] = (int32_t)p2[2 * i + 1];
  }
  int rc;
  if ((rc = ensure(c, c->r_pts, h.size() * 4))) return rc;
  if ((rc = ensure(c, c->r_npts, 16))) return rc;
  if ((rc = ensure(c, c->r_out, h.size() * 4))) return rc;
  if ((rc = ensure(c, c->r_on, 16))) return rc;
  if ((rc = ensure(c, c->r_oit, 16))) return rc;
  hipStream_t st;
  if ((rc = host_stream(c, &st))) return rc;
  const int32_t nn = (int32_t)n;
  HIPCHK(c, hipMemcpyAsync(c->r_pts.p, h.data(), h.size() * 4, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(c->r_npts.p, &nn, 4, hipMemcpyHostToDevice, st));
  if ((rc = ransac_impl(c, as<int32_t>(c->r_pts), as<int32_t>(c->r_npts), &nn, 1, nmax, iters, threshold,
                        as<int32_t>(c->r_out), as<int32_t>(c->r_on), as<int32_t>(c->r_oit), st)))
    return rc;
  int32_t k = 0, bi = -1;
  HIPCHK(c, hipMemcpyAsync(&k, c->r_on.p, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipMemcpyAsync(&bi, c->r_oit.p, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  if (k > n) return set_err(c, SFM_EDEVICE, "inlier count above the correspondence count");
  if (k > 0) {
    std::vector<int32_t> o((size_t)k * 4);
    HIPCHK(c, hipMemcpy(o.data(), c->r_out.p, o.size() * 4, hipMemcpyDeviceToHost));
    for (int i = 0; i < k; ++i) {
      if (in1) { in1[2 * i] = o[4 * i]; in1[2 * i + 1] = o[4 * i + 1]; }
      if (in2) { in2[2 * i] = o[4 * i + 2]; in2[2 * i + 1] = o[4 * i + 3]; }
    }
  }
  *n_out = k;
  if (best_iter) *best_iter = bi;
  return SFM_OK;
}

int32_t sfm_extract(sfm_ctx* c, const float* img, int32_t H, int32_t W, int64_t row_stride, int64_t* X,
                    int64_t* Y, float* desc, float* conf, int64_t cap, int64_t* n_out,
                    int32_t* level_counts) {
  if (!c || !img || !n_out) return SFM_EINVAL;
  if (H < 1 || W < 1 || row_stride < W) return set_err(c, SFM_EINVAL, "bad image shape or stride");
  HIPCHK(c, hipSetDevice(c->device));
  int rc = reserve_impl(c, 1, H, W);
  if (rc) return rc;
  const int64_t scap = std::max<int64_t>(c->cap, 1);
  if ((rc = ensure(c, c->d_xy, (size_t)scap * 8))) return rc;
  if ((rc = ensure(c, c->d_desc, (size_t)scap * 128 * 4))) return rc;
  if ((rc = ensure(c, c->d_count, 16))) return rc;
  if ((rc = ensure(c, c->d_conf, (size_t)scap * 4))) return rc;
  hipStream_t st;
  if ((rc = host_stream(c, &st))) return rc;
  HIPCHK(c, hipMemcpy2DAsync(c->d_img0.p, (size_t)W * 4, img, (size_t)row_stride * 4, (size_t)W * 4, H,
                             hipMemcpyHostToDevice, st));
  rc = extract_impl(c, as<float>(c->d_img0), 1, H, W, as<int32_t>(c->d_xy), as<float>(c->d_desc),
                    as<float>(c->d_conf), as<int32_t>(c->d_count), scap, st);
  if (rc) return rc;
  int32_t n = 0;
  std::vector<int32_t> lc(c->L);
  HIPCHK(c, hipMemcpyAsync(&n, c->d_count.p, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipMemcpyAsync(lc.data(), c->d_lc.p, (size_t)c->L * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  *n_out = n;
  if (level_counts) memcpy(level_counts, lc.data(), (size_t)c->L * 4);
  if (n > cap) return set_err(c, SFM_ERANGE, "output capacity too small");
  if (n > 0) {
    std::vector<int32_t> xy((size_t)n * 2);
    HIPCHK(c, hipMemcpyAsync(xy.data(), c->d_xy.p, (size_t)n * 8, hipMemcpyDeviceToHost, st));
    if (desc) HIPCHK(c, hipMemcpyAsync(desc, c->d_desc.p, (size_t)n * 128 * 4, hipMemcpyDeviceToHost, st));
    if (conf) HIPCHK(c, hipMemcpyAsync(conf, c->d_conf.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    for (int32_t i = 0; i < n; ++i) {
      if (X) X[i] = xy[2 * i];
      if (Y) Y[i] = xy[2 * i + 1];
    }
  }
  return SFM_OK;
}

int32_t sfm_match(sfm_ctx* c, const float* d1, int64_t n1, const float* d2, int64_t n2, float ratio,
                  int64_t* matches, float* conf, int64_t cap, int64_t* k_out) {
  if (!c || !k_out || n1 < 0 || n2 < 0) return SFM_EINVAL;
  if ((n1 > 0 && !d1) || (n2 > 0 && !d2)) return SFM_EINVAL;
  *k_out = 0;
  if (n1 >= 1 && n2 < 2) return set_err(c, SFM_EINDEX, "index 1 is out of bounds (fewer than 2 targets)");
  if (n1 == 0) return SFM_OK;
  HIPCHK(c, hipSetDevice(c->device));
  int64_t mcap = std::max(n1, n2);
  if (mcap > kMaxMatchRows) return set_err(c, SFM_EINVAL, "more than 16384 descriptors per side");
  int rc;
  hipStream_t st;
  if ((rc = host_stream(c, &st))) return rc;
  if ((rc = ensure(c, c->m_desc, (size_t)2 * mcap * 128 * 4))) return rc;
  if ((rc = ensure(c, c->m_count, 16))) return rc;
  if ((rc = ensure(c, c->m_pairs, 16))) return rc;
  if ((rc = ensure(c, c->m_matches, (size_t)mcap * 8))) return rc;
  if ((rc = ensure(c, c->m_conf, (size_t)mcap * 4))) return rc;
  if ((rc = ensure(c, c->m_nmatch, 16))) return rc;
  int32_t hcount[2] = {(int32_t)n1, (int32_t)n2};
  int32_t hpairs[2] = {0, 1};
  float* dd = as<float>(c->m_desc);
  HIPCHK(c, hipMemcpyAsync(dd, d1, (size_t)n1 * 128 * 4, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(dd + mcap * 128, d2, (size_t)n2 * 128 * 4, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(c->m_count.p, hcount, 8, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(c->m_pairs.p, hpairs, 8, hipMemcpyHostToDevice, st));
  rc = match_impl(c, dd, as<int32_t>(c->m_count), 2, mcap, as<int32_t>(c->m_pairs), 1, ratio,
                  as<int32_t>(c->m_matches), as<float>(c->m_conf), as<int32_t>(c->m_nmatch), st);
  if (rc) return rc;
  int32_t k = 0;
  HIPCHK(c, hipMemcpyAsync(&k, c->m_nmatch.p, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  if (k < 0) return set_err(c, SFM_EINDEX, "index 1 is out of bounds (fewer than 2 targets)");
  *k_out = k;
  if (k > cap) return set_err(c, SFM_ERANGE, "output capacity too small");
  if (k > 0) {
    std::vector<int32_t> mm((size_t)k * 2);
    HIPCHK(c, hipMemcpyAsync(mm.data(), c->m_matches.p, (size_t)k * 8, hipMemcpyDeviceToHost, st));
    if (conf) HIPCHK(c, hipMemcpyAsync(conf, c->m_conf.p, (size_t)k * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    if (matches)
      for (int64_t i = 0; i < 2 * k; ++i) matches[i] = mm[i];
  }
  return SFM_OK;
}

int32_t sfm_ctx_set_fused_prep(sfm_ctx* c, int32_t on) {
  if (!c) return SFM_EINVAL;
  c->fused_prep = on != 0;
  c->fp_desc = nullptr;
  c->fp_B = 0;
  return SFM_OK;
}

int32_t sfm_ctx_set_serial(sfm_ctx* c, int32_t serial) {
  if (!c) return SFM_EINVAL;
  c->serial = serial != 0;
  return SFM_OK;
}

int32_t sfm_ctx_set_priority(sfm_ctx* c, int32_t priority) {
  if (!c) return SFM_EINVAL;
  if (c->stream || c->aux) return set_err(c, SFM_EINVAL, "stream priority after the context's streams exist");
  c->prio = priority;
  return SFM_OK;
}

int32_t sfm_ctx_stream(sfm_ctx* c, void** stream) {
  if (!c || !stream) return SFM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t st;
  int rc;
  if ((rc = host_stream(c, &st))) return rc;
  *stream = (void*)st;
  return SFM_OK;
}

int32_t sfm_gate_create(int32_t device, sfm_gate** out) {
  if (!out) return SFM_EINVAL;
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) return SFM_EDEVICE;
  sfm_gate* g = new sfm_gate();
  g->device = device;
  if (hipEventCreateWithFlags(&g->ev, hipEventDisableTiming) != hipSuccess) {
    delete g;
    return SFM_EDEVICE;
  }
  *out = g;
  return SFM_OK;
}

int32_t sfm_gate_destroy(sfm_gate* g) {
  if (!g) return SFM_OK;
  (void)hipSetDevice(g->device);
  if (g->armed) (void)hipEventSynchronize(g->ev);
  (void)hipEventDestroy(g->ev);
  delete g;
  return SFM_OK;
}

int32_t sfm_ctx_set_gate(sfm_ctx* c, sfm_gate* g) {
  if (!c) return SFM_EINVAL;
  if (g && g->device != c->device) return set_err(c, SFM_EINVAL, "gate and context on different devices");
  c->gate = g;
  return SFM_OK;
}

int32_t sfm_profile_enable(sfm_ctx* c, int32_t on) {
  if (!c) return SFM_EINVAL;
  c->prof = on != 0;
  c->prof_mask = ~0u;
  return SFM_OK;
}

int32_t sfm_profile_stages(sfm_ctx* c, int32_t mask) {
  if (!c) return SFM_EINVAL;
  c->prof = mask != 0;
  c->prof_mask = (uint32_t)mask;
  return SFM_OK;
}

// diagnostics: copy level `l`'s R maps (what = 0) or level images (what = 1) of the last
// extraction, all planes [B][h][w], to the device buffer `out` on `stream`
int32_t sfm_debug_copy_level(sfm_ctx* c, int32_t l, int32_t what, float* out, void* stream) {
  if (!c || !out || l < 0 || l >= c->L || !c->last_B) return SFM_EINVAL;
  std::vector<Level> lv;
  if (geometry(&c->p, c->last_H, c->last_W, lv) != SFM_OK) return SFM_EINVAL;
  const int B = c->last_B;
  int64_t off = 0, offl = 0;
  for (int k = 0; k < l; ++k) off += (int64_t)B * lv[k].h * lv[k].w;
  for (int k = 1; k < l; ++k) offl += (int64_t)B * lv[k].h * lv[k].w;
  const size_t bytes = (size_t)B * lv[l].h * lv[l].w * 4;
  const float* src = what == 0 ? as<float>(c->d_R) + off : (l == 0 ? as<float>(c->d_img0) : as<float>(c->d_lvl) + offl);
  HIPCHK(c, hipMemcpyAsync(out, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return SFM_OK;
}

int32_t sfm_debug_select_stats(sfm_ctx* c, int32_t* fallback_planes, int32_t* total_planes) {
  if (!c || !fallback_planes || !total_planes) return SFM_EINVAL;
  *fallback_planes = 0;
  *total_planes = c->L * c->last_B;
  if (*total_planes == 0) return SFM_OK;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipDeviceSynchronize());
  std::vector<MedianState> ms((size_t)*total_planes);
  HIPCHK(c, hipMemcpy(ms.data(), c->d_med.p, ms.size() * sizeof(MedianState), hipMemcpyDeviceToHost));
  for (const MedianState& m : ms) *fallback_planes += m.fallback ? 1 : 0;
  return SFM_OK;
}

int32_t sfm_profile_read(sfm_ctx* c, double* ms, int64_t* launches, int32_t reset) {
  if (!c) return SFM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  for (auto& e : c->prof_pending) {
    HIPCHK(c, hipEventSynchronize(e.second.second));
    float t = 0.0f;
    HIPCHK(c, hipEventElapsedTime(&t, e.second.first, e.second.second));
    c->prof_ms[e.first] += t;
    c->prof_launches[e.first] += 1;
    c->prof_pool.push_back(e.second.first);
    c->prof_pool.push_back(e.second.second);
  }
  c->prof_pending.clear();
  for (int i = 0; i < SFM_PROF_STAGES; ++i) {
    if (ms) ms[i] = c->prof_ms[i];
    if (launches) launches[i] = c->prof_launches[i];
    if (reset) {
      c->prof_ms[i] = 0.0;
      c->prof_launches[i] = 0;
    }
  }
  return SFM_OK;
}

namespace {
// every span slot back to {~0, 0} (the kernels fold their workgroups in with atomic min / max)
int spans_reset(sfm_ctx* c) {
  c->span_n = 0;
  c->span_dropped = 0;
  c->span_level.clear();
  if (c->span_cap == 0) return SFM_OK;
  std::vector<unsigned long long> init((size_t)2 * c->span_cap, 0ull);
  for (int64_t i = 0; i < c->span_cap; ++i) init[2 * i] = ~0ull;
  HIPCHK(c, hipDeviceSynchronize());
  HIPCHK(c, hipMemcpy(c->d_spans.p, init.data(), init.size() * 8, hipMemcpyHostToDevice));
  return SFM_OK;
}
}  // namespace

int32_t sfm_profile_spans(sfm_ctx* c, int64_t capacity) {
  if (!c || capacity < 0) return SFM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if (capacity > 0 && (rc = ensure(c, c->d_spans, (size_t)capacity * 16))) return rc;
  c->span_cap = capacity;
  return spans_reset(c);
}

int32_t sfm_profile_spans_read(sfm_ctx* c, int64_t* spans_ns, int32_t* levels, int64_t cap, int64_t* n_out,
                               int64_t* dropped, int32_t reset) {
  if (!c || !n_out || cap < 0) return SFM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  *n_out = c->span_n;
  if (dropped) *dropped = c->span_dropped;
  if (c->span_n > 0 && spans_ns && cap > 0) {
    int khz = 0;
    HIPCHK(c, hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
    if (khz <= 0) return set_err(c, SFM_EDEVICE, "device reports no wall-clock rate");
    HIPCHK(c, hipDeviceSynchronize());
    const int64_t n = std::min(cap, c->span_n);
    std::vector<unsigned long long> h((size_t)2 * n);
    HIPCHK(c, hipMemcpy(h.data(), c->d_spans.p, h.size() * 8, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n; ++i) {
      for (int k = 0; k < 2; ++k) {  // ticks -> ns; an untouched slot reads -1
        const unsigned long long t = h[2 * i + k];
        spans_ns[2 * i + k] = (t == ~0ull || (k == 1 && t == 0ull)) ? -1 : (int64_t)((long double)t * 1.0e6L / khz);
      }
      if (levels) levels[i] = c->span_level[(size_t)i];
    }
  }
  return reset ? spans_reset(c) : SFM_OK;
}

int32_t sfm_match_pairs_dev(sfm_ctx* c, const float* desc, const int32_t* count, int32_t nimg,
                            int64_t cap, const int32_t* pairs, int32_t P, float ratio, int32_t* matches,
                            float* conf, int32_t* nmatch, void* stream) {
  if (!c || !desc || !count || !pairs || !matches || !conf || !nmatch || nimg < 1 || P < 0)
    return SFM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;  // exactly the caller's stream (NULL = null stream)
  return match_impl(c, desc, count, nimg, cap, pairs, P, ratio, matches, conf, nmatch, st);
}

int32_t sfm_match_prep_dev(sfm_ctx* c, const float* desc, const int32_t* count, int32_t nimg, int64_t cap,
                           int32_t slot_lo, int32_t slot_n, void* stream) {
  if (!c || !desc || !count || nimg < 1) return SFM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  return match_prep_range(c, desc, count, nimg, cap, slot_lo, slot_n, (hipStream_t)stream);
}

int32_t sfm_match_pairs_prepped_dev(sfm_ctx* c, const float* desc, const int32_t* count, int32_t nimg,
                                    int64_t cap, const int32_t* pairs, int32_t P, float ratio, int32_t* matches,
                                    float* conf, int32_t* nmatch, void* stream) {
  if (!c || !desc || !count || !pairs || !matches || !conf || !nmatch || nimg < 1 || P < 0)
    return SFM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  return match_impl(c, desc, count, nimg, cap, pairs, P, ratio, matches, conf, nmatch, (hipStream_t)stream,
                    false);
}

}  // extern "C"
