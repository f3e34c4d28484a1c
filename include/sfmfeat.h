/*
 * sfmfeat.h — C-ABI of the MI355X-native feature stage (detect + describe + match)
 * of reesque/SfmFromScratch.
 *
 * This is the drop-in boundary.  Every entry point replaces one reference interface;
 * the citation after each declaration is the reference file:line it stands in for
 * (paths relative to the reference repository root).  Plain C types only: pointers,
 * sizes and a POD parameter struct; no torch / HIP types cross this boundary (HIP
 * streams are passed as opaque `void*`).
 *
 * Error model: every function returns an int status and never aborts.
 *   SFM_OK      0  success
 *   SFM_EINVAL  1  bad argument          -> Python ValueError / AssertionError
 *                                          (Runner.py:29-30, ScaleRotInvSIFT.py:38)
 *   SFM_ESTATE  2  call out of order     -> RuntimeError (NaiveSIFT.py:49-50)
 *   SFM_EDEVICE 3  HIP runtime failure   -> RuntimeError, text via sfm_last_error()
 *   SFM_ERANGE  4  output capacity too small (n_out holds the required size)
 *   SFM_EINDEX  5  matcher with fewer than 2 target descriptors -> IndexError
 *                                          (NNRatioFeatureMatcher.py:41-43)
 *
 * Threading: the reference drives extractor and matcher from 8 Python threads
 * (Runner.py:183-191).  A context is NOT shared between threads; create one context
 * per thread (the Python wrapper keeps a thread-local context).  The library keeps no
 * global mutable state, so distinct contexts are fully re-entrant.
 */
#ifndef SFMFEAT_H_
#define SFMFEAT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SFM_OK 0
#define SFM_EINVAL 1
#define SFM_ESTATE 2
#define SFM_EDEVICE 3
#define SFM_ERANGE 4
#define SFM_EINDEX 5

/* Extractor plugin classes (FeatureExtractor/SIFT/NaiveSIFT.py, ScaleRotInvSIFT.py). */
#define SFM_MODE_SCALEROT 0 /* ScaleRotInvSIFT: pyramid + dominant orientation */
#define SFM_MODE_NAIVE 1    /* NaiveSIFT: one level, un-rotated descriptors */

#define SFM_DESC_DIM 128
#define SFM_MAX_GAUSS 15 /* largest gaussian_size accepted */
#define SFM_MAX_KSIZE 31 /* largest NMS ksize accepted */
#define SFM_MAX_FW 64    /* largest feature_width accepted */
#define SFM_MAX_LEVELS 12

/*
 * POD mirror of the reference's `extractor_params` dict keys.  Defaults are the
 * reference's `.get(key, default)` values:
 *   num_interest_points 2500  FeatureExtractor.py:11
 *   ksize 7, gaussian_size 7, sigma 5, alpha 0.05, feature_width 16  NaiveSIFT.py:35-39
 *   pyramid_level 4, pyramid_scale_factor 2                          ScaleRotInvSIFT.py:12-13
 * `gauss_kernel` optionally carries the float32 values of
 * NaiveSIFT._generate_gaussian_kernel (NaiveSIFT.py:175-199) computed by the caller
 * (the Python wrapper computes them with numpy exactly as the reference does); when
 * `gauss_kernel_set` is 0 the library computes them itself in double precision.
 */
typedef struct sfm_params {
  int32_t mode;
  int32_t num_interest_points;
  int32_t ksize;
  int32_t gaussian_size;
  int32_t feature_width;
  int32_t pyramid_level;
  double sigma;
  double alpha;
  double pyramid_scale_factor;
  int32_t gauss_kernel_set;
  int32_t reserved0;
  float gauss_kernel[SFM_MAX_GAUSS * SFM_MAX_GAUSS];
} sfm_params;

/* Fill `p` with the reference defaults for `mode`. */
void sfm_params_default(sfm_params* p, int32_t mode);

/* ABI version, bumped on any signature change. */
int32_t sfm_abi_version(void);

/* Build flags of this library: SFM_BUILD_ABLATIONS set only in the diagnostic build
 * (make ABLATIONS=1), whose timing switches (SFMFEAT_SKIP, SFMFEAT_*_ABL, SFMFEAT_NMS_DRY) skip
 * or hollow out work by design; the shipped build reads none of them.  (No reference
 * counterpart: build provenance for bench lines.) */
#define SFM_BUILD_ABLATIONS 1
int32_t sfm_build_flags(void);

/* Maximum number of keypoints one image can produce:
 * ScaleRot: pyramid_level * int(k / pyramid_level)  (ScaleRotInvSIFT.py:90 scaled_k)
 * Naive:    k                                       (NaiveSIFT.py:100-103) */
int64_t sfm_keypoint_capacity(const sfm_params* p);

/* Pyramid level sizes for an H x W image, chained int(w/s), int(h/s)
 * (ScaleRotInvSIFT.py:109-115).  dims receives 2*L ints (h0,w0,h1,w1,...). */
int32_t sfm_pyramid_dims(const sfm_params* p, int32_t H, int32_t W, int32_t* dims);

typedef struct sfm_ctx sfm_ctx;

/* Create a context bound to HIP device `device` with fixed extractor parameters. */
int32_t sfm_ctx_create(int32_t device, const sfm_params* p, sfm_ctx** out);
int32_t sfm_ctx_destroy(sfm_ctx* ctx);
/* Last error text for this context (never NULL). */
const char* sfm_last_error(const sfm_ctx* ctx);

/*
 * Per-image extraction from host memory — replaces the ScaleRotInvSIFT constructor
 * (ScaleRotInvSIFT.py:9-16, all work eager) and NaiveSIFT.detect_keypoints +
 * extract_descriptors (NaiveSIFT.py:42-52), chosen by params.mode.
 *   img: H x W float32 grayscale, row stride `row_stride` elements (>= W)
 *   X, Y: int64 column / row of each keypoint in level-0 pixels
 *         (ScaleRotInvSIFT.py:101-102: (x * s^l).astype(int))
 *   desc: n x 128 float32 RootSIFT descriptors (ScaleRotInvSIFT.py:79-85)
 *   conf: optional, n float32 Harris responses (NaiveSIFT.py:44 `self.confidences`)
 *   cap: capacity of X/Y/desc in keypoints; n_out: keypoints written
 *   level_counts: optional, pyramid_level ints — keypoints contributed per level
 *                 (the Python wrapper uses it to mirror ScaleRotInvSIFT.py:103's
 *                 ragged extend when a level yields exactly one keypoint)
 * Output order is the reference's: level by level, confidence descending.
 */
int32_t sfm_extract(sfm_ctx* ctx, const float* img, int32_t H, int32_t W, int64_t row_stride,
                    int64_t* X, int64_t* Y, float* desc, float* conf, int64_t cap,
                    int64_t* n_out, int32_t* level_counts);

/*
 * Brute-force L2 nearest neighbour with Lowe ratio test — replaces
 * NNRatioFeatureMatcher.match_features_ratio_test (NNRatioFeatureMatcher.py:8-60).
 *   d1: n1 x 128, d2: n2 x 128 float32 (row-major, contiguous)
 *   ratio: threshold, compared in float32 (`nndr <= float32(ratio)`, :49)
 *   matches: k x 2 int64 [row in d1, row in d2]; conf: k float32 nndr
 *   sorted by (conf ascending, row ascending).  cap >= n1 always suffices.
 * Returns SFM_EINDEX when n2 < 2 (the reference raises IndexError at :42).
 */
int32_t sfm_match(sfm_ctx* ctx, const float* d1, int64_t n1, const float* d2, int64_t n2,
                  float ratio, int64_t* matches, float* conf, int64_t cap, int64_t* k_out);

/*
 * Frame ingest of FeatureRunner (Runner.py:33-46): a decoded RGB frame ([H][W][3] uint8,
 * what _load_image reads, Runner.py:551-563) -> PIL BICUBIC resize to W2 x H2
 * (_PIL_resize, Runner.py:37-42,481-493; Pillow's 8-bit fixed-point resampler, bit
 * exact) -> /255 -> _rgb2gray (Runner.py:467-478) -> [H2][W2] float32, the image the
 * extractor classes take.  Host pointers; synchronous.
 */
int32_t sfm_ingest_rgb(sfm_ctx* ctx, const uint8_t* rgb, int32_t H, int32_t W, int32_t H2, int32_t W2,
                       float* gray);

/* (int(H * scale), int(W * scale)) — the PIL target size of Runner.py:37-42. */
int32_t sfm_resize_dims(int32_t H, int32_t W, double scale, int32_t* H2, int32_t* W2);

/*
 * RANSAC inlier filter — replaces CameraPose.find_inliers (SFM.py:126-160), the match
 * consumer of SFMRunner stage 1 (Runner.py:349-351).  p1, p2: n x 2 int64 pixel
 * coordinates (the pairs of _convert_matches_to_coords, Runner.py:423-434); iters =
 * max_iterations; samples replay numpy's legacy RandomState after np.random.seed(5).
 * in1 / in2 (capacity n x 2) receive the winning sample's inliers in input order,
 * n_out their count; n_out = -1 when n < 8 (the reference returns four Nones), 0 when
 * iters == 0 (the reference's empty arrays).  No limit on n.
 * best_iter (optional): the winning sample's index.
 */
int32_t sfm_ransac_find_inliers(sfm_ctx* ctx, const int64_t* p1, const int64_t* p2, int64_t n, int32_t iters,
                                double threshold, int64_t* in1, int64_t* in2, int64_t* n_out,
                                int32_t* best_iter);

/* The sample indices np.random.choice(n, 8, replace=False) draws on each of `iters`
 * iterations after np.random.seed(seed) (numpy legacy MT19937 + Fisher-Yates):
 * out [iters][8] int32.  Host-only. */
int32_t sfm_ransac_sample_indices(int32_t n, int32_t iters, uint32_t seed, int32_t* out);

/* ---------------- device-resident batch API (throughput path) ----------------
 * All pointers are device pointers on the context's device; `stream` is the
 * hipStream_t the work is enqueued on, exactly as given (NULL = HIP's null stream, as
 * in the HIP API — so a caller on PyTorch's default stream passes its handle, 0, and
 * stays ordered with its own work).  The calls are asynchronous with respect to the
 * host: results are valid once the stream has been synchronised.
 * Workspace is owned by the context; call sfm_reserve() once with the largest batch
 * so that the batch calls perform no device allocation (hipGraph-capturable).
 *
 * Slot table layout (also the RCCL all-gather unit):
 *   xy    [B][cap][2] int32   (X, Y) level-0 pixel coordinates
 *   desc  [B][cap][128] float32
 *   count [B] int32
 */
int32_t sfm_reserve(sfm_ctx* ctx, int32_t B, int32_t H, int32_t W);

/* sfm_ransac_find_inliers for P pairs at once: pts [P][nmax][4] int32 (x1, y1, x2, y2),
 * npts [P] on the device and npts_host [P] on the host (the sample streams depend on n);
 * out_pts [P][nmax][4] inliers in order, out_n [P] (-1 for n < 8, 0 when iters == 0),
 * out_iter [P] (-1 when no sample won).  Any nmax (the points are staged through LDS in
 * chunks).  Synchronises the stream before returning. */
int32_t sfm_ransac_find_inliers_dev(sfm_ctx* ctx, const int32_t* pts, const int32_t* npts,
                                    const int32_t* npts_host, int32_t P, int32_t nmax, int32_t iters,
                                    double threshold, int32_t* out_pts, int32_t* out_n, int32_t* out_iter,
                                    void* stream);

/* sfm_ingest_rgb for B frames: rgb [B][H][W][3] uint8 -> gray [B][H2][W2] float32. */
int32_t sfm_ingest_rgb_dev(sfm_ctx* ctx, const uint8_t* rgb, int32_t B, int32_t H, int32_t W,
                           int32_t H2, int32_t W2, float* gray, void* stream);

/* Extract B images of identical size H x W stored contiguously ([B][H][W] float32). */
int32_t sfm_extract_batch_dev(sfm_ctx* ctx, const float* imgs, int32_t B, int32_t H, int32_t W,
                              int32_t* xy, float* desc, int32_t* count, int64_t cap,
                              void* stream);

/* Same, from 8-bit grayscale frames ([B][H][W] uint8, value/255 as float32 —
 * the conversion of Runner.py:507-509,521 done on the device). */
int32_t sfm_extract_batch_u8_dev(sfm_ctx* ctx, const uint8_t* imgs, int32_t B, int32_t H,
                                 int32_t W, int32_t* xy, float* desc, int32_t* count,
                                 int64_t cap, void* stream);

/*
 * Match P image pairs out of a slot table of `nimg` images (the consecutive / all-pairs
 * schedule of Runner.py:183-191).  pairs: [P][2] int32 image indices into the table.
 * Output per pair p: matches [p][cap][2] int32 (row in first, row in second),
 * conf [p][cap] float32, nmatch [p] int32; sorted as sfm_match.  A pair whose second
 * image has fewer than 2 keypoints yields nmatch = -1 (the reference's IndexError).
 */
int32_t sfm_match_pairs_dev(sfm_ctx* ctx, const float* desc, const int32_t* count, int32_t nimg,
                            int64_t cap, const int32_t* pairs, int32_t P, float ratio,
                            int32_t* matches, float* conf, int32_t* nmatch, void* stream);

/*
 * The same matcher split in two for large resident tables (BASELINE configs[3]'s gathered
 * table of thousands of slots, matched a chunk of pairs at a time):
 *  - sfm_match_prep_dev builds the matcher's per-descriptor operands (split-f16 copies,
 *    norms, per-slot maxima) for slots [slot_lo, slot_lo + slot_n) of a table of `nimg`
 *    slots into ctx-owned buffers sized for the whole table;
 *  - sfm_match_pairs_prepped_dev matches pairs whose slots were all prepped by earlier
 *    calls on this ctx (same table, descriptors unchanged since) — sfm_match_pairs_dev
 *    without its prep of every slot.
 * Results are identical to sfm_match_pairs_dev.  Same pairs / outputs / status rules.
 * A prepped call whose table (desc, count, nimg, cap) is not the one last prepped on this
 * ctx returns SFM_ESTATE.  That every slot the device-resident pairs touch was prepped,
 * and that its descriptors did not change since, is the caller's (unchecked) contract.
 *
 * Matcher workspace (both calls): operands 520 B per slot (x capP = cap rounded up to
 * 128) for the table, plus per pair cap x 532 B (row results, overflow list and 128
 * admitted-target words per query row).  The per-pair part is bounded: a call with more
 * pairs than fit the budget (default 2 GiB, env SFMFEAT_MATCH_BUDGET_MB read at context
 * creation) runs as consecutive sub-launches over the same buffers.
 */
int32_t sfm_match_prep_dev(sfm_ctx* ctx, const float* desc, const int32_t* count, int32_t nimg,
                           int64_t cap, int32_t slot_lo, int32_t slot_n, void* stream);
int32_t sfm_match_pairs_prepped_dev(sfm_ctx* ctx, const float* desc, const int32_t* count,
                                    int32_t nimg, int64_t cap, const int32_t* pairs, int32_t P,
                                    float ratio, int32_t* matches, float* conf, int32_t* nmatch,
                                    void* stream);

/* ---------------- stream layout of a context ----------------
 * Replaces no reference interface (the reference has no device streams).
 * sfm_ctx_stream: the context's own HIP stream (created on first use; the host-pointer calls
 * run on it) for callers that enqueue the batch calls on it instead of a stream of their own.
 * sfm_ctx_set_serial: 1 = extractions run every stage on the caller's stream (no internal
 * aux stream, no fork/join); 0 = the two largest levels' selection and descriptors overlap
 * the later levels' Harris on the context's aux stream (default; SFMFEAT_SERIAL=1 flips the
 * default).  Each stream maps onto one of the HIP runtime's hardware queues, and streams
 * beyond GPU_MAX_HW_QUEUES share one, so a batch pipeline chooses how many it uses.
 * sfm_ctx_set_priority: HIP stream priority of the context's two streams (lower = higher
 * priority, hipDeviceGetStreamPriorityRange; default 0); only before either stream exists
 * (SFM_EINVAL after).  BatchPipeline's SFMFEAT_LANE_PRIO=1 gives its first lane the higher
 * priority (an A/B setting; DESIGN_LOG.md §B). */
int32_t sfm_ctx_stream(sfm_ctx* ctx, void** stream);
/* sfm_ctx_set_fused_prep: 1 = each batch extraction on this context also writes the matcher's
 * per-descriptor operands (split-f16 copies, norms, block maxima; sfm_match_prep_dev's work)
 * from its descriptor kernel, and the next sfm_match_pairs_dev on this context over the same
 * table (desc, count, cap) preps only the slots beyond the extraction's batch — one launch
 * fewer per batch (BatchPipeline turns it on for its own tables).  Contract: the
 * descriptors an extraction wrote are not modified before that match (or
 * sfm_match_prep_dev is called over them first); 0 (default) = off. */
int32_t sfm_ctx_set_fused_prep(sfm_ctx* ctx, int32_t on);
int32_t sfm_ctx_set_serial(sfm_ctx* ctx, int32_t serial);
int32_t sfm_ctx_set_priority(sfm_ctx* ctx, int32_t priority);

/* ---------------- batches in flight: the lane gate ----------------
 * Replaces no reference interface: the reference runs one pair per host thread
 * (Runner.py:183-191); this orders the device-resident batch path's lanes.  Contexts that
 * share a gate (set with sfm_ctx_set_gate) order their extractions in submission order:
 * each batched extraction's pyramid waits, on its stream, until the previous gated
 * extraction's level-0 Harris launch has finished, so the two batches' largest VALU
 * launches never compete, and one batch's level-0 Harris overlaps the other's level-0 NMS,
 * selection and descriptors.  The gated contexts must be driven from one host thread; a
 * gate must outlive the contexts that use it (or be unset with NULL first). */
typedef struct sfm_gate sfm_gate;
int32_t sfm_gate_create(int32_t device, sfm_gate** out);
int32_t sfm_gate_destroy(sfm_gate* gate);
int32_t sfm_ctx_set_gate(sfm_ctx* ctx, sfm_gate* gate);

/* ---------------- multi-GPU exchange over RCCL (SURVEY.md §8b "sfm_dist_*", §8e) ----------
 * The reference fans the extractor and matcher out over 8 threads of one process
 * (Runner.py:183-191, 336-355); sharded over GPUs (one process per GPU, frames in contiguous
 * shards), the only data exchanged is the slot table the match schedule needs: the halo slot
 * of the consecutive schedule and, for configs[3], each chunk's slots on every rank.  These
 * calls move exactly that over RCCL without torch: a host in any language creates one
 * communicator per rank (the 128-byte id made by one rank and handed to the others over any
 * channel), then enqueues the exchange on its stream next to sfm_extract_batch_dev /
 * sfm_match_pairs_dev.  RCCL is loaded at run time (the copy already in the process, e.g.
 * PyTorch's, else librccl.so.1 from the library path): without it every call returns
 * SFM_EDEVICE and the rest of the library is unaffected.  One device per rank (RCCL does not
 * allow two ranks of one communicator on the same GPU).  Slot-table layout as
 * sfm_extract_batch_dev writes it: xy [slot][cap][2] int32, desc [slot][cap][128] float32,
 * count [slot] int32.  Errors: SFM_EINVAL (arguments), SFM_EDEVICE (RCCL / HIP; text via
 * sfm_dist_last_error, which takes NULL for failures before a communicator exists). */
#define SFM_DIST_ID_BYTES 128
typedef struct sfm_dist sfm_dist;
int32_t sfm_dist_unique_id(uint8_t* id /* [SFM_DIST_ID_BYTES] */);
/* Collective over the `world` ranks: every rank calls it with the same id (blocks until all
 * have joined). */
int32_t sfm_dist_create(int32_t device, int32_t rank, int32_t world, const uint8_t* id, sfm_dist** out);
int32_t sfm_dist_destroy(sfm_dist* d);
const char* sfm_dist_last_error(const sfm_dist* d);
int32_t sfm_dist_rank(const sfm_dist* d, int32_t* rank, int32_t* world);
/* configs[3]'s chunk gather (distributed.py allgather_chunk): every rank's bc slots
 * (src_*) land at table slots [base + r * bc, base + (r + 1) * bc) of every rank r, all three
 * fields in one grouped RCCL launch on `stream`.  In place (no copy of the own slots) when
 * src_* point at the table's own slots base + rank * bc. */
int32_t sfm_dist_allgather_slots_dev(sfm_dist* d, int32_t bc, int32_t cap, const int32_t* src_xy,
                                     const float* src_desc, const int32_t* src_count, int32_t* tab_xy,
                                     float* tab_desc, int32_t* tab_count, int64_t base, void* stream);
/* The consecutive schedule's halo (distributed.py halo_exchange): rank r sends its slot
 * (src_*, one slot) to rank r - 1 and receives rank r + 1's into dst_* (one slot); the first
 * rank only receives, the last only sends, a single rank does nothing. */
int32_t sfm_dist_halo_dev(sfm_dist* d, int32_t cap, const int32_t* src_xy, const float* src_desc,
                          const int32_t* src_count, int32_t* dst_xy, float* dst_desc, int32_t* dst_count,
                          void* stream);

/* ---------------- stage profiling (bench.py's live roofline numbers) ----------------
 * When enabled, every stage's launches are bracketed by HIP events on the launch
 * stream; sfm_profile_read synchronises them and returns the accumulated device time
 * (ms) and bracket count per stage, indexed by SFM_PROF_*. */
#define SFM_PROF_PYRAMID 0
#define SFM_PROF_HARRIS 1
#define SFM_PROF_MEDIAN 2
#define SFM_PROF_NMS 3
#define SFM_PROF_TOPK 4
#define SFM_PROF_DESCRIBE 5
#define SFM_PROF_MATCH_PREP 6
#define SFM_PROF_MATCH 7
#define SFM_PROF_MATCH_POST 8
#define SFM_PROF_STAGES 9
int32_t sfm_profile_enable(sfm_ctx* ctx, int32_t on);
/* Bracket only the stages whose bit (1 << SFM_PROF_*) is set in `mask` (0 = off): the
 * bench times its headline run with the dominant stage's events alone. */
int32_t sfm_profile_stages(sfm_ctx* ctx, int32_t mask);
int32_t sfm_profile_read(sfm_ctx* ctx, double* ms, int64_t* launches, int32_t reset);
/* Kernel-active spans of the Harris launches (the dominant kernel of the headline step):
 * with capacity > 0, each of the context's next `capacity` Harris launches records
 * {earliest workgroup start, latest workgroup end} on the device's constant-rate realtime
 * clock (one atomic per workgroup, so it can stay on inside a timed region; unlike a pair of
 * stream events it excludes the time a launch waits on its stream for CUs another stream
 * holds).  capacity 0 turns it off.  Both calls reset the slots (and synchronise the device).
 * sfm_profile_spans_read: spans_ns [n][2] in ns on that clock (comparable across the contexts
 * of one device), levels [n] the first pyramid level of each launch, n_out the launches
 * recorded (at most `capacity`), dropped the launches beyond it.
 * (No reference counterpart: bench.py's roofline) */
int32_t sfm_profile_spans(sfm_ctx* ctx, int64_t capacity);
int32_t sfm_profile_spans_read(sfm_ctx* ctx, int64_t* spans_ns, int32_t* levels, int64_t cap, int64_t* n_out,
                               int64_t* dropped, int32_t reset);

/* ---------------- diagnostics (used by the parity tests) ----------------
 * Run individual stages of the same device code on host data. */
/* numpy-SVML-exact float32 atan2 on the device (np.arctan2, ScaleRotInvSIFT.py:42). */
int32_t sfm_debug_atan2(int32_t device, const float* y, const float* x, float* out, int64_t n);
/* Harris R map, exact median and candidate count of one plane (NaiveSIFT.py:59-97). */
int32_t sfm_debug_harris(int32_t device, const float* gauss, int32_t gs, double alpha,
                         int32_t ksize, const float* img, int32_t H, int32_t W, float* R_out,
                         float* median_out, int64_t* ncand_out);

/* Certified-mode NMS candidates (NaiveSIFT.py:77-95 with keys >= tnms[b]) of B planes:
 * unordered u64 keys ~fkey(R) << 32 | raster index in keys_out[b*H*W ...], counts_out[b] of
 * them.  tile = 1 forces the tiled kernel where the streaming one runs by default. */
int32_t sfm_debug_nms(int32_t device, const float* R, int32_t B, int32_t H, int32_t W, int32_t ksize,
                      const uint32_t* tnms, int32_t tile, uint64_t* keys_out, int64_t* counts_out);

/* Mean time (ms) of one fused Harris launch on synthetic planes, ablation variant abl
 * (0 full, 1 no digit histogram, 2 window sums over the first tap row only). */
float sfm_debug_time_harris(int32_t device, int32_t abl, int32_t B, int32_t H, int32_t W,
                            int32_t iters);
/* As sfm_debug_time_harris; abl = 3 (full kernel + timestamps) also copies the last launch's
   per-workgroup records into out[cap] (48 u64 per workgroup: start, end, CU id, tiles, then
   the end of each tile; s_memrealtime ticks of 10 ns). */
float sfm_debug_harris_stamps(int32_t device, int32_t abl, int32_t B, int32_t H, int32_t W,
                              int32_t iters, uint64_t* out, int64_t cap);

/* Diagnostic build only (make ABLATIONS=1; -1 in the shipped library): the matcher sweep's
 * per-wave shader-clock stamps of its last launch under SFMFEAT_MATCH_ABL=32, u64
 * [16 workgroups][8 waves][41][4] (stages 0..39: after the stage barrier, after each sub-tile
 * region, after the DMA issue; row 40: start clock, start / end realtime, pair | stages << 32),
 * then u64 [1024 workgroups][4]: start / end realtime, __smid(), pair | row0 << 32. */
int64_t sfm_debug_match_stamps(uint64_t* out, int64_t cap);

/* Exchange emulation for a single-GPU rehearsal of the multi-GPU job (bench.py
 * --emulate-exchange): copy `bytes` from src to dst (device pointers, 16-B aligned) on
 * `stream` with exactly `workgroups` persistent 256-thread workgroups — the launch shape of a
 * collective kernel (one workgroup per channel) receiving the same bytes. */
int32_t sfm_copy_wg(void* dst, const void* src, int64_t bytes, int32_t workgroups, void* stream);

/* Keypoint selection of the context's last extraction (synchronises the device): planes
 * (image x level) that took the exact-median path, and planes in total.  The default
 * certified select decides the others from the Harris histogram alone. */
int32_t sfm_debug_select_stats(sfm_ctx* ctx, int32_t* fallback_planes, int32_t* total_planes);
/* Level l's R maps (what 0) or level images (what 1) of the last extraction -> out [B][h][w]
 * (device, on `stream`; diagnostics). */
int32_t sfm_debug_copy_level(sfm_ctx* ctx, int32_t l, int32_t what, float* out, void* stream);


#ifdef __cplusplus
}
#endif

#endif /* SFMFEAT_H_ */
