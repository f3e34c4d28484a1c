/*
 * sfm_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C restatement of the reference's detect + describe + match path
 * (reesque/SfmFromScratch, FeatureExtractor/SIFT/NaiveSIFT.py, ScaleRotInvSIFT.py and
 * FeatureMatcher/NNRatioFeatureMatcher.py).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product (sfmfromscratch_amd/) never
 * links or calls it.
 *
 * Parity pinning: the .npz fixtures in tests/golden were produced by running the reference's own
 * Python code in the build container (tools/gen_golden.py) with the cv2 stand-in of
 * oracle/cv2_standin.py; tests/test_oracle_golden.py checks this file against them.
 * cv2.filter2D / cv2.resize themselves (OpenCV 4.10, absent from the image) are
 * restated by the documented rules below: parity with real OpenCV is UNPINNED for those
 * two calls.
 *
 * Numeric contract: compiled with -ffp-contract=off; every float
 * operation below is one IEEE-754 binary32 (or binary64 where marked) operation with
 * round-to-nearest-even; fmaf() only where the contract prescribes a fused op (the
 * SVML atan2f transcription).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/sfmfeat.h"

#define ORC_API __attribute__((visibility("default")))

static inline float f_from_bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t bits_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* ------------------------------------------------------------------------------- */
/* Gaussian window: NaiveSIFT._generate_gaussian_kernel, NaiveSIFT.py:175-199.       */
/* linspace(-m, m, ks) (numpy: i*step + start, last element = stop), exp in float64, */
/* normalised by the float64 sum (numpy pairwise for <=8 elems per row is sequential;*/
/* the 2-D sum reduces rows in order), then cast to float32 as filter2D does.        */
/* The Python wrapper passes numpy's own values; this is the native fallback.       */
/* ------------------------------------------------------------------------------- */
ORC_API void orc_linspace(double start, double stop, int num, double* out) {
  if (num <= 0) return;
  if (num == 1) { out[0] = start; return; }
  double step = (stop - start) / (double)(num - 1);
  for (int i = 0; i < num; ++i) out[i] = (double)i * step + start;
  out[num - 1] = stop;
}

ORC_API int orc_gaussian_kernel(int ks, double sigma, float* out) {
  if (ks < 1 || ks > SFM_MAX_GAUSS) return SFM_EINVAL;
  double ax[SFM_MAX_GAUSS];
  double k[SFM_MAX_GAUSS * SFM_MAX_GAUSS];
  int m = ks / 2;
  orc_linspace((double)-m, (double)m, ks, ax);
  const double PI = 3.141592653589793;
  double c = 1.0 / (2.0 * PI * (sigma * sigma));
  double den = 2.0 * (sigma * sigma);
  double total = 0.0;
  for (int i = 0; i < ks; ++i)
    for (int j = 0; j < ks; ++j) {
      double v = c * exp(-((ax[i] * ax[i]) + (ax[j] * ax[j])) / den);
      k[i * ks + j] = v;
    }
  /* np.sum over a 2-D contiguous array: pairwise over the flat buffer. */
  {
    int n = ks * ks;
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
  }
  for (int i = 0; i < ks * ks; ++i) out[i] = (float)(k[i] / total);
  return SFM_OK;
}

/* ------------------------------------------------------------------------------- */
/* cv2.filter2D(src, -1, kernel, borderType=BORDER_CONSTANT) restated               */
/* (call sites NaiveSIFT.py:67-69, 212-213): correlation, anchor at the kernel       */
/* centre, zero border.  acc starts at +0 and acc = fmaf(k, p, acc) for every NON-ZERO*/
/* tap in row-major kernel order — OpenCV's own float path (FilterVec_32f:           */
/* s = v_muladd(src, k, s) over preprocess2DKernel's row-major non-zero taps, FMA    */
/* under its AVX2 dispatch).  For the Sobel taps (+-1, +-2) k*p is exact, so the     */
/* gradients equal the unfused sum bit for bit.                                      */
/* ------------------------------------------------------------------------------- */
ORC_API void orc_filter2d(const float* src, int H, int W, const float* ker, int kh, int kw,
                          float* dst) {
  int ay = kh / 2, ax = kw / 2;
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      float acc = 0.0f;
      for (int i = 0; i < kh; ++i) {
        int yy = y + i - ay;
        for (int j = 0; j < kw; ++j) {
          float k = ker[i * kw + j];
          if (k == 0.0f) continue;
          int xx = x + j - ax;
          float p = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? src[(long)yy * W + xx] : 0.0f;
          acc = fmaf(k, p, acc);
        }
      }
      dst[(long)y * W + x] = acc;
    }
}

/* Sobel kernels NaiveSIFT.py:23-31 (float32). */
static const float SOBEL_X[9] = {-1, 0, 1, -2, 0, 2, -1, 0, 1};
static const float SOBEL_Y[9] = {-1, -2, -1, 0, 0, 0, 1, 2, 1};

/* NaiveSIFT._compute_image_gradients, NaiveSIFT.py:201-213. */
ORC_API void orc_gradients(const float* img, int H, int W, float* Ix, float* Iy) {
  orc_filter2d(img, H, W, SOBEL_X, 3, 3, Ix);
  orc_filter2d(img, H, W, SOBEL_Y, 3, 3, Iy);
}

/* ------------------------------------------------------------------------------- */
/* cv2.resize(src, (dw, dh)) INTER_LINEAR on float32 restated                       */
/* (ScaleRotInvSIFT.py:114).  Rule 1 (OpenCV's exact-2x switch to INTER_AREA fast):  */
/* when src == 2*dst in both axes, dst = ((a00 + a01) + (a10 + a11)) * 0.25f.        */
/* Rule 2 otherwise: half-pixel bilinear, coefficients                               */
/*   scale = 1/((double)dst/src);  f = (float)((d + 0.5)*scale - 0.5); s = floor(f);  */
/*   f -= s;  s < 0 -> (s=0, f=0);  s >= n-1 -> (s=n-1, f=0 and single tap)          */
/* horizontal h = S[s]*(1-f) + S[s+1]*f, vertical v = h0*(1-g) + h1*g (f32, no FMA). */
/* ------------------------------------------------------------------------------- */
static void linear_coeffs(int dn, int sn, int* ofs, float* a0, float* a1, int* single) {
  double inv = (double)dn / (double)sn;
  double scale = 1.0 / inv;
  for (int d = 0; d < dn; ++d) {
    float f = (float)(((double)d + 0.5) * scale - 0.5);
    int s = (int)floorf(f);
    f -= (float)s;
    int one = 0;
    if (s < 0) { s = 0; f = 0.0f; }
    if (s + 1 >= sn) { one = 1; if (s >= sn - 1) { s = sn - 1; f = 0.0f; } }
    ofs[d] = s;
    a0[d] = 1.0f - f;
    a1[d] = f;
    single[d] = one;
  }
}

ORC_API int orc_resize(const float* src, int H, int W, float* dst, int dH, int dW) {
  if (dH <= 0 || dW <= 0 || H <= 0 || W <= 0) return SFM_EINVAL;
  if (H == 2 * dH && W == 2 * dW) {
    for (int y = 0; y < dH; ++y)
      for (int x = 0; x < dW; ++x) {
        const float* r0 = src + (long)(2 * y) * W + 2 * x;
        const float* r1 = r0 + W;
        float t0 = r0[0] + r0[1];
        float t1 = r1[0] + r1[1];
        dst[(long)y * dW + x] = (t0 + t1) * 0.25f;
      }
    return SFM_OK;
  }
  int* xo = (int*)malloc(sizeof(int) * dW);
  int* xs = (int*)malloc(sizeof(int) * dW);
  float* xa0 = (float*)malloc(sizeof(float) * dW);
  float* xa1 = (float*)malloc(sizeof(float) * dW);
  int* yo = (int*)malloc(sizeof(int) * dH);
  int* ys = (int*)malloc(sizeof(int) * dH);
  float* ya0 = (float*)malloc(sizeof(float) * dH);
  float* ya1 = (float*)malloc(sizeof(float) * dH);
  float* h0 = (float*)malloc(sizeof(float) * dW);
  float* h1 = (float*)malloc(sizeof(float) * dW);
  linear_coeffs(dW, W, xo, xa0, xa1, xs);
  linear_coeffs(dH, H, yo, ya0, ya1, ys);
  for (int y = 0; y < dH; ++y) {
    int sy0 = yo[y];
    int sy1 = sy0 + 1 < H ? sy0 + 1 : H - 1;
    const float* rows[2] = {src + (long)sy0 * W, src + (long)sy1 * W};
    float* hb[2] = {h0, h1};
    for (int r = 0; r < 2; ++r)
      for (int x = 0; x < dW; ++x) {
        const float* S = rows[r];
        int sx = xo[x];
        if (xs[x]) {
          hb[r][x] = S[sx];
        } else {
          float p = S[sx] * xa0[x];
          float q = S[sx + 1] * xa1[x];
          hb[r][x] = p + q;
        }
      }
    for (int x = 0; x < dW; ++x) {
      float p = h0[x] * ya0[y];
      float q = h1[x] * ya1[y];
      dst[(long)y * dW + x] = p + q;
    }
  }
  free(xo); free(xs); free(xa0); free(xa1); free(yo); free(ys); free(ya0); free(ya1);
  free(h0); free(h1);
  return SFM_OK;
}

/* Pyramid sizes: ScaleRotInvSIFT._build_image_pyramid, ScaleRotInvSIFT.py:109-115. */
ORC_API int orc_pyramid_dims(int H, int W, int L, double s, int* dims) {
  if (L < 1 || L > SFM_MAX_LEVELS) return SFM_EINVAL;
  dims[0] = H; dims[1] = W;
  for (int l = 1; l < L; ++l) {
    dims[2 * l] = (int)((double)dims[2 * l - 2] / s);
    dims[2 * l + 1] = (int)((double)dims[2 * l - 1] / s);
    if (dims[2 * l] <= 0 || dims[2 * l + 1] <= 0) return SFM_EINVAL;
  }
  return SFM_OK;
}

/* ------------------------------------------------------------------------------- */
/* Harris response, NaiveSIFT.py:59-74.                                              */
/* ------------------------------------------------------------------------------- */
ORC_API void orc_harris_response(const float* img, int H, int W, const float* gk, int gs,
                                 double alpha, float* R) {
  long n = (long)H * W;
  float* Ix = (float*)malloc(sizeof(float) * n);
  float* Iy = (float*)malloc(sizeof(float) * n);
  float* P = (float*)malloc(sizeof(float) * n * 3);
  float* S = (float*)malloc(sizeof(float) * n * 3);
  orc_gradients(img, H, W, Ix, Iy);
  for (long i = 0; i < n; ++i) {
    P[i] = Ix[i] * Ix[i];          /* Ix ** 2   :61 */
    P[n + i] = Iy[i] * Iy[i];      /* Iy ** 2   :62 */
    P[2 * n + i] = Ix[i] * Iy[i];  /* Ix * Iy   :63 */
  }
  orc_filter2d(P, H, W, gk, gs, gs, S);              /* S_xx :67 */
  orc_filter2d(P + 2 * n, H, W, gk, gs, gs, S + 2 * n);  /* S_xy :68 */
  orc_filter2d(P + n, H, W, gk, gs, gs, S + n);      /* S_yy :69 */
  float a = (float)alpha; /* NEP 50: python float scalar is cast to float32 */
  for (long i = 0; i < n; ++i) {
    float sxx = S[i], syy = S[n + i], sxy = S[2 * n + i];
    float t1 = sxx * syy;
    float t2 = sxy * sxy;
    float det = t1 - t2;        /* :71 */
    float tr = sxx + syy;       /* :72 */
    float tr2 = tr * tr;
    float at = a * tr2;
    R[i] = det - at;            /* :74 */
  }
  free(Ix); free(Iy); free(P); free(S);
}

static int cmp_float(const void* a, const void* b) {
  float x = *(const float*)a, y = *(const float*)b;
  return (x < y) ? -1 : (x > y) ? 1 : 0;
}

/* np.median on float32 (NaiveSIFT.py:91): even n -> float32 (lo + hi) / 2, odd -> middle. */
ORC_API float orc_median(const float* R, long n) {
  float* c = (float*)malloc(sizeof(float) * n);
  memcpy(c, R, sizeof(float) * n);
  qsort(c, n, sizeof(float), cmp_float);
  float m;
  if (n % 2 == 1) {
    m = c[n / 2];
  } else {
    float s = c[n / 2 - 1] + c[n / 2];
    m = s / 2.0f;
  }
  free(c);
  return m;
}

typedef struct { float c; int64_t idx; } cand_t;

/* Order of np.argsort(conf)[::-1] made deterministic: conf descending, raster index
 * ascending (ties are compared as sets by the tests; SURVEY.md §8.1 'top-k ties'). */
static int cmp_cand(const void* a, const void* b) {
  const cand_t* p = (const cand_t*)a;
  const cand_t* q = (const cand_t*)b;
  if (p->c > q->c) return -1;
  if (p->c < q->c) return 1;
  return (p->idx < q->idx) ? -1 : (p->idx > q->idx) ? 1 : 0;
}

/*
 * NaiveSIFT._find_harris_interest_points, NaiveSIFT.py:54-120.
 * Returns the number of keypoints written to x, y, c (<= k).  dbg (nullable) gets
 * {median, number of candidates before top-k, number after top-k}.
 */
ORC_API long orc_detect(const float* img, int H, int W, int k, int fw, int ksize,
                        const float* gk, int gs, double alpha, int64_t* xo, int64_t* yo,
                        float* co, double* dbg) {
  long n = (long)H * W;
  float* R = (float*)malloc(sizeof(float) * n);
  orc_harris_response(img, H, W, gk, gs, alpha, R);
  int kh = ksize / 2;
  float med = orc_median(R, n); /* :91 */
  cand_t* cand = (cand_t*)malloc(sizeof(cand_t) * (n > 0 ? n : 1));
  long nc = 0;
  for (int r = 0; r < H; ++r) {
    int r0 = r - kh < 0 ? 0 : r - kh, r1 = r + kh + 1 > H ? H : r + kh + 1;
    for (int c = 0; c < W; ++c) {
      int c0 = c - kh < 0 ? 0 : c - kh, c1 = c + kh + 1 > W ? W : c + kh + 1;
      float v = R[(long)r * W + c];
      float mp = R[(long)r0 * W + c0];
      for (int yy = r0; yy < r1; ++yy)
        for (int xx = c0; xx < c1; ++xx) {
          float t = R[(long)yy * W + xx];
          if (t > mp) mp = t;                   /* np.max of the clipped window :85-88 */
        }
      double rmp = (v < med) ? 0.0 : (double)mp;  /* R_maxpool[R_map < median] = 0 :92 */
      if ((double)v == rmp) {                   /* R_map == R_maxpool :95 */
        cand[nc].c = v;
        cand[nc].idx = (int64_t)r * W + c;
        ++nc;
      }
    }
  }
  qsort(cand, nc, sizeof(cand_t), cmp_cand);   /* argsort desc :100 */
  long ntop = nc < k ? nc : k;                  /* [:k] :100 */
  int hw = fw / 2;                              /* :105 */
  long m = 0;
  for (long i = 0; i < ntop; ++i) {
    int64_t y = cand[i].idx / W, x = cand[i].idx % W;
    if (y >= hw && y < H - hw && x >= hw && x < W - hw) { /* edge filter :107-112 */
      xo[m] = x; yo[m] = y; co[m] = cand[i].c; ++m;
    }
  }
  /* re-sort desc :115-118 is the identity on an already (conf desc, idx asc) list */
  if (dbg) { dbg[0] = med; dbg[1] = (double)nc; dbg[2] = (double)ntop; }
  free(R); free(cand);
  return m;
}

/* ------------------------------------------------------------------------------- */
/* np.arctan2 on float32 = numpy's bundled SVML __svml_atan2f16 on AVX-512 hosts.    */
/* Transcription pinned bit-exactly against np.arctan2 (tests/golden/atan2.npz).     */
/* ------------------------------------------------------------------------------- */
ORC_API float orc_atan2f(float y, float x) {
  if (isnan(x) || isnan(y)) return x + y;
  const float PI = f_from_bits(0x40490fdbu), PI_2 = f_from_bits(0x3fc90fdbu);
  float ax = fabsf(x), ay = fabsf(y);
  if (ay == 0.0f) return signbit(x) ? copysignf(PI, y) : copysignf(0.0f, y);
  if (ax == 0.0f) return copysignf(PI_2, y);
  int k = ay < ax;
  float num = k ? ay : -ax;
  float den = k ? ax : ay;
  float off = k ? 0.0f : PI_2;
  float q = num / den;
  float z2 = q * q;
  float z4 = z2 * z2;
  const float c0 = f_from_bits(0x3b322cc0u), c1 = f_from_bits(0xbc7f2631u),
              c2 = f_from_bits(0x3d2bc384u), c3 = f_from_bits(0xbd987629u),
              c4 = f_from_bits(0x3dd96474u), c5 = f_from_bits(0xbe1161f8u),
              c6 = f_from_bits(0x3e4cb79fu), c7 = f_from_bits(0xbeaaaa49u);
  float A = fmaf(fmaf(fmaf(fmaf(c0, z4, c2), z4, c4), z4, c6), z4, 1.0f);
  float B = fmaf(fmaf(fmaf(c1, z4, c3), z4, c5), z4, c7);
  float r = fmaf(fmaf(B, z2, A), q, off);
  if (signbit(x)) {
    r = f_from_bits(bits_of(r) | 0x80000000u);
    r = r + PI;
  }
  return f_from_bits(bits_of(r) | (bits_of(y) & 0x80000000u));
}

ORC_API void orc_atan2f_vec(const float* y, const float* x, float* out, long n) {
  for (long i = 0; i < n; ++i) out[i] = orc_atan2f(y[i], x[i]);
}

/* ------------------------------------------------------------------------------- */
/* np.histogram(a, bins=<float64 edges>, weights=w) — numpy's cumulative path:       */
/* argsort(a) (restated as a STABLE sort), cw = [0, cumsum(w_sorted)] in float32,    */
/* bin boundaries by searchsorted in float64 ('left', last edge 'right'),            */
/* n = diff(cw[idx]) in float32.  (numpy/lib/_histograms_impl.py, cumulative branch; */
/* used at NaiveSIFT.py:140-141, ScaleRotInvSIFT.py:26,73-76.)                        */
/* ------------------------------------------------------------------------------- */
ORC_API void orc_histogram(const double* v, const float* w, int n, const double* edges, int nb,
                           float* out) {
  int ord[4096];
  double sv[4096];
  float cw[4097];
  int idx[64];
  /* stable insertion sort by value */
  for (int i = 0; i < n; ++i) {
    int j = i;
    while (j > 0 && v[ord[j - 1]] > v[i]) { ord[j] = ord[j - 1]; --j; }
    ord[j] = i;
  }
  cw[0] = 0.0f;
  for (int i = 0; i < n; ++i) { sv[i] = v[ord[i]]; cw[i + 1] = cw[i] + w[ord[i]]; }
  for (int e = 0; e <= nb; ++e) {
    int cnt = 0;
    if (e < nb) { while (cnt < n && sv[cnt] < edges[e]) ++cnt; }
    else        { while (cnt < n && sv[cnt] <= edges[e]) ++cnt; }
    idx[e] = cnt;
  }
  for (int b = 0; b < nb; ++b) out[b] = cw[idx[b + 1]] - cw[idx[b]];
}

/* Fixed-order L2 norm of a 128-vector (restatement of np.linalg.norm's BLAS sdot, whose
 * summation order is CPU-dependent; SURVEY.md §8.1 'L2 norm'):  s_l = w_l^2 + w_{l+64}^2,
 * then a halving tree s_l += s_{l+off}, off = 32..1; sqrt. */
static float norm128(const float* w) {
  float s[64];
  for (int l = 0; l < 64; ++l) {
    float a = w[l] * w[l];
    float b = w[l + 64] * w[l + 64];
    s[l] = a + b;
  }
  for (int off = 32; off >= 1; off >>= 1)
    for (int l = 0; l < off; ++l) s[l] = s[l] + s[l + off];
  return sqrtf(s[0]);
}

/*
 * Descriptors for one pyramid level.
 * rotate = 1: ScaleRotInvSIFT._get_SIFT_descriptors, ScaleRotInvSIFT.py:33-87
 * rotate = 0: NaiveSIFT._get_SIFT_descriptors,       NaiveSIFT.py:122-173
 * out: n x 128.  Caller guarantees the edge filter (windows inside the image).
 */
ORC_API void orc_descriptors(const float* img, int H, int W, const int64_t* X, const int64_t* Y,
                             long n, int fw, int rotate, float* out) {
  long np_ = (long)H * W;
  float* Ix = (float*)malloc(sizeof(float) * np_);
  float* Iy = (float*)malloc(sizeof(float) * np_);
  float* mag = (float*)malloc(sizeof(float) * np_);
  float* ori = (float*)malloc(sizeof(float) * np_);
  orc_gradients(img, H, W, Ix, Iy);        /* :40 */
  for (long i = 0; i < np_; ++i) {
    float a = Ix[i] * Ix[i], b = Iy[i] * Iy[i];
    float s = a + b;
    mag[i] = sqrtf(s);                      /* :41 */
    ori[i] = orc_atan2f(Iy[i], Ix[i]);      /* :42 */
  }
  double e37[37], e9[9], cen36[36];
  const double PI = 3.141592653589793;
  orc_linspace(-PI, PI, 37, e37);          /* :25 */
  orc_linspace(-PI, PI, 9, e9);            /* :66 */
  for (int b = 0; b < 36; ++b) cen36[b] = (e37[b] + e37[b + 1]) / 2.0; /* :29 */
  int h = fw / 2;                           /* :51 */
  int ws = 2 * h;
  double* wv = (double*)malloc(sizeof(double) * ws * ws);
  float* ww = (float*)malloc(sizeof(float) * ws * ws);
  for (long p = 0; p < n; ++p) {
    long x = X[p], y = Y[p];
    long r0 = y - h + 1, c0 = x - h + 1;   /* window [y-h+1, y+h+1) :53-56 */
    double dom = 0.0;
    if (rotate) {
      for (int i = 0; i < ws; ++i)
        for (int j = 0; j < ws; ++j) {
          long o = (r0 + i) * W + (c0 + j);
          wv[i * ws + j] = (double)ori[o];
          ww[i * ws + j] = mag[o];
        }
      float hist[36];
      orc_histogram(wv, ww, ws * ws, e37, 36, hist);  /* :26 */
      int am = 0;
      for (int b = 1; b < 36; ++b) if (hist[b] > hist[am]) am = b; /* first argmax :30 */
      dom = cen36[am];
    }
    float wgh[128];
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 4; ++c) {
        double cv[16];
        float cwt[16];
        int cn = 0;
        for (int i = 4 * r; i < 4 * r + 4 && i < ws; ++i)   /* [r*4:(r+1)*4] :68-71 */
          for (int j = 4 * c; j < 4 * c + 4 && j < ws; ++j) {
            long o = (r0 + i) * W + (c0 + j);
            double ov = (double)ori[o];
            cv[cn] = rotate ? ov - dom : ov;   /* float64 relative angle :62 */
            cwt[cn] = mag[o];
            ++cn;
          }
        orc_histogram(cv, cwt, cn, e9, 8, wgh + (r * 4 + c) * 8); /* :73-76 */
      }
    float nrm = norm128(wgh);                 /* :82 */
    float* d = out + p * 128;
    for (int i = 0; i < 128; ++i) {
      float v = wgh[i];
      if (nrm > 0.0f) v = v / nrm;            /* :83-84 */
      d[i] = sqrtf(v);                        /* :85 RootSIFT */
    }
  }
  free(Ix); free(Iy); free(mag); free(ori); free(wv); free(ww);
}

/*
 * Whole extractor for one image, params->mode selects the plugin class:
 * ScaleRotInvSIFT.compute (ScaleRotInvSIFT.py:89-107) or NaiveSIFT detect+describe.
 * Returns the number of keypoints (or -SFM_E* on error).  level_counts: L ints.
 */
ORC_API long orc_extract(const float* img, int H, int W, const sfm_params* p, int64_t* X,
                         int64_t* Y, float* desc, float* conf, long cap, int32_t* level_counts) {
  float gk[SFM_MAX_GAUSS * SFM_MAX_GAUSS];
  int gs = p->gaussian_size;
  if (p->gauss_kernel_set) memcpy(gk, p->gauss_kernel, sizeof(float) * gs * gs);
  else if (orc_gaussian_kernel(gs, p->sigma, gk) != SFM_OK) return -SFM_EINVAL;
  int naive = p->mode == SFM_MODE_NAIVE;
  int L = naive ? 1 : p->pyramid_level;
  int dims[2 * SFM_MAX_LEVELS];
  if (naive) { dims[0] = H; dims[1] = W; }
  else if (orc_pyramid_dims(H, W, L, p->pyramid_scale_factor, dims) != SFM_OK) return -SFM_EINVAL;
  int scaled_k = naive ? p->num_interest_points
                       : (int)((double)p->num_interest_points / (double)L); /* :90 */
  long total = 0;
  float* cur = (float*)malloc(sizeof(float) * (long)H * W);
  memcpy(cur, img, sizeof(float) * (long)H * W);
  int64_t* xs = (int64_t*)malloc(sizeof(int64_t) * (scaled_k > 0 ? scaled_k : 1));
  int64_t* ys = (int64_t*)malloc(sizeof(int64_t) * (scaled_k > 0 ? scaled_k : 1));
  float* cs = (float*)malloc(sizeof(float) * (scaled_k > 0 ? scaled_k : 1));
  for (int l = 0; l < L; ++l) {
    int h = dims[2 * l], w = dims[2 * l + 1];
    if (l > 0) {
      float* nx = (float*)malloc(sizeof(float) * (long)h * w);
      orc_resize(cur, dims[2 * l - 2], dims[2 * l - 1], nx, h, w);
      free(cur);
      cur = nx;
    }
    double scale = naive ? 1.0 : pow(p->pyramid_scale_factor, (double)l); /* :95 */
    int fwl = naive ? p->feature_width : (int)((double)p->feature_width / scale);
    if (!naive && fwl < 3) fwl = 3;                                       /* :96 */
    long m = orc_detect(cur, h, w, scaled_k, fwl, p->ksize, gk, gs, p->alpha, xs, ys, cs, NULL);
    if (total + m > cap) { total = -SFM_ERANGE; break; }
    orc_descriptors(cur, h, w, xs, ys, m, fwl, naive ? 0 : 1, desc + total * 128);
    for (long i = 0; i < m; ++i) {
      X[total + i] = (int64_t)((double)xs[i] * scale);   /* (x * scale).astype(int) :101 */
      Y[total + i] = (int64_t)((double)ys[i] * scale);   /* :102 */
      if (conf) conf[total + i] = cs[i];
    }
    if (level_counts) level_counts[l] = (int32_t)m;
    total += m;
  }
  free(cur); free(xs); free(ys); free(cs);
  return total;
}

/* ------------------------------------------------------------------------------- */
/* NNRatioFeatureMatcher.match_features_ratio_test, NNRatioFeatureMatcher.py:8-60.   */
/* ------------------------------------------------------------------------------- */

/* sum((a-b)**2) over 128 float32 = numpy pairwise_sum with 8 accumulators (n = 128):
 * r[j] = sq[j]; r[j] += sq[i+j] for i = 8..120; ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)). */
ORC_API float orc_sqdist128(const float* a, const float* b) {
  float r[8];
  for (int j = 0; j < 8; ++j) { float d = a[j] - b[j]; r[j] = d * d; }
  for (int i = 8; i < 128; i += 8)
    for (int j = 0; j < 8; ++j) { float d = a[i + j] - b[i + j]; float s = d * d; r[j] = r[j] + s; }
  float t01 = r[0] + r[1], t23 = r[2] + r[3], t45 = r[4] + r[5], t67 = r[6] + r[7];
  float u0 = t01 + t23, u1 = t45 + t67;
  return u0 + u1;
}

typedef struct { float conf; int64_t row; int64_t col; } match_t;

static int cmp_match(const void* a, const void* b) {
  const match_t* p = (const match_t*)a;
  const match_t* q = (const match_t*)b;
  if (p->conf < q->conf) return -1;
  if (p->conf > q->conf) return 1;
  return (p->row < q->row) ? -1 : (p->row > q->row) ? 1 : 0;
}

/* Returns k >= 0 matches, or -SFM_EINDEX when n1 >= 1 and n2 < 2 (IndexError at :42). */
ORC_API long orc_match(const float* f1, long n1, const float* f2, long n2, float ratio,
                       int64_t* mo, float* co) {
  if (n1 >= 1 && n2 < 2) return -SFM_EINDEX;
  match_t* ms = (match_t*)malloc(sizeof(match_t) * (n1 > 0 ? n1 : 1));
  long k = 0;
  for (long i = 0; i < n1; ++i) {
    /* argsort of sqrt(sum) rows (:34,:41): smallest and second smallest by
     * (distance, index); sqrt is monotone, so track the sums. */
    float b1 = INFINITY, b2 = INFINITY;
    long j1 = -1, j2 = -1;
    for (long j = 0; j < n2; ++j) {
      float s = orc_sqdist128(f1 + i * 128, f2 + j * 128);
      if (j1 < 0 || s < b1) { b2 = b1; j2 = j1; b1 = s; j1 = j; }
      else if (j2 < 0 || s < b2) { b2 = s; j2 = j; }
    }
    float d1 = sqrtf(b1), d2 = sqrtf(b2);
    if (d2 > 0.0f) {                     /* :46 */
      float nndr = d1 / d2;              /* :47 */
      if (nndr <= ratio) {               /* :49 */
        ms[k].conf = nndr; ms[k].row = i; ms[k].col = j1; ++k;
      }
    }
  }
  qsort(ms, k, sizeof(match_t), cmp_match); /* argsort(confidences) :56-58 */
  for (long i = 0; i < k; ++i) { mo[2 * i] = ms[i].row; mo[2 * i + 1] = ms[i].col; co[i] = ms[i].conf; }
  free(ms);
  return k;
}
