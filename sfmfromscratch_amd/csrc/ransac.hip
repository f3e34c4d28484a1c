// ransac.hip — the match consumer CameraPose.find_inliers (SFM.py:126-160, SURVEY.md §8f
// row 2): 8-point RANSAC over a pair's correspondences, max_iterations samples drawn by
// numpy's legacy RandomState after np.random.seed(5), the first sample with the most
// inliers (epipolar distance < threshold) wins.
//
// * Samples: `np.random.choice(n, 8, replace=False)` is permutation(n)[:8] — a full
//   Fisher-Yates shuffle of arange(n) whose j = random_interval(i) draws are MT19937
//   outputs masked to the next power of two, rejected above i (numpy legacy
//   _shuffle_raw / random_interval).  The stream depends only on (seed, n, iterations),
//   is inherently sequential, and is replayed on the host (ransac_sample_indices,
//   pinned bit-exactly against numpy by tests/test_ransac_cpu.py), cached per n.
// * Fundamental matrix per sample (CameraPose._compute_fundamental_matrix, SFM.py:
//   190-236), one thread per (pair, sample), float64: Hartley normalisation (mean,
//   mean distance, sqrt(2) scale), the 8 x 9 system's null vector by Gaussian
//   elimination with partial pivoting (the reference takes SVD's last right singular
//   vector: the same line, up to scale and sign, for a rank-8 system), rank 2 by
//   removing the smallest singular direction (F - (F v3) v3^T, v3 from a Jacobi
//   eigen-decomposition of F^T F: equal to U diag(d1, d2, 0) V^T), un-normalised.
//   Distances are invariant to F's scale and sign.
// * Inlier counts (SFM.py:147-156): one thread per sample, the pair's points staged in LDS
//   and read as broadcasts, d = |lb . p2| / sqrt(lb0^2 + lb1^2) with lb = F p1 in
//   float64, d < threshold (decided without the division away from the threshold).
// * Selection: the first sample with the largest count (strict > updates, SFM.py:156),
//   its mask recomputed and the inliers compacted in input order.
// Bar: the inlier sets equal the reference's on the golden pairs; float64 rounding of
// the SVD vs the elimination can only flip a point whose distance is within ~1e-12
// of the threshold.
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <vector>

#include "kernels.h"

namespace sfm {

// ---------------- host: numpy legacy RandomState replay ----------------
namespace {
struct MT19937 {
  uint32_t mt[624];
  int pos = 624;
  explicit MT19937(uint32_t seed) {  // init_genrand (numpy legacy seeding of an int)
    mt[0] = seed;
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
  }
  void twist() {
    for (int i = 0; i < 624; ++i) {
      const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
      mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    pos = 0;
  }
  uint32_t next() {
    if (pos >= 624) twist();
    uint32_t y = mt[pos++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
};

// The tempered output stream of one seed, generated once per process in fixed chunks
// that never move: every pair restarts from np.random.seed(5) (SFM.py:133), so all
// pairs read the same raw words and differ only in how their n consumes them.
class RawStream {
 public:
  static constexpr size_t kChunk = size_t(1) << 20;
  explicit RawStream(uint32_t seed) : g_(seed) {}
  const uint32_t* chunk(size_t k) {
    std::lock_guard<std::mutex> lock(mu_);
    while (chunks_.size() <= k) {
      std::unique_ptr<uint32_t[]> c(new uint32_t[kChunk]);
      for (size_t i = 0; i < kChunk; ++i) c[i] = g_.next();
      chunks_.push_back(std::move(c));
    }
    return chunks_[k].get();
  }

 private:
  std::mutex mu_;
  MT19937 g_;
  std::vector<std::unique_ptr<uint32_t[]>> chunks_;
};

RawStream& raw_stream(uint32_t seed) {
  static std::mutex mu;
  static std::vector<std::pair<uint32_t, std::unique_ptr<RawStream>>> streams;
  std::lock_guard<std::mutex> lock(mu);
  for (auto& s : streams)
    if (s.first == seed) return *s.second;
  streams.emplace_back(seed, std::unique_ptr<RawStream>(new RawStream(seed)));
  return *streams.back().second;
}

struct Cursor {
  RawStream& s;
  size_t k = 0, i = 0;
  const uint32_t* c;
  explicit Cursor(RawStream& st) : s(st), c(st.chunk(0)) {}
  uint32_t next() {
    if (i == RawStream::kChunk) {
      c = s.chunk(++k);
      i = 0;
    }
    return c[i++];
  }
};
}  // namespace

void ransac_sample_indices(int n, int iters, uint32_t seed, int32_t* out) {
  Cursor g(raw_stream(seed));
  std::vector<int32_t> a(std::max(n, 1));
  uint32_t top = 0;  // random_interval's mask for i = n - 1: the smallest 2^b - 1 >= i
  if (n > 1) {
    top = (uint32_t)(n - 1);
    top |= top >> 1;
    top |= top >> 2;
    top |= top >> 4;
    top |= top >> 8;
    top |= top >> 16;
  }
  for (int it = 0; it < iters; ++it) {
    for (int i = 0; i < n; ++i) a[i] = i;
    uint32_t mask = top;
    for (int i = n - 1; i >= 1; --i) {  // _shuffle_raw: j = random_interval(i)
      if ((uint32_t)i <= (mask >> 1)) mask >>= 1;  // i drops by one: one halving keeps it minimal
      uint32_t v;
      while ((v = (g.next() & mask)) > (uint32_t)i) {
      }
      const int32_t t = a[i];
      a[i] = a[v];
      a[v] = t;
    }
    for (int k = 0; k < 8; ++k) out[(size_t)it * 8 + k] = a[k];
  }
}

// ---------------- device ----------------
struct Mat3 {
  double m[9];
};

SFM_DEV void normalise8(const double (&x)[8], const double (&y)[8], double (&nx)[8], double (&ny)[8], double& s,
                        double& cx, double& cy) {
  // CameraPose.normalize_points (SFM.py:164-178)
  double mx = 0.0, my = 0.0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    mx += x[i];
    my += y[i];
  }
  mx /= 8.0;
  my /= 8.0;
  double md = 0.0;
#pragma unroll
  for (int i = 0; i < 8; ++i) md += sqrt((x[i] - mx) * (x[i] - mx) + (y[i] - my) * (y[i] - my));
  md /= 8.0;
  s = sqrt(2.0) / md;
  cx = mx;
  cy = my;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    nx[i] = s * x[i] + (-s * mx);
    ny[i] = s * y[i] + (-s * my);
  }
}

// null vector of the 8 x 9 system (rows [x1x2, y1x2, x2, x1y2, y1y2, y2, x1, y1, 1])
SFM_DEV bool null_vector_8x9(double (&A)[8][9], double (&f)[9]) {
  int piv_col[8];
  int r = 0;
  for (int c = 0; c < 9 && r < 8; ++c) {
    int best = r;
    double bv = fabs(A[r][c]);
    for (int i = r + 1; i < 8; ++i)
      if (fabs(A[i][c]) > bv) { bv = fabs(A[i][c]); best = i; }
    if (bv < 1e-300) continue;  // free column
    if (best != r)
      for (int k = 0; k < 9; ++k) { const double t = A[r][k]; A[r][k] = A[best][k]; A[best][k] = t; }
    for (int i = r + 1; i < 8; ++i) {
      const double fct = A[i][c] / A[r][c];
      for (int k = c; k < 9; ++k) A[i][k] -= fct * A[r][k];
    }
    piv_col[r++] = c;
  }
  if (r < 8) return false;  // rank-deficient sample (degenerate points)
  int free_col = 8;         // the one column without a pivot
  {
    bool used[9] = {false, false, false, false, false, false, false, false, false};
    for (int i = 0; i < 8; ++i) used[piv_col[i]] = true;
    for (int c = 0; c < 9; ++c)
      if (!used[c]) free_col = c;
  }
  for (int k = 0; k < 9; ++k) f[k] = 0.0;
  f[free_col] = 1.0;
  for (int i = 7; i >= 0; --i) {
    const int c = piv_col[i];
    double acc = 0.0;
    for (int k = c + 1; k < 9; ++k) acc += A[i][k] * f[k];
    f[c] = -acc / A[i][c];
  }
  return true;
}

// The same elimination when every column 0..7 has a pivot (the usual case), with every
// index compile-time: row exchanges are selects, so A stays in registers (the general
// routine's runtime row indices put it in scratch).  Returns false on a zero pivot; the
// caller then rebuilds A and takes the general routine, which handles free columns.
SFM_DEV bool null_vector_8x9_regs(double (&A)[8][9], double (&f)[9]) {
#pragma unroll
  for (int c = 0; c < 8; ++c) {
#pragma unroll
    for (int i = c + 1; i < 8; ++i) {  // the first row of largest |A[.][c]| ends in row c
      const bool sw = fabs(A[i][c]) > fabs(A[c][c]);
#pragma unroll
      for (int k = c; k < 9; ++k) {
        const double u = A[c][k], v = A[i][k];
        A[c][k] = sw ? v : u;
        A[i][k] = sw ? u : v;
      }
    }
    if (!(fabs(A[c][c]) >= 1e-300)) return false;
#pragma unroll
    for (int i = c + 1; i < 8; ++i) {
      const double fct = A[i][c] / A[c][c];
#pragma unroll
      for (int k = c; k < 9; ++k) A[i][k] -= fct * A[c][k];
    }
  }
  f[8] = 1.0;
#pragma unroll
  for (int i = 7; i >= 0; --i) {
    double acc = 0.0;
#pragma unroll
    for (int k = i + 1; k < 9; ++k) acc += A[i][k] * f[k];
    f[i] = -acc / A[i][i];
  }
  return true;
}

// smallest-eigenvalue eigenvector of a symmetric 3 x 3 (cyclic Jacobi)
SFM_DEV void smallest_eigvec3(double (&S)[3][3], double (&v)[3]) {
  double V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  for (int sweep = 0; sweep < 12; ++sweep) {
    const double off = fabs(S[0][1]) + fabs(S[0][2]) + fabs(S[1][2]);
    const double dia = fabs(S[0][0]) + fabs(S[1][1]) + fabs(S[2][2]);
    if (off <= 1e-18 * dia) break;
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int q = p + 1; q < 3; ++q) {
        if (fabs(S[p][q]) < 1e-300) continue;
        const double theta = (S[q][q] - S[p][p]) / (2.0 * S[p][q]);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 3; ++k) {  // S = J^T S J
          const double skp = S[k][p], skq = S[k][q];
          S[k][p] = c * skp - s * skq;
          S[k][q] = s * skp + c * skq;
        }
        for (int k = 0; k < 3; ++k) {
          const double spk = S[p][k], sqk = S[q][k];
          S[p][k] = c * spk - s * sqk;
          S[q][k] = s * spk + c * sqk;
        }
        for (int k = 0; k < 3; ++k) {
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq;
          V[k][q] = s * vkp + c * vkq;
        }
      }
  }
  const int mi = (S[1][1] < S[0][0]) ? ((S[2][2] < S[1][1]) ? 2 : 1) : ((S[2][2] < S[0][0]) ? 2 : 0);
#pragma unroll
  for (int k = 0; k < 3; ++k) v[k] = mi == 0 ? V[k][0] : (mi == 1 ? V[k][1] : V[k][2]);  // no runtime index
}

// one thread per (pair, sample): F as 9 doubles (NaN for degenerate samples)
__global__ void __launch_bounds__(128) k_ransac_F(const int32_t* __restrict__ pts, const int32_t* __restrict__ npts,
                                                  int nmax, const int32_t* __restrict__ idx,
                                                  const int32_t* __restrict__ idx_off, int iters,
                                                  double* __restrict__ Fout) {
  const int it = blockIdx.x * 128 + threadIdx.x;
  const int p = blockIdx.y;
  if (it >= iters) return;
  double* F = Fout + ((int64_t)p * iters + it) * 9;
  const int n = npts[p];
  if (n < 8) return;
  const int32_t* id = idx + (int64_t)idx_off[p] + (int64_t)it * 8;
  const int32_t* P = pts + (int64_t)p * nmax * 4;
  double x1[8], y1[8], x2[8], y2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int j = id[k];
    x1[k] = (double)P[4 * j + 0];
    y1[k] = (double)P[4 * j + 1];
    x2[k] = (double)P[4 * j + 2];
    y2[k] = (double)P[4 * j + 3];
  }
  double a1[8], b1[8], a2[8], b2[8], s1, c1x, c1y, s2, c2x, c2y;
  normalise8(x1, y1, a1, b1, s1, c1x, c1y);
  normalise8(x2, y2, a2, b2, s2, c2x, c2y);
  double A[8][9];
  auto build = [&]() {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const double u1 = a1[i], v1 = b1[i], u2 = a2[i], v2 = b2[i];
      A[i][0] = u1 * u2; A[i][1] = v1 * u2; A[i][2] = u2;
      A[i][3] = u1 * v2; A[i][4] = v1 * v2; A[i][5] = v2;
      A[i][6] = u1;      A[i][7] = v1;      A[i][8] = 1.0;
    }
  };
  build();
  double f[9];
  bool ok = null_vector_8x9_regs(A, f);
  if (!ok) {  // a zero pivot: the general elimination (free-column search) on a fresh system
    build();
    ok = null_vector_8x9(A, f);
  }
  if (!ok) {
#pragma unroll
    for (int k = 0; k < 9; ++k) F[k] = NAN;
    return;
  }
  // scale to unit norm (the SVD's vector), then rank 2: F - (F v3) v3^T
  double nn = 0.0;
#pragma unroll
  for (int k = 0; k < 9; ++k) nn += f[k] * f[k];
  nn = 1.0 / sqrt(nn);
#pragma unroll
  for (int k = 0; k < 9; ++k) f[k] *= nn;
  double S[3][3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) S[r][c] = f[0 + r] * f[0 + c] + f[3 + r] * f[3 + c] + f[6 + r] * f[6 + c];
  double v[3];
  smallest_eigvec3(S, v);
  double Fv[3];
  for (int r = 0; r < 3; ++r) Fv[r] = f[3 * r] * v[0] + f[3 * r + 1] * v[1] + f[3 * r + 2] * v[2];
  double F2[3][3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) F2[r][c] = f[3 * r + c] - Fv[r] * v[c];
  // un-normalise: T2^T F2 T1 (SFM.py:181-182), T = [[s,0,-s cx],[0,s,-s cy],[0,0,1]]
  const double T1[3][3] = {{s1, 0, -s1 * c1x}, {0, s1, -s1 * c1y}, {0, 0, 1}};
  const double T2[3][3] = {{s2, 0, -s2 * c2x}, {0, s2, -s2 * c2y}, {0, 0, 1}};
  double M[3][3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) M[r][c] = F2[r][0] * T1[0][c] + F2[r][1] * T1[1][c] + F2[r][2] * T1[2][c];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) F[3 * r + c] = T2[0][r] * M[0][c] + T2[1][r] * M[1][c] + T2[2][r] * M[2][c];
}

// d = |l . p2| / sqrt(l0^2 + l1^2) < thr (SFM.py:148-153).  Decided as num^2 vs thr^2 den2
// unless the two are within a relative 2^-40 of each other, where the reference's own
// expression decides: the squared comparison cannot flip a point farther than that from
// the threshold, and spares the float64 division and square root almost everywhere.
// lb = F p1 as fmas (numpy's F @ a_h goes through BLAS, whose order and fusing are its
// own; the bar is set by F's float64 rounding anyway).  thr2lo / thr2hi = thr^2 (1 -+ 2^-40).
SFM_DEV bool epi_inlier(const double* F, double x1, double y1, double x2, double y2, double thr, double thr2lo,
                        double thr2hi) {
  const double l0 = __builtin_fma(F[0], x1, __builtin_fma(F[1], y1, F[2]));
  const double l1 = __builtin_fma(F[3], x1, __builtin_fma(F[4], y1, F[5]));
  const double l2 = __builtin_fma(F[6], x1, __builtin_fma(F[7], y1, F[8]));
  const double num = fabs(__builtin_fma(l0, x2, __builtin_fma(l1, y2, l2)));
  const double den2 = __builtin_fma(l0, l0, l1 * l1);
  const double a = num * num;
  if (a < thr2lo * den2) return true;
  if (a > thr2hi * den2) return false;
  return num / sqrt(den2) < thr;  // near the threshold, or NaN (degenerate F) -> false
}

struct EpiThr {
  double thr, lo, hi;
};
SFM_DEV EpiThr epi_thr(double thr) {  // thr <= 0 (or NaN): nothing is an inlier (d >= 0)
  const double t2 = thr * thr;
  const bool on = thr > 0.0;
  return {thr, on ? t2 * (1.0 - 0x1p-40) : -1.0, on ? t2 * (1.0 + 0x1p-40) : -1.0};
}

// inlier count per (pair, sample): one thread per sample, its F in registers for the whole
// sweep; the pair's points are staged in LDS as float64 (x1, y1, x2, y2) in chunks of
// kRansacChunk points and every lane reads the same point (a broadcast) — no per-sample
// reduction, F reload or conversion.  Any n: larger sets take several chunks.
constexpr int kRansacChunk = 2560;
__global__ void __launch_bounds__(256) k_ransac_count(const int32_t* __restrict__ pts,
                                                      const int32_t* __restrict__ npts, int nmax,
                                                      const double* __restrict__ Fs, int iters, double thr,
                                                      int32_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) double s_pd[];  // [chunk][4]
  const int p = blockIdx.y;
  const int n = npts[p];
  const int4* P = reinterpret_cast<const int4*>(pts + (int64_t)p * nmax * 4);
  const int it = blockIdx.x * 256 + threadIdx.x;
  const bool live = it < iters;
  double f[9];
  if (live) {
    const double* F = Fs + ((int64_t)p * iters + it) * 9;
#pragma unroll
    for (int k = 0; k < 9; ++k) f[k] = F[k];
  }
  const EpiThr t = epi_thr(thr);
  uint32_t c = 0;
  for (int i0 = 0; i0 < n; i0 += kRansacChunk) {
    const int m = min(kRansacChunk, n - i0);
    if (i0) __syncthreads();  // every lane is done with the previous chunk
    for (int i = threadIdx.x; i < m; i += 256) {
      const int4 q = P[i0 + i];
      s_pd[4 * i + 0] = (double)q.x;
      s_pd[4 * i + 1] = (double)q.y;
      s_pd[4 * i + 2] = (double)q.z;
      s_pd[4 * i + 3] = (double)q.w;
    }
    __syncthreads();
    if (live)
      for (int i = 0; i < m; ++i) {
        const double4 q = reinterpret_cast<const double4*>(s_pd)[i];
        c += epi_inlier(f, q.x, q.y, q.z, q.w, t.thr, t.lo, t.hi) ? 1u : 0u;
      }
  }
  if (live) counts[(int64_t)p * iters + it] = n < 8 ? 0 : (int32_t)c;
}

// per pair: the first sample with the most inliers, its inliers compacted in order
__global__ void __launch_bounds__(256) k_ransac_select(const int32_t* __restrict__ pts,
                                                       const int32_t* __restrict__ npts, int nmax,
                                                       const double* __restrict__ Fs,
                                                       const int32_t* __restrict__ counts, int iters, double thr,
                                                       int32_t* __restrict__ out_pts, int32_t* __restrict__ out_n,
                                                       int32_t* __restrict__ out_iter) {
  __shared__ int s_bc[256], s_bi[256];
  __shared__ uint32_t s_scan[8];
  const int p = blockIdx.x, tid = threadIdx.x;
  const int n = npts[p];
  int bc = -1, bi = 0x7fffffff;
  for (int it = tid; it < iters; it += 256) {
    const int c = counts[(int64_t)p * iters + it];
    if (c > bc) { bc = c; bi = it; }  // ascending it per thread: first max kept
  }
  s_bc[tid] = bc;
  s_bi[tid] = bi;
  __syncthreads();
  for (int off = 128; off >= 1; off >>= 1) {
    if (tid < off) {
      const int oc = s_bc[tid + off], oi = s_bi[tid + off];
      if (oc > s_bc[tid] || (oc == s_bc[tid] && oi < s_bi[tid])) { s_bc[tid] = oc; s_bi[tid] = oi; }
    }
    __syncthreads();
  }
  const int best = s_bi[0];
  if (n < 8 || s_bc[0] <= 0) {  // (< 8 points: the reference returns None; 0 inliers: empty)
    if (tid == 0) { out_n[p] = n < 8 ? -1 : 0; out_iter[p] = -1; }
    return;
  }
  const double* F = Fs + ((int64_t)p * iters + best) * 9;
  const int4* P = reinterpret_cast<const int4*>(pts + (int64_t)p * nmax * 4);
  int4* O = reinterpret_cast<int4*>(out_pts + (int64_t)p * nmax * 4);
  const EpiThr t = epi_thr(thr);  // the same test as k_ransac_count, so the mask has the count
  uint32_t base = 0;
  for (int i0 = 0; i0 < n; i0 += 256) {
    const int i = i0 + tid;
    bool in = false;
    int4 q = make_int4(0, 0, 0, 0);
    if (i < n) {
      q = P[i];
      in = epi_inlier(F, (double)q.x, (double)q.y, (double)q.z, (double)q.w, t.thr, t.lo, t.hi);
    }
    uint32_t total;
    const uint32_t pos = block_exclusive_scan(in ? 1u : 0u, s_scan, &total);
    if (in) O[base + pos] = q;
    base += total;
  }
  if (tid == 0) { out_n[p] = (int32_t)base; out_iter[p] = best; }
}

void launch_ransac(const int32_t* pts, const int32_t* npts, int nmax, int P, const int32_t* idx,
                   const int32_t* idx_off, int iters, double thr, double* Fs, int32_t* counts, int32_t* out_pts,
                   int32_t* out_n, int32_t* out_iter, hipStream_t st) {
  if (iters > 0) {
    hipLaunchKernelGGL(k_ransac_F, dim3((iters + 127) / 128, P), dim3(128), 0, st, pts, npts, nmax, idx, idx_off,
                       iters, Fs);
    static const bool lds_attr = [] {  // up to kRansacChunk x 32 B of staged points
      return hipFuncSetAttribute((const void*)k_ransac_count, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 kRansacChunk * 32) == hipSuccess;
    }();
    (void)lds_attr;
    hipLaunchKernelGGL(k_ransac_count, dim3((iters + 255) / 256, P), dim3(256),
                       (size_t)std::min(nmax, kRansacChunk) * 32, st, pts, npts, nmax, Fs, iters, thr, counts);
  }
  // always: with iters == 0 no sample exists and every pair gets the reference's empty
  // result (n >= 8) or None (n < 8), out_iter -1
  hipLaunchKernelGGL(k_ransac_select, dim3(P), dim3(256), 0, st, pts, npts, nmax, Fs, counts, iters, thr, out_pts,
                     out_n, out_iter);
}

}  // namespace sfm
