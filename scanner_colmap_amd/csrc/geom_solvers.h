// fp64 two-view-geometry primitives shared by the HIP verification kernels
// (device), the product's host-side RANSAC replay, and the CPU oracle.
//
// These restate the estimator arithmetic that the reference op reaches through
// colmap::TwoViewGeometry::Estimate (integration/op_cpp/sequential_matching.cc:98-99)
// [upstream COLMAP 3.4/3.5, un-vendored: estimators/fundamental_matrix.cc,
// estimators/homography_matrix.cc, estimators/translation_transform.h,
// estimators/utils.cc, util/math.h].  Every function is written so that the
// SAME source evaluated by gcc (x86-64 SSE2, -ffp-contract=off) and by hipcc
// (gfx950, -ffp-contract=off) performs the same sequence of correctly rounded
// IEEE-754 binary64 operations: only + - * / sqrt fabs and comparisons, fixed
// loop orders, no libm transcendental.  That makes a hypothesis solved on the
// GPU bit-identical to the one the oracle solves on the CPU, so RANSAC
// trajectories (inlier counts, model selection, dynamic trial counts) can be
// compared exactly.  (gfx950 f64 div/sqrt were verified correctly rounded on
// 2^20 random operands: probes/probe_mfma.hip.)
//
// Documented deviations from Eigen-based COLMAP (parity at the COLMAP boundary
// is unpinned — no COLMAP build exists in this environment):
//  * minimal-sample null spaces (7-pt F, 4-pt H) come from a Householder QR of
//    A^T instead of Eigen::JacobiSVD (same subspace, orthonormal basis);
//  * least-squares null vectors (8-pt F, N-pt H local optimisation) come from
//    a cyclic Jacobi eigen-decomposition of A^T A on Hartley-normalised
//    coordinates instead of JacobiSVD of A;
//  * real roots of the 7-pt cubic come from a bracketed Newton/bisection
//    solver, returned in ascending order, instead of companion-matrix
//    eigenvalues (Eigen::EigenSolver order);
//  * sums over a variable number of points inside the estimators (centroid,
//    RMS distance, A^T A, translation mean) use the CANONICAL order defined
//    below (64 lane-strided partial sums, then a fixed binary tree), so a
//    64-lane wavefront reproduces them exactly;
//  * RANSAC::ComputeNumTrials evaluates pow/log with basic operations
//    (num_trials() below) instead of libm, so host and device agree; the
//    power is rounded once (as std::pow), and the counts equal the libm
//    formula's on every (inliers <= samples <= 16384) checked exhaustively
//    (tests/test_num_trials.py).
#pragma once

#if defined(__HIPCC__)
#define SCM_HD __host__ __device__
#define SCM_UNROLL _Pragma("unroll")
#else
#define SCM_HD
#define SCM_UNROLL
#endif

#include <math.h>
#include <stdint.h>

namespace scm {
namespace geom {

// ---------------------------------------------------------------------------
// Canonical reduction order: item i goes to partial (i mod 64), each partial
// accumulates its items in ascending order starting from -0.0 (the additive
// identity: -0.0 + x == x for every x, so an empty partial changes nothing),
// then the partials are combined as p[l] += p[l + w] for w = 32, 16, ..., 1.
// A 64-lane wavefront evaluates exactly the same additions (one partial per
// lane, the tree as shuffle-downs with the same pairing).
// ---------------------------------------------------------------------------
constexpr int kCanon = 64;
constexpr double kCanonZero = -0.0;

SCM_HD inline double canon_tree(double* p) {
  for (int w = kCanon / 2; w >= 1; w >>= 1)
    for (int l = 0; l < w; ++l) p[l] = p[l] + p[l + w];
  return p[0];
}

// ---------------------------------------------------------------------------
// Deterministic natural log (basic operations only): x = m * 2^e with
// m in [sqrt(1/2), sqrt(2)), log(m) = 2 atanh(s), s = (m - 1) / (m + 1).
// Accurate to ~1 ulp for normal positive x; log(0) = -inf; x < 0 -> NaN.
// ---------------------------------------------------------------------------
SCM_HD inline double det_log(double x) {
  if (!(x > 0.0)) return x == 0.0 ? -1.0 / 0.0 : 0.0 / 0.0;
  if (x == 1.0 / 0.0) return x;
  uint64_t u;
  __builtin_memcpy(&u, &x, 8);
  int e = (int)((u >> 52) & 0x7FF);
  if (e == 0) {  // subnormal: scale up by 2^54
    x = x * 18014398509481984.0;
    __builtin_memcpy(&u, &x, 8);
    e = (int)((u >> 52) & 0x7FF) - 54;
  }
  e -= 1023;
  u = (u & 0x800FFFFFFFFFFFFFull) | (0x3FFull << 52);  // m in [1, 2)
  double m;
  __builtin_memcpy(&m, &u, 8);
  if (m > 1.4142135623730951) {
    m = m * 0.5;
    e += 1;
  }
  const double s = (m - 1.0) / (m + 1.0);
  const double s2 = s * s;
  // 2 * (s + s^3/3 + ... + s^27/27); |s| <= 0.1716 -> truncation < 1e-21.
  double t = 1.0 / 27.0;
  for (int k = 25; k >= 1; k -= 2) t = t * s2 + 1.0 / (double)k;
  const double logm = 2.0 * s * t;
  const double ln2_hi = 6.93147180369123816490e-01;  // fdlibm split of ln 2
  const double ln2_lo = 1.90821492927058770002e-10;
  return ((double)e * ln2_lo + logm) + (double)e * ln2_hi;
}

// ratio^k rounded once: the power in double-double (Dekker products, exact
// for the normal doubles ratio^k reaches here), so the result is the
// correctly rounded value that std::pow returns (glibc's pow is correctly
// rounded outside hard cases).  Repeated double multiplication is not: one ulp
// of ratio^k moves 1 - ratio^k across a rounding boundary and, for small
// ratios, the trial count by more than one (tests/num_trials_check.cc).
SCM_HD inline void two_prod(double a, double b, double* p, double* e) {
  *p = a * b;
  const double c = 134217729.0;  // 2^27 + 1 (Dekker split)
  double t = c * a;
  const double ah = t - (t - a), al = a - ah;
  t = c * b;
  const double bh = t - (t - b), bl = b - bh;
  *e = ((ah * bh - *p) + ah * bl + al * bh) + al * bl;
}

SCM_HD inline double pow_int_rounded(double x, int k) {
  if (k <= 1) return k == 1 ? x : 1.0;
  double h = x, l = 0.0;
  for (int i = 1; i < k; ++i) {
    double p, e;
    two_prod(h, x, &p, &e);
    e = e + l * x;
    h = p + e;  // quick two-sum: |e| <= ulp(p)
    l = e - (h - p);
  }
  return h;
}

// colmap::RANSAC::ComputeNumTrials [upstream optim/ransac.h] with
// pow(ratio, kmin) by pow_int_rounded and log by det_log.  The final
// static_cast<size_t> mirrors gcc/x86-64 for out-of-range values
// (-inf -> 2^63, >= 2^64 -> 0).  Equal to the libm formula on every
// (inliers <= samples <= 16384) at kmin 1/4/7/8 and several confidences and
// multipliers (tests/test_num_trials.py).
SCM_HD inline uint64_t num_trials(uint64_t num_inliers, uint64_t num_samples,
                                  double confidence, double multiplier, int kmin) {
  const double inlier_ratio = (double)num_inliers / (double)num_samples;
  const double nom = 1.0 - confidence;
  if (nom <= 0.0) return ~0ull;
  const double denom = 1.0 - pow_int_rounded(inlier_ratio, kmin);
  if (denom <= 0.0) return 1;
  const double q = det_log(nom) / det_log(denom) * multiplier;
  // ceil without libm: integers >= 2^52 are already integral.
  double v = q;
  if (q == q && q < 4503599627370496.0 && q > -4503599627370496.0) {
    const double tq = (double)(int64_t)q;  // truncation toward zero
    v = (tq < q) ? tq + 1.0 : tq;
  }
  if (!(v >= 0.0)) return 1ull << 63;
  if (v >= 18446744073709551616.0) return 0;
  if (v >= 9223372036854775808.0)
    return ((uint64_t)(v - 9223372036854775808.0)) ^ (1ull << 63);
  return (uint64_t)v;
}

// Per-pair RANSAC PRNG seed (include/scm.h scm_pair_seed): the reference's
// PRNG is thread-local and time-seeded; here each pair gets a fresh
// std::mt19937 seeded with this hash of (base seed, image_id1, image_id2).
SCM_HD inline uint32_t pair_seed(uint32_t base, uint32_t id1, uint32_t id2) {
  uint32_t h = base ^ 0x9E3779B9u;
  h ^= id1 + 0x7F4A7C15u + (h << 6) + (h >> 2);
  h ^= id2 + 0x85EBCA77u + (h << 6) + (h >> 2);
  return h;
}

// Base seed of the k-th Estimate of TwoViewGeometry::EstimateMultiple
// (multiple_models; k = 0 is the plain Estimate's): the reference continues
// its one time-seeded generator from Estimate to Estimate, so any fresh
// per-iteration seeding is an equally valid realisation of it.
SCM_HD inline uint32_t iteration_seed(uint32_t base, uint32_t k) { return base ^ (k * 0x9E3779B1u); }

// Seed of the pair's second stream: the homography LO-RANSAC (and the
// watermark RANSAC after it) draw from std::mt19937(pair_seed_h(...)), so
// that the F and H estimations are independent and run concurrently.  (In
// the reference both continue one thread-local, time-seeded generator; any
// seeding is an equally valid realisation of it.)
SCM_HD inline uint32_t pair_seed_h(uint32_t base, uint32_t id1, uint32_t id2) {
  return pair_seed(base ^ 0x6A09E667u, id1, id2);
}

// ---------------------------------------------------------------------------
// Residuals.  Term order follows the reference formulas exactly.
// ---------------------------------------------------------------------------

// colmap::ComputeSquaredSampsonError [upstream estimators/utils.cc]; F row-major.
SCM_HD inline double sampson_sq(const double* F, double x1_0, double x1_1,
                                double x2_0, double x2_1) {
  const double Fx1_0 = F[0] * x1_0 + F[1] * x1_1 + F[2];
  const double Fx1_1 = F[3] * x1_0 + F[4] * x1_1 + F[5];
  const double Fx1_2 = F[6] * x1_0 + F[7] * x1_1 + F[8];
  const double Ftx2_0 = F[0] * x2_0 + F[3] * x2_1 + F[6];
  const double Ftx2_1 = F[1] * x2_0 + F[4] * x2_1 + F[7];
  const double x2tFx1 = x2_0 * Fx1_0 + x2_1 * Fx1_1 + Fx1_2;
  return x2tFx1 * x2tFx1 /
         (Fx1_0 * Fx1_0 + Fx1_1 * Fx1_1 + Ftx2_0 * Ftx2_0 + Ftx2_1 * Ftx2_1);
}

// colmap::HomographyMatrixEstimator::Residuals [upstream]; H row-major.
SCM_HD inline double homography_sq(const double* H, double s_0, double s_1,
                                   double d_0, double d_1) {
  const double pd_0 = H[0] * s_0 + H[1] * s_1 + H[2];
  const double pd_1 = H[3] * s_0 + H[4] * s_1 + H[5];
  const double pd_2 = H[6] * s_0 + H[7] * s_1 + H[8];
  const double inv_pd_2 = 1.0 / pd_2;
  const double dd_0 = d_0 - pd_0 * inv_pd_2;
  const double dd_1 = d_1 - pd_1 * inv_pd_2;
  return dd_0 * dd_0 + dd_1 * dd_1;
}

// colmap::TranslationTransformEstimator<2>::Residuals [upstream].
SCM_HD inline double translation_sq(const double* t, double x1_0, double x1_1,
                                    double x2_0, double x2_1) {
  const double d0 = x2_0 - x1_0 - t[0];
  const double d1 = x2_1 - x1_1 - t[1];
  return d0 * d0 + d1 * d1;
}

// ---------------------------------------------------------------------------
// Small dense linear algebra.
// ---------------------------------------------------------------------------

// C = A * B for row-major 3x3, k summed in ascending order.
SCM_HD inline void mat3_mul(const double* A, const double* B, double* C) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      C[3 * i + j] = A[3 * i + 0] * B[0 + j] + A[3 * i + 1] * B[3 + j] +
                     A[3 * i + 2] * B[6 + j];
}

// colmap::CenterAndNormalizeImagePoints [upstream estimators/utils.cc]:
// centroid, RMS distance to it, scale sqrt(2)/rms; sums in canonical order.
// xy interleaved (x0,y0,...).  Writes T (row-major 3x3).
SCM_HD inline void normalize_transform(const double* xy, int n, double* T) {
  double p0[kCanon], p1[kCanon];
  for (int l = 0; l < kCanon; ++l) { p0[l] = kCanonZero; p1[l] = kCanonZero; }
  for (int i = 0; i < n; ++i) {
    p0[i & (kCanon - 1)] += xy[2 * i];
    p1[i & (kCanon - 1)] += xy[2 * i + 1];
  }
  const double c0 = canon_tree(p0) / (double)n;
  const double c1 = canon_tree(p1) / (double)n;
  for (int l = 0; l < kCanon; ++l) p0[l] = kCanonZero;
  for (int i = 0; i < n; ++i) {
    const double d0 = xy[2 * i] - c0;
    const double d1 = xy[2 * i + 1] - c1;
    p0[i & (kCanon - 1)] += d0 * d0 + d1 * d1;
  }
  const double rms = sqrt(canon_tree(p0) / (double)n);
  const double s = sqrt(2.0) / rms;
  T[0] = s;   T[1] = 0.0; T[2] = -s * c0;
  T[3] = 0.0; T[4] = s;   T[5] = -s * c1;
  T[6] = 0.0; T[7] = 0.0; T[8] = 1.0;
}

// Apply a normalisation transform to one point (homogeneous divide kept, as
// in the reference).
SCM_HD inline void apply_normalize(const double* T, double p0, double p1, double* o0,
                                   double* o1) {
  const double np0 = T[0] * p0 + T[1] * p1 + T[2];
  const double np1 = T[3] * p0 + T[4] * p1 + T[5];
  const double np2 = T[6] * p0 + T[7] * p1 + T[8];
  const double inv = 1.0 / np2;
  *o0 = np0 * inv;
  *o1 = np1 * inv;
}

// Rows of the linear systems (reference row layouts).
SCM_HD inline void f_row(double x0, double y0, double x1, double y1, double* a) {
  a[0] = x1 * x0; a[1] = x1 * y0; a[2] = x1;
  a[3] = y1 * x0; a[4] = y1 * y0; a[5] = y1;
  a[6] = x0;      a[7] = y0;      a[8] = 1.0;
}
SCM_HD inline void h_rows(double s0, double s1, double d0, double d1, double* a, double* b) {
  a[0] = -s0; a[1] = -s1; a[2] = -1.0; a[3] = 0.0; a[4] = 0.0; a[5] = 0.0;
  a[6] = s0 * d0; a[7] = s1 * d0; a[8] = d0;
  b[0] = 0.0; b[1] = 0.0; b[2] = 0.0; b[3] = -s0; b[4] = -s1; b[5] = -1.0;
  b[6] = s0 * d1; b[7] = s1 * d1; b[8] = d1;
}

// Upper-triangle index of (p, q), p <= q, in a packed 45-entry A^T A.
SCM_HD inline int ata_index(int p, int q) { return p * 9 - (p * (p - 1)) / 2 + (q - p); }

// Contribution of one constraint row to the packed A^T A partial.
SCM_HD inline void ata_accumulate(double* part45, const double* a) {
  int k = 0;
  for (int p = 0; p < 9; ++p)
    for (int q = p; q < 9; ++q) part45[k++] += a[p] * a[q];
}

// Orthonormal basis of the null space of a full-row-rank M x 9 matrix A
// (row-major, M <= 8) from a Householder QR of A^T: the last 9-M columns of Q.
// Reflector k is stored in place in column k of W = A^T.  ns receives (9-M)
// vectors of 9 entries each, ns[j*9 + r].  Fixed trip counts: the loops
// unroll completely, so on the GPU everything stays in registers.
template <int M>
SCM_HD inline void householder_nullspace(const double* A, double* ns) {
  double W[9][M];
  double vn2[M];
SCM_UNROLL
  for (int r = 0; r < 9; ++r)
SCM_UNROLL
    for (int c = 0; c < M; ++c) W[r][c] = A[c * 9 + r];
SCM_UNROLL
  for (int k = 0; k < M; ++k) {
    double nrm2 = 0.0;
SCM_UNROLL
    for (int r = k; r < 9; ++r) nrm2 += W[r][k] * W[r][k];
    const double nrm = sqrt(nrm2);
    vn2[k] = 0.0;
    if (nrm == 0.0) continue;
    const double x0 = W[k][k];
    const double alpha = x0 > 0.0 ? -nrm : nrm;
    W[k][k] = x0 - alpha;  // v = (x0 - alpha, x1, ..., x_{8-k})
    double v2 = 0.0;
SCM_UNROLL
    for (int r = k; r < 9; ++r) v2 += W[r][k] * W[r][k];
    vn2[k] = v2;
    if (v2 == 0.0) continue;
SCM_UNROLL
    for (int c = k + 1; c < M; ++c) {
      double dot = 0.0;
SCM_UNROLL
      for (int r = k; r < 9; ++r) dot += W[r][k] * W[r][c];
      const double f = 2.0 * dot / v2;
SCM_UNROLL
      for (int r = k; r < 9; ++r) W[r][c] = W[r][c] - f * W[r][k];
    }
  }
SCM_UNROLL
  for (int j = M; j < 9; ++j) {
    double q[9];
SCM_UNROLL
    for (int r = 0; r < 9; ++r) q[r] = (r == j) ? 1.0 : 0.0;
SCM_UNROLL
    for (int k = M - 1; k >= 0; --k) {
      if (vn2[k] == 0.0) continue;
      double dot = 0.0;
SCM_UNROLL
      for (int r = k; r < 9; ++r) dot += W[r][k] * q[r];
      const double f = 2.0 * dot / vn2[k];
SCM_UNROLL
      for (int r = k; r < 9; ++r) q[r] = q[r] - f * W[r][k];
    }
SCM_UNROLL
    for (int r = 0; r < 9; ++r) ns[(j - M) * 9 + r] = q[r];
  }
}

// Cyclic Jacobi eigen-decomposition of a symmetric N x N matrix (row-major).
// On return the diagonal of a holds the eigenvalues and column j of v
// (row-major, v[r*N+j]) the j-th eigenvector.  Returns the index of the
// smallest eigenvalue (lowest index on ties).  Used for the 3 x 3 rank-2
// projection of the 8-point estimator (host and device run this same code).
constexpr int kJacobiMaxSweeps = 64;

SCM_HD inline void jacobi_params(double app, double aqq, double apq, double* c, double* s) {
  const double theta = (aqq - app) / (2.0 * apq);
  double t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
  if (theta < 0.0) t = -t;
  *c = 1.0 / sqrt(t * t + 1.0);
  *s = t * *c;
}

template <int N>
SCM_HD inline int jacobi_eigen_min(double* a, double* v) {
SCM_UNROLL
  for (int r = 0; r < N; ++r)
SCM_UNROLL
    for (int c = 0; c < N; ++c) v[r * N + c] = (r == c) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < kJacobiMaxSweeps; ++sweep) {
    double off = 0.0, diag = 0.0;
SCM_UNROLL
    for (int p = 0; p < N; ++p) {
      diag += a[p * N + p] * a[p * N + p];
SCM_UNROLL
      for (int q = p + 1; q < N; ++q) off += a[p * N + q] * a[p * N + q];
    }
    if (off <= 1e-36 * diag || off == 0.0) break;
SCM_UNROLL
    for (int p = 0; p < N - 1; ++p) {
SCM_UNROLL
      for (int q = p + 1; q < N; ++q) {
        const double apq = a[p * N + q];
        if (apq == 0.0) continue;
        double c, s;
        jacobi_params(a[p * N + p], a[q * N + q], apq, &c, &s);
SCM_UNROLL
        for (int k = 0; k < N; ++k) {
          const double akp = a[k * N + p], akq = a[k * N + q];
          a[k * N + p] = c * akp - s * akq;
          a[k * N + q] = s * akp + c * akq;
        }
SCM_UNROLL
        for (int k = 0; k < N; ++k) {
          const double apk = a[p * N + k], aqk = a[q * N + k];
          a[p * N + k] = c * apk - s * aqk;
          a[q * N + k] = s * apk + c * aqk;
        }
        a[p * N + q] = 0.0;
        a[q * N + p] = 0.0;
SCM_UNROLL
        for (int k = 0; k < N; ++k) {
          const double vkp = v[k * N + p], vkq = v[k * N + q];
          v[k * N + p] = c * vkp - s * vkq;
          v[k * N + q] = s * vkp + c * vkq;
        }
      }
    }
  }
  int best = 0;
  double bv = a[0];
SCM_UNROLL
  for (int j = 1; j < N; ++j)
    if (a[j * N + j] < bv) {
      bv = a[j * N + j];
      best = j;
    }
  return best;
}

// ---------------------------------------------------------------------------
// Polynomial roots (colmap::FindPolynomialRootsCompanionMatrix degree logic
// [upstream util/polynomial.cc]; cubic solved by bracketed Newton).
// ---------------------------------------------------------------------------

SCM_HD inline double cubic_eval(double B, double C, double D, double x) {
  return ((x + B) * x + C) * x + D;
}

// Real root of the monic cubic in (lo, hi) where p(lo), p(hi) differ in sign.
SCM_HD inline double cubic_refine(double B, double C, double D, double lo,
                                  double hi, double plo) {
  double x = 0.5 * (lo + hi);
  for (int it = 0; it < 200; ++it) {
    const double px = cubic_eval(B, C, D, x);
    if (px == 0.0) return x;
    if ((px < 0.0) == (plo < 0.0)) {
      lo = x;
      plo = px;
    } else {
      hi = x;
    }
    const double dpx = (3.0 * x + 2.0 * B) * x + C;
    double xn = (dpx != 0.0) ? x - px / dpx : lo;
    if (!(xn > lo && xn < hi)) xn = 0.5 * (lo + hi);
    if (xn == x || xn == lo || xn == hi) {
      // No representable progress left: bracket has collapsed.
      const double m = 0.5 * (lo + hi);
      if (m == lo || m == hi) return fabs(cubic_eval(B, C, D, lo)) <=
                                             fabs(cubic_eval(B, C, D, hi))
                                         ? lo
                                         : hi;
      xn = m;
    }
    x = xn;
  }
  return x;
}

// Real roots, ascending, of c[0] x^3 + c[1] x^2 + c[2] x + c[3].  Returns the
// number of roots written to r (<= 3); 0 when the polynomial is degenerate.
// Complex roots are kept only in the quadratic branch, where COLMAP keeps a
// pair whose imaginary part is <= 1e-10 (FindQuadraticPolynomialRoots).
SCM_HD inline int poly3_real_roots(const double* c, double* r) {
  int lead = 0;
  while (lead < 4 && c[lead] == 0.0) ++lead;  // RemoveLeadingZeros
  const int degree = 3 - lead;
  if (degree <= 0) return 0;
  if (degree == 1) {
    r[0] = -c[3] / c[2];
    return 1;
  }
  if (degree == 2) {
    const double a = c[1], b = c[2], cc = c[3];
    if (b == 0.0 && cc == 0.0) {
      r[0] = 0.0;
      return 1;
    }
    const double d = b * b - 4.0 * a * cc;
    if (d >= 0.0) {
      const double sd = sqrt(d);
      double r0, r1;
      if (b >= 0.0) {
        r0 = (-b - sd) / (2.0 * a);
        r1 = (2.0 * cc) / (-b - sd);
      } else {
        r0 = (2.0 * cc) / (-b + sd);
        r1 = (-b + sd) / (2.0 * a);
      }
      if (r1 < r0) { const double t = r0; r0 = r1; r1 = t; }
      r[0] = r0;
      r[1] = r1;
      return 2;
    }
    const double im = sqrt(-d) / (2.0 * a);
    if (fabs(im) <= 1e-10) {
      r[0] = -b / (2.0 * a);
      r[1] = r[0];
      return 2;
    }
    return 0;
  }
  // Cubic: monic form x^3 + B x^2 + C x + D.
  const double B = c[1] / c[0], C = c[2] / c[0], D = c[3] / c[0];
  double R = fabs(B);
  if (fabs(C) > R) R = fabs(C);
  if (fabs(D) > R) R = fabs(D);
  R = 1.0 + R;  // Cauchy bound: every root has |x| < R.
  // Bracket points -R <= e0 <= e1 <= R; e0 / e1 are the critical points of p
  // (3x^2 + 2Bx + C = 0, stable quadratic formula) when they exist inside
  // (-R, R), otherwise duplicates of the neighbouring point (an empty
  // interval, skipped).
  double e0 = -R, e1 = -R;
  const double disc = B * B - 3.0 * C;
  if (disc > 0.0) {
    const double sd = sqrt(disc);
    const double q = (B >= 0.0) ? -(B + sd) : -(B - sd);
    double c0 = q / 3.0, c1 = C / q;
    if (c1 < c0) { const double t = c0; c0 = c1; c1 = t; }
    if (c0 > -R && c0 < R) e0 = c0;
    e1 = e0;
    if (c1 > -R && c1 < R && c1 > e0) e1 = c1;
  }
  const double pts[4] = {-R, e0, e1, R};
  int nr = 0;
  double r0 = 0.0, r1 = 0.0, r2 = 0.0;
  double plo = cubic_eval(B, C, D, pts[0]);
  SCM_UNROLL
  for (int k = 0; k < 3; ++k) {
    const double lo = pts[k], hi = pts[k + 1];
    if (!(lo < hi)) continue;  // empty interval (plo unchanged: p(hi) == p(lo))
    const double phi = cubic_eval(B, C, D, hi);
    double x = 0.0;
    bool found = false;
    if (plo == 0.0) {
      const double last = nr == 1 ? r0 : (nr == 2 ? r1 : r2);
      if (nr == 0 || last != lo) { x = lo; found = true; }
    } else if (phi != 0.0 && ((plo < 0.0) != (phi < 0.0))) {
      x = cubic_refine(B, C, D, lo, hi, plo);
      found = true;
    }
    if (found && nr < 3) {
      if (nr == 0) r0 = x; else if (nr == 1) r1 = x; else r2 = x;
      ++nr;
    }
    if (phi == 0.0 && k == 2 && nr < 3) {
      if (nr == 0) r0 = hi; else if (nr == 1) r1 = hi; else r2 = hi;
      ++nr;
    }
    plo = phi;
  }
  r[0] = r0;
  r[1] = r1;
  r[2] = r2;
  return nr;
}

// ---------------------------------------------------------------------------
// Estimators.
// ---------------------------------------------------------------------------

// colmap::FundamentalMatrixSevenPointEstimator::Estimate [upstream
// estimators/fundamental_matrix.cc].  x1, x2: 7 interleaved (x, y) points of
// image 1 / image 2 in pixels (no normalisation, as in COLMAP).  Writes up to
// three row-major F (F(2,2) == 1) to models; returns their count.
SCM_HD inline int fundamental_7pt(const double* x1, const double* x2,
                                  double* models) {
  double A[7 * 9];
  for (int i = 0; i < 7; ++i) {
    const double x0 = x1[2 * i], y0 = x1[2 * i + 1];
    const double xx1 = x2[2 * i], yy1 = x2[2 * i + 1];
    double* a = A + 9 * i;
    a[0] = xx1 * x0; a[1] = xx1 * y0; a[2] = xx1;
    a[3] = yy1 * x0; a[4] = yy1 * y0; a[5] = yy1;
    a[6] = x0;       a[7] = y0;       a[8] = 1.0;
  }
  double ns[2 * 9];
  householder_nullspace<7>(A, ns);
  double f1[9], f2[9];
  for (int i = 0; i < 9; ++i) {
    f2[i] = ns[9 + i];
    f1[i] = ns[i] - f2[i];  // f1 -= f2
  }
  // det(lambda * f1 + f2) as a cubic in lambda (COLMAP's closed form).
  const double t0 = f1[4] * f1[8] - f1[5] * f1[7];
  const double t1 = f1[3] * f1[8] - f1[5] * f1[6];
  const double t2 = f1[3] * f1[7] - f1[4] * f1[6];
  const double t3 = f2[4] * f2[8] - f2[5] * f2[7];
  const double t4 = f2[3] * f2[8] - f2[5] * f2[6];
  const double t5 = f2[3] * f2[7] - f2[4] * f2[6];
  double coeffs[4];
  coeffs[0] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2;
  coeffs[1] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2 -
              f2[3] * (f1[1] * f1[8] - f1[2] * f1[7]) +
              f2[4] * (f1[0] * f1[8] - f1[2] * f1[6]) -
              f2[5] * (f1[0] * f1[7] - f1[1] * f1[6]) +
              f2[6] * (f1[1] * f1[5] - f1[2] * f1[4]) -
              f2[7] * (f1[0] * f1[5] - f1[2] * f1[3]) +
              f2[8] * (f1[0] * f1[4] - f1[1] * f1[3]);
  coeffs[2] = f1[0] * t3 - f1[1] * t4 + f1[2] * t5 -
              f1[3] * (f2[1] * f2[8] - f2[2] * f2[7]) +
              f1[4] * (f2[0] * f2[8] - f2[2] * f2[6]) -
              f1[5] * (f2[0] * f2[7] - f2[1] * f2[6]) +
              f1[6] * (f2[1] * f2[5] - f2[2] * f2[4]) -
              f1[7] * (f2[0] * f2[5] - f2[2] * f2[3]) +
              f1[8] * (f2[0] * f2[4] - f2[1] * f2[3]);
  coeffs[3] = f2[0] * t3 - f2[1] * t4 + f2[2] * t5;
  double roots[3];
  const int nroots = poly3_real_roots(coeffs, roots);
  // Models in root order, skipping |F(2,2)| < 1e-10; written with static
  // indices (register-resident on the GPU).
  double out[3][9];
  int nm = 0;
  SCM_UNROLL
  for (int k = 0; k < 3; ++k) {
    if (k >= nroots) continue;
    const double lambda = roots[k];
    double F[9];
    // Eigen: lambda * f1 + mu * f2 with mu = 1, reshaped column-major 3x3 and
    // transposed on return => row-major F[r][c] = f[3r + c].
    SCM_UNROLL
    for (int i = 0; i < 9; ++i) F[i] = lambda * f1[i] + 1.0 * f2[i];
    if (fabs(F[8]) < 1e-10) continue;
    const double s = F[8];
    SCM_UNROLL
    for (int i = 0; i < 9; ++i) {
      const double v = F[i] / s;
      if (nm == 0) out[0][i] = v;
      else if (nm == 1) out[1][i] = v;
      else out[2][i] = v;
    }
    ++nm;
  }
  SCM_UNROLL
  for (int k = 0; k < 3; ++k)
    SCM_UNROLL
    for (int i = 0; i < 9; ++i) models[9 * k + i] = k < nm ? out[k][i] : 0.0;
  return nm;
}

// Least-squares null vector of the 9 x 9 normal equations of the local
// estimators (the right singular vector of the smallest singular value that
// the reference's Eigen JacobiSVD returns), by
// repeated squaring of the inverse:
//   M0 = (A + delta I)^-1, delta = 2^-40 trace(A)   (Gauss-Jordan, no pivoting:
//        A + delta I is SPD, its pivots stay >= delta), symmetrised;
//   M_{s+1} = M_s M_s / trace(M_s M_s)               (entry (i, j) summed over
//        k = 0..8 in order: bitwise symmetric);
// M_s -> v v^T at rate ((l1 + delta) / (l2 + delta))^(2^s).  Squaring stops
// one step after the column j* of the largest diagonal passes the rank-one
// test |1 - sum_i M_ij*^2 / M_j*j*| <= 2^-44 (at least 4, at most 16
// squarings); v = column j* / its norm.  Every entry's arithmetic is fixed by
// this definition, so the GPU's lane-per-entry version (verify_kernels.hip,
// invsq9_null_wave) agrees bit for bit.  Accuracy is the eigenproblem's own
// (tests/test_oracle_geometry.py pins it against LAPACK); a zero matrix
// returns e_0.
constexpr int kInvSqMin = 4, kInvSqMax = 16;
constexpr double kInvSqTol = 0x1p-44;

// One Gauss-Jordan step on pivot k: entry (i, j) of the new matrix from the
// old one (every entry reads only row k, column k and itself).
SCM_HD inline double gj9_entry(double mij, double mik, double mkj, double inv, int i, int j, int k) {
  if (i == k && j == k) return inv;
  if (i == k) return mkj * inv;
  if (j == k) return -(mik * inv);
  return mij - mik * (mkj * inv);
}

SCM_HD inline double sq9_entry(const double* m, int i, int j) {
  double acc = m[i * 9 + 0] * m[0 * 9 + j];
SCM_UNROLL
  for (int k = 1; k < 9; ++k) acc = acc + m[i * 9 + k] * m[k * 9 + j];
  return acc;
}

// Trace-normalisation factor, column of the largest diagonal (lowest index on
// ties) and the rank-one test of a squared iterate.
SCM_HD inline double sq9_trace_inv(const double* m) {
  double t = m[0];
SCM_UNROLL
  for (int i = 1; i < 9; ++i) t = t + m[i * 9 + i];
  return 1.0 / t;
}

SCM_HD inline int sq9_argmax_diag(const double* m) {
  int j = 0;
  double d = m[0];
SCM_UNROLL
  for (int i = 1; i < 9; ++i)
    if (m[i * 9 + i] > d) {
      d = m[i * 9 + i];
      j = i;
    }
  return j;
}

SCM_HD inline bool sq9_rank_one(const double* m, int j) {
  double c = m[j] * m[j];
SCM_UNROLL
  for (int i = 1; i < 9; ++i) c = c + m[i * 9 + j] * m[i * 9 + j];
  const double r = c / m[j * 9 + j];
  return fabs(1.0 - r) <= kInvSqTol;
}

SCM_HD inline void sq9_column_unit(const double* m, int j, double* out9) {
  double n2 = m[j] * m[j];
SCM_UNROLL
  for (int i = 1; i < 9; ++i) n2 = n2 + m[i * 9 + j] * m[i * 9 + j];
  const double nrm = sqrt(n2);
SCM_UNROLL
  for (int i = 0; i < 9; ++i) out9[i] = m[i * 9 + j] / nrm;
}

SCM_HD inline double ata9_trace(const double* ata45) {
  // diagonal entries of the packed upper triangle: offsets 0, 9, 17, ...
  double t = ata45[0];
  int k = 9;
SCM_UNROLL
  for (int p = 1; p < 9; ++p) {
    t = t + ata45[k];
    k += 9 - p;
  }
  return t;
}

#if defined(SCM_GEOM_ATA_HOOK) && !defined(__HIP_DEVICE_COMPILE__)
void SCM_GEOM_ATA_HOOK(const double* ata45);  // diagnostics builds only (probes/)
#endif
SCM_HD inline void ata_null_vector(const double* ata45, double* out9) {
#if defined(SCM_GEOM_ATA_HOOK) && !defined(__HIP_DEVICE_COMPILE__)
  SCM_GEOM_ATA_HOOK(ata45);
#endif
  double a[81], b[81];
  const double tr = ata9_trace(ata45);
  if (!(tr > 0.0)) {
    for (int i = 0; i < 9; ++i) out9[i] = i == 0 ? 1.0 : 0.0;
    return;
  }
  const double delta = tr * 0x1p-40;
  int k = 0;
  for (int p = 0; p < 9; ++p)
    for (int q = p; q < 9; ++q) {
      const double v = p == q ? ata45[k] + delta : ata45[k];
      a[p * 9 + q] = v;
      a[q * 9 + p] = v;
      ++k;
    }
  for (int kk = 0; kk < 9; ++kk) {
    const double inv = 1.0 / a[kk * 9 + kk];
    for (int e = 0; e < 81; ++e) {
      const int i = e / 9, j = e % 9;
      b[e] = gj9_entry(a[e], a[i * 9 + kk], a[kk * 9 + j], inv, i, j, kk);
    }
    for (int e = 0; e < 81; ++e) a[e] = b[e];
  }
  for (int e = 0; e < 81; ++e) b[e] = 0.5 * (a[e] + a[(e % 9) * 9 + e / 9]);
  // b = symmetrised M0
  int jstar = 0;
  bool done = false;
  for (int sq = 0; sq < kInvSqMax; ++sq) {
    for (int e = 0; e < 81; ++e) a[e] = sq9_entry(b, e / 9, e % 9);
    const double ti = sq9_trace_inv(a);
    for (int e = 0; e < 81; ++e) b[e] = a[e] * ti;
    jstar = sq9_argmax_diag(b);
    if (done) break;
    done = sq + 1 >= kInvSqMin && sq9_rank_one(b, jstar);
  }
  sq9_column_unit(b, jstar, out9);
}

// Final step of colmap::FundamentalMatrixEightPointEstimator::Estimate
// [upstream]: rank-2 projection of the null vector and de-normalisation
// F = T2^T * F * T1.  F' = F0 - (F0 v3) v3^T with v3 the right singular
// vector of the smallest singular value (eigenvector of F0^T F0).
SCM_HD inline void fundamental_8pt_finish(const double* f, const double* T1,
                                          const double* T2, double* F) {
  double g[9];
  for (int p = 0; p < 3; ++p)
    for (int q = 0; q < 3; ++q)
      g[p * 3 + q] = f[0 + p] * f[0 + q] + f[3 + p] * f[3 + q] + f[6 + p] * f[6 + q];
  double w[9];
  const int kmin = jacobi_eigen_min<3>(g, w);
  double v3[3];
SCM_UNROLL
  for (int r = 0; r < 3; ++r)
    v3[r] = kmin == 0 ? w[r * 3] : (kmin == 1 ? w[r * 3 + 1] : w[r * 3 + 2]);
  double Fr[9];
  for (int r = 0; r < 3; ++r) {
    const double fv = f[3 * r] * v3[0] + f[3 * r + 1] * v3[1] + f[3 * r + 2] * v3[2];
    for (int c = 0; c < 3; ++c) Fr[3 * r + c] = f[3 * r + c] - fv * v3[c];
  }
  const double T2t[9] = {T2[0], T2[3], T2[6], T2[1], T2[4], T2[7], T2[2], T2[5], T2[8]};
  double tmp[9];
  mat3_mul(T2t, Fr, tmp);
  mat3_mul(tmp, T1, F);
}

// colmap::FundamentalMatrixEightPointEstimator::Estimate [upstream]
// (LO-RANSAC local estimator), n >= 8, canonical summation order.
SCM_HD inline int fundamental_8pt(const double* xy1, const double* xy2, int n, double* F) {
  double T1[9], T2[9];
  normalize_transform(xy1, n, T1);
  normalize_transform(xy2, n, T2);
  double part[kCanon][45];
  for (int l = 0; l < kCanon; ++l)
    for (int k = 0; k < 45; ++k) part[l][k] = kCanonZero;
  for (int i = 0; i < n; ++i) {
    double x0, y0, x1, y1, a[9];
    apply_normalize(T1, xy1[2 * i], xy1[2 * i + 1], &x0, &y0);
    apply_normalize(T2, xy2[2 * i], xy2[2 * i + 1], &x1, &y1);
    f_row(x0, y0, x1, y1, a);
    ata_accumulate(part[i & (kCanon - 1)], a);
  }
  double ata[45];
  for (int k = 0; k < 45; ++k) {
    double p[kCanon];
    for (int l = 0; l < kCanon; ++l) p[l] = part[l][k];
    ata[k] = canon_tree(p);
  }
  double f[9];
  ata_null_vector(ata, f);
  fundamental_8pt_finish(f, T1, T2, F);
  return 1;
}

// De-normalisation of a homography null vector: H = T2^-1 * h * T1, with
// T2^-1 = [1/s 0 cx; 0 1/s cy; 0 0 1] written analytically (cx = -T2[2]/s).
SCM_HD inline void homography_finish(const double* h, const double* T1, const double* T2,
                                     double* H) {
  const double s2 = T2[0];
  const double T2inv[9] = {1.0 / s2, 0.0, -T2[2] / s2, 0.0, 1.0 / s2, -T2[5] / s2,
                           0.0, 0.0, 1.0};
  double tmp[9];
  mat3_mul(T2inv, h, tmp);
  mat3_mul(tmp, T1, H);
}

// colmap::HomographyMatrixEstimator::Estimate [upstream
// estimators/homography_matrix.cc]: normalised DLT.  n == 4 (minimal sample)
// uses the exact Householder null space; n > 4 (local optimisation) the
// least-squares null vector of A^T A in canonical order.  Returns 1.
SCM_HD inline int homography_dlt(const double* xy1, const double* xy2, int n, double* H) {
  double T1[9], T2[9];
  normalize_transform(xy1, n, T1);
  normalize_transform(xy2, n, T2);
  double h[9];
  if (n == 4) {
    double A[8 * 9];
    for (int i = 0; i < 4; ++i) {
      double s0, s1, d0, d1;
      apply_normalize(T1, xy1[2 * i], xy1[2 * i + 1], &s0, &s1);
      apply_normalize(T2, xy2[2 * i], xy2[2 * i + 1], &d0, &d1);
      h_rows(s0, s1, d0, d1, A + 9 * i, A + 9 * (i + 4));
    }
    householder_nullspace<8>(A, h);
  } else {
    double part[kCanon][45];
    for (int l = 0; l < kCanon; ++l)
      for (int k = 0; k < 45; ++k) part[l][k] = kCanonZero;
    for (int i = 0; i < n; ++i) {
      double s0, s1, d0, d1, a[9], b[9];
      apply_normalize(T1, xy1[2 * i], xy1[2 * i + 1], &s0, &s1);
      apply_normalize(T2, xy2[2 * i], xy2[2 * i + 1], &d0, &d1);
      h_rows(s0, s1, d0, d1, a, b);
      ata_accumulate(part[i & (kCanon - 1)], a);
      ata_accumulate(part[i & (kCanon - 1)], b);
    }
    double ata[45];
    for (int k = 0; k < 45; ++k) {
      double p[kCanon];
      for (int l = 0; l < kCanon; ++l) p[l] = part[l][k];
      ata[k] = canon_tree(p);
    }
    ata_null_vector(ata, h);
  }
  homography_finish(h, T1, T2, H);
  return 1;
}

// colmap::TranslationTransformEstimator<2>::Estimate [upstream]:
// t = mean(x2) - mean(x1), sums in canonical order.
SCM_HD inline void translation_estimate(const double* xy1, const double* xy2, int n,
                                        double* t) {
  double p[4][kCanon];
  for (int c = 0; c < 4; ++c)
    for (int l = 0; l < kCanon; ++l) p[c][l] = kCanonZero;
  for (int i = 0; i < n; ++i) {
    const int l = i & (kCanon - 1);
    p[0][l] += xy1[2 * i];
    p[1][l] += xy1[2 * i + 1];
    p[2][l] += xy2[2 * i];
    p[3][l] += xy2[2 * i + 1];
  }
  const double s0 = canon_tree(p[0]) / (double)n;
  const double s1 = canon_tree(p[1]) / (double)n;
  const double d0 = canon_tree(p[2]) / (double)n;
  const double d1 = canon_tree(p[3]) / (double)n;
  t[0] = d0 - s0;
  t[1] = d1 - s1;
}

}  // namespace geom
}  // namespace scm
