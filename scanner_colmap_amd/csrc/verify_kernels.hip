// Kernel 2 of the sequential-matching stage: GPU-resident two-view geometry
// (replaces verifyTwoViewGeometry + colmap::TwoViewGeometry::Estimate +
// the op's post-filter, reference integration/op_cpp/sequential_matching.cc:
// 84-101 and 164-178; upstream EstimateUncalibrated).
//
// One 256-thread workgroup owns one image pair and runs, in order and with
// the pair's own std::mt19937 stream (LDS-resident):
//   LO-RANSAC<7-pt F, 8-pt F>  ->  LO-RANSAC<4-pt H, N-pt H>
//   -> configuration -> DetectWatermark (LO-RANSAC<translation>) -> post-filter.
// Each RANSAC round solves kTrialBatch hypotheses in parallel (one lane per
// trial), scores every resulting model with one wavefront per model over the
// pair's matches (fp64 Sampson / transfer error, exact inlier counts), then
// replays the trials in order exactly as the sequential LO-RANSAC does
// (Compare, recursive local optimisation, dynamic trial bound, early abort);
// hypotheses past the abort point are discarded and the PRNG is rewound to
// the last consumed draw.  Residual sums that decide a Compare are summed
// sequentially in index order, as InlierSupportMeasurer::Evaluate does.  The
// estimator arithmetic is the shared geom_solvers.h, so every model is
// bit-identical to the CPU oracle's.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/scm.h"
#include "geom_solvers.h"
#include "verify_kernels.h"

namespace scm {

using namespace geom;

enum { KIND_F = 0, KIND_H = 1, KIND_T = 2 };

template <int K> struct KindTraits;
template <> struct KindTraits<KIND_F> { static constexpr int kmin = 7, kmin_local = 8, max_models = 3, msize = 9; };
template <> struct KindTraits<KIND_H> { static constexpr int kmin = 4, kmin_local = 4, max_models = 1, msize = 9; };
template <> struct KindTraits<KIND_T> { static constexpr int kmin = 1, kmin_local = 1, max_models = 1, msize = 2; };

struct __attribute__((aligned(16))) VerifyLds {
  double models[kTrialBatch][3][9];
  double red[45 * kCanon];
  double best_model[9];
  double local_model[9];
  double T1[9], T2[9];
  double best_sum;
  double bcast_d;
  uint32_t mt[624];
  uint32_t mt_snap[624];
  uint32_t sidx[kLdsSampleIdx];
  uint32_t samples[kTrialBatch][8];
  int32_t nmodels[kTrialBatch];
  int32_t counts[kTrialBatch][3];
  int32_t wave_cnt[kVerifyThreads / 64];
  int32_t scan[kVerifyThreads];
  int32_t mt_idx, mt_idx_snap;
  int32_t best_n;
  int32_t bcast_i;
};

// ---------------------------------------------------------------------------
// std::mt19937 + std::uniform_int_distribution<uint32_t> (libstdc++ 11,
// Lemire nearly-divisionless downscaling), single lane.
// ---------------------------------------------------------------------------
__device__ void mt_seed(VerifyLds& s, uint32_t seed) {
  s.mt[0] = seed;
  for (int i = 1; i < 624; ++i)
    s.mt[i] = 1812433253u * (s.mt[i - 1] ^ (s.mt[i - 1] >> 30)) + (uint32_t)i;
  s.mt_idx = 624;
}

__device__ uint32_t mt_next(VerifyLds& s) {
  if (s.mt_idx >= 624) {
    for (int k = 0; k < 624; ++k) {
      const uint32_t y = (s.mt[k] & 0x80000000u) | (s.mt[k + 1 < 624 ? k + 1 : 0] & 0x7fffffffu);
      const int km = k + 397 < 624 ? k + 397 : k + 397 - 624;
      s.mt[k] = s.mt[km] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    s.mt_idx = 0;
  }
  uint32_t y = s.mt[s.mt_idx++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

__device__ uint32_t uniform_u32(VerifyLds& s, uint32_t a, uint32_t b) {
  const uint32_t urange = b - a;
  if (urange == 0xFFFFFFFFu) return mt_next(s);
  const uint32_t uerange = urange + 1u;
  uint64_t product = (uint64_t)mt_next(s) * (uint64_t)uerange;
  uint32_t low = (uint32_t)product;
  if (low < uerange) {
    const uint32_t threshold = (0u - uerange) % uerange;
    while (low < threshold) {
      product = (uint64_t)mt_next(s) * (uint64_t)uerange;
      low = (uint32_t)product;
    }
  }
  return a + (uint32_t)(product >> 32);
}

// ---------------------------------------------------------------------------
// Workgroup helpers.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
  return v;
}

// Sum of v over the workgroup (all threads receive it).
__device__ int wg_sum_i(VerifyLds& s, int v) {
  v = wave_sum_i(v);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) s.wave_cnt[wave] = v;
  __syncthreads();
  int t = 0;
#pragma unroll
  for (int w = 0; w < kVerifyThreads / 64; ++w) t += s.wave_cnt[w];
  __syncthreads();
  return t;
}

template <int K>
__device__ __forceinline__ double residual(const double* m, const double* xy1,
                                           const double* xy2, int i) {
  const double a0 = xy1[2 * i], a1 = xy1[2 * i + 1];
  const double b0 = xy2[2 * i], b1 = xy2[2 * i + 1];
  if (K == KIND_F) return sampson_sq(m, a0, a1, b0, b1);
  if (K == KIND_H) return homography_sq(m, a0, a1, b0, b1);
  return translation_sq(m, a0, a1, b0, b1);
}

// Residuals of one model over all points into res, returns the inlier count.
template <int K>
__device__ int residuals_wg(VerifyLds& s, const double* m, const double* xy1,
                            const double* xy2, int n, double maxr, double* res) {
  int c = 0;
  for (int i = threadIdx.x; i < n; i += kVerifyThreads) {
    const double r = residual<K>(m, xy1, xy2, i);
    res[i] = r;
    c += (r <= maxr) ? 1 : 0;
  }
  return wg_sum_i(s, c);
}

// InlierSupportMeasurer::Evaluate's residual_sum: inlier residuals summed in
// index order (one lane), broadcast to the workgroup.
__device__ double seq_inlier_sum(VerifyLds& s, const double* res, int n, double maxr) {
  __syncthreads();
  if (threadIdx.x == 0) {
    double sum = 0.0;
    for (int i = 0; i < n; ++i) {
      const double r = res[i];
      if (r <= maxr) sum += r;
    }
    s.bcast_d = sum;
  }
  __syncthreads();
  const double v = s.bcast_d;
  __syncthreads();
  return v;
}

// Ordered compaction of the points whose residual is <= maxr into
// xin1 / xin2; returns the number of inliers.
__device__ int gather_inliers(VerifyLds& s, const double* res, int n, double maxr,
                              const double* xy1, const double* xy2, double* xin1,
                              double* xin2) {
  const int tid = threadIdx.x;
  const int per = (n + kVerifyThreads - 1) / kVerifyThreads;
  const int i0 = min(n, tid * per), i1 = min(n, i0 + per);
  int c = 0;
  for (int i = i0; i < i1; ++i) c += (res[i] <= maxr) ? 1 : 0;
  s.scan[tid] = c;
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int t = 0; t < kVerifyThreads; ++t) {
      const int v = s.scan[t];
      s.scan[t] = acc;
      acc += v;
    }
    s.bcast_i = acc;
  }
  __syncthreads();
  int o = s.scan[tid];
  for (int i = i0; i < i1; ++i) {
    if (res[i] <= maxr) {
      xin1[2 * o] = xy1[2 * i];
      xin1[2 * o + 1] = xy1[2 * i + 1];
      xin2[2 * o] = xy2[2 * i];
      xin2[2 * o + 1] = xy2[2 * i + 1];
      ++o;
    }
  }
  const int total = s.bcast_i;
  __syncthreads();
  return total;
}

// Canonical partial sums (geom_solvers.h kCanon order) of up to 4 per-point
// quantities, computed by wave 0 (lane l owns points i = l mod 64), then the
// fixed tree by one lane per quantity.  Results in s.red[q * 64].
template <typename F>
__device__ void canon_sums(VerifyLds& s, int n, int nq, F f) {
  const int tid = threadIdx.x;
  if (tid < kCanon) {
    double p[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = tid; i < n; i += kCanon) {
      double v[4];
      f(i, v);
      for (int q = 0; q < nq; ++q) p[q] += v[q];
    }
    for (int q = 0; q < nq; ++q) s.red[q * kCanon + tid] = p[q];
  }
  __syncthreads();
  if (tid < nq) canon_tree(&s.red[tid * kCanon]);
  __syncthreads();
}

// normalize_transform (geom_solvers.h) of both point sets, in parallel.
__device__ void normalize_pair_wg(VerifyLds& s, const double* xy1, const double* xy2, int n) {
  canon_sums(s, n, 4, [&](int i, double* v) {
    v[0] = xy1[2 * i];
    v[1] = xy1[2 * i + 1];
    v[2] = xy2[2 * i];
    v[3] = xy2[2 * i + 1];
  });
  const double c10 = s.red[0] / (double)n, c11 = s.red[kCanon] / (double)n;
  const double c20 = s.red[2 * kCanon] / (double)n, c21 = s.red[3 * kCanon] / (double)n;
  __syncthreads();
  canon_sums(s, n, 2, [&](int i, double* v) {
    const double d0 = xy1[2 * i] - c10, d1 = xy1[2 * i + 1] - c11;
    const double e0 = xy2[2 * i] - c20, e1 = xy2[2 * i + 1] - c21;
    v[0] = d0 * d0 + d1 * d1;
    v[1] = e0 * e0 + e1 * e1;
  });
  if (threadIdx.x == 0) {
    const double rms1 = sqrt(s.red[0] / (double)n);
    const double rms2 = sqrt(s.red[kCanon] / (double)n);
    const double sc1 = sqrt(2.0) / rms1, sc2 = sqrt(2.0) / rms2;
    double* T1 = s.T1;
    double* T2 = s.T2;
    T1[0] = sc1; T1[1] = 0.0; T1[2] = -sc1 * c10;
    T1[3] = 0.0; T1[4] = sc1; T1[5] = -sc1 * c11;
    T1[6] = 0.0; T1[7] = 0.0; T1[8] = 1.0;
    T2[0] = sc2; T2[1] = 0.0; T2[2] = -sc2 * c20;
    T2[3] = 0.0; T2[4] = sc2; T2[5] = -sc2 * c21;
    T2[6] = 0.0; T2[7] = 0.0; T2[8] = 1.0;
  }
  __syncthreads();
}

// Local (least-squares) estimators on n gathered inliers; result in
// s.local_model.  Same arithmetic as geom_solvers.h fundamental_8pt /
// homography_dlt (n > 4) / translation_estimate.
template <int K>
__device__ void local_estimate_wg(VerifyLds& s, const double* xin1, const double* xin2, int n) {
  const int tid = threadIdx.x;
  if (K == KIND_T) {
    canon_sums(s, n, 4, [&](int i, double* v) {
      v[0] = xin1[2 * i];
      v[1] = xin1[2 * i + 1];
      v[2] = xin2[2 * i];
      v[3] = xin2[2 * i + 1];
    });
    if (tid == 0) {
      const double s0 = s.red[0] / (double)n, s1 = s.red[kCanon] / (double)n;
      const double d0 = s.red[2 * kCanon] / (double)n, d1 = s.red[3 * kCanon] / (double)n;
      s.local_model[0] = d0 - s0;
      s.local_model[1] = d1 - s1;
    }
    __syncthreads();
    return;
  }
  normalize_pair_wg(s, xin1, xin2, n);
  // A^T A partials: wave w owns entries k = w, w+4, ...; lane l owns points l mod 64.
  {
    const int wave = tid >> 6, lane = tid & 63;
    double part[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) part[j] = 0.0;
    const double* T1 = s.T1;
    const double* T2 = s.T2;
    for (int i = lane; i < n; i += kCanon) {
      double x0, y0, x1, y1;
      apply_normalize(T1, xin1[2 * i], xin1[2 * i + 1], &x0, &y0);
      apply_normalize(T2, xin2[2 * i], xin2[2 * i + 1], &x1, &y1);
      double a[9], b[9];
      if (K == KIND_F) f_row(x0, y0, x1, y1, a);
      else h_rows(x0, y0, x1, y1, a, b);
      int k = 0, j = 0;
#pragma unroll
      for (int p = 0; p < 9; ++p)
#pragma unroll
        for (int q = p; q < 9; ++q) {
          if ((k & 3) == wave) {
            double v = part[j] + a[p] * a[q];
            if (K == KIND_H) v = v + b[p] * b[q];
            part[j] = v;
          }
          if ((k & 3) == wave) ++j;
          ++k;
        }
    }
    int k = 0, j = 0;
#pragma unroll
    for (int p = 0; p < 9; ++p)
#pragma unroll
      for (int q = p; q < 9; ++q) {
        if ((k & 3) == wave) s.red[k * kCanon + lane] = part[j++];
        ++k;
      }
  }
  __syncthreads();
  if (tid < 45) canon_tree(&s.red[tid * kCanon]);
  __syncthreads();
  if (tid == 0) {
    double ata[45];
    for (int k = 0; k < 45; ++k) ata[k] = s.red[k * kCanon];
    double f[9];
    ata_null_vector(ata, f);
    if (K == KIND_F) fundamental_8pt_finish(f, s.T1, s.T2, s.local_model);
    else homography_finish(f, s.T1, s.T2, s.local_model);
  }
  __syncthreads();
}

struct RansacResult {
  int success;
  int num_inliers;
  int num_trials;
  int res_sel;  // which residual buffer holds the best model's residuals
};

// LORANSAC<Estimator, LocalEstimator>::Estimate on n points (xy1, xy2).
// res[0] / res[1]: residual buffers (n doubles each); xin1 / xin2 inlier
// gather buffers (2n doubles each).  Best model ends in s.best_model.
template <int K>
__device__ RansacResult loransac_wg(VerifyLds& s, const double* xy1, const double* xy2,
                                    int n, int max_trials, const VerifyParams& P,
                                    double* res0, double* res1, double* xin1, double* xin2,
                                    uint32_t* sidx_global) {
  using Tr = KindTraits<K>;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const double maxr = P.max_residual;
  RansacResult out = {0, 0, 0, 0};
  if (tid < 9) s.best_model[tid] = 0.0;  // report.model when no model is found
  __syncthreads();
  if (n < Tr::kmin) return out;

  uint32_t* sidx = (n <= kLdsSampleIdx) ? s.sidx : sidx_global;
  for (int i = tid; i < n; i += kVerifyThreads) sidx[i] = (uint32_t)i;
  if (tid == 0) {
    s.best_n = 0;
    s.best_sum = 1.7976931348623157e308;  // DBL_MAX
  }
  double* res[2] = {res0, res1};
  int best_sel = 0;          // res[best_sel] = residuals of the best model
  int dyn_max = max_trials;
  int trial = 0;
  bool abort = false;
  int abort_trial = -1;
  __syncthreads();

  while (trial < max_trials && !abort) {
    const int B = min(kTrialBatch, max_trials - trial);
    // -- snapshot the PRNG, draw B samples (Shuffle of the persistent index vector).
    for (int i = tid; i < 624; i += kVerifyThreads) s.mt_snap[i] = s.mt[i];
    if (tid == 0) s.mt_idx_snap = s.mt_idx;
    __syncthreads();
    if (tid == 0) {
      const uint32_t last = (uint32_t)(n - 1);
      for (int b = 0; b < B; ++b)
        for (int i = 0; i < Tr::kmin; ++i) {
          const uint32_t j = uniform_u32(s, (uint32_t)i, last);
          const uint32_t t = sidx[i];
          sidx[i] = sidx[j];
          sidx[j] = t;
          s.samples[b][i] = sidx[i];
        }
    }
    __syncthreads();
    // -- solve the B minimal samples, one lane each.
    if (tid < B) {
      double a[2 * 7], b[2 * 7];
      for (int i = 0; i < Tr::kmin; ++i) {
        const uint32_t k = s.samples[tid][i];
        a[2 * i] = xy1[2 * k];
        a[2 * i + 1] = xy1[2 * k + 1];
        b[2 * i] = xy2[2 * k];
        b[2 * i + 1] = xy2[2 * k + 1];
      }
      int nm = 0;
      if (K == KIND_F) {
        nm = fundamental_7pt(a, b, &s.models[tid][0][0]);
      } else if (K == KIND_H) {
        homography_dlt(a, b, 4, &s.models[tid][0][0]);
        nm = 1;
      } else {
        translation_estimate(a, b, 1, &s.models[tid][0][0]);
        nm = 1;
      }
      s.nmodels[tid] = nm;
    }
    __syncthreads();
    // -- score: one wavefront per model, exact inlier counts.
    for (int slot = wave; slot < B * Tr::max_models; slot += kVerifyThreads / 64) {
      const int b = slot / Tr::max_models, k = slot % Tr::max_models;
      if (k >= s.nmodels[b]) continue;
      const double* m = &s.models[b][k][0];
      int c = 0;
      for (int i = lane; i < n; i += 64) c += (residual<K>(m, xy1, xy2, i) <= maxr) ? 1 : 0;
      c = wave_sum_i(c);
      if (lane == 0) s.counts[b][k] = c;
    }
    __syncthreads();
    // -- replay the trials in order.
    for (int b = 0; b < B && !abort; ++b) {
      const int t = trial + b;
      const int nm = s.nmodels[b];
      for (int k = 0; k < nm; ++k) {
        const int c = s.counts[b][k];
        const int bn = s.best_n;
        if (c >= bn) {
          const double* m = &s.models[b][k][0];
          double* rt = res[best_sel ^ 1];
          residuals_wg<K>(s, m, xy1, xy2, n, maxr, rt);
          const double sum = seq_inlier_sum(s, rt, n, maxr);
          const bool better = (c > bn) || (sum < s.best_sum);
          if (better) {
            if (tid == 0) {
              s.best_n = c;
              s.best_sum = sum;
            }
            if (tid < Tr::msize) s.best_model[tid] = m[tid];
            best_sel ^= 1;
            __syncthreads();
            // Recursive local optimisation.
            if (c > Tr::kmin && c >= Tr::kmin_local) {
              for (int lt = 0; lt < 10; ++lt) {
                const int ni = gather_inliers(s, res[best_sel], n, maxr, xy1, xy2, xin1, xin2);
                local_estimate_wg<K>(s, xin1, xin2, ni);
                const int prev = s.best_n;
                double* rl = res[best_sel ^ 1];
                const int lc = residuals_wg<K>(s, s.local_model, xy1, xy2, n, maxr, rl);
                bool lbetter = lc > prev;
                double lsum = 0.0;
                if (lc >= prev) {
                  lsum = seq_inlier_sum(s, rl, n, maxr);
                  lbetter = (lc > prev) || (lsum < s.best_sum);
                }
                if (lbetter) {
                  if (tid == 0) {
                    s.best_n = lc;
                    s.best_sum = lsum;
                  }
                  if (tid < Tr::msize) s.best_model[tid] = s.local_model[tid];
                  best_sel ^= 1;
                }
                __syncthreads();
                if (s.best_n <= prev) break;
              }
            }
            dyn_max = (int)min((uint64_t)0x7FFFFFFF,
                               num_trials((uint64_t)s.best_n, (uint64_t)n, P.confidence,
                                          P.dyn_num_trials_multiplier, Tr::kmin));
          }
        }
        if (t >= dyn_max && t >= P.min_num_trials) {
          abort = true;
          abort_trial = t;
          break;
        }
      }
    }
    if (abort) {
      // Rewind the PRNG to the state after trial abort_trial's sample.
      __syncthreads();
      for (int i = tid; i < 624; i += kVerifyThreads) s.mt[i] = s.mt_snap[i];
      if (tid == 0) s.mt_idx = s.mt_idx_snap;
      __syncthreads();
      if (tid == 0) {
        const uint32_t last = (uint32_t)(n - 1);
        for (int b = 0; b <= abort_trial - trial; ++b)
          for (int i = 0; i < Tr::kmin; ++i) (void)uniform_u32(s, (uint32_t)i, last);
      }
      __syncthreads();
      out.num_trials = abort_trial + 2;
    } else {
      trial += B;
      out.num_trials = trial;
    }
  }
  // res[best_sel] holds the residuals of the best model (every accepted
  // model had its residuals written to the buffer that became res[best_sel]).
  out.num_inliers = s.best_n;
  out.success = s.best_n >= Tr::kmin ? 1 : 0;
  out.res_sel = best_sel;
  __syncthreads();
  return out;
}

__global__ __launch_bounds__(kVerifyThreads) void verify_kernel(
    const VerifyPair* __restrict__ pairs, const double* __restrict__ xy1_all,
    const double* __restrict__ xy2_all, double* __restrict__ scratch,
    uint32_t* __restrict__ idx_scratch, uint8_t* __restrict__ masks,
    VerifyOut* __restrict__ out, VerifyParams P) {
  __shared__ VerifyLds s;
  const VerifyPair pp = pairs[blockIdx.x];
  const int tid = threadIdx.x;
  const int n = pp.m;
  VerifyOut o;
  o.config = 0;
  o.num_inliers = 0;
  o.f_trials = o.h_trials = 0;
  o.f_inliers_raw = o.h_inliers_raw = 0;
  o.watermark = 0;
  o.pad_ = 0;
  for (int i = 0; i < 9; ++i) { o.F[i] = 0.0; o.H[i] = 0.0; }
  uint8_t* mask = masks + pp.mask_off;
  for (int i = tid; i < n; i += kVerifyThreads) mask[i] = 0;

  if (n >= P.min_num_inliers && n > 0) {
    const double* xy1 = xy1_all + pp.pts_off;
    const double* xy2 = xy2_all + pp.pts_off;
    double* res0 = scratch + pp.scr_off;
    double* res1 = res0 + n;
    double* xin1 = res1 + n;
    double* xin2 = xin1 + 2 * n;
    uint32_t* sg = idx_scratch + pp.idx_off;
    if (tid == 0) mt_seed(s, pair_seed(P.base_seed, pp.id1, pp.id2));
    __syncthreads();

    // ---- F: LORANSAC<7-pt, 8-pt>.
    const RansacResult rf = loransac_wg<KIND_F>(s, xy1, xy2, n, P.max_trials_F, P, res0, res1,
                                                xin1, xin2, sg);
    double Fm[9];
    for (int i = 0; i < 9; ++i) Fm[i] = s.best_model[i];
    const double* resF = rf.res_sel ? res1 : res0;
    // F inlier mask (ExtractInlierMatches input) before the buffers are reused.
    if (rf.success)
      for (int i = tid; i < n; i += kVerifyThreads) mask[i] = resF[i] <= P.max_residual ? 1 : 0;
    __syncthreads();
    // ---- H: LORANSAC<H, H> (same PRNG stream).
    const RansacResult rh = loransac_wg<KIND_H>(s, xy1, xy2, n, P.max_trials_H, P, res0, res1,
                                                xin1, xin2, sg);
    double Hm[9];
    for (int i = 0; i < 9; ++i) Hm[i] = s.best_model[i];
    o.f_trials = rf.num_trials;
    o.h_trials = rh.num_trials;
    o.f_inliers_raw = rf.num_inliers;
    o.h_inliers_raw = rh.num_inliers;
    for (int i = 0; i < 9; ++i) {
      o.F[i] = Fm[i];  // F = F_report.model, H = H_report.model
      o.H[i] = Hm[i];
    }
    const int mni = P.min_num_inliers;
    if ((!rf.success && !rh.success) || (rf.num_inliers < mni && rh.num_inliers < mni)) {
      o.config = SCM_TVG_DEGENERATE;
    } else {
      const double ratio = (double)rh.num_inliers / (double)rf.num_inliers;
      o.config = ratio > P.max_H_inlier_ratio ? SCM_TVG_PLANAR_OR_PANORAMIC : SCM_TVG_UNCALIBRATED;
      o.num_inliers = rf.success ? rf.num_inliers : 0;
      if (P.detect_watermark && rf.success) {
        // DetectWatermark with the dummy cameras (width = height = 0): a point
        // is inside the [0,0]x[0,0] box only if it is exactly (0, 0).
        int nb = 0;
        for (int i = tid; i < n; i += kVerifyThreads) {
          if (!mask[i]) continue;
          const bool in1 = xy1[2 * i] >= 0.0 && xy1[2 * i] <= 0.0 && xy1[2 * i + 1] >= 0.0 &&
                           xy1[2 * i + 1] <= 0.0;
          const bool in2 = xy2[2 * i] >= 0.0 && xy2[2 * i] <= 0.0 && xy2[2 * i + 1] >= 0.0 &&
                           xy2[2 * i + 1] <= 0.0;
          nb += (!in1 && !in2) ? 1 : 0;
        }
        nb = wg_sum_i(s, nb);
        const int ni = rf.num_inliers;
        const double bratio = (double)nb / (double)ni;
        if (!(bratio < P.watermark_min_inlier_ratio)) {
          // Inlier points in index order -> translation LO-RANSAC.  Scratch
          // layout (10n doubles per pair, res0 = base): tin1 [0,2ni) tin2
          // [2n,2n+2ni) tres0 [4n,4n+ni) tres1 [5n,5n+ni) tx1 [6n,6n+2ni)
          // tx2 [8n,8n+2ni).
          double* base = res0;
          double* tin1 = base;
          double* tin2 = base + 2 * n;
          {
            const int per = (n + kVerifyThreads - 1) / kVerifyThreads;
            const int i0 = min(n, tid * per), i1 = min(n, i0 + per);
            int c = 0;
            for (int i = i0; i < i1; ++i) c += mask[i] ? 1 : 0;
            s.scan[tid] = c;
            __syncthreads();
            if (tid == 0) {
              int acc = 0;
              for (int t = 0; t < kVerifyThreads; ++t) {
                const int v = s.scan[t];
                s.scan[t] = acc;
                acc += v;
              }
            }
            __syncthreads();
            int w = s.scan[tid];
            for (int i = i0; i < i1; ++i)
              if (mask[i]) {
                tin1[2 * w] = xy1[2 * i];
                tin1[2 * w + 1] = xy1[2 * i + 1];
                tin2[2 * w] = xy2[2 * i];
                tin2[2 * w + 1] = xy2[2 * i + 1];
                ++w;
              }
            __syncthreads();
          }
          double* tres0 = base + 4 * n;
          double* tres1 = base + 5 * n;
          double* tx1 = base + 6 * n;
          double* tx2 = base + 8 * n;
          const RansacResult rt = loransac_wg<KIND_T>(s, tin1, tin2, ni, P.max_trials_T, P, tres0,
                                                      tres1, tx1, tx2, sg);
          const double iratio = (double)rt.num_inliers / (double)ni;
          if (iratio >= P.watermark_min_inlier_ratio) {
            o.config = SCM_TVG_WATERMARK;
            o.watermark = 1;
          }
        }
      }
    }
    // ---- post-filter (sequential_matching.cc:173-178): TwoViewGeometry().
    if (o.num_inliers < P.min_num_inliers) {
      o.config = 0;
      o.num_inliers = 0;
      for (int i = 0; i < 9; ++i) { o.F[i] = 0.0; o.H[i] = 0.0; }
    }
  } else {
    o.config = 0;  // DEGENERATE, then the post-filter's TwoViewGeometry()
  }
  if (tid == 0) out[blockIdx.x] = o;
}

__global__ void gather_kernel(const GatherPair* __restrict__ pairs, const uint2* __restrict__ matches,
                              const float2* __restrict__ kpxy, double* __restrict__ xy1,
                              double* __restrict__ xy2, uint2* __restrict__ packed) {
  const GatherPair g = pairs[blockIdx.x];
  for (int i = threadIdx.x; i < g.m; i += blockDim.x) {
    const uint2 mt = matches[g.match_off + i];
    packed[g.pts_off + i] = mt;
    const float2 a = kpxy[g.kp1_off + mt.x];
    const float2 b = kpxy[g.kp2_off + mt.y];
    xy1[2 * (g.pts_off + i)] = (double)a.x;
    xy1[2 * (g.pts_off + i) + 1] = (double)a.y;
    xy2[2 * (g.pts_off + i)] = (double)b.x;
    xy2[2 * (g.pts_off + i) + 1] = (double)b.y;
  }
}

hipError_t launch_verify(const VerifyPair* pairs, int npairs, const double* xy1,
                         const double* xy2, double* scratch, uint32_t* idx_scratch,
                         uint8_t* masks, VerifyOut* out, const VerifyParams& params,
                         hipStream_t stream) {
  if (npairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(verify_kernel, dim3(npairs), dim3(kVerifyThreads), 0, stream, pairs, xy1,
                     xy2, scratch, idx_scratch, masks, out, params);
  return hipGetLastError();
}

hipError_t launch_gather(const GatherPair* pairs, int npairs, const uint2* matches,
                         const float2* kpxy, double* xy1, double* xy2, uint2* packed,
                         hipStream_t stream) {
  if (npairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_kernel, dim3(npairs), dim3(256), 0, stream, pairs, matches, kpxy,
                     xy1, xy2, packed);
  return hipGetLastError();
}

}  // namespace scm
