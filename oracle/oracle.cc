// CPU ORACLE — test infrastructure only.
//
// A plain, sequential C++ restatement of the reference's hot path
//   SequentialMatchingCPUKernel::execute
//     (reference integration/op_cpp/sequential_matching.cc:103-185)
// and of the COLMAP 3.4/3.5 functions it calls (un-vendored upstream code,
// restated from its published algorithm):
//   colmap::MatchSiftFeaturesCPU / ComputeSiftDistanceMatrix /
//     FindBestMatchesOneWay / FindBestMatches      [feature/sift.cc]
//   colmap::TwoViewGeometry::Estimate -> EstimateUncalibrated,
//     DetectWatermark                               [estimators/two_view_geometry.cc]
//   colmap::LORANSAC / RANSAC::ComputeNumTrials / RandomSampler / Shuffle /
//     InlierSupportMeasurer                         [optim/*.h, util/random.h]
// plus the io.cc byte codecs (reference integration/op_cpp/io.cc).
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
// this library, always as the checker / the timed CPU baseline — never as part
// of the product path.
//
// Parity status: the reference cannot be compiled or imported here (Scanner,
// COLMAP, Eigen, protoc and CUDA are all absent) and ships no
// tests, fixtures or golden vectors, so this oracle is "parity unpinned" at
// the COLMAP boundary.  It is pinned instead by known-answer tests
// (tests/test_oracle_*.py): hand-built top-2/tie/ratio cases, the acosf
// threshold of SURVEY.md §8a (d = 200,499), exact synthetic geometry, and the
// libstdc++ std::mt19937 + std::uniform_int_distribution draw sequence.
//
// The RANSAC PRNGs are std::mt19937 seeded per pair: F with scm_pair_seed(),
// H and the watermark RANSAC with the second stream's seed (geom_solvers.h
// pair_seed_h); the reference's single generator is time-seeded, SURVEY.md §0
// fact 4.  The fp64 estimator
// primitives are the shared header geom_solvers.h so that the GPU path can be
// checked bit-for-bit; they are pinned separately by known-answer tests.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <random>
#include <vector>

#include "../include/scm.h"
#include "../scanner_colmap_amd/csrc/geom_solvers.h"

extern "C" uint32_t oracle_pair_seed(uint32_t base, uint32_t id1, uint32_t id2);

namespace {

using scm::geom::fundamental_7pt;

struct Match {
  uint32_t idx1, idx2;
};

// ===========================================================================
// Matching (a4-a7): COLMAP 3.4 MatchSiftFeaturesCPU.
// ===========================================================================

// ComputeSiftDistanceMatrix: descriptors cast to Eigen::Matrix<int,Dynamic,128>
// (default ColMajor: element (i, d) at d * n + i, so each row dot is a scalar
// strided loop) into a RowMajor int32 N1 x N2 matrix.
void compute_sift_distance_matrix(const uint8_t* d1, int64_t n1,
                                  const uint8_t* d2, int64_t n2,
                                  std::vector<int32_t>* dists_rowmajor) {
  std::vector<int32_t> a((size_t)n1 * 128), b((size_t)n2 * 128);
  for (int64_t i = 0; i < n1; ++i)
    for (int d = 0; d < 128; ++d) a[(size_t)d * n1 + i] = d1[i * 128 + d];
  for (int64_t i = 0; i < n2; ++i)
    for (int d = 0; d < 128; ++d) b[(size_t)d * n2 + i] = d2[i * 128 + d];
  dists_rowmajor->assign((size_t)n1 * n2, 0);
  for (int64_t i1 = 0; i1 < n1; ++i1) {
    for (int64_t i2 = 0; i2 < n2; ++i2) {
      int32_t dot = 0;
      for (int d = 0; d < 128; ++d)
        dot += a[(size_t)d * n1 + i1] * b[(size_t)d * n2 + i2];
      (*dists_rowmajor)[(size_t)i1 * n2 + i2] = dot;
    }
  }
}

// The distance / ratio decision of FindBestMatchesOneWay for one scanned row
// (best_i2 == -1 is tested by the caller).  float kDistNorm = 1/(512*512),
// float max_ratio and max_distance (the function takes float parameters
// [upstream]).
bool passes_ratio_test(int best_dist, int second_best_dist, float max_ratio,
                       float max_distance) {
  const float kDistNorm = 1.0f / (512.0f * 512.0f);
  const float best_dist_normed = std::acos(std::min(kDistNorm * best_dist, 1.0f));
  if (best_dist_normed > max_distance) return false;
  const float second_best_dist_normed =
      std::acos(std::min(kDistNorm * second_best_dist, 1.0f));
  return !(best_dist_normed >= max_ratio * second_best_dist_normed);
}

// FindBestMatchesOneWay over a ColMajor rows x cols int matrix (element (r, c)
// at c * rows + r).
size_t find_best_matches_one_way(const std::vector<int32_t>& colmajor,
                                 int64_t rows, int64_t cols, float max_ratio,
                                 float max_distance, std::vector<int>* matches) {
  size_t num_matches = 0;
  matches->assign((size_t)rows, -1);
  for (int64_t i1 = 0; i1 < rows; ++i1) {
    int best_i2 = -1;
    int best_dist = 0;
    int second_best_dist = 0;
    for (int64_t i2 = 0; i2 < cols; ++i2) {
      const int dist = colmajor[(size_t)i2 * rows + i1];
      if (dist > best_dist) {
        best_i2 = (int)i2;
        second_best_dist = best_dist;
        best_dist = dist;
      } else if (dist > second_best_dist) {
        second_best_dist = dist;
      }
    }
    if (best_i2 == -1) continue;
    if (!passes_ratio_test(best_dist, second_best_dist, max_ratio, max_distance)) continue;
    num_matches += 1;
    (*matches)[(size_t)i1] = best_i2;
  }
  return num_matches;
}

// MatchSiftFeaturesCPU: dists (RowMajor) -> const Eigen::MatrixXi (ColMajor
// copy) -> FindBestMatches(cross_check): one pass on dists, one on the
// materialised transpose.
void match_sift_features_cpu(const scm_matching_options& o, const uint8_t* d1,
                             int64_t n1, const uint8_t* d2, int64_t n2,
                             std::vector<Match>* out) {
  out->clear();
  std::vector<int32_t> rowmajor;
  compute_sift_distance_matrix(d1, n1, d2, n2, &rowmajor);
  // const Eigen::MatrixXi dists = <RowMajor>  : ColMajor copy.
  std::vector<int32_t> dists((size_t)n1 * n2);
  for (int64_t i1 = 0; i1 < n1; ++i1)
    for (int64_t i2 = 0; i2 < n2; ++i2)
      dists[(size_t)i2 * n1 + i1] = rowmajor[(size_t)i1 * n2 + i2];
  std::vector<int32_t>().swap(rowmajor);
  const float max_ratio = (float)o.max_ratio;
  const float max_distance = (float)o.max_distance;
  std::vector<int> m12;
  find_best_matches_one_way(dists, n1, n2, max_ratio, max_distance, &m12);
  if (o.cross_check) {
    // dists.transpose() bound to const MatrixXi&: materialised ColMajor copy.
    std::vector<int32_t> dt((size_t)n1 * n2);
    for (int64_t i2 = 0; i2 < n2; ++i2)
      for (int64_t i1 = 0; i1 < n1; ++i1)
        dt[(size_t)i1 * n2 + i2] = dists[(size_t)i2 * n1 + i1];
    std::vector<int> m21;
    find_best_matches_one_way(dt, n2, n1, max_ratio, max_distance, &m21);
    for (size_t i1 = 0; i1 < m12.size(); ++i1) {
      if (m12[i1] != -1 && m21[(size_t)m12[i1]] != -1 &&
          m21[(size_t)m12[i1]] == (int)i1)
        out->push_back({(uint32_t)i1, (uint32_t)m12[i1]});
    }
  } else {
    for (size_t i1 = 0; i1 < m12.size(); ++i1)
      if (m12[i1] != -1) out->push_back({(uint32_t)i1, (uint32_t)m12[i1]});
  }
}

// FindBestMatches on a precomputed RowMajor dot matrix (test support: the
// tests compute the exact integer dots with a float32 BLAS product, every
// partial sum being an integer below 2^24).  The decisions are those of
// find_best_matches_one_way on dists and on dists.transpose(); only the loop
// order differs: the column scans of the transposed pass run as per-column
// state updated row by row, so each column still visits i1 in ascending
// order (same ties, same "second"), without the two 256 MiB copies.
void match_from_rowmajor_dots(const scm_matching_options& o, const int32_t* d,
                              int64_t n1, int64_t n2, std::vector<Match>* out) {
  out->clear();
  const float max_ratio = (float)o.max_ratio;
  const float max_distance = (float)o.max_distance;
  std::vector<int> m12((size_t)n1, -1), m21((size_t)n2, -1);
  std::vector<int> cbest((size_t)n2, 0), csecond((size_t)n2, 0), cidx((size_t)n2, -1);
  for (int64_t i1 = 0; i1 < n1; ++i1) {
    const int32_t* row = d + (size_t)i1 * n2;
    int best_i2 = -1, best_dist = 0, second_best_dist = 0;
    for (int64_t i2 = 0; i2 < n2; ++i2) {
      const int dist = row[i2];
      if (dist > best_dist) {
        best_i2 = (int)i2;
        second_best_dist = best_dist;
        best_dist = dist;
      } else if (dist > second_best_dist) {
        second_best_dist = dist;
      }
      if (dist > cbest[(size_t)i2]) {
        cidx[(size_t)i2] = (int)i1;
        csecond[(size_t)i2] = cbest[(size_t)i2];
        cbest[(size_t)i2] = dist;
      } else if (dist > csecond[(size_t)i2]) {
        csecond[(size_t)i2] = dist;
      }
    }
    if (best_i2 != -1 &&
        passes_ratio_test(best_dist, second_best_dist, max_ratio, max_distance))
      m12[(size_t)i1] = best_i2;
  }
  for (int64_t i2 = 0; i2 < n2; ++i2)
    if (cidx[(size_t)i2] != -1 &&
        passes_ratio_test(cbest[(size_t)i2], csecond[(size_t)i2], max_ratio, max_distance))
      m21[(size_t)i2] = cidx[(size_t)i2];
  for (size_t i1 = 0; i1 < m12.size(); ++i1) {
    if (m12[i1] == -1) continue;
    if (o.cross_check && m21[(size_t)m12[i1]] != (int)i1) continue;
    out->push_back({(uint32_t)i1, (uint32_t)m12[i1]});
  }
}

// ===========================================================================
// Geometry (a8-a14): LO-RANSAC restatement.
// ===========================================================================

struct Support {
  size_t num_inliers = 0;
  double residual_sum = DBL_MAX;
};

// InlierSupportMeasurer::Evaluate / Compare [upstream optim/support_measurement.cc]
Support evaluate(const std::vector<double>& r, double max_residual) {
  Support s;
  s.num_inliers = 0;
  s.residual_sum = 0;
  for (double x : r)
    if (x <= max_residual) {
      s.num_inliers += 1;
      s.residual_sum += x;
    }
  return s;
}
bool compare(const Support& a, const Support& b) {
  if (a.num_inliers > b.num_inliers) return true;
  return a.num_inliers == b.num_inliers && a.residual_sum < b.residual_sum;
}

// RANSAC::ComputeNumTrials [upstream optim/ransac.h]: the shared
// basic-operation evaluation (geom_solvers.h num_trials, see its header for
// the documented deviation from libm pow/log).
size_t compute_num_trials(size_t num_inliers, size_t num_samples,
                          double confidence, double multiplier, int kmin) {
  return (size_t)scm::geom::num_trials(num_inliers, num_samples, confidence,
                                       multiplier, kmin);
}

// The RANSAC constructor's cap on max_num_trials [upstream optim/ransac.h]:
// ComputeNumTrials(min_inlier_ratio * 1e5, 1e5) with the host libm
// (std::pow, std::log, std::ceil) and static_cast<size_t> as gcc emits it on
// x86-64 for out-of-range values.
size_t constructor_num_trials(double min_inlier_ratio, double confidence, double multiplier,
                              int kmin) {
  auto cast = [](double v) -> size_t {
    if (!(v < 9223372036854775808.0)) {
      if (!(v < 18446744073709551616.0)) return v == v ? 0 : (size_t)1 << 63;
      return (size_t)(int64_t)(v - 9223372036854775808.0) ^ ((size_t)1 << 63);
    }
    if (!(v > -9223372036854775808.0)) return (size_t)1 << 63;
    return (size_t)(int64_t)v;
  };
  const size_t kNumSamples = 100000;
  const size_t num_inliers = cast(min_inlier_ratio * kNumSamples);
  const double inlier_ratio = num_inliers / static_cast<double>(kNumSamples);
  const double nom = 1 - confidence;
  if (nom <= 0) return std::numeric_limits<size_t>::max();
  const double denom = 1 - std::pow(inlier_ratio, kmin);
  if (denom <= 0) return 1;
  return cast(std::ceil(std::log(nom) / std::log(denom) * multiplier));
}

using Model = std::vector<double>;  // 9 (F, H) or 2 (translation) doubles

// Estimator policies.  kind: 0 = F (7-pt min / 8-pt local), 1 = H, 2 = T.
struct Problem {
  const std::vector<double>* x1;  // interleaved x,y
  const std::vector<double>* x2;
  int kind;
};

int min_samples(int kind, bool local) {
  if (kind == 0) return local ? 8 : 7;
  if (kind == 1) return 4;
  return 1;
}

std::vector<Model> estimate(int kind, bool local, const std::vector<double>& a,
                            const std::vector<double>& b) {
  const int n = (int)(a.size() / 2);
  std::vector<Model> out;
  if (kind == 0 && !local) {
    double models[27];
    const int nm = fundamental_7pt(a.data(), b.data(), models);
    for (int k = 0; k < nm; ++k) out.emplace_back(models + 9 * k, models + 9 * k + 9);
  } else if (kind == 0) {
    Model F(9);
    scm::geom::fundamental_8pt(a.data(), b.data(), n, F.data());
    out.push_back(F);
  } else if (kind == 1) {
    Model H(9);
    scm::geom::homography_dlt(a.data(), b.data(), n, H.data());
    out.push_back(H);
  } else {
    Model t(2);
    scm::geom::translation_estimate(a.data(), b.data(), n, t.data());
    out.push_back(t);
  }
  return out;
}

void residuals(int kind, const std::vector<double>& x1,
               const std::vector<double>& x2, const Model& m,
               std::vector<double>* r) {
  const size_t n = x1.size() / 2;
  r->resize(n);
  for (size_t i = 0; i < n; ++i) {
    const double a0 = x1[2 * i], a1 = x1[2 * i + 1];
    const double b0 = x2[2 * i], b1 = x2[2 * i + 1];
    if (kind == 0)
      (*r)[i] = scm::geom::sampson_sq(m.data(), a0, a1, b0, b1);
    else if (kind == 1)
      (*r)[i] = scm::geom::homography_sq(m.data(), a0, a1, b0, b1);
    else
      (*r)[i] = scm::geom::translation_sq(m.data(), a0, a1, b0, b1);
  }
}

struct RansacOptions {
  double max_error;
  double min_inlier_ratio;
  double confidence;
  double dyn_num_trials_multiplier;
  size_t min_num_trials;
  size_t max_num_trials;
};

struct Report {
  bool success = false;
  size_t num_trials = 0;
  Support support;
  Model model;
  std::vector<char> inlier_mask;
};

// Shuffle [upstream util/random.h] with RandomInteger<uint32_t> =
// std::uniform_int_distribution<uint32_t>(i, last) over the shared PRNG.
void shuffle_prefix(uint32_t num_to_shuffle, std::vector<uint32_t>* elems,
                    std::mt19937* prng) {
  const uint32_t last_idx = (uint32_t)(elems->size() - 1);
  for (uint32_t i = 0; i < num_to_shuffle; ++i) {
    std::uniform_int_distribution<uint32_t> dist(i, last_idx);
    const uint32_t j = dist(*prng);
    std::swap((*elems)[i], (*elems)[j]);
  }
}

// LORANSAC<Estimator, LocalEstimator>::Estimate [upstream optim/loransac.h],
// recursive local optimisation (at most 10 local iterations while the inlier
// count grows), dynamic trial count, early abort inside the model loop.
Report loransac(int kind, const RansacOptions& opt_in,
                const std::vector<double>& X, const std::vector<double>& Y,
                std::mt19937* prng) {
  const int kmin = min_samples(kind, false);
  const int kmin_local = min_samples(kind, true);
  RansacOptions opt = opt_in;
  opt.max_num_trials = std::min<size_t>(
      opt.max_num_trials, constructor_num_trials(opt.min_inlier_ratio, opt.confidence,
                                                 opt.dyn_num_trials_multiplier, kmin));
  Report report;
  const size_t num_samples = X.size() / 2;
  if (num_samples < (size_t)kmin) return report;

  Support best_support;
  Model best_model;
  bool best_model_is_local = false;
  bool abort = false;
  const double max_residual = opt.max_error * opt.max_error;
  std::vector<double> res, best_local_res;
  std::vector<double> X_rand(2 * kmin), Y_rand(2 * kmin);
  std::vector<uint32_t> sample_idxs(num_samples);
  for (size_t i = 0; i < num_samples; ++i) sample_idxs[i] = (uint32_t)i;

  // RandomSampler::MaxNumSamples() is unbounded.
  const size_t max_num_trials = opt.max_num_trials;
  size_t dyn_max_num_trials = max_num_trials;

  for (report.num_trials = 0; report.num_trials < max_num_trials;
       ++report.num_trials) {
    if (abort) {
      report.num_trials += 1;
      break;
    }
    shuffle_prefix((uint32_t)kmin, &sample_idxs, prng);
    for (int i = 0; i < kmin; ++i) {
      const uint32_t s = sample_idxs[(size_t)i];
      X_rand[2 * i] = X[2 * s];
      X_rand[2 * i + 1] = X[2 * s + 1];
      Y_rand[2 * i] = Y[2 * s];
      Y_rand[2 * i + 1] = Y[2 * s + 1];
    }
    const std::vector<Model> sample_models = estimate(kind, false, X_rand, Y_rand);
    for (const Model& sample_model : sample_models) {
      residuals(kind, X, Y, sample_model, &res);
      const Support support = evaluate(res, max_residual);
      if (compare(support, best_support)) {
        best_support = support;
        best_model = sample_model;
        best_model_is_local = false;
        if (support.num_inliers > (size_t)kmin &&
            support.num_inliers >= (size_t)kmin_local) {
          const size_t kMaxNumLocalTrials = 10;
          for (size_t lt = 0; lt < kMaxNumLocalTrials; ++lt) {
            std::vector<double> Xi, Yi;
            Xi.reserve(2 * num_samples);
            Yi.reserve(2 * num_samples);
            for (size_t i = 0; i < res.size(); ++i)
              if (res[i] <= max_residual) {
                Xi.push_back(X[2 * i]);
                Xi.push_back(X[2 * i + 1]);
                Yi.push_back(Y[2 * i]);
                Yi.push_back(Y[2 * i + 1]);
              }
            const std::vector<Model> local_models = estimate(kind, true, Xi, Yi);
            const size_t prev_best_num_inliers = best_support.num_inliers;
            for (const Model& local_model : local_models) {
              residuals(kind, X, Y, local_model, &res);
              const Support local_support = evaluate(res, max_residual);
              if (compare(local_support, best_support)) {
                best_support = local_support;
                best_model = local_model;
                best_model_is_local = true;
                std::swap(res, best_local_res);
              }
            }
            if (best_support.num_inliers <= prev_best_num_inliers) break;
            std::swap(res, best_local_res);
          }
        }
        dyn_max_num_trials = compute_num_trials(
            best_support.num_inliers, num_samples, opt.confidence,
            opt.dyn_num_trials_multiplier, kmin);
      }
      if (report.num_trials >= dyn_max_num_trials &&
          report.num_trials >= opt.min_num_trials) {
        abort = true;
        break;
      }
    }
  }

  report.support = best_support;
  report.model = best_model;
  if (report.support.num_inliers < (size_t)kmin) return report;
  report.success = true;
  residuals(kind, X, Y, report.model, &res);
  (void)best_model_is_local;  // same residual function for both estimators
  report.inlier_mask.resize(num_samples);
  for (size_t i = 0; i < res.size(); ++i)
    report.inlier_mask[i] = res[i] <= max_residual;
  return report;
}

struct TVG {
  int32_t config = SCM_TVG_UNDEFINED;
  double F[9] = {0}, H[9] = {0};  // row-major
  std::vector<Match> inlier_matches;
  double tri_angle = 0;
};

RansacOptions ransac_options(const scm_matching_options& o) {
  RansacOptions r;
  r.max_error = (double)o.max_error;
  r.min_inlier_ratio = o.min_inlier_ratio;
  r.confidence = o.confidence;
  r.dyn_num_trials_multiplier = o.dyn_num_trials_multiplier;
  r.min_num_trials = (size_t)o.min_num_trials;
  r.max_num_trials = (size_t)o.max_num_trials;
  return r;
}

// TwoViewGeometry::DetectWatermark with the reference's dummy cameras
// (width = height = 0, sequential_matching.cc:88-89).
bool detect_watermark(const scm_matching_options& o, const std::vector<double>& p1,
                      const std::vector<double>& p2, size_t num_inliers,
                      const std::vector<char>& mask, std::mt19937* prng) {
  const double diagonal1 = std::sqrt(0.0), diagonal2 = std::sqrt(0.0);
  const double minx1 = o.watermark_border_size * diagonal1, miny1 = minx1;
  const double maxx1 = 0.0 - minx1, maxy1 = 0.0 - miny1;
  const double minx2 = o.watermark_border_size * diagonal2, miny2 = minx2;
  const double maxx2 = 0.0 - minx2, maxy2 = 0.0 - miny2;
  std::vector<double> ip1(2 * num_inliers), ip2(2 * num_inliers);
  size_t in_border = 0, j = 0;
  for (size_t i = 0; i < mask.size(); ++i) {
    if (!mask[i]) continue;
    ip1[2 * j] = p1[2 * i];
    ip1[2 * j + 1] = p1[2 * i + 1];
    ip2[2 * j] = p2[2 * i];
    ip2[2 * j + 1] = p2[2 * i + 1];
    j += 1;
    const bool in1 = p1[2 * i] >= minx1 && p1[2 * i] <= maxx1 &&
                     p1[2 * i + 1] >= miny1 && p1[2 * i + 1] <= maxy1;
    const bool in2 = p2[2 * i] >= minx2 && p2[2 * i] <= maxx2 &&
                     p2[2 * i + 1] >= miny2 && p2[2 * i + 1] <= maxy2;
    if (!in1 && !in2) in_border += 1;
  }
  const double ratio = static_cast<double>(in_border) / num_inliers;
  if (ratio < o.watermark_min_inlier_ratio) return false;
  RansacOptions ro = ransac_options(o);
  ro.min_inlier_ratio = o.watermark_min_inlier_ratio;
  const Report rep = loransac(2, ro, ip1, ip2, prng);
  const double inlier_ratio = static_cast<double>(rep.support.num_inliers) / num_inliers;
  return inlier_ratio >= o.watermark_min_inlier_ratio;
}

// verifyTwoViewGeometry (sequential_matching.cc:84-101) -> Estimate ->
// EstimateUncalibrated (dummy cameras have no prior focal length); the op's
// post-filter is verify_pair_filtered below.
TVG verify_pair(const scm_matching_options& o, const float* kp1, const float* kp2,
                const std::vector<Match>& matches, uint32_t id1, uint32_t id2,
                uint32_t iteration = 0) {
  TVG tvg;
  // Two PRNG streams per pair: F from pair_seed, H (then the watermark
  // RANSAC) from pair_seed_h (geom_solvers.h; the reference's single
  // thread-local generator is time-seeded, so either is a realisation of it).
  // Estimate number `iteration` of EstimateMultiple starts from
  // geom::iteration_seed (0: the plain Estimate).
  const uint32_t base = scm::geom::iteration_seed(o.ransac_seed, iteration);
  std::mt19937 prng(oracle_pair_seed(base, id1, id2));
  std::mt19937 prng_h(oracle_pair_seed(base ^ 0x6A09E667u, id1, id2));
  const size_t min_num_inliers = (size_t)o.min_num_inliers;
  if (matches.size() < min_num_inliers) {
    tvg.config = SCM_TVG_DEGENERATE;
  } else {
    // FeatureKeypointsToPointsVector: float x, y -> Eigen::Vector2d.
    std::vector<double> p1(2 * matches.size()), p2(2 * matches.size());
    for (size_t i = 0; i < matches.size(); ++i) {
      p1[2 * i] = (double)kp1[6 * (size_t)matches[i].idx1];
      p1[2 * i + 1] = (double)kp1[6 * (size_t)matches[i].idx1 + 1];
      p2[2 * i] = (double)kp2[6 * (size_t)matches[i].idx2];
      p2[2 * i + 1] = (double)kp2[6 * (size_t)matches[i].idx2 + 1];
    }
    const RansacOptions ro = ransac_options(o);
    const Report F_report = loransac(0, ro, p1, p2, &prng);
    if (!F_report.model.empty()) std::copy(F_report.model.begin(), F_report.model.end(), tvg.F);
    const Report H_report = loransac(1, ro, p1, p2, &prng_h);
    if (!H_report.model.empty()) std::copy(H_report.model.begin(), H_report.model.end(), tvg.H);
    if ((!F_report.success && !H_report.success) ||
        (F_report.support.num_inliers < min_num_inliers &&
         H_report.support.num_inliers < min_num_inliers)) {
      tvg.config = SCM_TVG_DEGENERATE;
    } else {
      const double H_F_inlier_ratio =
          static_cast<double>(H_report.support.num_inliers) /
          F_report.support.num_inliers;
      tvg.config = H_F_inlier_ratio > o.max_H_inlier_ratio
                       ? SCM_TVG_PLANAR_OR_PANORAMIC
                       : SCM_TVG_UNCALIBRATED;
      // ExtractInlierMatches (an unsuccessful F report has no mask: no inliers).
      if (F_report.success)
        for (size_t i = 0; i < matches.size(); ++i)
          if (F_report.inlier_mask[i]) tvg.inlier_matches.push_back(matches[i]);
      if (o.detect_watermark && F_report.success &&
          detect_watermark(o, p1, p2, F_report.support.num_inliers,
                           F_report.inlier_mask, &prng_h))
        tvg.config = SCM_TVG_WATERMARK;
    }
  }
  return tvg;
}

// TwoViewGeometry::EstimateMultiple [upstream estimators/two_view_geometry.cc],
// taken when multiple_models is set (sequential_matching.cc:94-96):
// Estimate on the remaining matches until it is DEGENERATE, keeping every
// geometry except WATERMARK ones (Options::multiple_ignore_watermark, default
// true), the remaining matches being ExtractOutlierMatches(remaining,
// inlier_matches); one kept geometry is the result, several give MULTIPLE
// with their inlier matches concatenated (F, H unset: zeros), none gives
// DEGENERATE.  Estimate k draws from the iteration-k seeds.  (The reference
// would loop forever on a non-degenerate Estimate without inlier matches;
// the loop stops there.)
TVG verify_pair_multiple(const scm_matching_options& o, const float* kp1, const float* kp2,
                         const std::vector<Match>& matches, uint32_t id1, uint32_t id2) {
  std::vector<Match> remaining = matches;
  std::vector<TVG> kept;
  for (uint32_t k = 0;; ++k) {
    const TVG g = verify_pair(o, kp1, kp2, remaining, id1, id2, k);
    if (g.config == SCM_TVG_DEGENERATE) break;
    if (g.config != SCM_TVG_WATERMARK) kept.push_back(g);
    if (g.inlier_matches.empty()) break;
    std::vector<Match> out;  // ExtractOutlierMatches (matches are unique pairs)
    size_t j = 0;
    for (const Match& m : remaining) {
      if (j < g.inlier_matches.size() && g.inlier_matches[j].idx1 == m.idx1 &&
          g.inlier_matches[j].idx2 == m.idx2)
        ++j;  // the inlier matches are a subsequence of `remaining`
      else
        out.push_back(m);
    }
    remaining.swap(out);
  }
  TVG tvg;
  if (kept.empty()) {
    tvg.config = SCM_TVG_DEGENERATE;
  } else if (kept.size() == 1) {
    tvg = kept[0];
  } else {
    tvg.config = SCM_TVG_MULTIPLE;
    for (const TVG& g : kept)
      tvg.inlier_matches.insert(tvg.inlier_matches.end(), g.inlier_matches.begin(),
                                g.inlier_matches.end());
  }
  return tvg;
}

// verifyTwoViewGeometry (Estimate, or EstimateMultiple with multiple_models)
// followed by the op's post-filter (sequential_matching.cc:173-178): too few
// inliers -> TwoViewGeometry() (config 0, zero models).
TVG verify_pair_filtered(const scm_matching_options& o, const float* kp1, const float* kp2,
                         const std::vector<Match>& matches, uint32_t id1, uint32_t id2) {
  TVG tvg = o.multiple_models ? verify_pair_multiple(o, kp1, kp2, matches, id1, id2)
                              : verify_pair(o, kp1, kp2, matches, id1, id2);
  if (tvg.inlier_matches.size() < (size_t)o.min_num_inliers) tvg = TVG();
  return tvg;
}

// ===========================================================================
// io.cc codecs (reference integration/op_cpp/io.cc).
// ===========================================================================

template <typename T>
void put(std::vector<uint8_t>* b, const T& v) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
  b->insert(b->end(), p, p + sizeof(T));
}

// Per-TVG layout of create_two_view_geometries_buffer (io.cc:279-292):
// int config, E, F, H (Eigen::Matrix3d, column-major), qvec[4], tvec[3],
// tri_angle, size_t n, n x FeatureMatch{uint32, uint32}.  E/qvec/tvec are
// never written by EstimateUncalibrated; they are emitted as zeros.
void put_tvg(std::vector<uint8_t>* b, const TVG& t) {
  put<int32_t>(b, t.config);
  for (int i = 0; i < 9; ++i) put<double>(b, 0.0);
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) put<double>(b, t.F[3 * r + c]);
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) put<double>(b, t.H[3 * r + c]);
  for (int i = 0; i < 7; ++i) put<double>(b, 0.0);
  put<double>(b, t.tri_angle);
  put<uint64_t>(b, (uint64_t)t.inlier_matches.size());
  for (const Match& m : t.inlier_matches) {
    put<uint32_t>(b, m.idx1);
    put<uint32_t>(b, m.idx2);
  }
}

// create_two_view_geometries_buffer (io.cc:256-297): size_t total, int count.
std::vector<uint8_t> tvg_list_blob(const std::vector<TVG>& list) {
  std::vector<uint8_t> body;
  for (const TVG& t : list) put_tvg(&body, t);
  std::vector<uint8_t> b;
  const uint64_t total = sizeof(uint64_t) + sizeof(int32_t) + body.size();
  put<uint64_t>(&b, total);
  put<int32_t>(&b, (int32_t)list.size());
  b.insert(b.end(), body.begin(), body.end());
  return b;
}

// createVectorBuffer (io.cc:151-162) for vector<image_t>.
std::vector<uint8_t> id_list_blob(const std::vector<uint32_t>& ids) {
  std::vector<uint8_t> b;
  put<uint64_t>(&b, (uint64_t)ids.size());
  for (uint32_t id : ids) put<uint32_t>(&b, id);
  return b;
}

struct Row {
  uint32_t id = 0;
  const float* kp = nullptr;
  int64_t nkp = 0;
  const uint8_t* desc = nullptr;
  int64_t ndesc = 0;
};

bool decode_row(const scm_element& id, const scm_element& kp,
                const scm_element& desc, Row* r) {
  // read_single_from_element<image_t> (io.cc:67-69): low 4 bytes of size_t.
  if (id.size < 4 || kp.size < 8 || desc.size < 16) return false;
  std::memcpy(&r->id, id.buffer, 4);
  uint64_t n;
  std::memcpy(&n, kp.buffer, 8);
  if (kp.size < 8 + n * 24) return false;
  r->nkp = (int64_t)n;
  r->kp = reinterpret_cast<const float*>(kp.buffer + 8);
  uint64_t rows, cols;
  std::memcpy(&rows, desc.buffer, 8);
  std::memcpy(&cols, desc.buffer + 8, 8);
  if (cols != 128 || desc.size < 16 + rows * cols) return false;
  r->ndesc = (int64_t)rows;
  r->desc = desc.buffer + 16;
  return true;
}

uint8_t* to_heap(const std::vector<uint8_t>& v, size_t* size) {
  uint8_t* p = (uint8_t*)std::malloc(v.size() ? v.size() : 1);
  if (!v.empty()) std::memcpy(p, v.data(), v.size());
  *size = v.size();
  return p;
}

// SequentialMatchingCPUKernel::execute (sequential_matching.cc:103-185).
bool execute_rows(const scm_matching_options& o, const std::vector<Row>& st,
                  std::vector<uint8_t>* ids_blob, std::vector<uint8_t>* tvg_blob) {
  const Row& pivot = st[0];
  std::vector<uint32_t> pair_ids;
  std::vector<TVG> tvgs;
  for (size_t i = 1; i < st.size(); ++i) {
    const uint32_t id2 = st[i].id;
    if (id2 == pivot.id ||
        std::count(pair_ids.begin(), pair_ids.end(), id2) > 0)
      continue;
    pair_ids.push_back(id2);
    std::vector<Match> matches;
    match_sift_features_cpu(o, pivot.desc, pivot.ndesc, st[i].desc, st[i].ndesc,
                            &matches);
    tvgs.push_back(verify_pair_filtered(o, pivot.kp, st[i].kp, matches, pivot.id, id2));
  }
  *ids_blob = id_list_blob(pair_ids);
  *tvg_blob = tvg_list_blob(tvgs);
  return true;
}

}  // namespace

// ===========================================================================
// C API (ctypes: tests/, bench.py cpu_baseline, __graft_entry__.smoke()).
// ===========================================================================
extern "C" {

// Reference-semantics options defaults (colmap.proto:6-65 + COLMAP defaults).
// Deliberately independent of the product's scm_default_options.
void oracle_default_options(scm_matching_options* o) {
  std::memset(o, 0, sizeof(*o));
  o->use_gpu = 0;
  o->gpu_index = -1;
  o->max_ratio = 0.8;
  o->max_distance = 0.7;
  o->cross_check = 1;
  o->max_num_matches = 32768;
  o->max_error = 4.0f;
  o->confidence = 0.999;
  o->min_num_trials = 30;
  o->max_num_trials = 10000;
  o->min_inlier_ratio = 0.25;
  o->min_num_inliers = 15;
  o->multiple_models = 0;
  o->guided_matching = 0;
  o->loop_detection = 0;
  o->overlap = 10;
  o->quadratic_overlap = 0;
  o->min_E_F_inlier_ratio = 0.95;
  o->max_H_inlier_ratio = 0.8;
  o->watermark_min_inlier_ratio = 0.7;
  o->watermark_border_size = 0.1;
  o->detect_watermark = 1;
  o->dyn_num_trials_multiplier = 3.0;
  o->ransac_seed = 0;
}

// Per-pair RANSAC seed: the definition include/scm.h documents for
// scm_pair_seed, restated here so the oracle links without the product.
uint32_t oracle_pair_seed(uint32_t base, uint32_t id1, uint32_t id2) {
  uint32_t h = base ^ 0x9E3779B9u;
  h ^= id1 + 0x7F4A7C15u + (h << 6) + (h >> 2);
  h ^= id2 + 0x85EBCA77u + (h << 6) + (h >> 2);
  return h;
}

// ComputeNumTrials as the oracle evaluates it (test support: the
// libm-free restatement is compared with std::log/std::pow in tests).
uint64_t oracle_num_trials(uint64_t num_inliers, uint64_t num_samples,
                           double confidence, double multiplier, int32_t kmin) {
  return (uint64_t)compute_num_trials(num_inliers, num_samples, confidence,
                                      multiplier, kmin);
}

// Least-squares null vector of a packed 9 x 9 normal matrix (45 entries) as
// the LO estimators compute it (geom_solvers.h ata_null_vector).
void oracle_ata_null_vector(const double* ata45, double* out9) {
  scm::geom::ata_null_vector(ata45, out9);
}

// The shared estimator arithmetic (geom_solvers.h, compiled into the product
// and into this oracle) exposed for the independent numpy restatement of
// COLMAP's SVD / companion-matrix formulation (tests/test_estimators_independent.py).
int oracle_fundamental_7pt(const double* x1, const double* x2, double* models27) {
  return scm::geom::fundamental_7pt(x1, x2, models27);
}
int oracle_fundamental_8pt(const double* x1, const double* x2, int32_t n, double* F9) {
  return scm::geom::fundamental_8pt(x1, x2, n, F9);
}
int oracle_homography_dlt(const double* x1, const double* x2, int32_t n, double* H9) {
  return scm::geom::homography_dlt(x1, x2, n, H9);
}

int oracle_match_pair(const scm_matching_options* o, const uint8_t* d1,
                      int64_t n1, const uint8_t* d2, int64_t n2,
                      uint32_t* out, int64_t cap, int64_t* m) {
  std::vector<Match> matches;
  match_sift_features_cpu(*o, d1, n1, d2, n2, &matches);
  *m = (int64_t)matches.size();
  if ((int64_t)matches.size() > cap) return SCM_E_CAPACITY;
  for (size_t i = 0; i < matches.size(); ++i) {
    out[2 * i] = matches[i].idx1;
    out[2 * i + 1] = matches[i].idx2;
  }
  return SCM_OK;
}

// FindBestMatches on an exact RowMajor int32 dot matrix (test support, see
// match_from_rowmajor_dots).
int oracle_match_from_dots(const scm_matching_options* o, const int32_t* dots,
                           int64_t n1, int64_t n2, uint32_t* out, int64_t cap,
                           int64_t* m) {
  std::vector<Match> matches;
  match_from_rowmajor_dots(*o, dots, n1, n2, &matches);
  *m = (int64_t)matches.size();
  if ((int64_t)matches.size() > cap) return SCM_E_CAPACITY;
  for (size_t i = 0; i < matches.size(); ++i) {
    out[2 * i] = matches[i].idx1;
    out[2 * i + 1] = matches[i].idx2;
  }
  return SCM_OK;
}

// One-way best / second / argmax per row of A against B (test support):
// FindBestMatchesOneWay's scan state before the ratio / distance tests.
int oracle_row_top2(const uint8_t* d1, int64_t n1, const uint8_t* d2, int64_t n2,
                    int32_t* best, int32_t* second, int32_t* best_idx) {
  for (int64_t i1 = 0; i1 < n1; ++i1) {
    int b = 0, s = 0, bi = -1;
    for (int64_t i2 = 0; i2 < n2; ++i2) {
      int dot = 0;
      for (int d = 0; d < 128; ++d) dot += (int)d1[i1 * 128 + d] * (int)d2[i2 * 128 + d];
      if (dot > b) {
        bi = (int)i2;
        s = b;
        b = dot;
      } else if (dot > s) {
        s = dot;
      }
    }
    best[i1] = b;
    second[i1] = s;
    best_idx[i1] = bi;
  }
  return SCM_OK;
}

float oracle_acosf_normed(int32_t d) {
  const float kDistNorm = 1.0f / (512.0f * 512.0f);
  return std::acos(std::min(kDistNorm * d, 1.0f));
}

int oracle_verify_pair(const scm_matching_options* o, const float* kp1,
                       int64_t n1, const float* kp2, int64_t n2,
                       const uint32_t* matches, int64_t m, uint32_t id1,
                       uint32_t id2, uint8_t** blob, size_t* size) {
  (void)n1;
  (void)n2;
  std::vector<Match> mm((size_t)m);
  for (int64_t i = 0; i < m; ++i) mm[(size_t)i] = {matches[2 * i], matches[2 * i + 1]};
  const TVG t = verify_pair_filtered(*o, kp1, kp2, mm, id1, id2);
  std::vector<uint8_t> b;
  put_tvg(&b, t);
  *blob = to_heap(b, size);
  return SCM_OK;
}

// The configuration EstimateUncalibrated / DetectWatermark decide BEFORE the
// op's post-filter, and the number of F-inlier matches (test support: shows
// which branch a scene takes even when the post-filter then empties the row,
// e.g. DEGENERATE with >= 15 matches).
int oracle_verify_pair_config(const scm_matching_options* o, const float* kp1,
                              const float* kp2, const uint32_t* matches, int64_t m,
                              uint32_t id1, uint32_t id2, int64_t* num_inliers) {
  std::vector<Match> mm((size_t)m);
  for (int64_t i = 0; i < m; ++i) mm[(size_t)i] = {matches[2 * i], matches[2 * i + 1]};
  const TVG t = verify_pair(*o, kp1, kp2, mm, id1, id2);
  *num_inliers = (int64_t)t.inlier_matches.size();
  return t.config;
}

// One LO-RANSAC run (kind 0 = F, 1 = H, 2 = translation) on explicit points
// with a fresh mt19937(seed): test support for the GPU replay.
int oracle_loransac(const scm_matching_options* o, int32_t kind,
                    const double* x1, const double* x2, int64_t n, uint32_t seed,
                    double* model, int64_t* num_inliers, double* residual_sum,
                    int64_t* num_trials, uint8_t* inlier_mask) {
  std::mt19937 prng(seed);
  std::vector<double> a(x1, x1 + 2 * n), b(x2, x2 + 2 * n);
  const Report r = loransac(kind, ransac_options(*o), a, b, &prng);
  for (size_t i = 0; i < r.model.size(); ++i) model[i] = r.model[i];
  *num_inliers = (int64_t)r.support.num_inliers;
  *residual_sum = r.support.residual_sum;
  *num_trials = (int64_t)r.num_trials;
  for (int64_t i = 0; i < n; ++i)
    inlier_mask[i] = r.success ? (uint8_t)r.inlier_mask[(size_t)i] : 0;
  return r.success ? 1 : 0;
}

// std::uniform_int_distribution<uint32_t>(lo[i], hi[i]) over std::mt19937(seed)
// (test support: pins the product's explicit sampler restatement).
int oracle_std_uniform(uint32_t seed, const uint32_t* lo, const uint32_t* hi,
                       int64_t n, uint32_t* out) {
  std::mt19937 prng(seed);
  for (int64_t i = 0; i < n; ++i) {
    std::uniform_int_distribution<uint32_t> d(lo[i], hi[i]);
    out[i] = d(prng);
  }
  return SCM_OK;
}

int oracle_execute_stencil(const scm_matching_options* o, int64_t k,
                           const scm_element* ids, const scm_element* kps,
                           const scm_element* descs, uint8_t** ids_out,
                           size_t* ids_size, uint8_t** tvg_out,
                           size_t* tvg_size) {
  std::vector<Row> st((size_t)k);
  for (int64_t i = 0; i < k; ++i)
    if (!decode_row(ids[i], kps[i], descs[i], &st[(size_t)i])) return SCM_E_INVALID;
  std::vector<uint8_t> a, b;
  execute_rows(*o, st, &a, &b);
  *ids_out = to_heap(a, ids_size);
  *tvg_out = to_heap(b, tvg_size);
  return SCM_OK;
}

// Scanner stencil range(0, overlap) over a table (feature_matching.py:43):
// row i sees rows i .. i+overlap-1, clamped to the last row.
int oracle_table_run(const scm_matching_options* o, int64_t num_rows,
                     const scm_element* ids, const scm_element* kps,
                     const scm_element* descs, int64_t overlap,
                     int64_t row_begin, int64_t row_end, uint8_t** ids_out,
                     size_t* ids_sizes, uint8_t** tvg_out, size_t* tvg_sizes) {
  std::vector<Row> rows((size_t)num_rows);
  for (int64_t i = 0; i < num_rows; ++i)
    if (!decode_row(ids[i], kps[i], descs[i], &rows[(size_t)i])) return SCM_E_INVALID;
  for (int64_t r = row_begin; r < row_end; ++r) {
    std::vector<Row> st;
    for (int64_t s = 0; s < overlap; ++s)
      st.push_back(rows[(size_t)std::min(r + s, num_rows - 1)]);
    std::vector<uint8_t> a, b;
    execute_rows(*o, st, &a, &b);
    ids_out[r - row_begin] = to_heap(a, &ids_sizes[r - row_begin]);
    tvg_out[r - row_begin] = to_heap(b, &tvg_sizes[r - row_begin]);
  }
  return SCM_OK;
}

void oracle_free(uint8_t* p) { std::free(p); }

}  // extern "C"
