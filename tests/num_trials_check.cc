// Exhaustive check of geom::num_trials (scanner_colmap_amd/csrc/geom_solvers.h,
// the libm-free ComputeNumTrials the GPU's LO-RANSAC replay evaluates) against
// COLMAP's formula on the host libm [upstream optim/ransac.h ComputeNumTrials]:
//   ratio = num_inliers / (double)num_samples
//   nom   = 1 - confidence                      (<= 0 -> SIZE_MAX)
//   denom = 1 - std::pow(ratio, kMinNumSamples) (<= 0 -> 1)
//   trials = (size_t)std::ceil(std::log(nom) / std::log(denom) * multiplier)
// over every (num_inliers, num_samples) with 0 <= num_inliers <= num_samples
// <= NMAX.  Counts are compared after min(count, 2^31): the trial cap
// max_num_trials is an int, so a larger count can never bound the loop.
// usage: num_trials_check KMIN CONFIDENCE MULTIPLIER [NMAX]
// prints: "evals=N mismatches=M" and the first few mismatches.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

#include "../scanner_colmap_amd/csrc/geom_solvers.h"

static uint64_t colmap_num_trials(uint64_t ni, uint64_t ns, double conf, double mult, int kmin) {
  const double ratio = ni / static_cast<double>(ns);
  const double nom = 1 - conf;
  if (nom <= 0) return ~0ull;
  const double denom = 1 - std::pow(ratio, kmin);
  if (denom <= 0) return 1;
  const double v = std::ceil(std::log(nom) / std::log(denom) * mult);
  // static_cast<size_t> on x86-64 (cvttsd2si with the 2^63 split gcc emits)
  if (!(v >= 0.0)) return 1ull << 63;
  if (v >= 18446744073709551616.0) return 0;
  if (v >= 9223372036854775808.0) return ((uint64_t)(v - 9223372036854775808.0)) ^ (1ull << 63);
  return (uint64_t)v;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s KMIN CONFIDENCE MULTIPLIER [NMAX]\n", argv[0]);
    return 2;
  }
  const int kmin = std::atoi(argv[1]);
  const double conf = std::atof(argv[2]), mult = std::atof(argv[3]);
  const int64_t nmax = argc > 4 ? std::atoll(argv[4]) : 16384;
  const uint64_t cap = 1ull << 31;
  unsigned T = std::thread::hardware_concurrency();
  if (const char* e = std::getenv("OMP_NUM_THREADS")) T = (unsigned)std::atoi(e);
  T = T < 1 ? 1 : (T > 16 ? 16 : T);
  std::mutex mu;
  std::vector<std::vector<uint64_t>> bad;
  uint64_t nbad = 0, evals = 0;
  std::vector<std::thread> ts;
  for (unsigned t = 0; t < T; ++t)
    ts.emplace_back([&, t] {
      uint64_t lb = 0, le = 0;
      std::vector<std::vector<uint64_t>> mine;
      for (int64_t ns = 1 + t; ns <= nmax; ns += T)
        for (int64_t ni = 0; ni <= ns; ++ni) {
          ++le;
          uint64_t a = scm::geom::num_trials((uint64_t)ni, (uint64_t)ns, conf, mult, kmin);
          uint64_t b = colmap_num_trials((uint64_t)ni, (uint64_t)ns, conf, mult, kmin);
          a = a < cap ? a : cap;
          b = b < cap ? b : cap;
          if (a != b) {
            ++lb;
            if (mine.size() < 8) mine.push_back({(uint64_t)ni, (uint64_t)ns, a, b});
          }
        }
      std::lock_guard<std::mutex> g(mu);
      nbad += lb;
      evals += le;
      for (auto& m : mine)
        if (bad.size() < 8) bad.push_back(m);
    });
  for (auto& th : ts) th.join();
  std::printf("kmin=%d confidence=%.17g multiplier=%.17g nmax=%lld evals=%llu mismatches=%llu\n", kmin,
              conf, mult, (long long)nmax, (unsigned long long)evals, (unsigned long long)nbad);
  for (auto& m : bad)
    std::printf("  inliers=%llu samples=%llu product=%llu libm=%llu\n", (unsigned long long)m[0],
                (unsigned long long)m[1], (unsigned long long)m[2], (unsigned long long)m[3]);
  return nbad == 0 ? 0 : 1;
}
