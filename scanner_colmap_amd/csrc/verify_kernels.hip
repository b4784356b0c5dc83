// Kernel 2 of the sequential-matching stage: GPU-resident two-view geometry
// (replaces verifyTwoViewGeometry + colmap::TwoViewGeometry::Estimate +
// the op's post-filter, reference integration/op_cpp/sequential_matching.cc:
// 84-101 and 164-178; upstream EstimateUncalibrated).
//
// Every pair of a batch runs, in order and with the pair's own std::mt19937
// stream:
//   LO-RANSAC<7-pt F, 8-pt F>  ->  LO-RANSAC<4-pt H, N-pt H>
//   -> configuration -> DetectWatermark (LO-RANSAC<translation>) -> post-filter.
// F and H run as the windowed kernels below (rs_begin / rs_sample / rs_solve /
// rs_score / rs_replay: all pairs advance one window of W rounds of 64
// hypotheses at a time, scoring is one wide regular kernel, the sequential
// LO-RANSAC decisions are replayed per pair in trial order and hypotheses past
// the abort point are discarded with the PRNG rewound), the rest in
// verify_final_kernel (one wavefront per pair).  Residual sums are only needed
// when two inlier counts tie; they are then summed in index order, as
// InlierSupportMeasurer::Evaluate does.  Inlier tests run on packed fp32 with
// rigorous error bounds and fall back to the exact fp64 residual for every
// point the bound cannot decide.  The estimator arithmetic is the shared
// geom_solvers.h (the 9x9 Jacobi is its lane-distributed twin), so every model
// is bit-identical to the CPU oracle's.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <functional>
#include <mutex>

#include "../../include/scm.h"
#include "geom_solvers.h"
#include "verify_kernels.h"

namespace scm {

using namespace geom;

enum { KIND_F = 0, KIND_H = 1, KIND_T = 2 };

template <int K> struct KindTraits;
// tb: hypotheses per round of the sequential (watermark) LO-RANSAC.
template <> struct KindTraits<KIND_F> { static constexpr int kmin = 7, kmin_local = 8, mm = 3, ms = 9, tb = kTrialBatch; };
template <> struct KindTraits<KIND_H> { static constexpr int kmin = 4, kmin_local = 4, mm = 1, ms = 9, tb = kTrialBatch; };
template <> struct KindTraits<KIND_T> { static constexpr int kmin = 1, kmin_local = 1, mm = 1, ms = 2, tb = kTrialBatch; };

// Per-pair LDS (one wavefront); the sample-index vector of RandomSampler
// (uint32, one per match) lives in the pair's global scratch so that the LDS
// footprint does not grow with the match count.
struct __attribute__((aligned(16))) VerifyLds {
  // Head: everything the windowed kernels (rs_begin / rs_draw / rs_replay)
  // touch.  They allocate only kVerifyLdsHead bytes, so more of their
  // wave-per-pair blocks fit on a CU.
  double best_model[9];
  double ata[45];
  double jA[81], jV[81];
  double best_sum;
  uint64_t prof_t;
  uint32_t mt[624];
  uint32_t counts[kTrialBatch * 3];
  int32_t nmodels[kTrialBatch];
  uint32_t jbuf[kTrialBatch * 7];  // Shuffle targets of one batch of samples
  double redd[16];  // cross-wave exchange of the multi-wave replay (NW > 1)
  double fvec[9];
  int32_t redi[16];
  int32_t mt_idx;
  int32_t best_n;
  int32_t best_sum_valid;
  int32_t pad_;
  // Tail: the sequential LO-RANSAC of verify_final_kernel only (the watermark).
  uint32_t samples[kTrialBatch][8];
};
constexpr size_t kVerifyLdsHead = __builtin_offsetof(VerifyLds, samples);

// ---------------------------------------------------------------------------
// Diagnostic phase timer (only when the launcher passes a profile buffer; no
// stamp executes in the production launch).
// ---------------------------------------------------------------------------
struct Prof {  // passed by value; the last stamp lives in *tp (LDS)
  uint64_t* p;
  uint64_t* tp;
  __device__ void start() {
    if (p && threadIdx.x == 0) *tp = __builtin_amdgcn_s_memtime();
  }
  __device__ void lap(int k) {
    if (p && threadIdx.x == 0) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      p[k] += now - *tp;
      *tp = now;
    }
  }
  __device__ void count(int k, uint64_t v = 1) {
    if (p && threadIdx.x == 0) p[k] += v;
  }
};
enum { PR_SAMPLE = 0, PR_SOLVE, PR_SCORE, PR_CAND, PR_SEQSUM, PR_GATHER, PR_LOEST, PR_LORES,
       PR_OTHER, PR_N_BATCH, PR_N_CAND, PR_N_LO, PR_N_TRIALS, PR_N_POINTS, PR_N_SEQSUM,
       PR_SCORE_H, PR_N_HCHUNK, PR_N_HSLOW };

__device__ __forceinline__ void wsync() { __syncthreads(); }  // one wavefront: cheap
// Barrier of a region one wave runs alone inside a multi-wave block (its LDS
// operations complete in order; this keeps the compiler from moving them).
__device__ __forceinline__ void wave_only_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), lane);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
  return v;
}

// Canonical tree (geom_solvers.h): lane l accumulates p[l] + p[l + w] for
// w = 32 .. 1; lane 0 holds the canonical sum, returned to every lane.
__device__ __forceinline__ double canon_tree_wave(double v) {
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) v = v + __shfl_down(v, w);
  return readlane_d(v, 0);
}

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

// Wave-parallel form of the same generator, used for the sample draws of a
// whole hypothesis batch at once.
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// mt19937 state regeneration in three dependency phases: words [0,227) read
// only old words, [227,454) read the new words k-227 of phase one, and
// [454,624) the new words k-227 of phase two (k = 623 also reads the new
// word 0) -- exactly the values the sequential loop in mt_next sees.
__device__ void mt_twist_wave(VerifyLds& s) {
  const int lane = threadIdx.x & 63;  // (several waves: each computes the same words)
  const int bounds[4] = {0, 227, 454, 624};
#pragma unroll
  for (int ph = 0; ph < 3; ++ph) {
    uint32_t nv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = bounds[ph] + q * 64 + lane;
      nv[q] = 0u;
      if (k < bounds[ph + 1]) {
        const uint32_t y = (s.mt[k] & 0x80000000u) | (s.mt[k + 1 < 624 ? k + 1 : 0] & 0x7fffffffu);
        const int km = k + 397 < 624 ? k + 397 : k + 397 - 624;
        nv[q] = s.mt[km] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      }
    }
    wsync();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = bounds[ph] + q * 64 + lane;
      if (k < bounds[ph + 1]) s.mt[k] = nv[q];
    }
    wsync();
  }
}

// The D = B * kmin uniform_u32(i, n - 1) draws of one batch (i = r mod kmin
// for draw r), computed in parallel under the assumption that no draw needs
// Lemire's rejection step; the generator state advances by exactly D words.
// Returns false (state untouched except through the snapshot the caller
// holds) when some draw might need a rejection; the caller then replays the
// batch serially.  Draw r's target index goes to s.jbuf[r].
template <int KMIN>
__device__ bool draw_targets_wave(VerifyLds& s, int D, uint32_t n) {
  const int lane = threadIdx.x & 63;  // (several waves: each computes the same draws)
  const int idx0 = s.mt_idx;
  const int avail = 624 - idx0;
  uint32_t outv[KMIN];
#pragma unroll
  for (int q = 0; q < KMIN; ++q) {
    const int r = lane + 64 * q;
    outv[q] = (r < D && r < avail) ? mt_temper(s.mt[idx0 + r]) : 0u;
  }
  if (D > avail) {
    wsync();
    mt_twist_wave(s);
#pragma unroll
    for (int q = 0; q < KMIN; ++q) {
      const int r = lane + 64 * q;
      if (r < D && r >= avail) outv[q] = mt_temper(s.mt[r - avail]);
    }
  }
  bool bad = false;
#pragma unroll
  for (int q = 0; q < KMIN; ++q) {
    const int r = lane + 64 * q;
    if (r < D) {
      const uint32_t i = (uint32_t)(r % KMIN);
      const uint32_t range = n - i;
      const uint64_t prod = (uint64_t)outv[q] * (uint64_t)range;
      if ((uint32_t)prod < range) bad = true;
      s.jbuf[r] = i + (uint32_t)(prod >> 32);
    }
  }
  const bool ok = __ballot(bad) == 0;
  wsync();
  if (lane == 0) s.mt_idx = D > avail ? D - avail : idx0 + D;
  wsync();
  return ok;
}

// Trials of the pair's run not drawn yet that its sequential loop can still
// reach: the loop stops after the first trial tt with tt >= dyn_max and tt >=
// min_num_trials, and dyn_max only falls as the best grows, so with the last
// dyn_max a replay stored (rst.dyn_max; a lagging value only bounds higher)
// no trial past max(dyn_max, min_num_trials) is ever needed -- the window
// is not drawn (and scored) past it.  Same trials, same order: only the
// window's length changes.
__device__ __forceinline__ int trials_left(const RansacState* st, int drawn, int min_trials) {
  int cap = st->max_trials;
  const int last = max(st->dyn_max, min_trials);
  if (last < cap) cap = last + 1;
  return cap - drawn;
}

// One round's D draws into s.jbuf, as the sequential generator makes them:
// wave-parallel, or -- when some draw might need Lemire's rejection step --
// serially from the round's start state, kept in registers (no round
// snapshot in memory: its stores would hold every later barrier of the round
// until they complete).  Any block size from 64 threads up.
template <int KMIN>
__device__ void draw_round(VerifyLds& s, int D, uint32_t n) {
  constexpr int KW = (624 + 63) / 64;
  uint32_t keep[KW];
#pragma unroll
  for (int k = 0; k < KW; ++k) {
    const int i = threadIdx.x + blockDim.x * k;
    keep[k] = i < 624 ? s.mt[i] : 0u;
  }
  const int kidx = s.mt_idx;
  if (!draw_targets_wave<KMIN>(s, D, n)) {
#pragma unroll
    for (int k = 0; k < KW; ++k) {
      const int i = threadIdx.x + blockDim.x * k;
      if (i < 624) s.mt[i] = keep[k];
    }
    wsync();
    if (threadIdx.x == 0) {
      s.mt_idx = kidx;
      const uint32_t last = n - 1u;
      for (int r = 0; r < D; ++r) s.jbuf[r] = uniform_u32(s, (uint32_t)(r % KMIN), last);
    }
    wsync();
  }
}

// The abort rewind of a window: from the window's start state (the one
// snapshot its draws keep), the draws of its first `rounds` rounds (full:
// kTrialBatch trials each) and then `extra` more.
template <int KMIN>
__device__ void mt_advance_draws(VerifyLds& s, int rounds, int extra, uint32_t n) {
  for (int r = 0; r < rounds; ++r) {
    draw_round<KMIN>(s, kTrialBatch * KMIN, n);
    wsync();
  }
  if (extra > 0) draw_round<KMIN>(s, extra, n);
  wsync();
}

// RandomSampler::Sample's Shuffle for B samples with precomputed targets:
// the kmin hot positions live in registers, cold targets are read from LDS
// once per sample (several reads in flight) and written back in order.
template <int KMIN>
__device__ void shuffle_batch_lane0(VerifyLds& s, uint32_t* sidx, int B) {
  uint32_t R[KMIN];
#pragma unroll
  for (int i = 0; i < KMIN; ++i) R[i] = sidx[i];
  for (int b = 0; b < B; ++b) {
    uint32_t j[KMIN], v[KMIN], w[KMIN];
#pragma unroll
    for (int i = 0; i < KMIN; ++i) j[i] = s.jbuf[b * KMIN + i];
#pragma unroll
    for (int i = 0; i < KMIN; ++i) v[i] = j[i] >= (uint32_t)KMIN ? sidx[j[i]] : 0u;
#pragma unroll
    for (int i = 0; i < KMIN; ++i) {
      w[i] = 0xFFFFFFFFu;
      if (j[i] < (uint32_t)KMIN) {  // hot swap R[i] <-> R[j] (j >= i)
        uint32_t rj = R[i];
#pragma unroll
        for (int t = 0; t < KMIN; ++t) rj = (t == (int)j[i]) ? R[t] : rj;
#pragma unroll
        for (int t = 0; t < KMIN; ++t) R[t] = (t == (int)j[i]) ? R[i] : R[t];
        R[i] = rj;
      } else {
        uint32_t cur = v[i];
#pragma unroll
        for (int i2 = 0; i2 < i; ++i2) cur = (j[i2] == j[i]) ? w[i2] : cur;
        w[i] = R[i];
        sidx[j[i]] = R[i];
        R[i] = cur;
      }
      s.samples[b][i] = R[i];
    }
  }
#pragma unroll
  for (int i = 0; i < KMIN; ++i) sidx[i] = R[i];
}

// ---------------------------------------------------------------------------
// Residuals and supports.
// ---------------------------------------------------------------------------
template <int K>
__device__ __forceinline__ double residual_pt(const double* m, double a0, double a1, double b0,
                                              double b1) {
  if (K == KIND_F) return sampson_sq(m, a0, a1, b0, b1);
  if (K == KIND_H) return homography_sq(m, a0, a1, b0, b1);
  return translation_sq(m, a0, a1, b0, b1);
}

// Inlier test r <= maxr of the squared Sampson error WITHOUT the division in
// the common case: num and den are computed exactly as sampson_sq does, and
// the correctly rounded quotient fl(num / den) <= maxr is decided from
// num <= maxr * den * (1 - 2^-50)  (surely inside) and
// num >= maxr * den * (1 + 2^-50)  (surely outside: exceeds maxr by > 2 ulp),
// each side carrying at most 2^-52 relative rounding; anything else
// (ties within the band, den <= 0, overflow, NaN) takes the exact division.
__device__ __forceinline__ bool sampson_inlier(const double* F, double x1_0, double x1_1,
                                               double x2_0, double x2_1, double maxr) {
  const double Fx1_0 = F[0] * x1_0 + F[1] * x1_1 + F[2];
  const double Fx1_1 = F[3] * x1_0 + F[4] * x1_1 + F[5];
  const double Fx1_2 = F[6] * x1_0 + F[7] * x1_1 + F[8];
  const double Ftx2_0 = F[0] * x2_0 + F[3] * x2_1 + F[6];
  const double Ftx2_1 = F[1] * x2_0 + F[4] * x2_1 + F[7];
  const double x2tFx1 = x2_0 * Fx1_0 + x2_1 * Fx1_1 + Fx1_2;
  const double num = x2tFx1 * x2tFx1;
  const double den = Fx1_0 * Fx1_0 + Fx1_1 * Fx1_1 + Ftx2_0 * Ftx2_0 + Ftx2_1 * Ftx2_1;
  const double md = maxr * den;
  const bool sane = den > 0.0 && den < 1e300 && num < 1e300;
  const bool in = sane && num <= md * (1.0 - 0x1p-50);
  const bool out = sane && num >= md * (1.0 + 0x1p-50);
  if (in | out) return in;
  return num / den <= maxr;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// Constants of the packed-fp32 homography inlier filter (score_h_chunk).
// The reference test fl64(transfer error) <= maxr is, on exact values,
// W_0^2 + W_1^2 <= maxr P_2^2 with P_i = H_i0 s0 + H_i1 s1 + H_i2 and
// W_j = d_j P_2 - P_j (up to the reference's own fp64 rounding, 2^29 times
// finer than the margin below).  The filter divides it by maxr: with
// r = 1/sqrt(maxr), rows 0 and 1 of H scaled by r and the destination point
// scaled by r when the chunk is loaded (d' = fl(d fl(r)): exact for maxr =
// 4^k, e.g. the default 16), it evaluates in fp32 with explicit FMAs
//   q_i = h'_i0 s0 + h'_i1 s1 + h'_i2,  w_j = d'_j q_2 - q_j,
//   diff = w_0^2 + w_1^2 - q_2^2           (11 packed ops per 2 points)
// against one per-model margin M: diff < -M is surely inside, diff > M
// surely outside, anything else undecided (exact fp64 test).
// Error bound (u = 2^-24; |coordinates| <= S, exact in fp32; A'_i = (|H'_i0|
// + |H'_i1|) S + |H'_i2| with H' = H r in rows 0, 1 and H in row 2):
//   |q_i - P'_i| <= al_i = 3.01u A'_i,
//   |w_j - W'_j| <= b + u|W'_j|,  b = S r (1.0001 al_2 + 2.02u A'_2) + max(al_0, al_1)
//   (the 2.02u term is the rounding of d'), so with L = W'_0^2 + W'_1^2,
//   |lhs - L| <= 2.85 b sqrt(L) + 2.01 b^2 + 4.1u L, |q_2^2 - P_2^2| <= al_2 (2|P_2| + al_2),
//   and the final rounding adds u max(lhs, q_2^2).  For D = L - P_2^2 <= 0,
//   sqrt(L) <= |P_2| <= A'_2; for D > 0 the decision error is largest at
//   L = P_2^2 (or, when |P_2| < 1.43 b, at sqrt(L) = 1.43 b: the 6.1 b^2 term),
// so |diff - D| <= E = (2.85 b + 2 al_2) A'_2 + 6.1 b^2 + al_2^2 + 5.2u A'_2^2 on
// every point the decision depends on; M = 1.5 E (rounded up) also covers the
// reference's fp64 rounding.  A model whose fp32 evaluation could overflow
// gets constants that leave every point undecided (q = 0, M = 1).
__device__ __forceinline__ void h_filter_consts(const double* H, double S, double maxr,
                                                float* c) {
  const double u = 0x1p-24;
  const double r = 1.0 / sqrt(maxr);
  double Hs[9];
#pragma unroll
  for (int j = 0; j < 6; ++j) Hs[j] = H[j] * r;
#pragma unroll
  for (int j = 6; j < 9; ++j) Hs[j] = H[j];
  const double A0 = (fabs(Hs[0]) + fabs(Hs[1])) * S + fabs(Hs[2]);
  const double A1 = (fabs(Hs[3]) + fabs(Hs[4])) * S + fabs(Hs[5]);
  const double A2 = (fabs(Hs[6]) + fabs(Hs[7])) * S + fabs(Hs[8]);
  const double al0 = 3.01 * u * A0, al1 = 3.01 * u * A1, al2 = 3.01 * u * A2;
  const double b = S * r * (1.0001 * al2 + 2.02 * u * A2) + fmax(al0, al1);
  const double E = (2.85 * b + 2.0 * al2) * A2 + 6.1 * b * b + al2 * al2 + 5.2 * u * A2 * A2;
  const double M = 1.5 * E + 1e-30;
  const double wmax = S * r * A2 + fmax(A0, A1);
  const double lmax = 2.0 * wmax * wmax, rmax = A2 * A2;
#pragma unroll
  for (int j = 0; j < 9; ++j) c[j] = (float)Hs[j];
  c[9] = __double2float_ru(M);
  c[10] = 0.0f;
  c[11] = 0.0f;
  if (!(lmax < 1e36 && rmax < 1e36 && M < 1e36)) {
    // fp32 evaluation unsafe: q = 0, M = 1 marks every point undecided, so
    // every point takes the exact test.
#pragma unroll
    for (int j = 0; j < 9; ++j) c[j] = 0.0f;
    c[9] = 1.0f;
  }
}

// The destination-point scale fl32(1/sqrt(maxr)) of the homography filter
// (h_filter_consts), applied to d when a chunk is loaded.
__device__ __forceinline__ float h_point_scale(double maxr) { return (float)(1.0 / sqrt(maxr)); }

// Lanes of point slot p (point base + 64 p + lane) that hold a point.
__device__ __forceinline__ uint64_t slot_mask(int n, int base, int p) {
  const int rem = n - base - 64 * p;
  return rem >= 64 ? ~0ull : (rem <= 0 ? 0ull : ((1ull << rem) - 1ull));
}

// Packed-fp32 FMA whose first and third operands are single dwords of
// constant pairs broadcast to both halves by op_sel (the constants stay in the
// registers their LDS loads landed in: no v_mov pairs per model).  SA / SC
// pick the dword (0 = low, 1 = high) of a / c; b is a regular pair.
// Bitwise the same as __builtin_elementwise_fma on splats (probes/opsel_probe.hip).
#define SCM_PKFMA_BB(d, a, b, c, SA, SC)                                                 \
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[" #SA ",0," #SC "] op_sel_hi:[" #SA ",1," #SC "]" \
      : "=v"(d) : "v"(a), "v"(b), "v"(c))
#define SCM_PKFMA_BV(d, a, b, c, SA)                                                   \
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[" #SA ",0,0] op_sel_hi:[" #SA ",1,1]"      \
      : "=v"(d) : "v"(a), "v"(b), "v"(c))

// Filter constants as the register pairs of their LDS loads:
// (h'0,h'1) (h'2,h'3) (h'4,h'5) (h6,h7) (h8,M).
struct HFilt {
  f32x2 p01, p23, p45, p67, p8m;
};

// diff of one packed pair of points (s0, s1, scaled d0', d1'): surely inside
// iff diff < -M, undecided iff |diff| <= M, surely outside otherwise.
__device__ __forceinline__ f32x2 h_filter_pair(const HFilt& f, f32x2 s0, f32x2 s1, f32x2 d0,
                                               f32x2 d1) {
  f32x2 t0, t1, t2, q0, q1, q2;
  SCM_PKFMA_BB(t0, f.p01, s1, f.p23, 1, 0);  // h'1 s1 + h'2
  SCM_PKFMA_BB(t1, f.p45, s1, f.p45, 0, 1);  // h'4 s1 + h'5
  SCM_PKFMA_BB(t2, f.p67, s1, f.p8m, 1, 0);  // h7 s1 + h8
  SCM_PKFMA_BV(q0, f.p01, s0, t0, 0);        // h'0 s0 + (h'1 s1 + h'2)
  SCM_PKFMA_BV(q1, f.p23, s0, t1, 1);        // h'3 s0 + (h'4 s1 + h'5)
  SCM_PKFMA_BV(q2, f.p67, s0, t2, 0);        // h6 s0 + (h7 s1 + h8)
  const f32x2 w0 = __builtin_elementwise_fma(d0, q2, -q0);
  const f32x2 w1 = __builtin_elementwise_fma(d1, q2, -q1);
  const f32x2 lhs = __builtin_elementwise_fma(w0, w0, w1 * w1);
  return __builtin_elementwise_fma(-q2, q2, lhs);
}

// Exact fp64 test (HomographyMatrixEstimator::Residuals) of the undecided
// points of one packed slot pair; the fp32 coordinates widen exactly to the
// doubles the reference uses.
// Exact reference test of one point (rare path; not inlined so that its
// fp64 registers do not add to the hot loop's budget).
__device__ __attribute__((noinline)) bool h_exact_pt(const double* mk, float sx, float sy,
                                                     float dx, float dy, double maxr) {
  return homography_sq(mk, (double)sx, (double)sy, (double)dx, (double)dy) <= maxr;
}

// The hypothesis' constants (LDS, broadcast read), kept in vector registers:
// no readfirstlane / SGPR copies per model (filter loop 20 % faster,
// probes/score_bench.hip).
__device__ __forceinline__ HFilt h_filter_load(const float* hc) {
  const float4 c0 = reinterpret_cast<const float4*>(hc)[0];
  const float4 c1 = reinterpret_cast<const float4*>(hc)[1];
  const float2 c2 = reinterpret_cast<const float2*>(hc)[4];
  HFilt f;
  f.p01 = f32x2{c0.x, c0.y};
  f.p23 = f32x2{c0.z, c0.w};
  f.p45 = f32x2{c1.x, c1.y};
  f.p67 = f32x2{c1.z, c1.w};
  f.p8m = f32x2{c2.x, c2.y};
  return f;
}

// Inlier count of one hypothesis (filter f, fp64 model mk in LDS) over the
// points [base, base + 64 PCH) (point base + 64 p + lane in slot p; FULL:
// every slot holds a point).
// Deferred exact tests of the scoring kernel: the filter's undecided
// (model, point) elements of a round are queued in LDS and tested after the
// round's model loop, 64 at a time (every lane busy), instead of one or two
// lanes at a time inside it.  A full queue falls back to the immediate test.
constexpr int kDeferCap = 256;
struct DeferQ {
  uint32_t* q;  // LDS: model << 16 | point offset within the chunk
  int n;        // entries queued (wave-uniform)
  int cap = kDeferCap;
};

// Queue the undecided lanes um of point slot p for model m; false when the
// queue is full (the caller then tests them at once).
__device__ __forceinline__ bool defer_push(DeferQ* d, uint64_t um, int p, int m) {
  const int c = __popcll(um);
  if (d->n + c > d->cap) return false;
  const uint32_t lane = threadIdx.x;
  if (um & (1ull << lane)) {
    const int pos = d->n + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(um >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)um, 0u));
    d->q[pos] = ((uint32_t)m << 16) | (uint32_t)(64 * p + lane);
  }
  d->n += c;
  return true;
}

// Inlier count of one homography (filter f, fp64 model mk) over the points
// [base, base + 64 PCH) (point base + 64 p + lane in slot p, destination
// coordinates pre-scaled, h_filter_consts; FULL: every slot holds a point).
// NOTOUT: one compare per point, no exact tests -- return the number of
// points not surely outside, an upper bound of the count (the first pass of
// the split scoring; rs_exact_kernel counts exactly the models whose bound
// reaches the pair's best).  Otherwise the sure inliers plus the exact fp64
// test (the point reloaded from xyf) of the undecided ones; the sure count
// goes to *nsure (when given) before the exact tests.
template <int PCH, bool FULL, bool NOTOUT = false>
__device__ __forceinline__ int score_h_chunk(const HFilt& f, const double* mk, const float4* xyf,
                                             const f32x2* s0, const f32x2* s1, const f32x2* d0,
                                             const f32x2* d1, int n, int base, double maxr,
                                             int* nslow, DeferQ* dq = nullptr, int dm = 0,
                                             int* nsure = nullptr) {
  const float M = f.p8m.y;
  int cnt = 0;
  if (NOTOUT) {
#pragma unroll
    for (int q = 0; q < PCH / 2; ++q) {
      if (!FULL && base + 128 * q >= n) continue;  // slot pair past the last point
      const f32x2 diff = h_filter_pair(f, s0[q], s1[q], d0[q], d1[q]);
      uint64_t o0 = __ballot(diff.x <= M), o1 = __ballot(diff.y <= M);
      if (!FULL) {
        o0 &= slot_mask(n, base, 2 * q);
        o1 &= slot_mask(n, base, 2 * q + 1);
      }
      cnt += __popcll(o0) + __popcll(o1);
    }
    return cnt;
  }
  uint64_t any = 0;
  uint64_t um[PCH];  // per point slot: lanes the filter left undecided
#pragma unroll
  for (int q = 0; q < PCH / 2; ++q) {
    if (!FULL && base + 128 * q >= n) {
      um[2 * q] = um[2 * q + 1] = 0;
      continue;
    }
    const f32x2 diff = h_filter_pair(f, s0[q], s1[q], d0[q], d1[q]);
    // strict: a point on the band's edge is undecided, never counted twice
    uint64_t i0 = __ballot(diff.x < -M), i1 = __ballot(diff.y < -M);
    uint64_t u0 = __ballot(fabsf(diff.x) <= M), u1 = __ballot(fabsf(diff.y) <= M);
    if (!FULL) {
      const uint64_t ok0 = slot_mask(n, base, 2 * q), ok1 = slot_mask(n, base, 2 * q + 1);
      i0 &= ok0;
      i1 &= ok1;
      u0 &= ok0;
      u1 &= ok1;
    }
    cnt += __popcll(i0) + __popcll(i1);
    um[2 * q] = u0;
    um[2 * q + 1] = u1;
    any |= u0 | u1;
  }
  if (nsure) *nsure = cnt;
  if (any) {  // rare: exact test of the undecided points only (queued when dq)
    ++*nslow;
    if (dq) {
#pragma unroll
      for (int p = 0; p < PCH; ++p)
        if (um[p] && defer_push(dq, um[p], p, dm)) um[p] = 0;
    }
    const uint64_t me = 1ull << threadIdx.x;
#pragma unroll
    for (int p = 0; p < PCH; ++p) {
      if (um[p]) {
        bool e = false;
        if (um[p] & me) {
          const float4 pt = xyf[base + 64 * p + threadIdx.x];
          e = h_exact_pt(mk, pt.x, pt.y, pt.z, pt.w, maxr);
        }
        cnt += __popcll(__ballot(e));
      }
    }
  }
  return cnt;
}

// Points not surely outside for NM homographies at once over one chunk (the
// split first pass): the models' independent chains interleave, and the loop
// overhead (constant loads, count selection) is paid once per NM models.
template <int PCH, bool FULL, int NM>
__device__ __forceinline__ void score_h_notout_n(const HFilt* f, const f32x2* s0, const f32x2* s1,
                                                 const f32x2* d0, const f32x2* d1, int n, int base,
                                                 int* c) {
#pragma unroll
  for (int k = 0; k < NM; ++k) c[k] = 0;
#pragma unroll
  for (int q = 0; q < PCH / 2; ++q) {
    if (!FULL && base + 128 * q >= n) continue;
    f32x2 d[NM];
#pragma unroll
    for (int k = 0; k < NM; ++k) d[k] = h_filter_pair(f[k], s0[q], s1[q], d0[q], d1[q]);
    const uint64_t ok0 = FULL ? ~0ull : slot_mask(n, base, 2 * q);
    const uint64_t ok1 = FULL ? ~0ull : slot_mask(n, base, 2 * q + 1);
#pragma unroll
    for (int k = 0; k < NM; ++k)
      c[k] += __popcll(__ballot(d[k].x <= f[k].p8m.y) & ok0) +
              __popcll(__ballot(d[k].y <= f[k].p8m.y) & ok1);
  }
}

// ---------------------------------------------------------------------------
// Packed-fp32 Sampson inlier filter (FundamentalMatrix*Estimator::Residuals,
// SURVEY.md §8a a12) with exact fp64 fallback.  With U = F x1 (rows 0..2),
// V = F^T x2 (rows 0, 1), e = x2^T F x1, the reference tests
// e^2 / (U0^2 + U1^2 + V0^2 + V1^2) <= maxr, i.e. E^2 <= maxr D on exact
// values up to its own fp64 rounding.  In fp32 (u = 2^-24, explicit FMAs):
//   |U_i - U~_i| <= 3u A_i = al_i, A_i = (|F_i0| + |F_i1|) S + |F_i2|,
//   |V_j - V~_j| <= 3u B_j = be_j, B_j = (|F_0j| + |F_1j|) S + |F_2j|,
//   |e - E| <= g = S (al_0 + al_1) + al_2 + 2.01u (S (A_0 + A_1) + A_2),
// so |num - E^2| <= 2 g |E| + g^2 + u num and, with d = max(al_0, al_1,
// be_0, be_1) and |U0| + |U1| + |V0| + |V1| <= 2 sqrt(D),
// |den - D| <= 4 d sqrt(D) + 2 d^2 + 4u den.  At the threshold |E| =
// sqrt(maxr D), and sqrt(D) <= (D / tau + tau) / 2 for any tau > 0 (tau =
// sqrt(den) at the image middle), so the decision is certain whenever
// |num - maxr den| > a1 maxr den + a0 with
//   c1 = 2 g sqrt(maxr) + 4 d maxr, c0 = g^2 + 2 maxr d^2,
//   a1 = 1.01 c1 / (2 tau maxr) + 5.1u, a0 = c1 tau / 2 + c0   (x 1.5).
// ---------------------------------------------------------------------------
// (f0,f1) (f2,f3) (f4,f5) (f6,f7) (f8,a0) (a1,-), and maxr splat (see HFilt).
struct FFilt {
  f32x2 p01, p23, p45, p67, p8a, pa1, mr;
};

__device__ __forceinline__ void f_filter_consts(const double* F, double S, double maxr,
                                                float* c) {
  const double u = 0x1p-24;
  const double A0 = (fabs(F[0]) + fabs(F[1])) * S + fabs(F[2]);
  const double A1 = (fabs(F[3]) + fabs(F[4])) * S + fabs(F[5]);
  const double A2 = (fabs(F[6]) + fabs(F[7])) * S + fabs(F[8]);
  const double B0 = (fabs(F[0]) + fabs(F[3])) * S + fabs(F[6]);
  const double B1 = (fabs(F[1]) + fabs(F[4])) * S + fabs(F[7]);
  const double al0 = 3.01 * u * A0, al1 = 3.01 * u * A1, al2 = 3.01 * u * A2;
  const double be0 = 3.01 * u * B0, be1 = 3.01 * u * B1;
  const double g = S * (al0 + al1) + al2 + 2.01 * u * (S * (A0 + A1) + A2);
  const double d = fmax(fmax(al0, al1), fmax(be0, be1));
  const double sq = sqrt(maxr);
  const double c1 = 2.0 * g * sq + 4.0 * d * maxr;
  const double c0 = g * g + 2.0 * maxr * d * d;
  const double h = 0.5 * S;
  const double m0 = F[0] * h + F[1] * h + F[2], m1 = F[3] * h + F[4] * h + F[5];
  const double n0 = F[0] * h + F[3] * h + F[6], n1 = F[1] * h + F[4] * h + F[7];
  double tau = sqrt(m0 * m0 + m1 * m1 + n0 * n0 + n1 * n1);
  const double tmax = A0 + A1 + B0 + B1;
  if (!(tau > 1e-30 && tau < 1e30)) tau = tmax > 1e-30 ? tmax : 1e-30;
  const double a1 = 1.5 * (1.01 * c1 / (2.0 * tau * maxr) + 5.1 * u);
  const double a0 = 1.5 * (0.5 * c1 * tau + c0) + 1e-30;
  const double emax = S * (A0 + A1) + A2;
  const double dmax = A0 * A0 + A1 * A1 + B0 * B0 + B1 * B1;
#pragma unroll
  for (int j = 0; j < 9; ++j) c[j] = (float)F[j];
  c[9] = __double2float_ru(a0);
  c[10] = __double2float_ru(a1);
  c[11] = 0.0f;
  if (!(emax * emax < 1e36 && maxr * dmax < 1e36 && a1 < 1e30 && a0 < 1e36)) {
    // fp32 evaluation unsafe: num = den = 0, margin 1 -> every point undecided.
#pragma unroll
    for (int j = 0; j < 9; ++j) c[j] = 0.0f;
    c[9] = 1.0f;
    c[10] = 0.0f;
  }
}

__device__ __forceinline__ FFilt f_filter_load(const float* fc, float maxrf) {
  const float4 c0 = reinterpret_cast<const float4*>(fc)[0];
  const float4 c1 = reinterpret_cast<const float4*>(fc)[1];
  const float4 c2 = reinterpret_cast<const float4*>(fc)[2];
  FFilt f;
  f.p01 = f32x2{c0.x, c0.y};
  f.p23 = f32x2{c0.z, c0.w};
  f.p45 = f32x2{c1.x, c1.y};
  f.p67 = f32x2{c1.z, c1.w};
  f.p8a = f32x2{c2.x, c2.y};
  f.pa1 = f32x2{c2.z, c2.w};
  f.mr = f32x2(maxrf);
  return f;
}

// diff = num - maxr den, mg = decision margin (see above).
__device__ __forceinline__ void f_filter_pair(const FFilt& f, f32x2 x0, f32x2 x1, f32x2 y0,
                                              f32x2 y1, f32x2* diff, f32x2* mg) {
  typedef f32x2 V;
  V t, U0, U1, U2, V0, V1, m;
  SCM_PKFMA_BB(t, f.p01, x1, f.p23, 1, 0);  // f1 x1 + f2
  SCM_PKFMA_BV(U0, f.p01, x0, t, 0);        // f0 x0 + .
  SCM_PKFMA_BB(t, f.p45, x1, f.p45, 0, 1);  // f4 x1 + f5
  SCM_PKFMA_BV(U1, f.p23, x0, t, 1);        // f3 x0 + .
  SCM_PKFMA_BB(t, f.p67, x1, f.p8a, 1, 0);  // f7 x1 + f8
  SCM_PKFMA_BV(U2, f.p67, x0, t, 0);        // f6 x0 + .
  SCM_PKFMA_BB(t, f.p23, y1, f.p67, 1, 0);  // f3 y1 + f6
  SCM_PKFMA_BV(V0, f.p01, y0, t, 0);        // f0 y0 + .
  SCM_PKFMA_BB(t, f.p45, y1, f.p67, 0, 1);  // f4 y1 + f7
  SCM_PKFMA_BV(V1, f.p01, y0, t, 1);        // f1 y0 + .
  const V e = __builtin_elementwise_fma(y0, U0, __builtin_elementwise_fma(y1, U1, U2));
  const V den = __builtin_elementwise_fma(
      U0, U0, __builtin_elementwise_fma(U1, U1, __builtin_elementwise_fma(V0, V0, V1 * V1)));
  const V rhs = f.mr * den;
  SCM_PKFMA_BB(m, f.pa1, rhs, f.p8a, 0, 1);  // a1 rhs + a0
  *mg = m;
  *diff = __builtin_elementwise_fma(e, e, -rhs);
}

__device__ __attribute__((noinline)) bool f_exact_pt(const double* mk, float x0, float x1,
                                                     float y0, float y1, double maxr) {
  return sampson_sq(mk, (double)x0, (double)x1, (double)y0, (double)y1) <= maxr;
}

// Inlier count of one 7-point model (filter f; fp64 model mk in LDS, read
// only for undecided points) over one chunk of points.
// UND: no exact tests -- return the sure inliers and write the number of
// undecided points to *nund (the exact pass, rs_exact_kernel, tests them
// only for models that can still reach the pair's best count).  Otherwise
// the sure count goes to *nsure (when given) before the exact tests.
template <int PCH, bool FULL, bool UND = false>
__device__ __forceinline__ int score_f_chunk(const FFilt& f, const double* mk, const f32x2* x0,
                                             const f32x2* x1, const f32x2* y0, const f32x2* y1,
                                             int n, int base, double maxr, int* nslow,
                                             DeferQ* dq = nullptr, int dm = 0,
                                             int* nund = nullptr, int* nsure = nullptr) {
  int cnt = 0;
  uint64_t any = 0;
  uint64_t um[PCH];  // per point slot: lanes the filter left undecided
#pragma unroll
  for (int q = 0; q < PCH / 2; ++q) {
    if (!FULL && base + 128 * q >= n) {  // slot pair past the last point
      um[2 * q] = um[2 * q + 1] = 0;
      continue;
    }
    f32x2 diff, mg;
    f_filter_pair(f, x0[q], x1[q], y0[q], y1[q], &diff, &mg);
    uint64_t i0 = __ballot(diff.x < -mg.x), i1 = __ballot(diff.y < -mg.y);
    uint64_t u0 = __ballot(fabsf(diff.x) <= mg.x), u1 = __ballot(fabsf(diff.y) <= mg.y);
    if (!FULL) {
      const uint64_t ok0 = slot_mask(n, base, 2 * q), ok1 = slot_mask(n, base, 2 * q + 1);
      i0 &= ok0;
      i1 &= ok1;
      u0 &= ok0;
      u1 &= ok1;
    }
    cnt += __popcll(i0) + __popcll(i1);
    um[2 * q] = u0;
    um[2 * q + 1] = u1;
    any |= u0 | u1;
  }
  if (UND) {
    int u = 0;
#pragma unroll
    for (int p = 0; p < PCH; ++p) u += __popcll(um[p]);
    *nund = u;
    return cnt;
  }
  if (nsure) *nsure = cnt;
  if (any) {  // rare: exact test of the undecided points only (queued when dq)
    ++*nslow;
    if (dq) {
#pragma unroll
      for (int p = 0; p < PCH; ++p)
        if (um[p] && defer_push(dq, um[p], p, dm)) um[p] = 0;
    }
    const uint64_t me = 1ull << threadIdx.x;
#pragma unroll
    for (int q = 0; q < PCH / 2; ++q) {
      if (um[2 * q]) {
        bool e = false;
        if (um[2 * q] & me) e = f_exact_pt(mk, x0[q].x, x1[q].x, y0[q].x, y1[q].x, maxr);
        cnt += __popcll(__ballot(e));
      }
      if (um[2 * q + 1]) {
        bool e = false;
        if (um[2 * q + 1] & me) e = f_exact_pt(mk, x0[q].y, x1[q].y, y0[q].y, y1[q].y, maxr);
        cnt += __popcll(__ballot(e));
      }
    }
  }
  return cnt;
}

// Point loops of the sequential (watermark) LO-RANSAC and the final kernel:
// latency-bound, so each lane keeps kSeqU points' loads in flight; items are
// consumed in index order per lane (canonical sums keep their order).
constexpr int kSeqU = 8;

// InlierSupportMeasurer::Evaluate's residual_sum: inlier residuals summed
// in index order.  The wave loads 64 x kSeqU residuals at a time; every lane
// runs the same ordered chain over the 64 lanes' values, broadcast with
// v_readlane at fixed lane indices (no per-inlier scan).  A point that is not
// an inlier contributes -0.0, the exact additive identity (x + -0.0 == x for
// every x, signed zeros included), so the chain performs exactly the
// reference's additions.
__device__ __forceinline__ void seq_inlier_load(const double* res, int n, int b0, double (&x)[4]) {
  const int lane = (int)(threadIdx.x & 63);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = b0 + 64 * u + lane;
    x[u] = i < n ? res[i] : 1.7976931348623157e308;
  }
}
// A batch of 64 with few inliers visits them by a scan of its ballot; a dense
// one runs the fixed chain over all 64 lanes with -0.0 for the others.
__device__ __noinline__ double seq_inlier_sum(const double* res, int n, double maxr) {
  double sum = 0.0;
  double cur[4];
  seq_inlier_load(res, n, 0, cur);
  for (int b0 = 0; b0 < n; b0 += 256) {
    double nxt[4];  // the next 256 residuals in flight during this chain
    seq_inlier_load(res, n, b0 + 256, nxt);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool in = cur[u] <= maxr;
      uint64_t bal = __ballot(in);
      if (__popcll(bal) <= 16) {
        while (bal) {
          sum += readlane_d(cur[u], __builtin_ctzll(bal));
          bal &= bal - 1;
        }
      } else {
        const double x = in ? cur[u] : -0.0;
#pragma unroll
        for (int l = 0; l < 64; ++l) sum += readlane_d(x, l);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) cur[u] = nxt[u];
  }
  return sum;
}

// ---------------------------------------------------------------------------
// Point loops of the windowed replay (candidate residuals and local
// optimisation) on the packed fp32 copy of the matches (xyf: x1, y1, x2, y2
// per point; keypoints are float32, so widening to double reproduces the
// reference's Eigen::Vector2d values exactly).  Each lane keeps kLoU loads in
// flight; items are still consumed in index order per lane, so every
// canonical-order sum performs the same additions as before.
// ---------------------------------------------------------------------------
constexpr int kLoU = 4;

__device__ __forceinline__ void load_pts(const float4* p, int b, int n, float4 (&v)[kLoU]) {
#pragma unroll
  for (int u = 0; u < kLoU; ++u) {
    const int i = b + 64 * u;
    v[u] = i < n ? p[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// apply_normalize (geom_solvers.h) for a transform with last row (0, 0, 1):
// np2 = 0 p0 + 0 p1 + 1 is exactly 1 and the homogeneous divide by it is the
// identity, so it is skipped (same values bit for bit).
__device__ __forceinline__ void apply_norm_affine(const double* T, double p0, double p1,
                                                  double* o0, double* o1) {
  *o0 = T[0] * p0 + T[1] * p1 + T[2];
  *o1 = T[3] * p0 + T[4] * p1 + T[5];
}

// A model's residuals and the ordered gather of its inliers in one pass: the
// model's residuals into res and, in index order, its inliers' points into
// xin (the gather the local optimisation runs next if the model becomes the
// best: a candidate's pass and every LO step's pass write it, so LO starts
// from it without another pass over the points).  Wave w takes block w of
// each round of 64 kLoU NW points; a prefix of the waves' counts places its
// inliers.  Returns the inlier count; residuals and inliers are visible to
// the block on return.
template <int K, int NW = 1>
__device__ int residuals_gather_f4(const double* m, const float4* xyf, int n, double maxr,
                                   double* res, float4* xin, int32_t* redi = nullptr) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int base_out = 0;
  for (int r0 = 0; r0 < n; r0 += 64 * kLoU * NW) {
    const int b0 = r0 + wv * 64 * kLoU;
    float4 v[kLoU];
    double r[kLoU];
    load_pts(xyf, b0 + lane, n, v);
    uint64_t bal[kLoU];
    int wc = 0;
#pragma unroll
    for (int u = 0; u < kLoU; ++u) {
      const int i = b0 + 64 * u + lane;
      r[u] = 1.7976931348623157e308;
      if (i < n) {
        r[u] = residual_pt<K>(m, (double)v[u].x, (double)v[u].y, (double)v[u].z, (double)v[u].w);
        res[i] = r[u];
      }
      bal[u] = __ballot(r[u] <= maxr);
      wc += __popcll(bal[u]);
    }
    int before = 0, total = wc;
    if (NW > 1) {
      if (lane == 0) redi[wv] = wc;
      __syncthreads();
      total = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const int x = redi[w];
        before += w < wv ? x : 0;
        total += x;
      }
      __syncthreads();
    }
    int o = base_out + before;
#pragma unroll
    for (int u = 0; u < kLoU; ++u) {
      if (r[u] <= maxr)
        xin[o + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal[u] >> 32),
                                               __builtin_amdgcn_mbcnt_lo((uint32_t)bal[u], 0u))] = v[u];
      o += __popcll(bal[u]);
    }
    base_out += total;
  }
  if (NW > 1) __syncthreads();
  return base_out;
}

// Wavefront twin of ata_null_vector (geom_solvers.h): lane e (and e + 64)
// owns entry e of the 9 x 9 iterate (row-major, LDS buffers A and B); each
// Gauss-Jordan step and each squaring computes every entry from the previous
// matrix with exactly the host's operations, so the result is bit-identical.
// The uniform scalars (pivot reciprocal, trace factor, j*, rank-one test) are
// evaluated by every lane from broadcast LDS reads.  Returns the unit null
// vector in f (every lane).
// SOLO: run by one wave of a multi-wave block (wave-only barriers).
template <bool SOLO = false>
__device__ void invsq9_null_wave(const double* ata45, double* A, double* B, double* f) {
  auto bar = [] {
    if (SOLO) wave_only_sync();
    else wsync();
  };
  const int lane = threadIdx.x;
  const int e0 = lane, e1 = lane + 64;  // e1 valid for lane < 17
  const bool has1 = e1 < 81;
  const double tr = ata9_trace(ata45);
  if (!(tr > 0.0)) {
#pragma unroll
    for (int i = 0; i < 9; ++i) f[i] = i == 0 ? 1.0 : 0.0;
    return;
  }
  const double delta = tr * 0x1p-40;
  {
    // packed upper-triangle index of (p, q), p <= q
    auto load = [&](int e) {
      const int i = e / 9, j = e - 9 * (e / 9);
      const int p = i < j ? i : j, q = i < j ? j : i;
      const double v = ata45[ata_index(p, q)];
      A[e] = p == q ? v + delta : v;
    };
    load(e0);
    if (has1) load(e1);
  }
  bar();
  const int i0 = e0 / 9, j0 = e0 - 9 * (e0 / 9);
  const int i1 = e1 / 9, j1 = e1 - 9 * (e1 / 9);
#pragma unroll 1
  for (int k = 0; k < 9; ++k) {
    const double inv = 1.0 / A[k * 9 + k];
    const double n0 = gj9_entry(A[e0], A[i0 * 9 + k], A[k * 9 + j0], inv, i0, j0, k);
    const double n1 = has1 ? gj9_entry(A[e1], A[i1 * 9 + k], A[k * 9 + j1], inv, i1, j1, k) : 0.0;
    bar();
    A[e0] = n0;
    if (has1) A[e1] = n1;
    bar();
  }
  B[e0] = 0.5 * (A[e0] + A[j0 * 9 + i0]);
  if (has1) B[e1] = 0.5 * (A[e1] + A[j1 * 9 + i1]);
  bar();
  int jstar = 0;
  bool done = false;
#pragma unroll 1
  for (int sq = 0; sq < kInvSqMax; ++sq) {
    const double q0 = sq9_entry(B, i0, j0);
    const double q1 = has1 ? sq9_entry(B, i1, j1) : 0.0;
    A[e0] = q0;  // A is free: B holds the iterate
    if (has1) A[e1] = q1;
    bar();
    const double ti = sq9_trace_inv(A);
    B[e0] = q0 * ti;
    if (has1) B[e1] = q1 * ti;
    bar();
    jstar = sq9_argmax_diag(B);
    if (done) break;
    done = sq + 1 >= kInvSqMin && sq9_rank_one(B, jstar);
  }
  sq9_column_unit(B, jstar, f);
}

// Local estimator of the watermark LO-RANSAC (geom_solvers.h
// translation_estimate on n gathered inliers, packed fp32 points: keypoints
// are float32, so widening reproduces the reference's doubles exactly): the
// mean displacement, its four coordinate sums in canonical order.  NW > 1:
// wave w < 4 forms the sum of coordinate w with the one-wave lane mapping (the
// same sums), exchanged in s.redd.  Every lane returns the model.
template <int K, int NW = 1>
__device__ void local_estimate_wave(VerifyLds& s, const float4* xin, int n, double* model) {
  static_assert(K == KIND_T, "the F / H local estimators run on local_estimate_f4");
  const int lane = threadIdx.x & 63;
  if (NW > 1) {
    const int wv = threadIdx.x >> 6;
    double p = kCanonZero;
    if (wv < 4) {
      for (int b = lane; b < n; b += 64 * kSeqU) {
        double a[kSeqU];
        const float* xc = reinterpret_cast<const float*>(xin) + wv;  // coordinate wv only
#pragma unroll
        for (int u = 0; u < kSeqU; ++u) a[u] = (double)xc[4 * min(b + 64 * u, n - 1)];
#pragma unroll
        for (int u = 0; u < kSeqU; ++u)
          if (b + 64 * u < n) p += a[u];
      }
      p = canon_tree_wave(p);
      if (lane == 0) s.redd[wv] = p;
    }
    __syncthreads();
    const double s0 = s.redd[0] / (double)n, s1 = s.redd[1] / (double)n;
    const double d0 = s.redd[2] / (double)n, d1 = s.redd[3] / (double)n;
    __syncthreads();
    model[0] = d0 - s0;
    model[1] = d1 - s1;
    return;
  }
  double p0 = kCanonZero, p1 = kCanonZero, p2 = kCanonZero, p3 = kCanonZero;
  for (int b = lane; b < n; b += 64 * kSeqU) {
    float4 v[kSeqU];
#pragma unroll
    for (int u = 0; u < kSeqU; ++u) v[u] = xin[min(b + 64 * u, n - 1)];
#pragma unroll
    for (int u = 0; u < kSeqU; ++u)
      if (b + 64 * u < n) {
        p0 += (double)v[u].x;
        p1 += (double)v[u].y;
        p2 += (double)v[u].z;
        p3 += (double)v[u].w;
      }
  }
  const double s0 = canon_tree_wave(p0) / (double)n, s1 = canon_tree_wave(p1) / (double)n;
  const double d0 = canon_tree_wave(p2) / (double)n, d1 = canon_tree_wave(p3) / (double)n;
  model[0] = d0 - s0;
  model[1] = d1 - s1;
}

__device__ __forceinline__ void norm_transforms(double c10, double c11, double c20, double c21,
                                                double rms1, double rms2, double* T1, double* T2) {
  const double s1 = sqrt(2.0) / rms1, s2 = sqrt(2.0) / rms2;
  T1[0] = s1; T1[1] = 0.0; T1[2] = -s1 * c10;
  T1[3] = 0.0; T1[4] = s1; T1[5] = -s1 * c11;
  T1[6] = 0.0; T1[7] = 0.0; T1[8] = 1.0;
  T2[0] = s2; T2[1] = 0.0; T2[2] = -s2 * c20;
  T2[3] = 0.0; T2[4] = s2; T2[5] = -s2 * c21;
  T2[6] = 0.0; T2[7] = 0.0; T2[8] = 1.0;
}

// normalize_pair_f4 with four waves: wave w forms the canonical sum of
// coordinate w (then waves 0 / 1 the two RMS sums) with the lane mapping of
// the one-wave version, so every sum is the same.
__device__ void normalize_pair_f4_w4(const float4* xin, int n, double* T1, double* T2,
                                     double* redd) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double p = kCanonZero;
  for (int b = lane; b < n; b += 64 * kLoU) {
    float4 v[kLoU];
    load_pts(xin, b, n, v);
#pragma unroll
    for (int u = 0; u < kLoU; ++u)
      if (b + 64 * u < n)
        p += (double)(wv == 0 ? v[u].x : wv == 1 ? v[u].y : wv == 2 ? v[u].z : v[u].w);
  }
  p = canon_tree_wave(p);
  if (lane == 0) redd[wv] = p;
  __syncthreads();
  const double c10 = redd[0] / (double)n, c11 = redd[1] / (double)n;
  const double c20 = redd[2] / (double)n, c21 = redd[3] / (double)n;
  __syncthreads();
  if (wv < 2) {
    const double ca = wv == 0 ? c10 : c20, cb = wv == 0 ? c11 : c21;
    p = kCanonZero;
    for (int b = lane; b < n; b += 64 * kLoU) {
      float4 v[kLoU];
      load_pts(xin, b, n, v);
#pragma unroll
      for (int u = 0; u < kLoU; ++u)
        if (b + 64 * u < n) {
          const double d0 = (double)(wv == 0 ? v[u].x : v[u].z) - ca;
          const double d1 = (double)(wv == 0 ? v[u].y : v[u].w) - cb;
          p += d0 * d0 + d1 * d1;
        }
    }
    p = canon_tree_wave(p);
    if (lane == 0) redd[4 + wv] = p;
  }
  __syncthreads();
  norm_transforms(c10, c11, c20, c21, sqrt(redd[4] / (double)n), sqrt(redd[5] / (double)n), T1, T2);
  __syncthreads();
}

// normalize_transform (geom_solvers.h) of both point sets on packed points,
// canonical sums.
__device__ void normalize_pair_f4(const float4* xin, int n, double* T1, double* T2) {
  double p0 = kCanonZero, p1 = kCanonZero, p2 = kCanonZero, p3 = kCanonZero;
  for (int b = threadIdx.x; b < n; b += 64 * kLoU) {
    float4 v[kLoU];
    load_pts(xin, b, n, v);
#pragma unroll
    for (int u = 0; u < kLoU; ++u)
      if (b + 64 * u < n) {
        p0 += (double)v[u].x;
        p1 += (double)v[u].y;
        p2 += (double)v[u].z;
        p3 += (double)v[u].w;
      }
  }
  const double c10 = canon_tree_wave(p0) / (double)n, c11 = canon_tree_wave(p1) / (double)n;
  const double c20 = canon_tree_wave(p2) / (double)n, c21 = canon_tree_wave(p3) / (double)n;
  p0 = kCanonZero;
  p1 = kCanonZero;
  for (int b = threadIdx.x; b < n; b += 64 * kLoU) {
    float4 v[kLoU];
    load_pts(xin, b, n, v);
#pragma unroll
    for (int u = 0; u < kLoU; ++u)
      if (b + 64 * u < n) {
        const double d0 = (double)v[u].x - c10, d1 = (double)v[u].y - c11;
        const double e0 = (double)v[u].z - c20, e1 = (double)v[u].w - c21;
        p0 += d0 * d0 + d1 * d1;
        p1 += e0 * e0 + e1 * e1;
      }
  }
  const double rms1 = sqrt(canon_tree_wave(p0) / (double)n);
  const double rms2 = sqrt(canon_tree_wave(p1) / (double)n);
  const double s1 = sqrt(2.0) / rms1, s2 = sqrt(2.0) / rms2;
  T1[0] = s1; T1[1] = 0.0; T1[2] = -s1 * c10;
  T1[3] = 0.0; T1[4] = s1; T1[5] = -s1 * c11;
  T1[6] = 0.0; T1[7] = 0.0; T1[8] = 1.0;
  T2[0] = s2; T2[1] = 0.0; T2[2] = -s2 * c20;
  T2[3] = 0.0; T2[4] = s2; T2[5] = -s2 * c21;
  T2[6] = 0.0; T2[7] = 0.0; T2[8] = 1.0;
}

// Packed entries [K0, K1) of the normal equations A^T A of the local
// estimators, summed in canonical order into s.ata.
template <int K, int K0, int K1>
__device__ __forceinline__ void ata_range_f4(VerifyLds& s, const float4* xin, int n,
                                             const double* T1, const double* T2) {
  constexpr int NE = K1 - K0;
  const int lane = threadIdx.x & 63;
  double part[NE];
#pragma unroll
  for (int k = 0; k < NE; ++k) part[k] = kCanonZero;
#pragma unroll 1
  for (int b = lane; b < n; b += 64 * kLoU) {
    float4 v[kLoU];
    load_pts(xin, b, n, v);
#pragma unroll
    for (int u = 0; u < kLoU; ++u) {
      if (b + 64 * u >= n) break;
      double x0, y0, x1, y1;
      apply_norm_affine(T1, (double)v[u].x, (double)v[u].y, &x0, &y0);
      apply_norm_affine(T2, (double)v[u].z, (double)v[u].w, &x1, &y1);
      double a[9], c[9];
      if (K == KIND_F) f_row(x0, y0, x1, y1, a);
      else h_rows(x0, y0, x1, y1, a, c);
      int k = 0;
#pragma unroll
      for (int p = 0; p < 9; ++p)
#pragma unroll
        for (int q = p; q < 9; ++q) {
          if (k >= K0 && k < K1) part[k - K0] = part[k - K0] + a[p] * a[q];
          ++k;
        }
      if (K == KIND_H) {
        k = 0;
#pragma unroll
        for (int p = 0; p < 9; ++p)
#pragma unroll
          for (int q = p; q < 9; ++q) {
            if (k >= K0 && k < K1) part[k - K0] = part[k - K0] + c[p] * c[q];
            ++k;
          }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    const double t = canon_tree_wave(part[k]);
    if (lane == 0) s.ata[K0 + k] = t;
  }
}
template <int K, int PASS>
__device__ __forceinline__ void ata_pass_f4(VerifyLds& s, const float4* xin, int n,
                                            const double* T1, const double* T2) {
  ata_range_f4<K, 15 * PASS, 15 * PASS + 15>(s, xin, n, T1, T2);
}

// The F / H local estimators (geom_solvers.h fundamental_8pt / homography_dlt
// n > 4) on packed points, canonical sums.
// NW = 4: the coordinate sums and the A^T A entries are split between the
// waves (each sum whole on one wave), the 9 x 9 null vector runs on wave 0.
template <int K, int NW = 1>
__device__ void local_estimate_f4(VerifyLds& s, const float4* xin, int n, double* model,
                                  uint64_t* pl = nullptr) {
  static_assert(NW == 1 || NW == 4, "one wave or four");
  uint64_t t0 = pl ? __builtin_amdgcn_s_memtime() : 0;
  double T1[9], T2[9];
  if (NW == 1) normalize_pair_f4(xin, n, T1, T2);
  else normalize_pair_f4_w4(xin, n, T1, T2, s.redd);
  if (pl && threadIdx.x == 0) { const uint64_t t = __builtin_amdgcn_s_memtime(); pl[1] += t - t0; t0 = t; }
  if (NW == 1) {
    ata_pass_f4<K, 0>(s, xin, n, T1, T2);
    ata_pass_f4<K, 1>(s, xin, n, T1, T2);
    ata_pass_f4<K, 2>(s, xin, n, T1, T2);
  } else {
    switch (threadIdx.x >> 6) {
      case 0: ata_range_f4<K, 0, 12>(s, xin, n, T1, T2); break;
      case 1: ata_range_f4<K, 12, 24>(s, xin, n, T1, T2); break;
      case 2: ata_range_f4<K, 24, 35>(s, xin, n, T1, T2); break;
      default: ata_range_f4<K, 35, 45>(s, xin, n, T1, T2); break;
    }
  }
  wsync();
  if (pl && threadIdx.x == 0) { const uint64_t t = __builtin_amdgcn_s_memtime(); pl[2] += t - t0; t0 = t; }
  double f[9];
  if (NW == 1) {
    invsq9_null_wave(s.ata, s.jA, s.jV, f);
  } else {
    if (threadIdx.x < 64) {
      invsq9_null_wave<true>(s.ata, s.jA, s.jV, f);
      if (threadIdx.x < 9) s.fvec[threadIdx.x] = f[threadIdx.x];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 9; ++i) f[i] = s.fvec[i];
  }
  wsync();
  if (pl && threadIdx.x == 0) { const uint64_t t = __builtin_amdgcn_s_memtime(); pl[3] += t - t0; t0 = t; }
  if (K == KIND_F) fundamental_8pt_finish(f, T1, T2, model);
  else homography_finish(f, T1, T2, model);
  if (pl && threadIdx.x == 0) pl[6] += __builtin_amdgcn_s_memtime() - t0;
}

struct RansacResult {
  int success;
  int num_inliers;
  int num_trials;
  int res_sel;  // which residual buffer holds the best model's residuals
};

// Makes s.best_sum the exact (index-order) sum of the best model's inlier
// residuals, computing it lazily from res_best the first time a tie needs it.
__device__ void ensure_best_sum(VerifyLds& s, const double* res_best, int n, double maxr) {
  if (s.best_sum_valid) return;
  const double bs = seq_inlier_sum(res_best, n, maxr);
  wsync();
  if (threadIdx.x == 0) {
    s.best_sum = bs;
    s.best_sum_valid = 1;
  }
  wsync();
}

// A tie on the inlier count: InlierSupportMeasurer's Compare keeps the model
// with the smaller residual sum -- its inlier residuals summed in index order,
// a strictly ordered chain (~15 cycles per point).  The compare is decided
// from bounds first, with the chains only when they cannot decide it:
//  * residual arrays equal bit for bit have equal sums: not better;
//  * otherwise the inlier residuals (m of them, each >= 0) summed in any order
//    give T within gamma(m - 1) S of their exact sum S, and so does the index-
//    order chain; hence |chain - T| <= E = 2 (m + 2) u T (u = 2^-53, with
//    margin for the rounding of E and of the compares), and when the intervals
//    [T - E, T + E] of the two models (E = 0 for a best sum already exact) are
//    disjoint, they order the chains' sums exactly as the chains would.
// Every thread of the block calls it (block barriers).  Returns whether the
// new model is better; *sum / *exact: its index-order sum when the chains ran.
template <int NW>
__device__ bool tie_better(VerifyLds& s, const double* rt, const double* rb, int n, int m,
                           double maxr, double* sum, bool* exact) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double tn = 0.0, tb = 0.0;
  bool diff = false;
  for (int i0 = wv * 64 * kSeqU + lane; i0 < n; i0 += 64 * kSeqU * NW) {
    double a[kSeqU], b[kSeqU];
#pragma unroll
    for (int u = 0; u < kSeqU; ++u) {
      const int i = min(i0 + 64 * u, n - 1);
      a[u] = rt[i];
      b[u] = rb[i];
    }
#pragma unroll
    for (int u = 0; u < kSeqU; ++u)
      if (i0 + 64 * u < n) {
        diff |= __double_as_longlong(a[u]) != __double_as_longlong(b[u]);
        if (a[u] <= maxr) tn += a[u];
        if (b[u] <= maxr) tb += b[u];
      }
  }
  tn = canon_tree_wave(tn);
  tb = canon_tree_wave(tb);
  int d = __ballot(diff) != 0 ? 1 : 0;
  if (NW > 1) {
    if (lane == 0) {
      s.redd[2 * wv] = tn;
      s.redd[2 * wv + 1] = tb;
      s.redi[wv] = d;
    }
    __syncthreads();
    tn = 0.0;
    tb = 0.0;
    d = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      tn += s.redd[2 * w];
      tb += s.redd[2 * w + 1];
      d |= s.redi[w];
    }
    __syncthreads();
  }
  *exact = false;
  if (!d) return false;
  const double g = 2.0 * (double)(m + 2) * 1.1102230246251565e-16;
  const double en = g * tn + 1e-300;
  const bool bex = s.best_sum_valid != 0;
  const double Tb = bex ? s.best_sum : tb;
  const double eb = bex ? 0.0 : g * tb + 1e-300;
  if (tn + en < Tb - eb) return true;
  if (tn - en > Tb + eb) return false;
  *sum = seq_inlier_sum(rt, n, maxr);
  ensure_best_sum(s, rb, n, maxr);
  *exact = true;
  return *sum < s.best_sum;
}

// LORANSAC<Estimator, LocalEstimator>::Estimate on n points (pts: packed
// x1, y1, x2, y2; the watermark's translation RANSAC, KIND_T).  res0 / res1:
// residual buffers (n doubles each); xin: inlier gather buffer (n points);
// snap: 625-word PRNG snapshot (global).  The best model ends in s.best_model.
// NW waves (8: small batches, verify_final_kernel<8>; KIND_T): every wave runs
// the same decisions; the point loops split as in the windowed replay.
template <int K, int NW = 1>
__device__ __attribute__((always_inline)) RansacResult loransac_wave(VerifyLds& s, uint32_t* sidx,
                                      const float4* pts, int n, int max_trials,
                                      const VerifyParams P, double* res0, double* res1,
                                      float4* xin, uint32_t* snap, double* mbuf, Prof pf,
                                      uint32_t* scrib = nullptr) {
  using Tr = KindTraits<K>;
  constexpr int MM = Tr::mm, MS = Tr::ms;
  const int lane = threadIdx.x & 63;
  const bool t0th = threadIdx.x == 0;
  constexpr int BS = 64 * NW;
  const double maxr = P.max_residual;
  RansacResult out = {0, 0, 0, 0};
  if (threadIdx.x < 9) s.best_model[threadIdx.x] = 0.0;  // report.model when no model is found
  if (t0th) {
    s.best_n = 0;
    s.best_sum = 1.7976931348623157e308;  // Support() default: DBL_MAX
    s.best_sum_valid = 1;
  }
  wsync();
  if (n < Tr::kmin) return out;
  for (int i = threadIdx.x; i < n; i += BS) sidx[i] = (uint32_t)i;
  double* res[2] = {res0, res1};
  int best_sel = 0;
  int dyn_max = max_trials;
  int trial = 0;
  bool abort = false;
  int abort_trial = -1;
  wsync();

  while (trial < max_trials && !abort) {
    const int B = min(Tr::tb, max_trials - trial);
    pf.lap(PR_OTHER);
    pf.count(PR_N_BATCH);
    // -- snapshot the PRNG (global), draw B samples (Shuffle of the persistent
    //    index vector, RandomSampler::Sample).
    for (int i = threadIdx.x; i < 624; i += BS) snap[i] = s.mt[i];
    if (t0th) snap[624] = (uint32_t)s.mt_idx;
    if (scrib) {
      // Diagnostics (SCM_DIAG_SCRIBBLE_F_SIDX, verify_final_kernel): rewrite the
      // F area's index vector before every draw, as a speculative F window's
      // draws may at any point of this RANSAC.  It must change nothing.
      for (int i = threadIdx.x; i < n; i += BS) scrib[i] = 0u;
    }
    wsync();
    if (draw_targets_wave<Tr::kmin>(s, B * Tr::kmin, (uint32_t)n)) {
      if (t0th) shuffle_batch_lane0<Tr::kmin>(s, sidx, B);
    } else {  // a draw may need rejection sampling: serial replay from the snapshot
      for (int i = threadIdx.x; i < 624; i += BS) s.mt[i] = snap[i];
      wsync();
      if (t0th) {
        s.mt_idx = (int32_t)snap[624];
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
    }
    for (int i = threadIdx.x; i < kTrialBatch * 3; i += BS) s.counts[i] = 0u;
    wsync();
    pf.lap(PR_SAMPLE);
    // -- solve the B minimal samples, one lane each; models go to the pair's
    //    model buffer (global, L1/L2-resident), counts of models to LDS.
    if ((int)threadIdx.x < B) {  // wave 0
      double a[2 * 7], b[2 * 7];
#pragma unroll
      for (int i = 0; i < Tr::kmin; ++i) {
        const float4 v = pts[s.samples[lane][i]];
        a[2 * i] = (double)v.x;
        a[2 * i + 1] = (double)v.y;
        b[2 * i] = (double)v.z;
        b[2 * i + 1] = (double)v.w;
      }
      double* mo = mbuf + lane * (MM * MS);
      int nm = 1;
      if (K == KIND_F) nm = fundamental_7pt(a, b, mo);
      else if (K == KIND_H) homography_dlt(a, b, 4, mo);
      else translation_estimate(a, b, 1, mo);
      s.nmodels[lane] = nm;
    }
    wsync();
    pf.lap(PR_SOLVE);
    // -- score: every lane reloads its own trial's models into registers; the
    //    points are streamed once in register chunks and each model is
    //    broadcast with v_readlane; exact inlier counts via ballot.
    {
    double m[MM][MS];
    int nm = 0;
    if (lane < B) {
      nm = s.nmodels[lane];
      const double* src = mbuf + lane * (MM * MS);
#pragma unroll
      for (int k = 0; k < MM; ++k)
#pragma unroll
        for (int j = 0; j < MS; ++j) m[k][j] = src[k * MS + j];
    } else {
#pragma unroll
      for (int k = 0; k < MM; ++k)
#pragma unroll
        for (int j = 0; j < MS; ++j) m[k][j] = 0.0;
    }
    constexpr int PC = 8;  // points per lane per chunk
    for (int base = (int)(threadIdx.x >> 6) * 64 * PC; base < n; base += 64 * PC * NW) {
      double pa0[PC], pa1[PC], pb0[PC], pb1[PC];
      bool ok[PC];
#pragma unroll
      for (int p = 0; p < PC; ++p) {
        const int i = base + p * 64 + lane;
        ok[p] = i < n;
        const float4 v = pts[ok[p] ? i : 0];
        pa0[p] = (double)v.x;
        pa1[p] = (double)v.y;
        pb0[p] = (double)v.z;
        pb1[p] = (double)v.w;
      }
      for (int t = 0; t < B; ++t) {
        const int nmt = __builtin_amdgcn_readlane(nm, t);
#pragma unroll
        for (int k = 0; k < MM; ++k) {
          if (k < nmt) {
            double mk[MS];
#pragma unroll
            for (int j = 0; j < MS; ++j) mk[j] = readlane_d(m[k][j], t);
            int c = 0;
#pragma unroll
            for (int p = 0; p < PC; ++p) {
              bool in;
              if (K == KIND_F) in = sampson_inlier(mk, pa0[p], pa1[p], pb0[p], pb1[p], maxr);
              else in = residual_pt<K>(mk, pa0[p], pa1[p], pb0[p], pb1[p]) <= maxr;
              c += __popcll(__ballot(ok[p] && in));
            }
            if (lane == 0) {
              if (NW == 1) s.counts[t * MM + k] += (uint32_t)c;
              else atomicAdd(&s.counts[t * MM + k], (uint32_t)c);
            }
          }
        }
      }
    }
    }
    wsync();
    pf.lap(K == KIND_H ? PR_SCORE_H : PR_SCORE);
    // -- replay the trials in order.
    for (int t = 0; t < B && !abort; ++t) {
      const int tt = trial + t;
      const int nmt = s.nmodels[t];
      for (int k = 0; k < MM; ++k) {
        if (k < nmt && !abort) {
          const int c = (int)s.counts[t * MM + k];
          const int bn = s.best_n;
          if (c >= bn) {
            double mk[MS];
            const double* src = mbuf + (t * MM + k) * MS;
#pragma unroll
            for (int j = 0; j < MS; ++j) mk[j] = src[j];
            pf.lap(PR_OTHER);
            pf.count(PR_N_CAND);
            double* rt = res[best_sel ^ 1];
            residuals_gather_f4<K, NW>(mk, pts, n, maxr, rt, xin, s.redi);
            pf.lap(PR_CAND);
            bool better = c > bn, exact = false;
            double sum = 0.0;
            if (!better) {  // tie on the inlier count: Compare the residual sums
              better = tie_better<NW>(s, rt, res[best_sel], n, c, maxr, &sum, &exact);
              if (exact) pf.count(PR_N_SEQSUM);  // (the chains ran)
              pf.lap(PR_SEQSUM);
            }
            if (better) {
              wsync();
              if (t0th) {
#pragma unroll
                for (int j = 0; j < MS; ++j) s.best_model[j] = mk[j];
                s.best_n = c;
                s.best_sum = sum;
                s.best_sum_valid = exact ? 1 : 0;
              }
              best_sel ^= 1;
              wsync();
              // Recursive local optimisation.
              if (c > Tr::kmin && c >= Tr::kmin_local) {
                for (int lt = 0; lt < 10; ++lt) {
                  pf.lap(PR_OTHER);
                  pf.count(PR_N_LO);
                  const int ni = s.best_n;  // in xin from the best's residual pass
                  pf.lap(PR_GATHER);
                  double lm[9];
                  local_estimate_wave<K, NW>(s, xin, ni, lm);
                  pf.lap(PR_LOEST);
                  const int prev = s.best_n;
                  double* rl = res[best_sel ^ 1];
                  const int lc = residuals_gather_f4<K, NW>(lm, pts, n, maxr, rl, xin, s.redi);
                  pf.lap(PR_LORES);
                  bool lbetter = lc > prev, lexact = false;
                  double lsum = 0.0;
                  if (lc == prev) {
                    lbetter = tie_better<NW>(s, rl, res[best_sel], n, lc, maxr, &lsum, &lexact);
                    if (lexact) pf.count(PR_N_SEQSUM);
                    pf.lap(PR_SEQSUM);
                  }
                  if (lbetter) {
                    wsync();
                    if (t0th) {
#pragma unroll
                      for (int j = 0; j < MS; ++j) s.best_model[j] = lm[j];
                      s.best_n = lc;
                      s.best_sum = lsum;
                      s.best_sum_valid = lexact ? 1 : 0;
                    }
                    best_sel ^= 1;
                  }
                  wsync();
                  if (s.best_n <= prev) break;
                }
              }
              dyn_max = (int)min((uint64_t)0x7FFFFFFF,
                                 num_trials((uint64_t)s.best_n, (uint64_t)n, P.confidence,
                                            P.dyn_num_trials_multiplier, Tr::kmin));
            }
          }
          if (tt >= dyn_max && tt >= P.min_num_trials) {
            abort = true;
            abort_trial = tt;
          }
        }
      }
    }
    if (abort) {
      // Rewind the PRNG to the state right after trial abort_trial's sample.
      wsync();
      for (int i = threadIdx.x; i < 624; i += BS) s.mt[i] = snap[i];
      wsync();
      if (t0th) {
        s.mt_idx = (int32_t)snap[624];
        const uint32_t last = (uint32_t)(n - 1);
        for (int b = 0; b <= abort_trial - trial; ++b)
          for (int i = 0; i < Tr::kmin; ++i) (void)uniform_u32(s, (uint32_t)i, last);
      }
      wsync();
      out.num_trials = abort_trial + 2;
    } else {
      trial += B;
      out.num_trials = trial;
    }
  }
  pf.lap(PR_OTHER);
  pf.count(PR_N_TRIALS, (uint64_t)out.num_trials);
  pf.count(PR_N_POINTS, (uint64_t)n);
  // res[best_sel] holds the residuals of the best model (every accepted
  // model had its residuals written to the buffer that became res[best_sel]).
  out.num_inliers = s.best_n;
  out.success = s.best_n >= Tr::kmin ? 1 : 0;
  out.res_sel = best_sel;
  wsync();
  return out;
}

// ---------------------------------------------------------------------------
// Per-pair state shared by the windowed kernels and verify_final_kernel (one
// wavefront per pair): the F / H models and counts travel in the pair's
// VerifyOut record, the PRNG state in the pair's snapshot words.
// ---------------------------------------------------------------------------
struct PairSetup {
  VerifyPair pp;
  int n;
  uint32_t* state;  // 625 words: handed-on PRNG state
  uint32_t* snap;   // 625 words: per-batch snapshot (abort rewind)
  double* base;     // 10 n + kVerifyModelDoubles doubles of scratch
  VerifyOut* o;
};

__device__ __forceinline__ PairSetup pair_setup(const VerifyPair* pairs, double* scratch,
                                                uint32_t* snaps, VerifyOut* out,
                                                const int32_t* counts) {
  PairSetup ps;
  ps.pp = pairs[blockIdx.x];
  ps.n = ps.pp.cidx >= 0 ? counts[ps.pp.cidx] : ps.pp.m;
  // the watermark RANSAC continues the H stream; F's scratch area is free
  ps.state = snaps + (int64_t)blockIdx.x * kVerifySnapWords + kVerifyStreamWords;
  ps.snap = ps.state + kVerifyStreamWords / 2;
  ps.base = scratch + ps.pp.scr_off;
  ps.o = out + ps.pp.out_idx;
  return ps;
}

__device__ __forceinline__ void mt_save(const VerifyLds& s, uint32_t* st) {
  for (int i = threadIdx.x; i < 624; i += blockDim.x) st[i] = s.mt[i];
  if (threadIdx.x == 0) st[624] = (uint32_t)s.mt_idx;
}

__device__ __forceinline__ void mt_load(VerifyLds& s, const uint32_t* st) {
  for (int i = threadIdx.x; i < 624; i += blockDim.x) s.mt[i] = st[i];
  if (threadIdx.x == 0) s.mt_idx = (int32_t)st[624];
  wsync();
}

// NW waves per pair (4 for small batches: the watermark LO-RANSAC is on the
// critical path of one Scanner stencil).
template <int NW>
__global__ __launch_bounds__(64 * NW) void verify_final_kernel(
    const VerifyPair* __restrict__ pairs, const double* __restrict__ xy1_all,
    const double* __restrict__ xy2_all, double* __restrict__ scratch,
    uint32_t* __restrict__ snaps, const uint8_t* __restrict__ masks,
    VerifyOut* __restrict__ out, VerifyParams P, uint64_t* __restrict__ prof,
    const int32_t* __restrict__ counts, RansacState* __restrict__ rstF,
    const RansacState* __restrict__ rstH, int phase,
    const uint32_t* __restrict__ spec_state) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
  VerifyLds& s = *reinterpret_cast<VerifyLds*>(dyn_lds);
  if (P.prio) __builtin_amdgcn_s_setprio(2);
  // phase 1 (early, small batches): only pairs whose F and H RANSACs are both
  // done (read once, by thread 0: the replay of other pairs is still
  // running); phase 2: after every window, every pair; each pair is claimed
  // once, by whichever of the two runs first (rstF[q].pad_, atomically: the
  // two may run at once).  phase 0: every pair.
  // phase 3 (speculative, small batches; beside H's last window): the
  // watermark decision only, of the pairs whose F is done, into
  // VerifyOut::spec / spec_wm -- from H's final stream state when H is done
  // (spec 1), else from spec_state, the state after H's last window's draws
  // (spec 2), which that window's replay leaves as H's final state unless it
  // aborts H (RansacState::aborted).  Phases 1 / 2 take the decision when
  // spec is 1, or 2 and H did not abort, and run the watermark RANSAC
  // otherwise: the same decision either way.
  // Bit 8 of the argument: diagnostics (loransac_wave's scrib); bit 16:
  // diagnostics, phases 1 / 2 recompute a speculative decision they would
  // take and record whether it was equal (VerifyOut::spec_check).
  const bool scrib = (phase & 8) != 0;
  const bool chk = (phase & 16) != 0;
  phase &= 3;
  int src = 0;  // phase 3: the decision's state source (1 / 2)
  if (phase != 0) {
    if (threadIdx.x == 0) {
      const int q0 = blockIdx.x;
      const int fd = *reinterpret_cast<volatile const int32_t*>(&rstF[q0].done);
      const int hd = *reinterpret_cast<volatile const int32_t*>(&rstH[q0].done);
      const int mk = *reinterpret_cast<volatile const int32_t*>(&rstF[q0].pad_);
      int go;
      if (phase == 3) go = fd ? (hd ? 1 : 2) : 0;
      else go = (phase == 2 || (fd && hd)) && !mk && atomicCAS(&rstF[q0].pad_, 0, 1) == 0;
      s.redi[15] = go;
      __threadfence();
    }
    __syncthreads();
    const int go = s.redi[15];
    __syncthreads();
    if (!go) return;
    if (phase == 3) src = go;
  }
  Prof pf{prof ? prof + (int64_t)blockIdx.x * kVerifyProfSlots : nullptr, &s.prof_t};
  pf.start();
  const PairSetup ps = pair_setup(pairs, scratch, snaps, out, counts);
  const int n = ps.n, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // The watermark RANSAC's sample-index vector lives in the pair's H scratch
  // area, its points and residuals in the F area (layout below).  H is done
  // when this kernel runs for a pair and no H draws follow H's last window,
  // while the F area's index vector may still be rewritten: in a small batch
  // the early pass (phase 1) runs beside the later windows, whose F draws are
  // speculative -- window r + 1's draws take the pairs that were running one
  // window back, so a pair whose F stopped in window r (or whose stop phase 1
  // observes during window r + 1's replay) is drawn once more.  The draws
  // write nothing else in the pair's scratch (pair_sidx only).
  uint32_t* fsidx = reinterpret_cast<uint32_t*>(ps.base + 10 * (int64_t)n + kVerifyModelDoubles);
  uint32_t* sidx = reinterpret_cast<uint32_t*>(ps.base + verify_kind_scratch_doubles(n) +
                                               10 * (int64_t)n + kVerifyModelDoubles);
  if (!(n >= P.min_num_inliers && n > 0)) return;
  const double* xy1 = xy1_all + ps.pp.pts_off;
  const double* xy2 = xy2_all + ps.pp.pts_off;
  const uint8_t* mask = masks + ps.pp.mask_off;
  VerifyOut* o = ps.o;
  const int f_in = o->f_inliers_raw, h_in = o->h_inliers_raw;
  const bool f_ok = f_in >= KindTraits<KIND_F>::kmin, h_ok = h_in >= KindTraits<KIND_H>::kmin;
  const int mni = P.min_num_inliers;
  // DetectWatermark's decision (1: the F inliers are mostly one 2-D
  // translation) from the H stream state st: the watermark RANSAC continues
  // H's generator.
  auto detect_wm = [&](const uint32_t* st) -> int {
    // DetectWatermark with the dummy cameras (width = height = 0): a point
    // is inside the [0,0]x[0,0] box only if it is exactly (0, 0).
    int nb = 0;
    for (int b = wv * 64 * kSeqU + lane; b < n; b += 64 * kSeqU * NW) {
      uint8_t mk[kSeqU];
      double a0[kSeqU], a1[kSeqU], c0[kSeqU], c1[kSeqU];
#pragma unroll
      for (int u = 0; u < kSeqU; ++u) {
        const int i = min(b + 64 * u, n - 1);
        mk[u] = b + 64 * u < n ? mask[i] : 0;
        a0[u] = xy1[2 * i];
        a1[u] = xy1[2 * i + 1];
        c0[u] = xy2[2 * i];
        c1[u] = xy2[2 * i + 1];
      }
#pragma unroll
      for (int u = 0; u < kSeqU; ++u) {
        const bool in1 = a0[u] >= 0.0 && a0[u] <= 0.0 && a1[u] >= 0.0 && a1[u] <= 0.0;
        const bool in2 = c0[u] >= 0.0 && c0[u] <= 0.0 && c1[u] >= 0.0 && c1[u] <= 0.0;
        nb += (mk[u] && !in1 && !in2) ? 1 : 0;
      }
    }
    nb = wave_sum_i(nb);
    if (NW > 1) {
      if (lane == 0) s.redi[wv] = nb;
      __syncthreads();
      nb = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) nb += s.redi[w];
      __syncthreads();
    }
    const int ni = f_in;
    const double bratio = (double)nb / (double)ni;
    if (bratio < P.watermark_min_inlier_ratio) return 0;
    {
      // Inlier points in index order -> translation LO-RANSAC, on packed
      // fp32 points (the doubles are widened float32 keypoints: exact both
      // ways; half the bytes of every point loop).  Scratch layout (10n
      // doubles; float4 arrays 16-B aligned): tin [0,2ni+1) tres0
      // [2n+2,2n+2+ni) tres1 [3n+2,3n+2+ni) tx [4n+2,4n+3+2ni).
      double* base = ps.base;
      auto align16 = [](double* p) {
        return reinterpret_cast<float4*>((reinterpret_cast<uintptr_t>(p) + 15) & ~(uintptr_t)15);
      };
      float4* tin = align16(base);
      int w = 0;
      for (int r0 = 0; r0 < n; r0 += 64 * kSeqU * NW) {
        const int b0 = r0 + wv * 64 * kSeqU;
        uint8_t mk[kSeqU];
        double a0[kSeqU], a1[kSeqU], c0[kSeqU], c1[kSeqU];
#pragma unroll
        for (int u = 0; u < kSeqU; ++u) {
          const int i = b0 + 64 * u + lane, ic = min(i, n - 1);
          mk[u] = i < n ? mask[ic] : 0;
          a0[u] = xy1[2 * ic];
          a1[u] = xy1[2 * ic + 1];
          c0[u] = xy2[2 * ic];
          c1[u] = xy2[2 * ic + 1];
        }
        uint64_t bal[kSeqU];
        int wc = 0;
#pragma unroll
        for (int u = 0; u < kSeqU; ++u) {
          bal[u] = __ballot(mk[u] != 0);
          wc += __popcll(bal[u]);
        }
        int before = 0, total = wc;
        if (NW > 1) {
          if (lane == 0) s.redi[wv] = wc;
          __syncthreads();
          total = 0;
#pragma unroll
          for (int q = 0; q < NW; ++q) {
            const int x = s.redi[q];
            before += q < wv ? x : 0;
            total += x;
          }
          __syncthreads();
        }
        int o = w + before;
#pragma unroll
        for (int u = 0; u < kSeqU; ++u) {
          if (mk[u]) {
            const int o2 = o + (int)__builtin_amdgcn_mbcnt_hi(
                                   (uint32_t)(bal[u] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal[u], 0u));
            tin[o2] = make_float4((float)a0[u], (float)a1[u], (float)c0[u], (float)c1[u]);
          }
          o += __popcll(bal[u]);
        }
        w += total;
      }
      if (NW > 1) __syncthreads();
      mt_load(s, st);
      const RansacResult rt = loransac_wave<KIND_T, NW>(s, sidx, tin, ni, P.max_trials_T, P,
                                                    base + 2 * n + 2, base + 3 * n + 2,
                                                    align16(base + 4 * n + 2), ps.snap,
                                                    base + 10 * n, pf, scrib ? fsidx : nullptr);
      const double iratio = (double)rt.num_inliers / (double)ni;
      return iratio >= P.watermark_min_inlier_ratio ? 1 : 0;
    }
  };
  if (phase == 3) {
    const int wm = P.detect_watermark && f_ok
                       ? detect_wm(src == 2 ? spec_state + (int64_t)blockIdx.x * kVerifyStateWords
                                            : ps.state)
                       : 0;
    if (threadIdx.x == 0) {
      o->spec_wm = wm;
      o->spec = src;
    }
    return;
  }
  // a decision phase 3 took (thread 0 reads, every thread uses it)
  if (threadIdx.x == 0) {
    const int sp = o->spec;
    const bool valid = sp == 1 || (sp == 2 && !rstH[blockIdx.x].aborted);
    s.redi[14] = valid ? 1 + o->spec_wm : 0;
    s.redi[13] = sp == 2 && !valid ? 4 : 0;
  }
  __syncthreads();
  const int known = s.redi[14];
  int check = s.redi[13];
  __syncthreads();
  int config, num_inliers = 0, watermark = 0;
  if ((!f_ok && !h_ok) || (f_in < mni && h_in < mni)) {
    config = SCM_TVG_DEGENERATE;
  } else {
    const double ratio = (double)h_in / (double)f_in;
    config = ratio > P.max_H_inlier_ratio ? SCM_TVG_PLANAR_OR_PANORAMIC : SCM_TVG_UNCALIBRATED;
    num_inliers = f_ok ? f_in : 0;
    if (P.detect_watermark && f_ok) {
      int wm;
      if (known && chk) {
        wm = detect_wm(ps.state);
        check = wm == known - 1 ? 1 : 2;
      } else if (known) {
        wm = known - 1;
        check = 3;
      } else {
        wm = detect_wm(ps.state);
      }
      if (wm) {
        config = SCM_TVG_WATERMARK;
        watermark = 1;
      }
    }
  }
  if (threadIdx.x == 0) {
    o->spec = 0;
    o->spec_check = check;
  }
  // Post-filter (sequential_matching.cc:173-178): TwoViewGeometry().
  const bool keep = num_inliers >= mni;
  if (threadIdx.x == 0) {
    o->config = keep ? config : 0;
    o->num_inliers = keep ? num_inliers : 0;
    o->watermark = watermark;
    o->raw_config = config;  // EstimateMultiple (multiple_models) reads the unfiltered result
  }
  if (!keep && threadIdx.x < 9) {
    o->F[threadIdx.x] = 0.0;
    o->H[threadIdx.x] = 0.0;
  }
}

// ---------------------------------------------------------------------------
// Windowed LO-RANSAC (F and H).  All pairs of a batch advance together one
// window at a time; a window holds W rounds of up to 64 hypotheses per pair
// (W = 1, 2, 4, 8, 16, 16, ...: most F runs stop within a round or two, the
// long runs get wide windows):
//   rs_sample  (one wave per pair)  RandomSampler draws + Shuffle for every
//                                   trial of the window; the PRNG state at the
//                                   start of each round is kept for the rewind
//   rs_solve   (one thread per hypothesis) minimal solver + filter constants
//   rs_score   (blocks of 256 threads over (pair, 1024-point chunk)) inlier
//                                   counts of every model of the window
//   rs_replay  (one wave per pair)  the sequential LO-RANSAC decisions in
//                                   trial order (Compare, local optimisation,
//                                   dynamic trial bound, abort + PRNG rewind)
// Hypotheses past a pair's abort point are discarded, exactly as the serial
// algorithm never draws them; the expensive scoring runs as a wide, regular
// kernel and the sequential parts cost one short kernel per window.
// ---------------------------------------------------------------------------
// Kind K's PRNG stream words and scratch area of pair q (F and H run
// concurrently, each on its own).
template <int K>
__device__ __forceinline__ PairSetup pair_at(const VerifyPair* pairs, int q, double* scratch,
                                             uint32_t* snaps, VerifyOut* out) {
  PairSetup ps;
  ps.pp = pairs[q];
  ps.n = ps.pp.m;
  ps.state = snaps + (int64_t)q * kVerifySnapWords + (K == KIND_H ? kVerifyStreamWords : 0);
  ps.snap = ps.state + kVerifyStreamWords / 2;
  ps.base = scratch + ps.pp.scr_off + (K == KIND_H ? verify_kind_scratch_doubles(ps.n) : 0);
  ps.o = out + ps.pp.out_idx;
  return ps;
}

__device__ __forceinline__ uint32_t* pair_sidx(const PairSetup& ps) {
  return reinterpret_cast<uint32_t*>(ps.base + 10 * (int64_t)ps.n + kVerifyModelDoubles);
}

// Per-pair results of a finished RANSAC into the pair's VerifyOut (and, for
// F, the inlier mask ExtractInlierMatches reads).
template <int K>
__device__ void rs_finish(const PairSetup& ps, const RansacState& st, uint8_t* masks,
                          double maxr) {
  const int lane = threadIdx.x;  // block-wide (one or several waves)
  const int n = ps.n;
  if (K == KIND_F) {
    uint8_t* mask = masks + ps.pp.mask_off;
    const double* resb = ps.base + (st.res_sel ? n : 0);
    const bool ok = st.best_n >= KindTraits<K>::kmin;
    for (int i = lane; i < n; i += blockDim.x) mask[i] = (ok && resb[i] <= maxr) ? 1 : 0;
    if (lane < 9) ps.o->F[lane] = st.best_model[lane];
    if (lane == 0) {
      ps.o->f_trials = st.num_trials;
      ps.o->f_inliers_raw = st.best_n;
      ps.o->f_evals = st.evals;
    }
  } else {
    if (lane < 9) ps.o->H[lane] = st.best_model[lane];
    if (lane == 0) {
      ps.o->h_trials = st.num_trials;
      ps.o->h_inliers_raw = st.best_n;
      ps.o->h_evals = st.evals;
    }
  }
}

// Start of a RANSAC for every pair: state, sample-index vector, the kind's
// PRNG stream seeded (F: pair_seed, H: pair_seed_h).  Pairs with fewer points than
// the minimal sample finish at once (LORANSAC returns an empty report).
template <int K>
__device__ __attribute__((always_inline)) void rs_begin_body(
    const VerifyPair* __restrict__ pairs, int npairs, double* __restrict__ scratch,
    uint32_t* __restrict__ snaps, VerifyOut* __restrict__ out, uint8_t* __restrict__ masks,
    const float4* __restrict__ xyf_all, RansacState* __restrict__ rst,
    int32_t* __restrict__ act, int32_t* __restrict__ nact, uint32_t* __restrict__ pstate,
    int32_t* __restrict__ dtrial, VerifyParams P, int bid, int nblk) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
  VerifyLds& s = *reinterpret_cast<VerifyLds*>(dyn_lds);
  using Tr = KindTraits<K>;
  const int lane = threadIdx.x;
  for (int q = bid; q < npairs; q += nblk) {
    const PairSetup ps = pair_at<K>(pairs, q, scratch, snaps, out);
    const int n = ps.n;
    const float4* xyf = xyf_all + ps.pp.pts_off / 2;
    float smax = 0.0f;
    for (int i0 = lane; i0 < n; i0 += 64 * 8) {  // eight loads in flight (clamped: same max)
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = xyf[min(i0 + 64 * u, n - 1)];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        smax = fmaxf(smax, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) smax = fmaxf(smax, __shfl_xor(smax, d));
    wsync();
    if (lane == 0)
      mt_seed(s, K == KIND_F ? pair_seed(P.base_seed, ps.pp.id1, ps.pp.id2)
                             : pair_seed_h(P.base_seed, ps.pp.id1, ps.pp.id2));
    wsync();
    mt_save(s, ps.state);
    mt_save(s, pstate + (int64_t)q * kVerifyStateWords);  // where window 0's draws start
    uint32_t* sidx = pair_sidx(ps);
    for (int i = lane; i < n; i += 64) sidx[i] = (uint32_t)i;
    if (lane == 0) {
      dtrial[q] = 0;
      RansacState& st = rst[q];
      st.n = n;
      st.max_trials = K == KIND_F ? P.max_trials_F : P.max_trials_H;
      st.trial = 0;
      st.dyn_max = st.max_trials;
      st.best_n = 0;
      st.best_sum_valid = 1;
      st.res_sel = 0;
      st.B = 0;
      st.num_trials = 0;
      st.evals = 0;
      st.done = (n < Tr::kmin || st.max_trials <= 0) ? 1 : 0;
      st.pad_ = 0;
      st.aborted = 0;
      if (K == KIND_F) ps.o->spec = 0;  // (verify_final_kernel phase 3)
      st.best_sum = 1.7976931348623157e308;  // Support() default: DBL_MAX
      st.S = (double)smax;
#pragma unroll
      for (int j = 0; j < 9; ++j) st.best_model[j] = 0.0;
      if (!st.done) act[atomicAdd(nact, 1)] = q;
    }
    wsync();
    if (rst[q].done) rs_finish<K>(ps, rst[q], masks, P.max_residual);
  }
}

// Draws of one window: B = min(64 W, max_trials - trial) samples of kmin
// indices (RandomSampler::Sample); the PRNG state before each round of 64 is
// kept in wsnap for the abort rewind, the state after the window in snaps.
template <int K>
__device__ __attribute__((always_inline)) void rs_draw_body(
    const VerifyPair* __restrict__ pairs, double* __restrict__ scratch,
    uint32_t* __restrict__ snaps, VerifyOut* __restrict__ out, RansacState* __restrict__ rst,
    const int32_t* __restrict__ act, const int32_t* __restrict__ nact,
    int32_t* __restrict__ nact_next, uint32_t* __restrict__ samp, uint32_t* __restrict__ cnts,
    uint32_t* __restrict__ ucnt, uint32_t* __restrict__ wsnap, int32_t* __restrict__ wB,
    const uint32_t* __restrict__ pstate, uint32_t* __restrict__ wstate,
    int32_t* __restrict__ dtrial, const uint32_t* __restrict__ pcnts,
    const int32_t* __restrict__ pwB, const VerifyParams& P, bool spec, int W, int bid, int nblk,
    int WT) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
  VerifyLds& s = *reinterpret_cast<VerifyLds*>(dyn_lds);
  using Tr = KindTraits<K>;
  const int lane = threadIdx.x;
  if (bid == 0 && lane == 0) *nact_next = 0;
  const int na = *nact;
  for (int a = bid; a < na; a += nblk) {
    const int q = act[a];
    const PairSetup ps = pair_at<K>(pairs, q, scratch, snaps, out);
    const int n = ps.n;
    // (the trials drawn so far, not the replay's count: this window may be
    // drawn while the previous one is still replayed)
    int Btot = max(0, min(kTrialBatch * W, trials_left(rst + q, dtrial[q], P.min_num_trials)));
    if (spec && Btot > 0) {
      // Speculative window: skip a pair certain to stop in the previous window.
      // Its best count after that window is at least every count the window
      // scored (a model above the best becomes the best; LO only adds), so
      // its trial bound is at most ComputeNumTrials(cmax); if that bound
      // falls inside the previous window, the pair aborts there.
      const int Bp = pwB[q];
      const uint32_t* pc = pcnts + (int64_t)q * WT * 3;
      uint32_t cm = 0;
      for (int i = lane; i < Bp * Tr::mm; i += 64) cm = max(cm, pc[i]);
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) cm = max(cm, (uint32_t)__shfl_xor((int)cm, d));
      const int last = dtrial[q] - 1;  // the previous window's last trial
      const uint64_t bound = num_trials((uint64_t)cm, (uint64_t)n, P.confidence,
                                        P.dyn_num_trials_multiplier, Tr::kmin);
      if (Bp > 0 && last >= P.min_num_trials && (uint64_t)last >= bound) Btot = 0;
    }
    wsync();
    mt_load(s, pstate + (int64_t)q * kVerifyStateWords);
    uint32_t* sq = samp + (int64_t)q * WT * 8;
    for (int w = 0; w * kTrialBatch < Btot; ++w) {
      const int B = min(kTrialBatch, Btot - w * kTrialBatch);
      if (w == 0) {  // the window's start state, for the abort rewind
        uint32_t* snap = wsnap + (int64_t)q * 640;
        for (int i = lane; i < 624; i += 64) snap[i] = s.mt[i];
        if (lane == 0) snap[624] = (uint32_t)s.mt_idx;
      }
      // (the targets do not depend on the shuffle state)
      draw_round<Tr::kmin>(s, B * Tr::kmin, (uint32_t)n);
      wsync();
      for (int r = lane; r < B * Tr::kmin; r += 64)
        sq[(w * kTrialBatch + r / Tr::kmin) * 8 + r % Tr::kmin] = s.jbuf[r];
      wsync();
    }
    mt_save(s, wstate + (int64_t)q * kVerifyStateWords);
    uint32_t* cq = cnts + (int64_t)q * WT * 3;
    for (int i = lane; i < Btot * 3; i += 64) cq[i] = 0u;
    if (ucnt) {
      uint32_t* uq = ucnt + (int64_t)q * WT * 3;
      for (int i = lane; i < Btot * 3; i += 64) uq[i] = 0u;
    }
    if (lane == 0) {
      wB[q] = Btot;
      dtrial[q] += Btot;
    }
  }
}

// RandomSampler::Sample's Shuffle for every trial of the window: the swap
// chain of one pair is sequential, so each lane runs one pair's chain; the
// pairs' sample-index vectors are staged in LDS (kShuffleLdsKb per
// block) so that every swap costs one LDS round trip.  The targets drawn by
// rs_draw_kernel are read from samp and replaced by the trial's sample.
// One pair's swap chain over Btot trials: the trial's kmin targets are read
// from sq (next trial's in flight) and replaced by the trial's sample.  T:
// uint16 for an LDS-staged vector, uint32 in global memory.  (Keeping the kmin
// hot positions in registers with one batched read of the cold targets per
// trial measured slower: divergent per-lane selects, profiles/r02_l.)
template <int KM, typename T>
__device__ __forceinline__ void shuffle_chain(T* sid, uint32_t* sq, int Btot) {
  const uint4 z = make_uint4(0u, 0u, 0u, 0u);
  uint4 tn0 = Btot > 0 ? reinterpret_cast<const uint4*>(sq)[0] : z;
  uint4 tn1 = Btot > 0 && KM > 4 ? reinterpret_cast<const uint4*>(sq)[1] : z;
  for (int b = 0; b < Btot; ++b) {
    const uint32_t wv[8] = {tn0.x, tn0.y, tn0.z, tn0.w, tn1.x, tn1.y, tn1.z, tn1.w};
    if (b + 1 < Btot) {
      tn0 = reinterpret_cast<const uint4*>(sq + (b + 1) * 8)[0];
      if (KM > 4) tn1 = reinterpret_cast<const uint4*>(sq + (b + 1) * 8)[1];
    }
#pragma unroll
    for (int i = 0; i < KM; ++i) {  // std::swap(sidx[i], sidx[j]), as the reference writes it
      const uint32_t jj = wv[i];
      const T ti = sid[i];
      const T tj = sid[jj];
      sid[i] = tj;
      sid[jj] = ti;
    }
    uint4* o = reinterpret_cast<uint4*>(sq + b * 8);
    o[0] = make_uint4(sid[0], sid[1], sid[2], sid[3]);
    if (KM > 4) o[1] = make_uint4(sid[4], sid[5], sid[6], 0u);
  }
}

template <int K>
__device__ __attribute__((always_inline)) void rs_shuffle_body(
    const VerifyPair* __restrict__ pairs, double* __restrict__ scratch,
    uint32_t* __restrict__ snaps, VerifyOut* __restrict__ out,
    const int32_t* __restrict__ wB, const int32_t* __restrict__ act,
    const int32_t* __restrict__ nact, uint32_t* __restrict__ samp, int ppb, int stride, int bid, int nblk,
    int WT) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
  uint16_t* lsidx = reinterpret_cast<uint16_t*>(dyn_lds);
  const int na = *nact;
  const int a0 = bid * ppb;
  if (a0 >= na) return;
  const int np = min(ppb, na - a0);
  // Stage the sample-index vectors of this block's ppb pairs in LDS as uint16
  // (every thread helps; batches whose pairs have at most 65536 matches), run
  // one pair's swap chain per lane, write them back.  stride 0: larger pairs
  // -- one pair per block, swapped in place in global memory (uint32).
  const bool staged = stride > 0;
  if (staged)
    for (int l = 0; l < np; ++l) {
      const PairSetup pl = pair_at<K>(pairs, act[a0 + l], scratch, snaps, out);
      const uint32_t* g = pair_sidx(pl);
      for (int i = threadIdx.x; i < pl.n; i += 64) lsidx[l * stride + i] = (uint16_t)g[i];
    }
  __syncthreads();
  if ((int)threadIdx.x < np) {
    constexpr int KM = KindTraits<K>::kmin;
    const int q = act[a0 + threadIdx.x];
    uint32_t* sq = samp + (int64_t)q * WT * 8;
    const int Btot = wB[q];
    if (staged) shuffle_chain<KM>(lsidx + threadIdx.x * stride, sq, Btot);
    else shuffle_chain<KM>(pair_sidx(pair_at<K>(pairs, q, scratch, snaps, out)), sq, Btot);
  }
  __syncthreads();
  if (staged)
    for (int l = 0; l < np; ++l) {
      const PairSetup pl = pair_at<K>(pairs, act[a0 + l], scratch, snaps, out);
      uint32_t* g = pair_sidx(pl);
      for (int i = threadIdx.x; i < pl.n; i += 64) g[i] = lsidx[l * stride + i];
    }
}

// The same window's Shuffle with a whole wave per pair, for small batches
// (one Scanner stencil: a lane per pair leaves nearly every lane, and the
// GPU, idle while one pair's chain of kmin dependent LDS round trips per
// trial runs).  The swap chain is split in time: pass of 64 x kWsC trials,
// lane L takes trials L*kWsC .. and runs their swaps on symbols -- the
// position each value had at its chunk's start -- keeping its chunk's
// touched positions in a per-lane open-addressing table in LDS (key j, symbol
// at j) and its head (positions 0 .. kmin-1) in registers.  The wave then
// walks the chunks in order over the real vector: a chunk's samples are the
// vector at their symbols, and its exit map (every touched position p takes
// the value at its symbol) moves the vector to the next chunk's start; every
// read of a step is issued before its writes (one wave: LDS operations
// complete in order), so the map applies as a permutation.  Same samples and
// final vector as the sequential chain, bit for bit.
constexpr int kWsC = 16;               // trials per lane and pass
constexpr int kWsTab = 256;            // table slots per lane (>= 2 x kmin x kWsC)
// (Lane tables 1 KiB apart: a 16-byte skew per lane, against LDS bank
// conflicts of the phase-A bucket reads, measured no change, round 5.)
constexpr int kWsPass = 64 * kWsC;     // trials per pass
constexpr int kWsRow = 65;             // trial slots per row of ssym (64 lanes + 1: no bank conflicts)
constexpr int kWsMaxStride = 32768;    // vector positions staged as uint16
static_assert(kWsTab == 64 * 4, "phase B reads a chunk's table as one uint4 per lane");

// LDS: the lanes' tables, the pass's trial slots (8 uint16: targets, then the
// sample's symbols), head symbols, the vector plus one dummy entry per lane
// (the target of the reads and writes of empty table slots: no branches).
size_t wave_shuffle_lds_bytes(int stride) {
  return (size_t)64 * kWsTab * 4 + (size_t)kWsC * kWsRow * 16 + 64 * 8 * 2 +
         (size_t)(stride + 64) * 2;
}

// The window's first trial, beside its start state in wsnap (decoupled draws:
// rs_prune_body reads it while later windows' draws advance dtrial).
constexpr int kWsnapFirst = 632;

// DRAW: the window's draws (rs_draw_body's work: RandomSampler targets from
// the pair's PRNG stream, round snapshots for the abort rewind, the trial
// counts) happen here too, straight into the trial slots in LDS -- one launch
// and no round trip of the targets through memory (small batches).
constexpr size_t kWsDrawHead = (kVerifyLdsHead + 15) / 16 * 16;
struct WsDraw {
  RansacState* rst;
  int32_t* nact_next;
  uint32_t* cnts;
  uint32_t* ucnt;
  uint32_t* wsnap;
  const uint32_t* pstate;
  uint32_t* wstate;
  int32_t* dtrial;
  const uint32_t* pcnts;
  const int32_t* pwB;
  int spec, W;
  int clr;  // clear the list the window's replay fills (0: rs_prune2_kernel does)
};

template <int K, bool DRAW = false>
__device__ __attribute__((always_inline)) void rs_shuffle_wave_body(
    const VerifyPair* __restrict__ pairs, double* __restrict__ scratch,
    uint32_t* __restrict__ snaps, VerifyOut* __restrict__ out,
    int32_t* __restrict__ wB, const int32_t* __restrict__ act,
    const int32_t* __restrict__ nact, uint32_t* __restrict__ samp, uint64_t* __restrict__ prof,
    int WT, int stride, int bid, int nblk, const WsDraw& dr = WsDraw{},
    const VerifyParams* Pp = nullptr) {
  constexpr int KM = KindTraits<K>::kmin;
  using Tr = KindTraits<K>;
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
  VerifyLds& s = *reinterpret_cast<VerifyLds*>(dyn_lds);  // DRAW: the PRNG state
  uint32_t* tab = reinterpret_cast<uint32_t*>(dyn_lds + (DRAW ? kWsDrawHead : 0));  // 64 x kWsTab: (j << 16) | symbol
  // Trial k of lane L's chunk lives in slot k * kWsRow + L (16 bytes).
  uint4* slots = reinterpret_cast<uint4*>(tab + 64 * kWsTab);
  uint16_t* hsym = reinterpret_cast<uint16_t*>(slots + kWsC * kWsRow);  // 64 x 8 head symbols
  uint16_t* V = hsym + 64 * 8;                                           // the vector (+ dummies)
  const int lane = threadIdx.x;
  const uint32_t dummy = (uint32_t)(stride + lane);
  if (DRAW && dr.clr && bid == 0 && lane == 0) *dr.nact_next = 0;
  const int na = *nact;
  for (int a = bid; a < na; a += nblk) {
    const int q = act[a];
    const PairSetup ps = pair_at<K>(pairs, q, scratch, snaps, out);
    uint32_t* g = pair_sidx(ps);
    const int n = ps.n;
    int Bdraw = 0;
    if (DRAW) {  // as rs_draw_body
      const VerifyParams& P = *Pp;
      Bdraw = max(0, min(kTrialBatch * dr.W,
                              trials_left(dr.rst + q, dr.dtrial[q], P.min_num_trials)));
      if (dr.spec && Bdraw > 0) {
        const int Bp = dr.pwB[q];
        const uint32_t* pc2 = dr.pcnts + (int64_t)q * WT * 3;
        uint32_t cm = 0;
        for (int i = lane; i < Bp * Tr::mm; i += 64) cm = max(cm, pc2[i]);
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) cm = max(cm, (uint32_t)__shfl_xor((int)cm, d));
        const int last = dr.dtrial[q] - 1;
        const uint64_t bound = num_trials((uint64_t)cm, (uint64_t)n, P.confidence,
                                          P.dyn_num_trials_multiplier, Tr::kmin);
        if (Bp > 0 && last >= P.min_num_trials && (uint64_t)last >= bound) Bdraw = 0;
      }
      wsync();
      mt_load(s, dr.pstate + (int64_t)q * kVerifyStateWords);
    }
    // Diagnostic phase cycles (SCM_PROFILE=1 only): staging, phase A, phase B, write-back.
    uint64_t* pc = prof ? prof + (int64_t)q * kVerifyProfSlots + (K == KIND_F ? 60 : 65) : nullptr;
    uint64_t tp = pc ? __builtin_amdgcn_s_memtime() : 0;
    auto lap = [&](int k) {
      if (pc && lane == 0) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        pc[k] += t - tp;
        tp = t;
      }
    };
    for (int b = lane; b < n; b += 64 * 8) {
      uint32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = g[min(b + 64 * u, n - 1)];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (b + 64 * u < n) V[b + 64 * u] = (uint16_t)v[u];
    }
    __syncthreads();
    lap(0);
    uint32_t* sq = samp + (int64_t)q * WT * 8;
    const int Btot = DRAW ? Bdraw : wB[q];
    for (int p0 = 0; p0 < Btot; p0 += kWsPass) {
      const int np = min(kWsPass, Btot - p0);
      {
        uint4* t4 = reinterpret_cast<uint4*>(tab);
        for (int i = lane; i < 64 * kWsTab / 4; i += 64) t4[i] = make_uint4(0u, 0u, 0u, 0u);
      }
      // The pass's targets (drawn by rs_draw into samp) into the trial slots
      // as uint16 pairs, coalesced.
      // (All of a lane's loads are issued before the first LDS write: one
      // memory latency per pass, not one per trial.)
      if (DRAW) {
        // The pass's rounds of 64 draws: snapshot, targets into the slots.
        // (Measured round 5: drawing a whole pass per state stretch, each
        // draw's target stored straight into its slot, is slower -- F
        // targets 549K -> 777K cycles per pair: the per-draw slot addressing
        // and scattered 16-bit stores cost more than the round's barriers.)
        for (int w0 = 0; w0 * kTrialBatch < np; ++w0) {
          const int B = min(kTrialBatch, np - w0 * kTrialBatch);
          const int wg = p0 / kTrialBatch + w0;  // round of the window
          if (wg == 0) {  // the window's start state, for the abort rewind
            uint32_t* snap = dr.wsnap + (int64_t)q * 640;
            for (int i = lane; i < 624; i += 64) snap[i] = s.mt[i];
            if (lane == 0) snap[624] = (uint32_t)s.mt_idx;
          }
          draw_round<KM>(s, B * KM, (uint32_t)n);
          wsync();
          if (lane < B) {
            uint32_t tg[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) tg[i] = i < KM ? s.jbuf[lane * KM + i] : 0u;
            const int idx = w0 * kTrialBatch + lane;
            slots[(idx % kWsC) * kWsRow + idx / kWsC] =
                make_uint4(tg[0] | (tg[1] << 16), tg[2] | (tg[3] << 16), tg[4] | (tg[5] << 16),
                           tg[6] | (tg[7] << 16));
          }
          wsync();
        }
      } else {
        constexpr int U = kWsPass / 64;
        uint4 a0[U], a1[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int idx = min(lane + 64 * u, np - 1);
          a0[u] = reinterpret_cast<const uint4*>(sq + (p0 + idx) * 8)[0];
          a1[u] = KM > 4 ? reinterpret_cast<const uint4*>(sq + (p0 + idx) * 8)[1]
                         : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int idx = lane + 64 * u;
          if (idx < np)
            slots[(idx % kWsC) * kWsRow + idx / kWsC] =
                make_uint4(a0[u].x | (a0[u].y << 16), a0[u].z | (a0[u].w << 16),
                           a1[u].x | (a1[u].y << 16), a1[u].z | (a1[u].w << 16));
        }
      }
      __syncthreads();
      lap(4);
      // Phase A: this lane's chunk on symbols.
      uint32_t* mt = tab + lane * kWsTab;
      uint32_t R[KM];
#pragma unroll
      for (int i = 0; i < KM; ++i) R[i] = (uint32_t)i;
      const int kn = min(kWsC, max(0, np - lane * kWsC));
      uint4 nx = kn > 0 ? slots[lane] : make_uint4(0u, 0u, 0u, 0u);
      for (int k = 0; k < kn; ++k) {
        const uint32_t wv[8] = {nx.x & 0xffffu, nx.x >> 16, nx.y & 0xffffu, nx.y >> 16,
                                nx.z & 0xffffu, nx.z >> 16, nx.w & 0xffffu, nx.w >> 16};
        if (k + 1 < kn) nx = slots[(k + 1) * kWsRow + lane];
#pragma unroll
        for (int i = 0; i < KM; ++i) {  // std::swap(sidx[i], sidx[j])
          const uint32_t j = wv[i];
          if (j < (uint32_t)KM) {
            uint32_t ri = R[i];
#pragma unroll
            for (int k2 = i + 1; k2 < KM; ++k2) {
              const bool m = j == (uint32_t)k2;
              const uint32_t rk = R[k2];
              R[k2] = m ? ri : rk;
              ri = m ? rk : ri;
            }
            R[i] = ri;
          } else {
            // Buckets of 8 slots (two b128 reads, one round trip), filled
            // from slot 0 up: j is in its bucket before the first empty slot
            // or absent; a full bucket continues in the next one.
            uint32_t b = (j * 0x9E3779B1u) >> 27;
            uint32_t slot, sym;
            for (;;) {
              const uint4 x0 = reinterpret_cast<const uint4*>(mt + b * 8)[0];
              const uint4 x1 = reinterpret_cast<const uint4*>(mt + b * 8)[1];
              const uint32_t w[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
              uint32_t stop = 0u;
#pragma unroll
              for (int e = 0; e < 8; ++e)
                stop |= (w[e] == 0u || (w[e] >> 16) == j) ? (1u << e) : 0u;
              if (stop) {
                const uint32_t e = (uint32_t)__builtin_ctz(stop);
                uint32_t we = w[0];
#pragma unroll
                for (int e2 = 1; e2 < 8; ++e2) we = e == (uint32_t)e2 ? w[e2] : we;
                slot = b * 8 + e;
                sym = we ? (we & 0xffffu) : j;
                break;
              }
              b = (b + 1) & (kWsTab / 8 - 1);
            }
            mt[slot] = (j << 16) | R[i];
            R[i] = sym;
          }
        }
        uint32_t o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = i < KM ? R[i] : 0u;
        slots[k * kWsRow + lane] = make_uint4(o[0] | (o[1] << 16), o[2] | (o[3] << 16),
                                              o[4] | (o[5] << 16), o[6] | (o[7] << 16));
      }
#pragma unroll
      for (int i = 0; i < KM; ++i) hsym[lane * 8 + i] = (uint16_t)R[i];
      __syncthreads();
      lap(1);
      // Phase B: the chunks in order over the vector.  Entry e = lane + 64 r
      // of a chunk's samples is trial e / 8, index e % 8.
      const int nch = (np + kWsC - 1) / kWsC;
      const uint16_t* ss = reinterpret_cast<const uint16_t*>(slots);
      // A chunk's symbols and exit map do not depend on the vector: the next
      // chunk's are read while this one's vector reads are in flight.
      auto chunk_syms = [&](int c, uint32_t* sy, uint4* wd, uint32_t* hs) {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const int e = lane + 64 * r, i = e & 7, k = e >> 3;
          sy[r] = i < KM && c * kWsC + k < np ? (uint32_t)ss[(k * kWsRow + c) * 8 + i] : dummy;
        }
        *wd = reinterpret_cast<const uint4*>(tab + c * kWsTab)[lane];
        *hs = lane < KM ? (uint32_t)hsym[c * 8 + lane] : dummy;
      };
      auto src_of = [&](uint32_t w) { return w ? (w & 0xffffu) : dummy; };
      auto dst_of = [&](uint32_t w) { return w ? (w >> 16) : dummy; };
      uint32_t sy[2], hs;
      uint4 wd;
      chunk_syms(0, sy, &wd, &hs);
      for (int c = 0; c < nch; ++c) {
        const int tc = p0 + c * kWsC;
        const uint32_t sv0 = V[sy[0]], sv1 = V[sy[1]];
        const uint32_t v0 = V[src_of(wd.x)], v1 = V[src_of(wd.y)];
        const uint32_t v2 = V[src_of(wd.z)], v3 = V[src_of(wd.w)];
        const uint32_t hv = V[hs];
        const uint32_t d0 = dst_of(wd.x), d1 = dst_of(wd.y), d2 = dst_of(wd.z), d3 = dst_of(wd.w);
        const uint32_t dh = lane < KM ? (uint32_t)lane : dummy;
        if (c + 1 < nch) chunk_syms(c + 1, sy, &wd, &hs);
        V[d0] = (uint16_t)v0;
        V[d1] = (uint16_t)v1;
        V[d2] = (uint16_t)v2;
        V[d3] = (uint16_t)v3;
        V[dh] = (uint16_t)hv;
        const uint32_t svr[2] = {sv0, sv1};
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const int e = lane + 64 * r, i = e & 7, t = tc + (e >> 3);
          // rows as shuffle_chain writes them: kmin samples (+ a zero pad for F)
          if (t < p0 + np && (i < KM || KM > 4)) sq[t * 8 + i] = i < KM ? svr[r] : 0u;
        }
      }
      __syncthreads();
      lap(2);
    }
    for (int i = lane; i < n; i += 64) g[i] = V[i];
    if (DRAW) {
      mt_save(s, dr.wstate + (int64_t)q * kVerifyStateWords);
      uint32_t* cq = dr.cnts + (int64_t)q * WT * 3;
      for (int i = lane; i < Btot * 3; i += 64) cq[i] = 0u;
      if (dr.ucnt) {
        uint32_t* uq = dr.ucnt + (int64_t)q * WT * 3;
        for (int i = lane; i < Btot * 3; i += 64) uq[i] = 0u;
      }
      if (lane == 0) {
        wB[q] = Btot;
        dr.wsnap[(int64_t)q * 640 + kWsnapFirst] = (uint32_t)dr.dtrial[q];
        dr.dtrial[q] += Btot;
      }
    }
    __syncthreads();
    lap(3);
  }
}

__global__ __launch_bounds__(64) void rs_shuffle_wave2_kernel(
    const VerifyPair* __restrict__ pairs, double* __restrict__ scratch,
    uint32_t* __restrict__ snaps, VerifyOut* __restrict__ out, VerifyRoundBufs rf,
    VerifyRoundBufs rh, int ain, uint64_t* __restrict__ prof, int stride, int split) {
  if ((int)blockIdx.x < split)
    rs_shuffle_wave_body<KIND_F>(pairs, scratch, snaps, out, rf.wB, rf.act[ain], rf.nact + ain,
                                 rf.samp, prof, rf.wt, stride, blockIdx.x, split);
  else
    rs_shuffle_wave_body<KIND_H>(pairs, scratch, snaps, out, rh.wB, rh.act[ain], rh.nact + ain,
                                 rh.samp, prof, rh.wt, stride, blockIdx.x - split, gridDim.x - split);
}

// Draws and Shuffle of a window in one launch (small batches).
__global__ __launch_bounds__(64) void rs_drawshuffle_wave2_kernel(
    const VerifyPair* __restrict__ pairs, double* __restrict__ scratch,
    uint32_t* __restrict__ snaps, VerifyOut* __restrict__ out, VerifyRoundBufs rf,
    VerifyRoundBufs rh, int ain, int aclr, VerifyParams P, int spec, int Wf, int Wh,
    uint64_t* __restrict__ prof, int stride, int split, int clr) {
  if (P.prio) __builtin_amdgcn_s_setprio(2);
  if ((int)blockIdx.x < split) {
    const WsDraw d{rf.rst, rf.nact + aclr, rf.cnts, rf.ucnt, rf.wsnap, rf.pstate, rf.wstate,
                   rf.dtrial, rf.pcnts, rf.pwB, spec, Wf, clr};
    rs_shuffle_wave_body<KIND_F, true>(pairs, scratch, snaps, out, rf.wB, rf.act[ain],
                                       rf.nact + ain, rf.samp, prof, rf.wt, stride, blockIdx.x, split, d,
                                       &P);
  } else {
    const WsDraw d{rh.rst, rh.nact + aclr, rh.cnts, rh.ucnt, rh.wsnap, rh.pstate, rh.wstate,
                   rh.dtrial, rh.pcnts, rh.pwB, spec, Wh, clr};
    rs_shuffle_wave_body<KIND_H, true>(pairs, scratch, snaps, out, rh.wB, rh.act[ain],
                                       rh.nact + ain, rh.samp, prof, rh.wt, stride, blockIdx.x - split,
                                       gridDim.x - split, d, &P);
  }
}

// Decoupled draws (small batches, run_windows): window r's draws run on their
// own stream beside window r - 1's scoring, so the two steps of a window's
// draws that need window r - 1 to be scored run here instead, on the scoring
// stream, right before window r's solves: the list window r's replay fills
// (aclr) is cleared, and a pair certain to stop in window r - 1 (the bound of
// rs_draw_body's speculative skip, over window r - 1's counts) gets no trials
// in window r (wB = 0: its solves and scores exit; its draws are never used,
// since window r - 1's replay rewinds the pair's PRNG to its stop).  Window
// r - 1's last trial is the one before window r's first (kept by its draws in
// wsnap: later windows' draws may already have advanced dtrial).
template <int K>
__device__ __forceinline__ void rs_prune_body(const VerifyPair* __restrict__ pairs,
                                              const VerifyRoundBufs& rb, int ain,
                                              const VerifyParams& P, int bid, int nblk) {
  using Tr = KindTraits<K>;
  const int lane = threadIdx.x;
  const int WT = rb.wt;
  const int na = rb.nact[ain];
  for (int a = bid; a < na; a += nblk) {
    const int q = rb.act[ain][a];
    const int B = rb.wB[q];
    const int Bp = rb.pwB[q];
    if (B <= 0 || Bp <= 0) continue;
    const uint32_t* pc = rb.pcnts + (int64_t)q * WT * 3;
    uint32_t cm = 0;
    for (int i = lane; i < Bp * Tr::mm; i += 64) cm = max(cm, pc[i]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) cm = max(cm, (uint32_t)__shfl_xor((int)cm, d));
    const int last = (int)rb.wsnap[(int64_t)q * 640 + kWsnapFirst] - 1;
    const uint64_t bound = num_trials((uint64_t)cm, (uint64_t)pairs[q].m, P.confidence,
                                      P.dyn_num_trials_multiplier, Tr::kmin);
    if (last >= P.min_num_trials && (uint64_t)last >= bound && lane == 0) rb.wB[q] = 0;
  }
}

__global__ __launch_bounds__(64) void rs_prune2_kernel(const VerifyPair* __restrict__ pairs,
                                                      VerifyRoundBufs rf, VerifyRoundBufs rh,
                                                      int ain, int aclr, VerifyParams P,
                                                      int skip, int split) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    rf.nact[aclr] = 0;
    rh.nact[aclr] = 0;
  }
  if (!skip) return;
  if ((int)blockIdx.x < split) rs_prune_body<KIND_F>(pairs, rf, ain, P, blockIdx.x, split);
  else rs_prune_body<KIND_H>(pairs, rh, ain, P, blockIdx.x - split, gridDim.x - split);
}

// Minimal solvers, one thread per hypothesis of the window, plus the fp32
// filter constants of every model.
constexpr int kSolveGrid = 4096;  // 1024 / 2048 / 3072: equal or slower (profiles/r02_m_solve_vbench.log)
template <int K>
__global__ __launch_bounds__(64) void rs_solve_kernel(
    const VerifyPair* __restrict__ pairs, const double* __restrict__ xy1_all,
    const double* __restrict__ xy2_all, const RansacState* __restrict__ rst,
    const int32_t* __restrict__ wB, const int32_t* __restrict__ act, const int32_t* __restrict__ nact,
    const uint32_t* __restrict__ samp, int32_t* __restrict__ nmod, float* __restrict__ fcon,
    double* __restrict__ mods, int W, double maxr, int WT) {
  using Tr = KindTraits<K>;
  constexpr int MM = Tr::mm, MS = Tr::ms;
  const int na = *nact;
  const int per = W;  // blocks of 64 hypotheses per pair
  for (int it = blockIdx.x; it < na * per; it += gridDim.x) {
    const int q = act[it / per];
    const int h = (it % per) * 64 + threadIdx.x;
    if (h >= wB[q]) continue;
    const VerifyPair pp = pairs[q];
    const double S = rst[q].S;
    const double* xy1 = xy1_all + pp.pts_off;
    const double* xy2 = xy2_all + pp.pts_off;
    const uint32_t* sq = samp + ((int64_t)q * WT + h) * 8;
    double a_[2 * 7], b_[2 * 7];
#pragma unroll
    for (int i = 0; i < Tr::kmin; ++i) {
      const uint32_t k = sq[i];
      a_[2 * i] = xy1[2 * k];
      a_[2 * i + 1] = xy1[2 * k + 1];
      b_[2 * i] = xy2[2 * k];
      b_[2 * i + 1] = xy2[2 * k + 1];
    }
    double* mo = mods + ((int64_t)q * WT * 3 + h * MM) * MS;
    int nm = 1;
    if (K == KIND_F) nm = fundamental_7pt(a_, b_, mo);
    else homography_dlt(a_, b_, 4, mo);
    nmod[(int64_t)q * WT + h] = nm;
    float* fc = fcon + ((int64_t)q * WT * 3 + h * MM) * 12;
    for (int k = 0; k < nm; ++k) {
      float c[12];
      if (K == KIND_F) f_filter_consts(mo + k * MS, S, maxr, c);
      else h_filter_consts(mo + k * MS, S, maxr, c);
#pragma unroll
      for (int j = 0; j < 12; ++j) fc[k * 12 + j] = c[j];
    }
  }
}

// Inlier counts of every model of the window: work item = (active pair,
// 1024-point chunk), one wave each (16 points per lane, packed in pairs);
// the filter constants of one round at a time are broadcast from LDS and
// lane t accumulates the count of hypothesis t of the round.
constexpr int kScoreThreads = 64;
// H split pass: models per loop iteration (2, 3: -0.5 %; 6, 8: no change,
// profiles/r03_hm_score_models_vbench.log)
constexpr int kScoreHm = 4;

constexpr int kScorePch = 8;  // points per lane
constexpr int kScoreChunk = kScoreThreads * kScorePch;
constexpr int kScorePchSmall = 4;  // small batches: points per lane
// work items per score launch (16K / 32K / 131K / 262K: -1.5 to -6 %, profiles/r02_j_*vbench.log)
constexpr int kScoreTargetItems = 65536;

// PCH: points per lane of a work item (kScorePch; small batches take more,
// so that each model's constants and loop overhead serve more points).
template <int K, bool SPLIT, int PCH = kScorePch>
__global__ __launch_bounds__(kScoreThreads) void rs_score_kernel(
    const VerifyPair* __restrict__ pairs, const float4* __restrict__ xyf_all,
    const RansacState* __restrict__ rst, const int32_t* __restrict__ wB,
    const int32_t* __restrict__ act, const int32_t* __restrict__ nact, const int32_t* __restrict__ nmod,
    const float* __restrict__ fcon, const double* __restrict__ mods,
    uint32_t* __restrict__ cnts, uint32_t* __restrict__ ucnt, int max_chunks, int W, double maxr,
    uint64_t* __restrict__ prof, int WT) {
  using Tr = KindTraits<K>;
  constexpr int MM = Tr::mm, MS = Tr::ms;
  __shared__ __attribute__((aligned(16))) float lc[kTrialBatch * MM][12];
  __shared__ int32_t lnm[kTrialBatch];
  constexpr int CH = kScoreThreads * PCH, QCAP = kDeferCap * (PCH / 8 > 1 ? PCH / 8 : 1);
  __shared__ uint32_t ldq[SPLIT ? 1 : QCAP];         // deferred exact tests (defer_push)
  __shared__ uint32_t ldc[SPLIT ? 1 : kTrialBatch * MM];  // their inliers per model of the round
  const int lane = threadIdx.x;
  const int na = *nact;
  const float maxrf = (float)maxr;
  const f32x2 dsc = f32x2(h_point_scale(maxr));
  // Work item = (active pair, chunk, run of rpi rounds of the window): late
  // windows (few far pairs left) split their rounds over separate items so
  // that they still fill the GPU; busy windows keep long runs (points loaded
  // once per run).
  const int rpi = max(1, min(W, (int)(((int64_t)na * max_chunks * W) / kScoreTargetItems)));
  const int nri = (W + rpi - 1) / rpi;
  const int per_pair = max_chunks * nri;
  for (int w = blockIdx.x; w < na * per_pair; w += gridDim.x) {
    const int q = act[w / per_pair];
    const int rem = w - (w / per_pair) * per_pair;
    const int chunk = rem / nri, ri = rem - (rem / nri) * nri;
    const VerifyPair pp = pairs[q];
    const int n = pp.m;
    const int base = chunk * CH;
    if (base >= n) continue;
    const int Bpair = wB[q];
    const int rbeg = ri * rpi * kTrialBatch;
    const int rend = min(Bpair, rbeg + rpi * kTrialBatch);
    if (rbeg >= rend) continue;
    const float4* xyf = xyf_all + pp.pts_off / 2;
    const uint64_t t_item = prof ? __builtin_amdgcn_s_memtime() : 0;
    f32x2 x0[PCH / 2], x1[PCH / 2], y0[PCH / 2], y1[PCH / 2];
#pragma unroll
    for (int qq = 0; qq < PCH / 2; ++qq) {
      const int i0 = base + (2 * qq) * 64 + lane, i1 = i0 + 64;
      const float4 v0 = i0 < n ? xyf[i0] : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 v1 = i1 < n ? xyf[i1] : make_float4(0.f, 0.f, 0.f, 0.f);
      x0[qq] = f32x2{v0.x, v1.x};
      x1[qq] = f32x2{v0.y, v1.y};
      y0[qq] = f32x2{v0.z, v1.z};
      y1[qq] = f32x2{v0.w, v1.w};
      if (K == KIND_H) {  // destination scaled by 1/sqrt(maxr) (h_filter_consts)
        y0[qq] *= dsc;
        y1[qq] *= dsc;
      }
    }
    const bool full = base + CH <= n;
    for (int r0 = rbeg; r0 < rend; r0 += kTrialBatch) {
      const int B = min(kTrialBatch, rend - r0);
      __syncthreads();
      if (lane < B) lnm[lane] = nmod[(int64_t)q * WT + r0 + lane];
      {
        const float4* src = reinterpret_cast<const float4*>(
            fcon + ((int64_t)q * WT * 3 + r0 * MM) * 12);
        float4* dst = reinterpret_cast<float4*>(&lc[0][0]);
        for (int i = lane; i < B * MM * 3; i += kScoreThreads) dst[i] = src[i];
      }
      if (!SPLIT)
        for (int i = lane; i < B * MM; i += kScoreThreads) ldc[i] = 0;
      __syncthreads();
      const double* mb = mods + ((int64_t)q * WT * 3 + r0 * MM) * MS;
      DeferQ dq{ldq, 0, QCAP};
      int nslow = 0;
      uint32_t c0 = 0, c1 = 0, c2 = 0;  // lane t: counts of hypothesis t's models
      uint32_t u0 = 0, u1 = 0, u2 = 0;  // SPLIT: lane t: their undecided points
      if (K == KIND_H && SPLIT) {
        // H split pass: kScoreHm models per iteration (one model per hypothesis)
        constexpr int NM = kScoreHm;
        for (int t = 0; t < B; t += NM) {
          HFilt f[NM];
#pragma unroll
          for (int k = 0; k < NM; ++k) f[k] = h_filter_load(&lc[min(t + k, B - 1)][0]);
          int uc[NM];
          if (full) score_h_notout_n<PCH, true, NM>(f, x0, x1, y0, y1, n, base, uc);
          else score_h_notout_n<PCH, false, NM>(f, x0, x1, y0, y1, n, base, uc);
#pragma unroll
          for (int k = 0; k < NM; ++k)
            if (t + k < B && lane == t + k) u0 += (uint32_t)uc[k];
        }
      } else
      for (int t = 0; t < B; ++t) {
        const int nmt = K == KIND_F ? __builtin_amdgcn_readfirstlane(lnm[t]) : 1;
        for (int k = 0; k < nmt; ++k) {
          const int m = t * MM + k;
          int c, u = 0;
          if (K == KIND_F) {
            const FFilt f = f_filter_load(&lc[m][0], maxrf);
            c = full ? score_f_chunk<PCH, true, SPLIT>(f, mb + m * MS, x0, x1, y0, y1, n,
                                                             base, maxr, &nslow,
                                                             SPLIT ? nullptr : &dq, m, &u)
                     : score_f_chunk<PCH, false, SPLIT>(f, mb + m * MS, x0, x1, y0, y1, n,
                                                              base, maxr, &nslow,
                                                              SPLIT ? nullptr : &dq, m, &u);
          } else {
            const HFilt f = h_filter_load(&lc[m][0]);
            if (SPLIT) {  // points not surely outside (bound); exact counts in rs_exact_kernel
              c = 0;
              u = full ? score_h_chunk<PCH, true, true>(f, mb + m * MS, xyf, x0, x1, y0, y1,
                                                              n, base, maxr, &nslow)
                       : score_h_chunk<PCH, false, true>(f, mb + m * MS, xyf, x0, x1, y0,
                                                               y1, n, base, maxr, &nslow);
            } else {
              c = full ? score_h_chunk<PCH, true>(f, mb + m * MS, xyf, x0, x1, y0, y1, n,
                                                        base, maxr, &nslow, &dq, m)
                       : score_h_chunk<PCH, false>(f, mb + m * MS, xyf, x0, x1, y0, y1, n,
                                                         base, maxr, &nslow, &dq, m);
            }
          }
          const uint32_t add = (lane == t) ? (uint32_t)c : 0u;
          const uint32_t uadd = (lane == t) ? (uint32_t)u : 0u;
          if (k == 0) { c0 += add; u0 += uadd; }
          else if (k == 1) { c1 += add; u1 += uadd; }
          else { c2 += add; u2 += uadd; }
        }
      }
      if (prof && lane == 0) {  // diagnostics: chunk-models scored, slow (exact) passes
        uint64_t* pc = prof + (int64_t)q * kVerifyProfSlots + (K == KIND_F ? 80 : 84);
        atomicAdd(reinterpret_cast<unsigned long long*>(pc), (unsigned long long)(B * MM));
        atomicAdd(reinterpret_cast<unsigned long long*>(pc + 1), (unsigned long long)nslow);
        atomicAdd(reinterpret_cast<unsigned long long*>(pc + 2), (unsigned long long)dq.n);
      }
      if (!SPLIT) {
        // The queued exact tests, 64 at a time.
        for (int e = lane; e < dq.n; e += kScoreThreads) {
          const uint32_t v = ldq[e];
          const int m = (int)(v >> 16), off = (int)(v & 0xFFFFu);
          const float4 pt = xyf[base + off];
          const bool in = K == KIND_F ? f_exact_pt(mb + m * MS, pt.x, pt.y, pt.z, pt.w, maxr)
                                      : h_exact_pt(mb + m * MS, pt.x, pt.y, pt.z, pt.w, maxr);
          if (in) atomicAdd(&ldc[m], 1u);
        }
        if (dq.n && lane < B) {
          c0 += ldc[lane * MM];
          if (MM > 1) c1 += ldc[lane * MM + 1];
          if (MM > 2) c2 += ldc[lane * MM + 2];
        }
      }
      uint32_t* cq = cnts + (int64_t)q * WT * 3 + r0 * MM;
      if (lane < B) {
        if (c0) atomicAdd(&cq[lane * MM], c0);
        if (MM > 1 && c1) atomicAdd(&cq[lane * MM + 1], c1);
        if (MM > 2 && c2) atomicAdd(&cq[lane * MM + 2], c2);
      }
      if (SPLIT && lane < B) {
        uint32_t* uq = ucnt + (int64_t)q * WT * 3 + r0 * MM;
        if (u0) atomicAdd(&uq[lane * MM], u0);
        if (MM > 1 && u1) atomicAdd(&uq[lane * MM + 1], u1);
        if (MM > 2 && u2) atomicAdd(&uq[lane * MM + 2], u2);
      }
    }
    if (prof && lane == 0)  // diagnostics: cycles of the pair's score items
      atomicAdd(reinterpret_cast<unsigned long long*>(prof + (int64_t)q * kVerifyProfSlots +
                                                      (K == KIND_F ? 83 : 87)),
                (unsigned long long)(__builtin_amdgcn_s_memtime() - t_item));
  }
}

// Exact pass of the split scoring (after rs_score_kernel<K, true>): a model's
// count is needed exactly only if it can be a candidate of the sequential
// replay, i.e. reach the pair's best count -- and the best only grows, so a
// model whose upper bound stays below the best at the start of the window
// (rst.best_n) can never be one.  F: the bound is sure + undecided inliers and
// the count stays the sure count; H: the bound is the number of points not
// surely outside and the count stays 0 -- either way a value below the best,
// which the replay reads exactly as it would read the exact count.  For the
// others the exact count is completed here (F: the undecided points' exact
// tests; H: the whole count).  Same work items as the scoring kernel; items
// with no such model exit without loading their points.
template <int K>
__global__ __launch_bounds__(kScoreThreads) void rs_exact_kernel(
    const VerifyPair* __restrict__ pairs, const float4* __restrict__ xyf_all,
    const RansacState* __restrict__ rst, const int32_t* __restrict__ wB,
    const int32_t* __restrict__ act, const int32_t* __restrict__ nact, const int32_t* __restrict__ nmod,
    const float* __restrict__ fcon, const double* __restrict__ mods,
    uint32_t* __restrict__ cnts, const uint32_t* __restrict__ ucnt, int max_chunks, int W,
    double maxr, int WT) {
  using Tr = KindTraits<K>;
  constexpr int MM = Tr::mm, MS = Tr::ms;
  const int lane = threadIdx.x;
  const int na = *nact;
  const float maxrf = (float)maxr;
  const f32x2 dsc = f32x2(h_point_scale(maxr));
  const int rpi = max(1, min(W, (int)(((int64_t)na * max_chunks * W) / kScoreTargetItems)));
  const int nri = (W + rpi - 1) / rpi;
  const int per_pair = max_chunks * nri;
  for (int w = blockIdx.x; w < na * per_pair; w += gridDim.x) {
    const int q = act[w / per_pair];
    const int rem = w - (w / per_pair) * per_pair;
    const int chunk = rem / nri, ri = rem - (rem / nri) * nri;
    const VerifyPair pp = pairs[q];
    const int n = pp.m;
    const int base = chunk * kScoreChunk;
    if (base >= n) continue;
    const int Bpair = wB[q];
    const uint32_t best0 = (uint32_t)rst[q].best_n;
    const int rbeg = ri * rpi * kTrialBatch;
    const int rend = min(Bpair, rbeg + rpi * kTrialBatch);
    if (rbeg >= rend) continue;
    const float4* xyf = xyf_all + pp.pts_off / 2;
    f32x2 x0[kScorePch / 2], x1[kScorePch / 2], y0[kScorePch / 2], y1[kScorePch / 2];
    bool loaded = false;
    for (int r0 = rbeg; r0 < rend; r0 += kTrialBatch) {
      const int B = min(kTrialBatch, rend - r0);
      const int64_t mo = (int64_t)q * WT * 3 + r0 * MM;
      // lane t: the qualifying models of hypothesis t (bit k)
      uint32_t qual = 0;
      if (lane < B) {
        const int nml = K == KIND_F ? nmod[(int64_t)q * WT + r0 + lane] : 1;
#pragma unroll
        for (int k = 0; k < MM; ++k) {
          const uint32_t u = k < nml ? ucnt[mo + lane * MM + k] : 0u;
          const uint32_t bound = K == KIND_H ? u : cnts[mo + lane * MM + k] + u;
          if (u && bound >= best0) qual |= 1u << k;
        }
      }
      uint64_t any = __ballot(qual != 0);
      if (!any) continue;
      if (!loaded) {
#pragma unroll
        for (int qq = 0; qq < kScorePch / 2; ++qq) {
          const int i0 = base + (2 * qq) * 64 + lane, i1 = i0 + 64;
          const float4 v0 = i0 < n ? xyf[i0] : make_float4(0.f, 0.f, 0.f, 0.f);
          const float4 v1 = i1 < n ? xyf[i1] : make_float4(0.f, 0.f, 0.f, 0.f);
          x0[qq] = f32x2{v0.x, v1.x};
          x1[qq] = f32x2{v0.y, v1.y};
          y0[qq] = f32x2{v0.z, v1.z};
          y1[qq] = f32x2{v0.w, v1.w};
          if (K == KIND_H) {
            y0[qq] *= dsc;
            y1[qq] *= dsc;
          }
        }
        loaded = true;
      }
      const bool full = base + kScoreChunk <= n;
      const double* mb = mods + mo * MS;
      const float* cb = fcon + mo * 12;
      while (any) {
        const int t = (int)__builtin_ctzll(any);
        any &= any - 1;
        const uint32_t qt = __builtin_amdgcn_readlane(qual, t);
        for (int k = 0; k < MM; ++k) {
          if (!(qt & (1u << k))) continue;
          const int m = t * MM + k;
          int nslow = 0, sure = 0, c;
          if (K == KIND_F) {
            const FFilt f = f_filter_load(cb + m * 12, maxrf);
            c = full ? score_f_chunk<kScorePch, true>(f, mb + m * MS, x0, x1, y0, y1, n, base,
                                                      maxr, &nslow, nullptr, 0, nullptr, &sure)
                     : score_f_chunk<kScorePch, false>(f, mb + m * MS, x0, x1, y0, y1, n, base,
                                                       maxr, &nslow, nullptr, 0, nullptr, &sure);
          } else {
            const HFilt f = h_filter_load(cb + m * 12);
            c = full ? score_h_chunk<kScorePch, true>(f, mb + m * MS, xyf, x0, x1, y0, y1, n,
                                                      base, maxr, &nslow)
                     : score_h_chunk<kScorePch, false>(f, mb + m * MS, xyf, x0, x1, y0, y1, n,
                                                       base, maxr, &nslow);
          }
          if (lane == 0 && c > sure) atomicAdd(&cnts[mo + m], (uint32_t)(c - sure));
        }
      }
    }
  }
}

// Parallel local optimisation (small batches, the first window; shipped by
// default since round 5, byte-identical to the inline chains: every
// small-batch GPU test, and tests/test_gpu_stencil.py::
// test_parallel_lo_more_records_than_slots with SCM_PARALLEL_LO=1 and =0):
// block (a, slot) takes active pair a's slot-th record model of the window --
// a model whose count reaches the running maximum of the counts before it,
// starting from the pair's best at the window start (rst.best_n; a stale,
// lower value only adds records) -- and runs the LO chain the replay would
// run if the model became the best: its residual pass (with the inlier
// gather), then the LO steps with their compares, all against the chain's own
// models, so the outcome depends on the record alone.  Only records can be
// candidates (the best after trial s is at least every count up to s), so
// the replay takes these outcomes instead of running the chains one after
// another (host model: tests/test_parallel_lo_model.py).  The record's own
// residuals stay in slot buffer 0 (a tie compare at acceptance needs them);
// the chain alternates buffers 1 and 2.
template <int K>
__device__ __attribute__((always_inline)) void rs_lo_chain_body(
    const VerifyPair* __restrict__ pairs, double* __restrict__ scratch,
    uint32_t* __restrict__ snaps, VerifyOut* __restrict__ out, const VerifyRoundBufs& rb, int ain,
    const VerifyParams& P, const float4* __restrict__ xyf_all, int bid) {
  constexpr int NW = 4;
  using Tr = KindTraits<K>;
  constexpr int MM = Tr::mm, MS = Tr::ms;
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
  VerifyLds& s = *reinterpret_cast<VerifyLds*>(dyn_lds);
  const int a = bid / kLoSlots, slot = bid % kLoSlots;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool t0th = threadIdx.x == 0;
  if (a >= rb.nact[ain]) return;
  const int q = rb.act[ain][a];
  const int WT = rb.wt;
  LoSlot* sl = rb.lo + (int64_t)q * kLoSlots + slot;
  const int B = rb.wB[q];
  // Records in order, found by wave 0 (prefix maxima over chunks of 64
  // entries); the slot-th one's index goes to s.redi[8], -1 if none.
  if (wv == 0) {
    int run = *reinterpret_cast<volatile const int32_t*>(&rb.rst[q].best_n);
    int found = 0, rec = -1;
    const int ne = B * MM;
    for (int e0 = 0; e0 < ne && rec < 0; e0 += 64) {
      const int e = e0 + lane;
      int v = -1;
      if (e < ne) {
        const int t = e / MM, k = e - t * MM;
        const int nm = K == KIND_F ? rb.nmod[(int64_t)q * WT + t] : 1;
        if (k < nm) v = (int)rb.cnts[(int64_t)q * WT * 3 + e];
      }
      // exclusive prefix maximum of v over the chunk, on top of run
      int incl = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(incl, d);
        if (lane >= d) incl = max(incl, o);
      }
      int excl = __shfl_up(incl, 1);
      if (lane == 0) excl = -1;
      const bool isrec = v >= 0 && v >= max(run, excl);
      const uint64_t bal = __ballot(isrec);
      const int nb = __popcll(bal);
      if (found + nb > slot) {  // the slot-th record is in this chunk
        uint64_t b = bal;
        for (int i = 0; i < slot - found; ++i) b &= b - 1;
        rec = e0 + (int)__builtin_ctzll(b);
      }
      found += nb;
      run = max(run, __shfl(incl, 63));
    }
    if (lane == 0) s.redi[8] = rec;
  }
  __syncthreads();
  const int e = s.redi[8];
  __syncthreads();
  if (e < 0) {
    if (t0th) sl->rec = -1;
    return;
  }
  const PairSetup ps = pair_at<K>(pairs, q, scratch, snaps, out);
  const int n = ps.n;
  const double maxr = P.max_residual;
  const float4* xyf = xyf_all + ps.pp.pts_off / 2;
  double* data = rb.lo_data + ((int64_t)q * kLoSlots + slot) * rb.lo_stride;
  double* buf[3] = {data, data + n, data + 2 * n};
  float4* xin = reinterpret_cast<float4*>((reinterpret_cast<uintptr_t>(data + 3 * n) + 15) &
                                          ~(uintptr_t)15);
  double mk[MS];
  const double* src = rb.mods + ((int64_t)q * WT * 3 + e) * MS;
#pragma unroll
  for (int j = 0; j < MS; ++j) mk[j] = src[j];
  // the record's count as the scoring counted it (the replay starts LO from it)
  const int c = (int)rb.cnts[(int64_t)q * WT * 3 + e];
  residuals_gather_f4<K, NW>(mk, xyf, n, maxr, buf[0], xin, s.redi);
  if (t0th) {
#pragma unroll
    for (int j = 0; j < MS; ++j) s.best_model[j] = mk[j];
    s.best_n = c;
    s.best_sum = 0.0;
    s.best_sum_valid = 0;
  }
  __syncthreads();
  int bi = 0;  // buffer of the chain's best
  if (c > Tr::kmin && c >= Tr::kmin_local) {
    for (int lt = 0; lt < 10; ++lt) {
      const int ni = s.best_n;  // in xin from the best's residual pass
      double lm[9];
      local_estimate_f4<K, NW>(s, xin, ni, lm);
      const int prev = s.best_n;
      const int li = bi == 1 ? 2 : 1;
      const int lcn = residuals_gather_f4<K, NW>(lm, xyf, n, maxr, buf[li], xin, s.redi);
      bool lbetter = lcn > prev, lexact = false;
      double lsum = 0.0;
      if (lcn == prev)
        lbetter = tie_better<NW>(s, buf[li], buf[bi], n, lcn, maxr, &lsum, &lexact);
      if (lbetter) {
        __syncthreads();
        if (t0th) {
#pragma unroll
          for (int j = 0; j < MS; ++j) s.best_model[j] = lm[j];
          s.best_n = lcn;
          s.best_sum = lsum;
          s.best_sum_valid = lexact ? 1 : 0;
        }
        bi = li;
      }
      __syncthreads();
      if (s.best_n <= prev) break;
    }
  }
  if (t0th) {
    sl->rec = e;
    sl->count = s.best_n;
    sl->sum = s.best_sum;
    sl->sum_valid = s.best_sum_valid;
    sl->buf = bi;
#pragma unroll
    for (int j = 0; j < 9; ++j) sl->model[j] = j < MS ? s.best_model[j] : 0.0;
  }
}

// Both kinds in one launch: blocks [0, split) the F records, the rest H's.
__global__ __launch_bounds__(256) void rs_lo_chain2_kernel(
    const VerifyPair* __restrict__ pairs, double* __restrict__ scratch,
    uint32_t* __restrict__ snaps, VerifyOut* __restrict__ out, VerifyRoundBufs rf,
    VerifyRoundBufs rh, int ain, VerifyParams P, const float4* __restrict__ xyf_all, int split) {
  if (P.prio) __builtin_amdgcn_s_setprio(2);
  if ((int)blockIdx.x < split)
    rs_lo_chain_body<KIND_F>(pairs, scratch, snaps, out, rf, ain, P, xyf_all, blockIdx.x);
  else
    rs_lo_chain_body<KIND_H>(pairs, scratch, snaps, out, rh, ain, P, xyf_all, blockIdx.x - split);
}

// The sequential part of one window, in trial order, for every active pair.
// NW waves per pair (4: small batches, see rs_replay2w_kernel): every wave
// runs the same decisions from the shared LDS state; thread 0 writes it.
template <int K, int NW = 1>
__device__ __attribute__((always_inline)) void rs_replay_body(
    const VerifyPair* __restrict__ pairs, double* __restrict__ scratch,
    uint32_t* __restrict__ snaps, VerifyOut* __restrict__ out, uint8_t* __restrict__ masks,
    RansacState* __restrict__ rst, const int32_t* __restrict__ act,
    const int32_t* __restrict__ nact, int32_t* __restrict__ act_next,
    int32_t* __restrict__ nact_next, const int32_t* __restrict__ nmod,
    const uint32_t* __restrict__ cnts, const double* __restrict__ mods,
    const uint32_t* __restrict__ wsnap, const int32_t* __restrict__ wB,
    const uint32_t* __restrict__ wstate, VerifyParams P, uint64_t* __restrict__ prof,
    const float4* __restrict__ xyf_all, int bid, int nblk, int WT,
    const LoSlot* __restrict__ lo = nullptr, double* __restrict__ lo_data = nullptr,
    int64_t lo_stride = 0) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
  VerifyLds& s = *reinterpret_cast<VerifyLds*>(dyn_lds);
  using Tr = KindTraits<K>;
  constexpr int MM = Tr::mm, MS = Tr::ms;
  const int lane = threadIdx.x & 63;
  const bool t0th = threadIdx.x == 0;
  const double maxr = P.max_residual;
  const int na = *nact;
  for (int a = bid; a < na; a += nblk) {
    const int q = act[a];
    // Diagnostic counters (SCM_PROFILE=1 only): windows, candidates, ties,
    // new bests, LO iterations; cycles in candidate residuals, tie sums, LO,
    // whole replay.
    uint64_t* pc = prof ? prof + (int64_t)q * kVerifyProfSlots + (K == KIND_F ? 20 : 30) : nullptr;
    const uint64_t t_enter = pc ? __builtin_amdgcn_s_memtime() : 0;
    if (pc && t0th) pc[0] += 1;
    const PairSetup ps = pair_at<K>(pairs, q, scratch, snaps, out);
    const int n = ps.n;
    double* base = ps.base;
    double* res[2] = {base, base + n};
    const float4* xyf = xyf_all + ps.pp.pts_off / 2;
    // compacted inliers (packed fp32) in the scratch after the two residual
    // buffers, 16-B aligned
    float4* xin = reinterpret_cast<float4*>(
        (reinterpret_cast<uintptr_t>(base + 2 * n) + 15) & ~(uintptr_t)15);
    const double* mq = mods + (int64_t)q * WT * 3 * MS;
    RansacState st = rst[q];
    wsync();
    if (threadIdx.x < 9) s.best_model[threadIdx.x] = st.best_model[threadIdx.x];
    if (t0th) {
      s.best_n = st.best_n;
      s.best_sum = st.best_sum;
      s.best_sum_valid = st.best_sum_valid;
    }
    int best_sel = st.res_sel;
    // The best's residuals: res[0] / res[1], or a slot buffer of the parallel
    // LO (rs_lo_chain2_kernel) after a record's outcome is taken.
    double* rbest = res[best_sel];
    const LoSlot* slots = lo ? lo + (int64_t)q * kLoSlots : nullptr;
    int si = 0;  // next slot (records in window order)
    int dyn_max = st.dyn_max;
    const int trial = st.trial;
    const int Btot = wB[q];
    bool abort = false;
    int abort_trial = -1;
    int64_t evals = st.evals;
    // Leading rounds with neither a candidate nor the abort trial are skipped
    // in one scan with several rounds' loads in flight (the round loop below
    // pays a load latency and two barriers per round: a window of 32 rounds
    // in which a pair's best is no longer reached was 32 of them).  Until the
    // first candidate the best and dyn_max keep their entry values, so a
    // candidate is a count >= the entry best and the abort trial is the first
    // trial >= max(dyn_max, min_num_trials); the scan finds the earliest of
    // them, and the loop starts at its round -- the trials before it pass
    // exactly as the loop would pass them (their models counted in evals).
    int rstart = 0;
    {
      const int bn0 = st.best_n;
      const int lim = min(Btot, max(0, max(dyn_max, P.min_num_trials) - trial));
      const int32_t* nm_q = nmod + (int64_t)q * WT;
      const uint32_t* c_q = cnts + (int64_t)q * WT * 3;
      int first = lim;
      constexpr int U = 4;
      for (int b0 = 0; b0 < lim; b0 += 64 * U) {
        int nmv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int t = b0 + 64 * u + lane;
          nmv[u] = t < lim ? nm_q[t] : 0;
        }
        uint32_t cv[U][MM];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int k = 0; k < MM; ++k)
            cv[u][k] = k < nmv[u] ? c_q[(b0 + 64 * u + lane) * MM + k] : 0u;
        int hit = -1;
#pragma unroll
        for (int u = U - 1; u >= 0; --u) {
          bool cand = false;
#pragma unroll
          for (int k = 0; k < MM; ++k) cand |= k < nmv[u] && (int)cv[u][k] >= bn0;
          const uint64_t bal = __ballot(cand);
          if (bal) hit = b0 + 64 * u + (int)__builtin_ctzll(bal);
        }
        if (hit >= 0) {
          first = min(first, hit);
          break;
        }
      }
      rstart = first / kTrialBatch * kTrialBatch;
      int ns = 0;
      for (int t = lane; t < rstart; t += 64) ns += nm_q[t];
      evals += (int64_t)wave_sum_i(ns) * n;
    }
    for (int r0 = rstart; r0 < Btot && !abort; r0 += kTrialBatch) {
      const int B = min(kTrialBatch, Btot - r0);
      wsync();
      for (int i = threadIdx.x; i < B; i += 64 * NW) s.nmodels[i] = nmod[(int64_t)q * WT + r0 + i];
      for (int i = threadIdx.x; i < B * MM; i += 64 * NW)
        s.counts[i] = cnts[(int64_t)q * WT * 3 + r0 * MM + i];
      wsync();
      // Trials of the round in order.  Only two kinds need the sequential
      // step: a candidate (a model whose inlier count reaches the best) and
      // the abort trial (tt >= dyn_max and >= min_num_trials); the lanes
      // find the next such trial in one ballot (lane = trial of the round),
      // and the trials in between -- no model to compare, no abort -- are
      // skipped as the sequential scan would pass them.
      int t = 0;
      while (t < B && !abort) {
        bool need = false;
        if (lane < B && lane >= t) {
          const int nml = s.nmodels[lane];
          const int bnl = s.best_n;
          bool cand = false;
#pragma unroll
          for (int k = 0; k < MM; ++k)
            cand |= k < nml && (int)s.counts[lane * MM + k] >= bnl;
          const int ttl = trial + r0 + lane;
          need = cand || (ttl >= dyn_max && ttl >= P.min_num_trials);
        }
        const uint64_t needm = __ballot(need);
        if (!needm) break;
        t = (int)__builtin_ctzll(needm);
        const int tt = trial + r0 + t;
        const int nmt = s.nmodels[t];
        for (int k = 0; k < MM; ++k) {
          if (k < nmt && !abort) {
            const int c = (int)s.counts[t * MM + k];
            const int bn = s.best_n;
            if (c >= bn) {
              uint64_t t0 = pc ? __builtin_amdgcn_s_memtime() : 0;
              const int e = (r0 + t) * MM + k;
              const LoSlot* sl = nullptr;
              if (slots) {
                while (si < kLoSlots && slots[si].rec >= 0 && slots[si].rec < e) ++si;
                if (si < kLoSlots && slots[si].rec == e) sl = slots + si;
              }
              if (sl) {
                // A record with its LO chain already run: the acceptance
                // compare here, the chain's outcome if accepted.
                double* sd = lo_data + ((int64_t)q * kLoSlots + si) * lo_stride;
                bool better = c > bn, exact = false;
                double sum = 0.0;
                if (!better) better = tie_better<NW>(s, sd, rbest, n, c, maxr, &sum, &exact);
                if (pc && t0th) {
                  pc[1] += 1;
                  if (c == bn) pc[2] += 1;
                  if (better) pc[3] += 1;
                }
                if (better) {
                  wsync();
                  if (t0th) {
#pragma unroll
                    for (int j = 0; j < MS; ++j) s.best_model[j] = sl->model[j];
                    s.best_n = sl->count;
                    s.best_sum = sl->sum;
                    s.best_sum_valid = sl->sum_valid;
                  }
                  rbest = sd + (int64_t)sl->buf * n;
                  wsync();
                  dyn_max = (int)min((uint64_t)0x7FFFFFFF,
                                     num_trials((uint64_t)s.best_n, (uint64_t)n, P.confidence,
                                                P.dyn_num_trials_multiplier, Tr::kmin));
                }
              } else {
              double mk[MS];
              const double* src = mq + e * MS;
#pragma unroll
              for (int j = 0; j < MS; ++j) mk[j] = src[j];
              double* rt = rbest == res[0] ? res[1] : res[0];
              residuals_gather_f4<K, NW>(mk, xyf, n, maxr, rt, xin, s.redi);
              bool better = c > bn, exact = false;
              double sum = 0.0;
              if (pc && t0th) {
                const uint64_t t1 = __builtin_amdgcn_s_memtime();
                pc[1] += 1;
                pc[5] += t1 - t0;
                t0 = t1;
              }
              if (!better) {  // tie on the inlier count: Compare the residual sums
                better = tie_better<NW>(s, rt, rbest, n, c, maxr, &sum, &exact);
                if (pc && t0th) {
                  pc[2] += 1;
                  pc[6] += __builtin_amdgcn_s_memtime() - t0;
                }
              }
              if (pc && t0th && better) pc[3] += 1;
              const uint64_t t_lo = pc ? __builtin_amdgcn_s_memtime() : 0;
              if (better) {
                wsync();
                if (t0th) {
#pragma unroll
                  for (int j = 0; j < MS; ++j) s.best_model[j] = mk[j];
                  s.best_n = c;
                  s.best_sum = sum;
                  s.best_sum_valid = exact ? 1 : 0;
                }
                rbest = rt;
                wsync();
                // Recursive local optimisation.
                if (c > Tr::kmin && c >= Tr::kmin_local) {
                  for (int lt = 0; lt < 10; ++lt) {
                    if (pc && t0th) pc[4] += 1;
                    uint64_t* pl = pc ? pc + 20 : nullptr;
                    uint64_t tl0 = pl ? __builtin_amdgcn_s_memtime() : 0;
                    const int ni = s.best_n;  // in xin from the best's residual pass
                    if (pl && t0th) { const uint64_t tq = __builtin_amdgcn_s_memtime(); pl[0] += tq - tl0; tl0 = tq; pl[5] += ni; }
                    double lm[9];
                    local_estimate_f4<K, NW>(s, xin, ni, lm, pl);
                    if (pl && t0th) tl0 = __builtin_amdgcn_s_memtime();
                    const int prev = s.best_n;
                    double* rl = rbest == res[0] ? res[1] : res[0];
                    const int lcn = residuals_gather_f4<K, NW>(lm, xyf, n, maxr, rl, xin, s.redi);
                    if (pl && t0th) pl[4] += __builtin_amdgcn_s_memtime() - tl0;
                    bool lbetter = lcn > prev, lexact = false;
                    double lsum = 0.0;
                    if (lcn == prev)
                      lbetter = tie_better<NW>(s, rl, rbest, n, lcn, maxr, &lsum, &lexact);
                    if (lbetter) {
                      wsync();
                      if (t0th) {
#pragma unroll
                        for (int j = 0; j < MS; ++j) s.best_model[j] = lm[j];
                        s.best_n = lcn;
                        s.best_sum = lsum;
                        s.best_sum_valid = lexact ? 1 : 0;
                      }
                      rbest = rl;
                    }
                    wsync();
                    if (s.best_n <= prev) break;
                  }
                }
                dyn_max = (int)min((uint64_t)0x7FFFFFFF,
                                   num_trials((uint64_t)s.best_n, (uint64_t)n, P.confidence,
                                              P.dyn_num_trials_multiplier, Tr::kmin));
              }
              if (pc && t0th) pc[7] += __builtin_amdgcn_s_memtime() - t_lo;
              }
            }
            if (tt >= dyn_max && tt >= P.min_num_trials) {
              abort = true;
              abort_trial = tt;
            }
          }
        }
        ++t;
      }
      // models scored by the trials of this round up to the stop
      {
        const int lastt = abort ? abort_trial - (trial + r0) : B - 1;
        const int nm = lane <= lastt && lane < B ? s.nmodels[lane] : 0;
        evals += (int64_t)wave_sum_i(nm) * n;
      }
    }
    wsync();
    if (abort) {
      // Rewind the PRNG to the state right after trial abort_trial's sample:
      // the window's start state, then its draws up to that trial.
      const int rel = abort_trial - trial, w = rel / kTrialBatch;
      const uint32_t* snap = wsnap + (int64_t)q * 640;
      for (int i = threadIdx.x; i < 624; i += 64 * NW) s.mt[i] = snap[i];
      if (t0th) s.mt_idx = (int32_t)snap[624];
      wsync();
      mt_advance_draws<Tr::kmin>(s, w, (rel - w * kTrialBatch + 1) * Tr::kmin, (uint32_t)n);
      mt_save(s, ps.state);
      st.num_trials = abort_trial + 2;
      st.done = 1;
      st.aborted = 1;
    } else {
      st.trial = trial + Btot;
      st.num_trials = st.trial;
      if (st.trial >= st.max_trials) {
        st.done = 1;
        // the stream continues (H: the watermark RANSAC) from the state after
        // the last window's draws
        const uint32_t* ws = wstate + (int64_t)q * kVerifyStateWords;
        for (int i = threadIdx.x; i < 625; i += blockDim.x) ps.state[i] = ws[i];
      }
    }
    if (rbest != res[0] && rbest != res[1]) {  // the best's residuals from a slot
      for (int i = threadIdx.x; i < n; i += 64 * NW) res[0][i] = rbest[i];
      wsync();
      rbest = res[0];
    }
    best_sel = rbest == res[1] ? 1 : 0;
    st.dyn_max = dyn_max;
    st.evals = evals;
    st.res_sel = best_sel;
    st.best_n = s.best_n;
    st.best_sum = s.best_sum;
    st.best_sum_valid = s.best_sum_valid;
#pragma unroll
    for (int j = 0; j < 9; ++j) st.best_model[j] = s.best_model[j];
    // The pair's outputs first, then its state: a reader that sees done
    // (the early verify_final pass of small batches, NW > 1) sees the
    // outputs too.
    if (st.done) rs_finish<K>(ps, st, masks, maxr);
    if (NW > 1) __threadfence();
    wsync();
    if (t0th) rst[q] = st;
    if (!st.done && t0th) act_next[atomicAdd(nact_next, 1)] = q;
    if (pc && t0th) {
      pc[8] += __builtin_amdgcn_s_memtime() - t_enter;
      pc[9] += (uint64_t)Btot;
    }
  }
}

// ---------------------------------------------------------------------------
// Window kernels over both RANSAC kinds at once: blocks [0, split) run the F
// LO-RANSAC of every active pair, blocks [split, grid) the H LO-RANSAC (its
// own PRNG stream, pair_seed_h), so one launch sequence advances both and the
// latency-bound per-pair kernels carry twice the pairs.  split == grid: F
// only (H has run out of windows).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void rs_begin2_kernel(
    const VerifyPair* __restrict__ pairs, int npairs, double* __restrict__ scratch,
    uint32_t* __restrict__ snaps, VerifyOut* __restrict__ out, uint8_t* __restrict__ masks,
    const float4* __restrict__ xyf, VerifyRoundBufs rf, VerifyRoundBufs rh, VerifyParams P,
    int split) {
  if ((int)blockIdx.x < split)
    rs_begin_body<KIND_F>(pairs, npairs, scratch, snaps, out, masks, xyf, rf.rst, rf.act[0],
                          rf.nact, rf.pstate, rf.dtrial, P, blockIdx.x, split);
  else
    rs_begin_body<KIND_H>(pairs, npairs, scratch, snaps, out, masks, xyf, rh.rst, rh.act[0],
                          rh.nact, rh.pstate, rh.dtrial, P, blockIdx.x - split, gridDim.x - split);
}

__global__ __launch_bounds__(64) void rs_draw2_kernel(
    const VerifyPair* __restrict__ pairs, double* __restrict__ scratch,
    uint32_t* __restrict__ snaps, VerifyOut* __restrict__ out, VerifyRoundBufs rf,
    VerifyRoundBufs rh, int ain, int aclr, VerifyParams P, int spec, int Wf, int Wh, int split) {
  if (P.prio) __builtin_amdgcn_s_setprio(2);
  if ((int)blockIdx.x < split)
    rs_draw_body<KIND_F>(pairs, scratch, snaps, out, rf.rst, rf.act[ain], rf.nact + ain,
                         rf.nact + aclr, rf.samp, rf.cnts, rf.ucnt, rf.wsnap, rf.wB, rf.pstate,
                         rf.wstate, rf.dtrial, rf.pcnts, rf.pwB, P, spec != 0, Wf, blockIdx.x,
                         split, rf.wt);
  else
    rs_draw_body<KIND_H>(pairs, scratch, snaps, out, rh.rst, rh.act[ain], rh.nact + ain,
                         rh.nact + aclr, rh.samp, rh.cnts, rh.ucnt, rh.wsnap, rh.wB, rh.pstate,
                         rh.wstate, rh.dtrial, rh.pcnts, rh.pwB, P, spec != 0, Wh,
                         blockIdx.x - split, gridDim.x - split, rh.wt);
}

__global__ __launch_bounds__(64) void rs_shuffle2_kernel(
    const VerifyPair* __restrict__ pairs, double* __restrict__ scratch,
    uint32_t* __restrict__ snaps, VerifyOut* __restrict__ out, VerifyRoundBufs rf,
    VerifyRoundBufs rh, int ain, int ppb, int stride, int split, int prio) {
  if (prio) __builtin_amdgcn_s_setprio(2);
  if ((int)blockIdx.x < split)
    rs_shuffle_body<KIND_F>(pairs, scratch, snaps, out, rf.wB, rf.act[ain], rf.nact + ain,
                            rf.samp, ppb, stride, blockIdx.x, split, rf.wt);
  else
    rs_shuffle_body<KIND_H>(pairs, scratch, snaps, out, rh.wB, rh.act[ain], rh.nact + ain,
                            rh.samp, ppb, stride, blockIdx.x - split, gridDim.x - split, rh.wt);
}

__global__ __launch_bounds__(64) void rs_replay2_kernel(
    const VerifyPair* __restrict__ pairs, double* __restrict__ scratch,
    uint32_t* __restrict__ snaps, VerifyOut* __restrict__ out, uint8_t* __restrict__ masks,
    VerifyRoundBufs rf, VerifyRoundBufs rh, int ain, int aout, VerifyParams P,
    uint64_t* __restrict__ prof, const float4* __restrict__ xyf, int split) {
  if (P.prio) __builtin_amdgcn_s_setprio(2);
  if ((int)blockIdx.x < split)
    rs_replay_body<KIND_F>(pairs, scratch, snaps, out, masks, rf.rst, rf.act[ain], rf.nact + ain,
                           rf.act[aout], rf.nact + aout, rf.nmod, rf.cnts, rf.mods,
                           rf.wsnap, rf.wB, rf.wstate, P, prof, xyf, blockIdx.x, split, rf.wt);
  else
    rs_replay_body<KIND_H>(pairs, scratch, snaps, out, masks, rh.rst, rh.act[ain], rh.nact + ain,
                           rh.act[aout], rh.nact + aout, rh.nmod, rh.cnts, rh.mods,
                           rh.wsnap, rh.wB, rh.wstate, P, prof, xyf, blockIdx.x - split, gridDim.x - split, rh.wt);
}

// rs_replay2_kernel with four waves per pair (small batches: the window's
// sequential decisions are the critical path of one Scanner stencil).
__global__ __launch_bounds__(256) void rs_replay2w_kernel(
    const VerifyPair* __restrict__ pairs, double* __restrict__ scratch,
    uint32_t* __restrict__ snaps, VerifyOut* __restrict__ out, uint8_t* __restrict__ masks,
    VerifyRoundBufs rf, VerifyRoundBufs rh, int ain, int aout, VerifyParams P,
    uint64_t* __restrict__ prof, const float4* __restrict__ xyf, int split) {
  if (P.prio) __builtin_amdgcn_s_setprio(2);
  if ((int)blockIdx.x < split)
    rs_replay_body<KIND_F, 4>(pairs, scratch, snaps, out, masks, rf.rst, rf.act[ain], rf.nact + ain,
                              rf.act[aout], rf.nact + aout, rf.nmod, rf.cnts, rf.mods,
                              rf.wsnap, rf.wB, rf.wstate, P, prof, xyf, blockIdx.x, split, rf.wt,
                              rf.lo, rf.lo_data, rf.lo_stride);
  else
    rs_replay_body<KIND_H, 4>(pairs, scratch, snaps, out, masks, rh.rst, rh.act[ain], rh.nact + ain,
                              rh.act[aout], rh.nact + aout, rh.nmod, rh.cnts, rh.mods,
                              rh.wsnap, rh.wB, rh.wstate, P, prof, xyf, blockIdx.x - split, gridDim.x - split, rh.wt,
                              rh.lo, rh.lo_data, rh.lo_stride);
}

// Points of the verified pairs: block (x, q) takes chunks x, x + gridDim.x,
// ... of kGatherChunk matches of pair q, kGatherU per thread with their loads
// in flight.  Small batches (the gather is on their critical path) spread a
// pair over max_m / kGatherChunk blocks; large ones take a block per pair (a
// grid of many more blocks beside the next batch's matcher takes its CUs).
constexpr int kGatherThreads = 256, kGatherU = 4, kGatherChunk = kGatherThreads * kGatherU;
constexpr int kGatherWidePairs = 256;
__global__ __launch_bounds__(kGatherThreads) void gather_kernel(
    const GatherPair* __restrict__ pairs, const uint2* __restrict__ matches,
    const float2* __restrict__ kpxy, double* __restrict__ xy1, double* __restrict__ xy2,
    const int32_t* __restrict__ counts, float4* __restrict__ xyf) {
  const GatherPair g = pairs[blockIdx.y];
  const int m = g.cidx >= 0 ? counts[g.cidx] : g.m;
  for (int i0 = blockIdx.x * kGatherChunk + threadIdx.x; i0 < m; i0 += gridDim.x * kGatherChunk) {
    uint2 mt[kGatherU];
#pragma unroll
    for (int u = 0; u < kGatherU; ++u) {
      const int i = i0 + u * kGatherThreads;
      mt[u] = matches[g.match_off + (i < m ? i : i0)];
    }
    float2 a[kGatherU], b[kGatherU];
#pragma unroll
    for (int u = 0; u < kGatherU; ++u) {
      a[u] = kpxy[g.kp1_off + mt[u].x];
      b[u] = kpxy[g.kp2_off + mt[u].y];
    }
#pragma unroll
    for (int u = 0; u < kGatherU; ++u) {
      const int i = i0 + u * kGatherThreads;
      if (i >= m) break;
      xy1[2 * (g.pts_off + i)] = (double)a[u].x;
      xy1[2 * (g.pts_off + i) + 1] = (double)a[u].y;
      xy2[2 * (g.pts_off + i)] = (double)b[u].x;
      xy2[2 * (g.pts_off + i) + 1] = (double)b[u].y;
      xyf[g.pts_off + i] = make_float4(a[u].x, a[u].y, b[u].x, b[u].y);
    }
  }
}

// Packs each pair's matches and F-inlier mask contiguously at offsets[p]
// (exclusive scan of the counts, computed on the host).
__global__ void compact_kernel(const int32_t* __restrict__ counts, const int64_t* __restrict__ offsets,
                               const int64_t* __restrict__ match_off, const uint2* __restrict__ matches,
                               const uint8_t* __restrict__ masks, uint2* __restrict__ out_matches,
                               uint8_t* __restrict__ out_masks) {
  const int p = blockIdx.x;
  const int m = counts[p];
  const int64_t o = offsets[p], s = match_off[p];
  for (int i = threadIdx.x; i < m; i += blockDim.x) {
    out_matches[o + i] = matches[s + i];
    out_masks[o + i] = masks[s + i];
  }
}

static_assert(sizeof(VerifyLds) <= 20 * 1024, "VerifyLds must allow 8 pairs per CU");

size_t verify_lds_bytes(int max_m) {
  (void)max_m;
  return sizeof(VerifyLds);
}

namespace {

// Blocks of the wave-per-pair kernels (rs_begin / rs_draw / rs_replay) per
// kind; pairs beyond it are taken in grid-stride order.
constexpr int kPairGrid = 4096;  // 2048: -1 %, 16384 (a block per pair): +0.4 %, within noise (profiles/r02_o_pairgrid_vbench.log)

// (a request past the CU's LDS together with the kernel's static LDS fails:
// launch_verify returns that error at once instead of leaving it for the next
// hipGetLastError)
template <typename F>
hipError_t set_lds_attr(F f, int static_bytes = 0) {
  return hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize,
                             160 * 1024 - static_bytes);
}

// Small-batch threshold: 1,024 pairs (Scanner op batches up to 53 stencils of
// 20): the table path's schedule -- one-wave replays, windows doubling from 1
// round -- left batches of 266-1,007 pairs latency-bound (op batch 16 = 304
// pairs: 22 ms per call vs 13.8 ms on the small-batch kernels, batch 32: 32
// vs 26 ms); at 1,216 pairs (batch 64) the small-batch schedule's wider
// speculative windows cost more than they save (49-50 vs 51-52 ms),
// profiles/r06_ad.
constexpr int kWaveShufflePairs = 1024;
constexpr int kMaxDevices = 64;  // launch_verify's per-device attribute set-up
constexpr int kSmallFirstWindow = 4;  // rounds of a small batch's first window (run_windows)
constexpr int kSmallSecondWindowF = 80;  // rounds of its second F window (run_windows)
// Small batches (up to kWaveShufflePairs pairs): a wave per pair
// (rs_shuffle_wave2_kernel), four waves per pair in the replay, speculative
// windows -- while the batch leaves most of the GPU idle, latency decides.

// Windows of both RANSAC kinds (W = 1, 2, 4, ..., kMaxWindow rounds) until
// each kind's trial cap: draw / shuffle / replay as dual-kind launches, the
// wide solve and score kernels per kind.  Kernels of windows with no active
// pair exit at once.
//
// Window r uses the parity r & 1 buffers (rb[r & 1]) and the active lists in
// rotation: its replay reads list r % 3 (the pairs still running) and writes
// list (r + 1) % 3.  Speculative schedule (spec: small batches with odd-parity
// buffers and a replay stream): the draws, shuffles, solves and scores of
// window r + 1 run on `stream` while window r is replayed on `rstream`; they
// take the pairs that were running at the start of window r (list (r - 1) %
// 3 after its replay -- that replay, two windows back, is waited for), so a
// pair that stops in window r has had one window drawn and scored in vain, and
// nothing else changes: the draws count their own trials (dtrial), read and
// write their parity's PRNG state, and the replay alone decides the pair's
// state, output and final PRNG state.
//
// np parities of window buffers (window r: rb[r % np]): 2, or 3 with decoupled
// draws, which then run two windows ahead of the replays -- window r's draws
// wait for the replay of window r - 3 (the last user of their parity's
// buffers) and take the pairs running after it (list (r - 2) % 3; before any
// replay, the begin kernel's list 0), a superset of the pairs its solves and
// scores take (list (r - 1) % 3, after window r - 2's replay, as above).  A
// pair drawn but no longer running is simply not read: its draws touch only
// its parity's buffers, its sample-index vectors and dtrial.
hipError_t run_windows(const VerifyPair* pairs, int npairs, const double* xy1, const double* xy2,
                       double* scratch, uint32_t* snaps, uint8_t* masks, VerifyOut* out,
                       const VerifyParams& P, const float4* xyf, const VerifyRoundBufs* rfp,
                       const VerifyRoundBufs* rhp, int max_chunks, int max_m, uint64_t* prof,
                       hipStream_t stream, hipEvent_t* score_ev, int* nwin, bool spec,
                       hipStream_t rstream, hipEvent_t* win_ev, int* last_h,
                       hipStream_t dstream, hipEvent_t* draw_ev, int np,
                       const std::function<void(int)>* before_last_h_replay) {
  const size_t lds = kVerifyLdsHead;  // rs_draw / rs_replay touch only the head
  const int gw = npairs < kPairGrid ? npairs : kPairGrid;
  constexpr int kShuffleLdsKb = 16;
  // Shuffle blocks: as many pairs per block as fit kShuffleLdsKb of LDS sample-index
  // vectors (the swap chains are latency-bound; LDS instead of global memory
  // shortens every step of them).
  // (pairs above 65536 matches: vectors in global memory, stride 0, one pair per block)
  const int sh_stride = max_m <= 65536 ? (max_m + 7) / 8 * 8 : 0;
  const int sh_ppb =
      sh_stride ? std::max(1, std::min(64, (kShuffleLdsKb * 1024) / (2 * sh_stride))) : 1;
  const int sh_blocks = (npairs + sh_ppb - 1) / sh_ppb;
  const int wave_stride = (max_m + 7) / 8 * 8;
  const bool wave_sh = verify_small_batch(npairs, max_m);
  const size_t wave_lds = wave_shuffle_lds_bytes(wave_stride);
  const int max_chunks_s = (max_m + kScoreThreads * kScorePchSmall - 1) / (kScoreThreads * kScorePchSmall);
  // Window sizes.  A batch that fills the GPU: 1, 2, 4, ... kMaxWindow rounds
  // (a pair's speculative rounds past its stop are GPU work).  A small batch
  // (a single Scanner stencil): its chain of windows is latency-bound, so
  // kSmallFirstWindow rounds -- enough for the near pairs' F, which stops
  // within ~64 trials -- and then the largest windows, each later window being
  // one more stage of the chain (19-pair stencil, profiles/r04_j: first window
  // 16 rounds then doubling 3.75 ms per call; first window 16 / 8 / 4 / 2 then
  // 32: 3.54 / 3.48 / 3.38 / 3.44 ms).
  const int maxw = rfp[0].wt / kTrialBatch;  // kMaxWindow, or kMaxWindowSmall
  int W = 1;
  if (wave_sh) W = std::min(kSmallFirstWindow, maxw);
  else
    while (W < maxw && (int64_t)npairs * 2 * W <= 1024) W *= 2;
  // (A run's last batch -- its window chain runs with nothing beside it --
  // starting at 4 / 8 / 16 rounds instead of the doubling rule's 1: 48.32 /
  // 48.40 / 46.86K vs 48.38K pairs/s, and the small-batch kernels on the table
  // schedule 47.98 vs 48.35K, profiles/r06_e, r06_h: fewer windows do not
  // shorten the tail, not kept.)
  // Per-kind window sizes: the same schedule for both kinds, except a small
  // batch's second F window, kSmallSecondWindowF rounds: F stops early on
  // most pairs, and that window's draws run beside the first window's solves,
  // scores and replay -- the two branches of a stencil's critical path
  // (19-pair stencil, profiles/r05_g, r05_h: 128 rounds 2.80-2.84 ms per
  // call, 96: 2.60-2.62, 80: 2.58-2.62, 64: 2.61-2.75, 48: 2.77-2.85, 32:
  // 2.93-2.97; F's 10,000 trials still take three windows).  The table
  // path's first windows per kind were measured at H 4 / 8 / 16 and F 2
  // rounds against the doubling schedule from W: no gain (round 5).
  int Wf = W, Wh = W;
  // Windows whose LO chains run in parallel (small batches with LO slots):
  // the first (later windows' records are many and mostly superseded; two
  // windows measured slower, profiles/r05_m).
  // (Two windows measured again in round 6, with three parities and the draw
  // stream: 2.18-2.30 vs 2.19-2.25 ms per batch-1 call, profiles/r06_s -- no
  // gain.)
  constexpr int lo_windows = 1;
  // Decoupled draws (speculative schedule with a draw stream): window r's
  // draws and shuffles run on dstream as soon as window r - 2 is replayed (its
  // active list) and window r - 1's prune has run (the lists and counts it
  // reads), i.e. beside window r - 1's solves and scores; rs_prune2_kernel
  // then does, on `stream`, the parts of the draws that need window r - 1's
  // scores.  draw_ev: 2r = window r drawn, 2r + 1 = window r pruned, and
  // 2 * kMaxVerifyWindows = the batch's begin kernel done.
  const bool dsplit = spec && wave_sh && dstream && draw_ev;
  if (dsplit) (void)hipEventRecord(draw_ev[2 * kMaxVerifyWindows], stream);
  int covered_f = 0, covered_h = 0, r = 0;
  while (covered_f < P.max_trials_F || covered_h < P.max_trials_H) {
    const VerifyRoundBufs& rf = rfp[r % np];
    const VerifyRoundBufs& rh = rhp[r % np];
    // lists: the replay's input and output, the wide kernels' input
    const int lin = r % 3, lout = (r + 1) % 3;
    const int lw = spec && r > 0 ? (r - 1) % 3 : lin;
    if (spec && r >= 2 && r - 2 < kMaxVerifyWindows)
      (void)hipStreamWaitEvent(stream, win_ev[2 * (r - 2) + 1], 0);
    const bool f = covered_f < P.max_trials_F, h = covered_h < P.max_trials_H;
    if (h && last_h) *last_h = r;
    const int g1 = (f ? gw : 0) + (h ? gw : 0), s1 = f ? gw : 0;
    const int g2 = (f ? sh_blocks : 0) + (h ? sh_blocks : 0), s2 = f ? sh_blocks : 0;
    if (dsplit && r < kMaxVerifyWindows) {
      int ld = lw;  // the list the draws take
      if (np == 3) {
        // two windows ahead (above), and after window r - 2's prune, the last
        // reader of this parity's counts and trial counts (as the previous
        // window's); not window r - 1's prune (it reads the first trial its
        // own draws kept, not dtrial)
        if (r >= 3) (void)hipStreamWaitEvent(dstream, win_ev[2 * (r - 3) + 1], 0);
        if (r >= 2) (void)hipStreamWaitEvent(dstream, draw_ev[2 * (r - 2) + 1], 0);
        if (r == 0) (void)hipStreamWaitEvent(dstream, draw_ev[2 * kMaxVerifyWindows], 0);
        ld = r < 2 ? 0 : (r - 2) % 3;
      } else {
        if (r >= 2) (void)hipStreamWaitEvent(dstream, win_ev[2 * (r - 2) + 1], 0);
        (void)hipStreamWaitEvent(dstream, draw_ev[r == 0 ? 2 * kMaxVerifyWindows : 2 * r - 1], 0);
      }
      hipLaunchKernelGGL(rs_drawshuffle_wave2_kernel, dim3(g1), dim3(64), kWsDrawHead + wave_lds,
                         dstream, pairs, scratch, snaps, out, rf, rh, ld, lout, P, 0, Wf, Wh, prof,
                         wave_stride, s1, 0);
      (void)hipEventRecord(draw_ev[2 * r], dstream);
      (void)hipStreamWaitEvent(stream, draw_ev[2 * r], 0);
      hipLaunchKernelGGL(rs_prune2_kernel, dim3(g1), dim3(64), 0, stream, pairs, rf, rh, lw, lout,
                         P, r > 0 ? 1 : 0, s1);
      (void)hipEventRecord(draw_ev[2 * r + 1], stream);
    } else if (wave_sh) {
      hipLaunchKernelGGL(rs_drawshuffle_wave2_kernel, dim3(g1), dim3(64), kWsDrawHead + wave_lds,
                         stream, pairs, scratch, snaps, out, rf, rh, lw, lout, P,
                         (spec && r > 0) ? 1 : 0, Wf, Wh, prof, wave_stride, s1, 1);
    } else {
      hipLaunchKernelGGL(rs_draw2_kernel, dim3(g1), dim3(64), lds, stream, pairs, scratch, snaps,
                         out, rf, rh, lw, lout, P, (spec && r > 0) ? 1 : 0, Wf, Wh, s1);
      hipLaunchKernelGGL(rs_shuffle2_kernel, dim3(g2), dim3(64),
                         (size_t)sh_ppb * sh_stride * sizeof(uint16_t), stream, pairs, scratch,
                         snaps, out, rf, rh, lw, sh_ppb, sh_stride, s2, P.prio);
    }
    if (f)
      hipLaunchKernelGGL(rs_solve_kernel<KIND_F>, dim3(kSolveGrid), dim3(64), 0, stream, pairs, xy1, xy2,
                         rf.rst, rf.wB, rf.act[lw], rf.nact + lw, rf.samp, rf.nmod, rf.fcon, rf.mods,
                         Wf, P.max_residual, rf.wt);
    if (h)
      hipLaunchKernelGGL(rs_solve_kernel<KIND_H>, dim3(kSolveGrid), dim3(64), 0, stream, pairs, xy1, xy2,
                         rh.rst, rh.wB, rh.act[lw], rh.nact + lw, rh.samp, rh.nmod, rh.fcon, rh.mods,
                         Wh, P.max_residual, rh.wt);
    if (score_ev && r < kMaxVerifyWindows) (void)hipEventRecord(score_ev[2 * r], stream);
    // Scoring per kind: split (filter counts + undecided counts, then exact
    // tests only for the models that can reach the best; the runtime's
    // choice for H) or one pass with the exact tests of every undecided point
    // (round buffers without ucnt; F).  (Speculative windows: the best a model
    // must reach may lag one window behind -- only more exact recounts.)
    if (f) {
      if (rf.ucnt) {
        hipLaunchKernelGGL((rs_score_kernel<KIND_F, true>), dim3(8192), dim3(kScoreThreads), 0,
                           stream, pairs, xyf, rf.rst, rf.wB, rf.act[lw], rf.nact + lw, rf.nmod, rf.fcon,
                           rf.mods, rf.cnts, rf.ucnt, max_chunks, Wf, P.max_residual, prof, rf.wt);

        hipLaunchKernelGGL(rs_exact_kernel<KIND_F>, dim3(8192), dim3(kScoreThreads), 0, stream,
                           pairs, xyf, rf.rst, rf.wB, rf.act[lw], rf.nact + lw, rf.nmod, rf.fcon,
                           rf.mods, rf.cnts, rf.ucnt, max_chunks, Wf, P.max_residual, rf.wt);
      } else {
        if (wave_sh)
          hipLaunchKernelGGL((rs_score_kernel<KIND_F, false, kScorePchSmall>), dim3(8192),
                             dim3(kScoreThreads), 0, stream, pairs, xyf, rf.rst, rf.wB, rf.act[lw],
                             rf.nact + lw, rf.nmod, rf.fcon, rf.mods, rf.cnts, nullptr, max_chunks_s,
                             Wf, P.max_residual, prof, rf.wt);
        else
          hipLaunchKernelGGL((rs_score_kernel<KIND_F, false>), dim3(8192), dim3(kScoreThreads), 0,
                             stream, pairs, xyf, rf.rst, rf.wB, rf.act[lw], rf.nact + lw, rf.nmod,
                             rf.fcon, rf.mods, rf.cnts, nullptr, max_chunks, Wf, P.max_residual, prof, rf.wt);
      }
    }
    if (h) {
      // The first window starts from best 0, where every model would need the
      // exact recount: it takes the one-pass kernel (exact tests inline).
      if (rh.ucnt && r > 0) {
        if (wave_sh)
          hipLaunchKernelGGL((rs_score_kernel<KIND_H, true, kScorePchSmall>), dim3(8192),
                             dim3(kScoreThreads), 0, stream, pairs, xyf, rh.rst, rh.wB, rh.act[lw],
                             rh.nact + lw, rh.nmod, rh.fcon, rh.mods, rh.cnts, rh.ucnt, max_chunks_s,
                             Wh, P.max_residual, prof, rh.wt);
        else
          hipLaunchKernelGGL((rs_score_kernel<KIND_H, true>), dim3(8192), dim3(kScoreThreads), 0,
                             stream, pairs, xyf, rh.rst, rh.wB, rh.act[lw], rh.nact + lw, rh.nmod,
                             rh.fcon, rh.mods, rh.cnts, rh.ucnt, max_chunks, Wh, P.max_residual, prof, rh.wt);
        hipLaunchKernelGGL(rs_exact_kernel<KIND_H>, dim3(8192), dim3(kScoreThreads), 0, stream,
                           pairs, xyf, rh.rst, rh.wB, rh.act[lw], rh.nact + lw, rh.nmod, rh.fcon,
                           rh.mods, rh.cnts, rh.ucnt, max_chunks, Wh, P.max_residual, rh.wt);
      } else {
        if (wave_sh)
          hipLaunchKernelGGL((rs_score_kernel<KIND_H, false, kScorePchSmall>), dim3(8192),
                             dim3(kScoreThreads), 0, stream, pairs, xyf, rh.rst, rh.wB, rh.act[lw],
                             rh.nact + lw, rh.nmod, rh.fcon, rh.mods, rh.cnts, nullptr, max_chunks_s,
                             Wh, P.max_residual, prof, rh.wt);
        else
          hipLaunchKernelGGL((rs_score_kernel<KIND_H, false>), dim3(8192), dim3(kScoreThreads), 0,
                             stream, pairs, xyf, rh.rst, rh.wB, rh.act[lw], rh.nact + lw, rh.nmod,
                             rh.fcon, rh.mods, rh.cnts, nullptr, max_chunks, Wh, P.max_residual, prof, rh.wt);
      }
    }
    if (score_ev && r < kMaxVerifyWindows) (void)hipEventRecord(score_ev[2 * r + 1], stream);
    // Small batches: the record models' LO chains of the first lo_windows
    // windows (where nearly all new bests occur), in parallel, before the
    // replay (rs_lo_chain2_kernel); later windows' replays run their few
    // chains inline (their slots are not read: lo = nullptr).
    hipStream_t rs = stream;
    if (spec && r < kMaxVerifyWindows) {
      (void)hipEventRecord(win_ev[2 * r], stream);
      (void)hipStreamWaitEvent(rstream, win_ev[2 * r], 0);
      rs = rstream;
      // (checks: work that must run before H's last window's replay is
      // enqueued -- launch_verify's SCM_DIAG_HOLD_LAST_REPLAY)
      if (h && before_last_h_replay && covered_h + Wh * kTrialBatch >= P.max_trials_H)
        (*before_last_h_replay)(r);
    }
    // (on the replay's stream: the next window's solves and scores do not wait
    // for the chains; over the replay's input list, complete there)
    VerifyRoundBufs rfr = rf, rhr = rh;
    const bool lo_win = wave_sh && rf.lo && rh.lo && r < lo_windows;
    if (lo_win) {
      const int ls = f ? npairs * kLoSlots : 0;
      hipLaunchKernelGGL(rs_lo_chain2_kernel, dim3(ls + (h ? npairs * kLoSlots : 0)), dim3(256), lds,
                         rs, pairs, scratch, snaps, out, rf, rh, lin, P, xyf, ls);
    } else {
      rfr.lo = rhr.lo = nullptr;
    }
    if (wave_sh)
      hipLaunchKernelGGL(rs_replay2w_kernel, dim3(g1), dim3(256), lds, rs, pairs, scratch,
                         snaps, out, masks, rfr, rhr, lin, lout, P, prof, xyf, s1);
    else
      hipLaunchKernelGGL(rs_replay2_kernel, dim3(g1), dim3(64), lds, rs, pairs, scratch, snaps,
                         out, masks, rf, rh, lin, lout, P, prof, xyf, s1);
    if (spec && r < kMaxVerifyWindows) (void)hipEventRecord(win_ev[2 * r + 1], rstream);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
    covered_f += Wf * kTrialBatch;
    covered_h += Wh * kTrialBatch;
    if (wave_sh) {
      // (H's second window at 96 / 64 / 48 / 32 rounds: 2.34-2.36 / 2.41-2.44 /
      // 2.48 / 2.53-2.58 vs 2.30-2.35 ms per batch-1 call, and F 64 with H
      // 64: 2.42-2.47, profiles/r06_q; window cap 160 / 192 rounds: within the
      // noise, profiles/r06_r -- not kept)
      Wf = r == 0 ? std::min(kSmallSecondWindowF, maxw) : maxw;
      Wh = maxw;
    } else {
      Wf = Wf * 2 > maxw ? maxw : Wf * 2;
      Wh = Wh * 2 > maxw ? maxw : Wh * 2;
    }
    ++r;
    if (spec && r >= kMaxVerifyWindows) spec = false;  // out of events: the rest in order
  }
  if (spec && r > 0) (void)hipStreamWaitEvent(stream, win_ev[2 * (r - 1) + 1], 0);
  if (nwin) *nwin = r < kMaxVerifyWindows ? r : kMaxVerifyWindows;
  return hipSuccess;
}

}  // namespace

int verify_small_batch_pairs() { return kWaveShufflePairs; }

bool verify_small_batch(int npairs, int max_m) {
  return npairs <= kWaveShufflePairs && (max_m + 7) / 8 * 8 <= kWsMaxStride;
}

hipError_t launch_verify(const VerifyPair* pairs, int npairs, int max_m, const double* xy1,
                         const double* xy2, double* scratch, uint32_t* snaps, uint8_t* masks,
                         VerifyOut* out, const VerifyParams& params_in, uint64_t* prof,
                         const int32_t* counts, const float4* xyf, const VerifyRoundBufs& rb_f,
                         const VerifyRoundBufs& rb_h, hipStream_t stream, hipEvent_t* score_ev,
                         int* nwin, const VerifySpec* spec) {
  if (npairs <= 0) return hipSuccess;
  hipError_t err;
  // Small batches: the latency-bound kernels (draws, LO chains, replays, final
  // passes) raise their waves' issue priority over the wide scoring kernels'
  // (2.34-2.35 vs 2.35-2.36 ms per batch-1 call, profiles/r05_o); the table
  // path keeps the default (the same priority there: within the noise,
  // profiles/r05_r, r05_s).
  VerifyParams params = params_in;
  params.prio = verify_small_batch(npairs, max_m) ? 1 : 0;
  // The kernels' dynamic LDS limit, once per device and process (contexts on
  // several threads may launch at once: std::call_once, not a plain flag).
  int dev = 0;
  if ((err = hipGetDevice(&dev)) != hipSuccess) return err;
  static std::once_flag attr_once[kMaxDevices];
  static hipError_t attr_err[kMaxDevices];
  if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
  std::call_once(attr_once[dev], [&] {
    const hipError_t es[] = {
        set_lds_attr(rs_begin2_kernel),
        set_lds_attr(rs_draw2_kernel),
        set_lds_attr(rs_shuffle2_kernel),
        set_lds_attr(rs_shuffle_wave2_kernel),
        set_lds_attr(rs_drawshuffle_wave2_kernel),
        set_lds_attr(rs_replay2_kernel),
        set_lds_attr(rs_replay2w_kernel),
        set_lds_attr(rs_lo_chain2_kernel),
        set_lds_attr(verify_final_kernel<1>),
        set_lds_attr(verify_final_kernel<8>)};
    attr_err[dev] = hipSuccess;
    for (hipError_t e : es)
      if (e != hipSuccess && attr_err[dev] == hipSuccess) attr_err[dev] = e;
  });
  if (attr_err[dev] != hipSuccess) return attr_err[dev];
  const size_t lds = sizeof(VerifyLds);
  const int gw = npairs < kPairGrid ? npairs : kPairGrid;
  const int max_chunks = (max_m + kScoreChunk - 1) / kScoreChunk;
  // Parity buffers: the odd ones from spec, else both parities alias (the
  // windows then run strictly in order on one stream).
  const bool sp = spec && spec->rb_f1 && spec->rb_h1 && spec->rstream && spec->win_ev &&
                  spec->fstream && spec->fin_ev && verify_small_batch(npairs, max_m);
  // A third parity with decoupled draws (run_windows: they run two windows ahead).
  const int np = sp && spec->dstream && spec->draw_ev && spec->rb_f2 && spec->rb_h2 ? 3 : 2;
  VerifyRoundBufs rfp[3] = {rb_f, sp ? *spec->rb_f1 : rb_f, np == 3 ? *spec->rb_f2 : rb_f};
  VerifyRoundBufs rhp[3] = {rb_h, sp ? *spec->rb_h1 : rb_h, np == 3 ? *spec->rb_h2 : rb_h};
  // each parity's draws start from the previous parity's state; its prune and
  // speculative skip read the previous window's counts
  VerifyRoundBufs pf[3] = {rfp[0], rfp[1], rfp[2]}, ph[3] = {rhp[0], rhp[1], rhp[2]};
  for (int k = 0; k < np; ++k) {
    const int o = (k + np - 1) % np;
    rfp[k].pstate = pf[o].wstate;
    rfp[k].pcnts = pf[o].cnts;
    rfp[k].pwB = pf[o].wB;
    rhp[k].pstate = ph[o].wstate;
    rhp[k].pcnts = ph[o].cnts;
    rhp[k].pwB = ph[o].wB;
  }
  // LORANSAC<7-pt, 8-pt> (F, then its inlier masks) and LORANSAC<H, H>, each
  // on its own PRNG stream, advanced together window by window.
  if (!(spec && spec->lists_zeroed)) {
    if ((err = hipMemsetAsync(rb_f.nact, 0, 3 * sizeof(int32_t), stream)) != hipSuccess) return err;
    if ((err = hipMemsetAsync(rb_h.nact, 0, 3 * sizeof(int32_t), stream)) != hipSuccess) return err;
  }
  hipLaunchKernelGGL(rs_begin2_kernel, dim3(2 * gw), dim3(64), kVerifyLdsHead, stream, pairs,
                     npairs, scratch, snaps, out, masks, xyf, rfp[0], rhp[0], params, gw);
  // Diagnostics: SCM_DIAG_SCRIBBLE_F_SIDX=1 makes the final kernel rewrite the
  // F area's index vector before every watermark draw (the worst the
  // speculative F draws beside the early pass can do; outputs must not move,
  // tests/test_gpu_stencil.py).  Read per call so a test can set it.
  const char* diag_env = getenv("SCM_DIAG_SCRIBBLE_F_SIDX");
  const char* chk_env = getenv("SCM_DIAG_SPEC_CHECK");  // (verify_final_kernel bit 16)
  const int diag = (diag_env && atoi(diag_env) ? 8 : 0) | (chk_env && atoi(chk_env) ? 16 : 0);
  // The speculative watermark pass (phase 3, below) reads the pairs' F / H
  // states while H's last window's replay may be writing them.
  // SCM_DIAG_HOLD_LAST_REPLAY=1 (checks, read per call) forces one extreme
  // order: phase 3 is enqueued before that replay and the replay waits for it,
  // so phase 3 sees every pair whose F or H ends in that window still running
  // (tests/test_gpu_stencil.py).
  const char* hold_env = getenv("SCM_DIAG_HOLD_LAST_REPLAY");
  const bool spec_pass = sp && spec->dstream && spec->draw_ev;
  const bool hold = spec_pass && spec->spec_ev && hold_env && atoi(hold_env);
  bool phase3_done = false;
  auto phase3 = [&](int lh) {
    (void)hipStreamWaitEvent(spec->fstream, spec->draw_ev[2 * lh], 0);
    (void)hipStreamWaitEvent(spec->fstream, spec->win_ev[2 * (lh - 1) + 1], 0);
    hipLaunchKernelGGL(verify_final_kernel<8>, dim3(npairs), dim3(512), lds, spec->fstream,
                       pairs, xy1, xy2, scratch, snaps, masks, out, params, prof, counts,
                       rb_f.rst, rb_h.rst, 3 | diag, rhp[lh % np].wstate);
  };
  const std::function<void(int)> hold_fn = [&](int lh) {
    if (lh < 1) return;  // (no phase 3 when H ends in the first window)
    phase3(lh);
    phase3_done = true;
    (void)hipEventRecord(spec->spec_ev, spec->fstream);
    (void)hipStreamWaitEvent(spec->rstream, spec->spec_ev, 0);
  };
  int last_h = -1;
  if ((err = run_windows(pairs, npairs, xy1, xy2, scratch, snaps, masks, out, params, xyf, rfp,
                         rhp, max_chunks, max_m, prof, stream, score_ev, nwin, sp,
                         sp ? spec->rstream : stream, sp ? spec->win_ev : nullptr, &last_h,
                         sp ? spec->dstream : nullptr, sp ? spec->draw_ev : nullptr, np,
                         hold ? &hold_fn : nullptr)) != hipSuccess)
    return err;
  if (sp && last_h >= 0 && last_h < kMaxVerifyWindows) {
    // Configuration + watermark of the pairs done when H's last window is
    // replayed (typically all but the far pairs' F), beside the later windows;
    // then the rest after the last window.  Nothing orders this pass against
    // the later windows' F draws on dstream: the watermark's index vector is
    // in the pair's H area (verify_final_kernel), which they never touch.
    // Before it, the speculative watermark decisions (phase 3): once H's last
    // window is drawn and the window before it replayed (F done for the near
    // pairs), beside H's last window's solves, scores and replay.
    if (last_h >= 1 && spec_pass && !phase3_done) phase3(last_h);
    // Phase 2 waits for phase 1 (the pairs it left), or, with an event after
    // phase 3, for phase 3 only (it must not run a pair's watermark RANSAC
    // while phase 3 may) and claims pairs beside phase 1.
    const bool beside = spec->spec_ev != nullptr;
    if (beside) (void)hipEventRecord(spec->spec_ev, spec->fstream);
    (void)hipStreamWaitEvent(spec->fstream, spec->win_ev[2 * last_h + 1], 0);
    hipLaunchKernelGGL(verify_final_kernel<8>, dim3(npairs), dim3(512), lds, spec->fstream, pairs,
                       xy1, xy2, scratch, snaps, masks, out, params, prof, counts, rb_f.rst,
                       rb_h.rst, 1 | diag, nullptr);
    (void)hipEventRecord(spec->fin_ev, spec->fstream);
    (void)hipStreamWaitEvent(stream, beside ? spec->spec_ev : spec->fin_ev, 0);
    hipLaunchKernelGGL(verify_final_kernel<8>, dim3(npairs), dim3(512), lds, stream, pairs, xy1,
                       xy2, scratch, snaps, masks, out, params, prof, counts, rb_f.rst, rb_h.rst,
                       2 | diag, nullptr);
    if (beside) (void)hipStreamWaitEvent(stream, spec->fin_ev, 0);
  } else if (verify_small_batch(npairs, max_m)) {
    hipLaunchKernelGGL(verify_final_kernel<8>, dim3(npairs), dim3(512), lds, stream, pairs, xy1,
                       xy2, scratch, snaps, masks, out, params, prof, counts, rb_f.rst, rb_h.rst,
                       diag, nullptr);
  } else {
    hipLaunchKernelGGL(verify_final_kernel<1>, dim3(npairs), dim3(kVerifyThreads), lds, stream,
                       pairs, xy1, xy2, scratch, snaps, masks, out, params, prof, counts, rb_f.rst,
                       rb_h.rst, diag, nullptr);
  }
  return hipGetLastError();
}

hipError_t launch_gather(const GatherPair* pairs, int npairs, int max_m, const uint2* matches,
                         const float2* kpxy, double* xy1, double* xy2, const int32_t* counts,
                         float4* xyf, hipStream_t stream) {
  if (npairs <= 0 || max_m <= 0) return hipSuccess;
  const unsigned gx =
      npairs <= kGatherWidePairs ? (unsigned)((max_m + kGatherChunk - 1) / kGatherChunk) : 1u;
  hipLaunchKernelGGL(gather_kernel, dim3(gx, npairs), dim3(kGatherThreads), 0, stream, pairs, matches,
                     kpxy, xy1, xy2, counts, xyf);
  return hipGetLastError();
}

hipError_t launch_compact(const int32_t* counts, int npairs, const int64_t* offsets,
                          const int64_t* match_off, const uint2* matches, const uint8_t* masks,
                          uint2* out_matches, uint8_t* out_masks, hipStream_t stream) {
  if (npairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(compact_kernel, dim3(npairs), dim3(256), 0, stream, counts, offsets,
                     match_off, matches, masks, out_matches, out_masks);
  return hipGetLastError();
}

}  // namespace scm
