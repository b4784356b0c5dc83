// Descriptors and launchers of the two-view-geometry kernel (verify_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace scm {

constexpr int kVerifyThreads = 64;    // one wavefront per pair
constexpr int kTrialBatch = 64;       // hypotheses solved in parallel per round (one per lane)
constexpr int kVerifyModelDoubles = kTrialBatch * 27;  // per-pair model buffer
// PRNG words per pair: for each of the two streams (F; H then watermark) the
// handed-on mt19937 state (640) and the abort-rewind snapshot (640).
constexpr int kVerifyStreamWords = 1280;
constexpr int kVerifySnapWords = 2 * kVerifyStreamWords;
// Per-pair scratch of one RANSAC kind (doubles): residuals / inlier gathers
// (10 m), the model buffer, then the uint32 sample-index vector.  F and H run
// concurrently, each in its own area (H's follows F's; the watermark RANSAC
// reuses F's after both finished).
__host__ __device__ inline int64_t verify_kind_scratch_doubles(int64_t m) {
  return 10 * m + kVerifyModelDoubles + (m + 1) / 2 + 1;
}
inline int64_t verify_scratch_doubles(int64_t m) { return 2 * verify_kind_scratch_doubles(m); }

// Scalar options of TwoViewGeometry::EstimateUncalibrated (SURVEY.md §8a a2,
// a9-a14) after the op's parseConfigs (sequential_matching.cc:64-75).
struct VerifyParams {
  double max_residual;            // max_error^2
  double confidence;
  double dyn_num_trials_multiplier;
  double max_H_inlier_ratio;
  double watermark_min_inlier_ratio;
  double watermark_border_size;
  int32_t min_num_trials;
  int32_t max_trials_F;           // min(max_num_trials, ComputeNumTrials(min_inlier_ratio))
  int32_t max_trials_H;
  int32_t max_trials_T;           // watermark translation RANSAC (ratio 0.7)
  int32_t min_num_inliers;
  int32_t detect_watermark;
  uint32_t base_seed;
  int32_t prio;  // small batches: the latency-bound kernels' waves issue at raised priority
};

struct VerifyPair {
  int64_t pts_off;   // double offset of xy1/xy2 (2 doubles per match)
  int64_t scr_off;   // double offset of the per-pair scratch (verify_scratch_doubles(m))
  int64_t mask_off;  // byte offset of the F inlier mask
  int32_t m;         // number of matches when cidx < 0
  int32_t cidx;      // index into the device match counts (>= 0: read m there)
  uint32_t id1, id2;
  int32_t out_idx;   // VerifyOut slot
  int32_t pad_;
};

struct VerifyOut {
  int32_t config;
  int32_t num_inliers;   // F inliers = |inlier_matches| (0 after the post-filter)
  int32_t f_trials, h_trials;
  int32_t f_inliers_raw, h_inliers_raw;
  int32_t watermark;
  int32_t raw_config;    // Estimate's configuration before the op's post-filter
  double F[9];
  double H[9];
  // (model, point) residual evaluations the sequential LO-RANSAC scores up to
  // its stop (speculative trials past the abort excluded): the scoring
  // kernels' algorithmic work (bench.py roofline_verify)
  int64_t f_evals, h_evals;
  // Small batches: the speculative watermark decision (verify_final_kernel
  // phase 3) -- spec 0: none, 1: from H's final stream state, 2: from the state
  // after H's last window's draws (valid unless that window's replay aborted
  // H); spec_wm the decision.
  int32_t spec, spec_wm;
  // How phases 1 / 2 took the watermark decision (counted by the runtime):
  // 0 no speculation, 3 the speculative decision, 1 the speculative decision
  // recomputed and equal (SCM_DIAG_SPEC_CHECK=1), 2 recomputed and different
  // (never: a test asserts it), 4 the speculation void (H aborted in its
  // last window) and recomputed.
  int32_t spec_check, pad3_;
};

// Per-pair state of the round-synchronous LO-RANSAC (verify_kernels.hip).
struct RansacState {
  int32_t n, done, trial, dyn_max;
  int32_t max_trials, best_n, best_sum_valid, res_sel;
  int32_t B, num_trials, pad_;
  int32_t aborted;  // the run ended by the abort (dynamic trial bound), not at its cap
  int64_t evals;  // (model, point) evaluations of the trials up to the stop
  double best_sum;
  double S;  // max |coordinate| of the pair's points (fp32 filter bound)
  double best_model[9];
};

// Windowed verifier: up to kMaxWindow rounds of kTrialBatch hypotheses.
constexpr int kMaxWindow = 32;  // rounds per window at most (16: -1.3 %, 64: -1 %, bench s35;
                                // 64 again after trials_left: -0.4 %, profiles/r04_l)
constexpr int kWindowTrials = kMaxWindow * kTrialBatch;
// Small batches (verify_small_batch): windows of up to 128 rounds -- every
// window is one more latency-bound stage of a stencil's chain (19-pair
// stencil: 3.35 ms per call with 32, 3.13 ms with 64, profiles/r04_k; 3.07-3.16
// with 64 vs 2.90-2.93 with 128, profiles/r04_n: H's 5,295 trials in two
// windows).
constexpr int kMaxWindowSmall = 128;
constexpr int kWindowTrialsSmall = kMaxWindowSmall * kTrialBatch;

// Device buffers of the windowed verifier (V = pairs of a batch, T =
// VerifyRoundBufs::wt): rst[V], samp[V][T*8], nmod[V][T], fcon[V][3T][12],
// mods[V][3T][9], cnts[V][3T], wsnap[V][640] (the window's start PRNG state), act[2][V],
// nact[2].
// One window parity's buffers of one RANSAC kind.  The per-window buffers
// (samp .. wstate) exist twice for small batches, so that the draws, shuffles,
// solves and scores of window r + 1 can run while window r is replayed
// (speculative windows, run_windows); rst, dtrial and the active lists are
// shared by both parities.  Large batches alias both parities.
// Parallel local optimisation of a small batch's window (rs_lo_chain2_kernel,
// DESIGN §10): the LO chain of each of a pair's first kLoSlots record models
// (counts reaching the running maximum of the window's counts before them,
// from the pair's best at the window start), computed on its own before the
// replay, which then takes a record's outcome instead of running its LO.
constexpr int kLoSlots = 8;
struct LoSlot {
  int32_t rec;        // record index (trial of the window x models per trial + model), -1: none
  int32_t count;      // the chain's final inlier count
  int32_t sum_valid;  // sum is the final model's exact index-order residual sum
  int32_t buf;        // slot buffer holding the final model's residuals (0: the record's own)
  double sum;
  double model[9];
};
// A slot's data: three residual buffers of n doubles and the inlier gather
// buffer (n float4, 16-B aligned) -- lo_stride doubles per slot.
inline int64_t lo_slot_doubles(int64_t max_m) { return 5 * max_m + 4; }

struct VerifyRoundBufs {
  RansacState* rst;
  uint32_t* samp;
  int32_t* nmod;
  float* fcon;
  double* mods;
  uint32_t* cnts;
  uint32_t* ucnt;  // split scoring: undecided points per model [V][3T]
  uint32_t* wsnap;
  int32_t* wB;       // trials of the pair's window
  uint32_t* wstate;  // PRNG state after the window's draws (kVerifyStateWords per pair)
  uint32_t* pstate;  // the other parity's wstate: where the window's draws start
  const uint32_t* pcnts;  // the other parity's cnts and wB (the previous window's, read
  const int32_t* pwB;     //   by speculative draws to skip pairs certain to stop)
  int32_t* dtrial;   // trials drawn so far
  int32_t* act[3];   // active-pair lists (rotating: window r's replay reads r % 3)
  int32_t* nact;     // their lengths [3]
  int wt;            // trials per pair the window buffers hold (T: kWindowTrials or
                     // kWindowTrialsSmall); the windows' rounds are at most wt / kTrialBatch
  LoSlot* lo = nullptr;       // small batches: [V][kLoSlots] outcomes (nullptr: LO inline)
  double* lo_data = nullptr;  // [V][kLoSlots][lo_stride]
  int64_t lo_stride = 0;
};
constexpr int kVerifyStateWords = 640;

// snaps: kVerifySnapWords uint32 per pair (PRNG states handed between the
// windowed kernels + the per-round snapshots for the abort rewind).  The F
// LO-RANSAC (round buffers rb_f) and the H LO-RANSAC (rb_h, its own PRNG
// stream) advance together in one launch sequence on `stream`; the
// configuration, watermark and post-filter kernel follows.
// score_ev (optional, 2 * kMaxVerifyWindows events): recorded around each
// window's scoring kernels; *nwin receives the number of windows launched.
constexpr int kMaxVerifyWindows = 64;
// Speculative windows (small batches): rb_f1 / rb_h1 are the odd parity's
// buffers (nullptr: none), rstream the replay stream and win_ev
// 2 * kMaxVerifyWindows events (window r's wide kernels done, its replay done).
// fstream / fin_ev: the early verify_final pass (pairs whose F and H are both
// done once H's last window is replayed) runs there beside the later windows.
struct VerifySpec {
  const VerifyRoundBufs* rb_f1 = nullptr;
  const VerifyRoundBufs* rb_h1 = nullptr;
  hipStream_t rstream = nullptr;
  hipEvent_t* win_ev = nullptr;
  hipStream_t fstream = nullptr;
  hipEvent_t fin_ev = nullptr;
  // (optional) the speculative watermark pass done: with it the last final
  // pass waits for that pass only and runs beside the early one, the two
  // claiming pairs (RansacState::pad_)
  hipEvent_t spec_ev = nullptr;
  // The caller zeroed both kinds' list lengths (rb_f.nact / rb_h.nact) on
  // `stream` already (the runtime does it before the count read-back).
  bool lists_zeroed = false;
  // Decoupled draws (optional): window r's draws run on dstream beside window
  // r - 1's scoring; draw_ev: 2 * kMaxVerifyWindows + 1 events.
  hipStream_t dstream = nullptr;
  hipEvent_t* draw_ev = nullptr;
  // A third parity's buffers (optional, with decoupled draws): the draws then
  // run two windows ahead of the replays.
  const VerifyRoundBufs* rb_f2 = nullptr;
  const VerifyRoundBufs* rb_h2 = nullptr;
};
hipError_t launch_verify(const VerifyPair* pairs, int npairs, int max_m, const double* xy1,
                         const double* xy2, double* scratch, uint32_t* snaps, uint8_t* masks,
                         VerifyOut* out, const VerifyParams& params, uint64_t* prof,
                         const int32_t* counts, const float4* xyf, const VerifyRoundBufs& rb_f,
                         const VerifyRoundBufs& rb_h, hipStream_t stream,
                         hipEvent_t* score_ev = nullptr, int* nwin = nullptr,
                         const VerifySpec* spec = nullptr);
// Whether launch_verify runs the small-batch kernels (wave-per-pair shuffle,
// four-wave replay, speculative windows) for a batch of npairs pairs with at
// most max_m matches.
bool verify_small_batch(int npairs, int max_m);
// The pair count at or below which a batch may take the small-batch kernels.
int verify_small_batch_pairs();
size_t verify_lds_bytes(int max_m);
constexpr int kVerifyProfSlots = 90;

// Gathers the matched keypoint coordinates of each pair (float -> double,
// FeatureKeypointsToPointsVector, sequential_matching.cc:91-92).
struct GatherPair {
  int64_t match_off;  // uint2 offset into the matcher's match buffer
  int64_t kp1_off;    // float2 offset of image 1 / image 2 keypoint xy
  int64_t kp2_off;
  int64_t pts_off;    // destination double offset / 2
  int32_t m;          // number of matches when cidx < 0
  int32_t cidx;       // index into the device match counts (>= 0: read m there)
};
// (max_m: at least every pair's match count)
hipError_t launch_gather(const GatherPair* pairs, int npairs, int max_m, const uint2* matches,
                         const float2* kpxy, double* xy1, double* xy2, const int32_t* counts,
                         float4* xyf, hipStream_t stream);
// Packs each pair's matches / F-inlier mask contiguously at offsets[p].
hipError_t launch_compact(const int32_t* counts, int npairs, const int64_t* offsets,
                          const int64_t* match_off, const uint2* matches, const uint8_t* masks,
                          uint2* out_matches, uint8_t* out_masks, hipStream_t stream);

}  // namespace scm
