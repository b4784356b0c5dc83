// Host runtime of the MI355X sequential-matching stage: implements the C ABI
// of include/scm.h on top of the two HIP kernels (match_kernels.hip,
// verify_kernels.hip).  Mirrors SequentialMatchingCPUKernel
// (reference integration/op_cpp/sequential_matching.cc:27-205): one context
// = one kernel instance bound to one device with its own stream and HBM
// workspace; execute() over a stencil, or the batched table path that keeps
// every descriptor resident in HBM.
//
// Batch pipeline (table path): pairs are cut into batches of whole pivot
// rows; each batch is enqueued as
//   match tiles -> finalize -> gather -> verify -> compact
// Matching runs on one stream with buffers laid out for the worst case (one
// match slot per pivot keypoint), so it never waits for the host.  Only the
// per-pair match counts come back early; the host then launches verification
// of exactly the pairs that need it (longest first) on the batch's own
// stream, compacts matches and F-inlier masks in HBM and DMAs the results to
// pinned memory.  Three batch buffer sets rotate: while batch b+1 is matched
// and batch b verified, the host serialises batch b-1's io.cc rows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "geom_solvers.h"
#include "scm_internal.h"
#include "scm_pool.h"
#include "verify_kernels.h"

namespace scm {

thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

namespace {

constexpr int64_t kMaxPairsPerBatch = 16384;
// (a batch's pairs index grid dimension y of the finalize, rowcheck, recheck and
// gather launches, at most 65,535; a batch exceeds the cap only with a single
// row of more pairs -- a stencil of over 16,385 images -- and a launch past
// 65,535 then fails with its error)
static_assert(kMaxPairsPerBatch <= 65535, "pairs of a batch on grid y");
constexpr int64_t kDefaultPairsPerBatch = 8192;
// Scanner op calls that fit one batch: cut into up to kOpCallBatches batches
// of at least verify_small_batch_pairs() pairs each (run_rows).
constexpr int64_t kOpCallBatches = 3;

struct ImageTable {
  int64_t n = 0;
  std::vector<uint32_t> ids;
  std::vector<int32_t> nkp, ndesc;
  std::vector<int64_t> desc_row;  // first (padded) bf16 descriptor row
  std::vector<int64_t> kp_off;    // first float2 keypoint
  std::vector<uint64_t> max_norm2;
  int64_t total_rows = 0, total_kp = 0;
  DevBuf desc;   // uint16 bf16 [total_rows][128] (bf16 matcher, SCM_MATCH_BF16=1)
  DevBuf desc8;  // a ^ 0x80 [total_rows][128] (i8 matcher, default)
  DevBuf csum;   // int32 128 * sum_d a_d [total_rows] (i8 matcher)
  DevBuf kpxy;   // float2 [total_kp]
  DevBuf u8;     // upload staging
  void release() {
    desc.release();
    desc8.release();
    csum.release();
    kpxy.release();
    u8.release();
  }
};

struct PairSpec {
  int32_t a, b;  // image indices in the table
};

// Identity of one execute() image: the reference decodes every stencil
// element's own bytes (sequential_matching.cc:115-122) and its image ids come
// from PrepareImage's per-instance counter starting at 0 (prepare_image.cc:
// 11-20), so an id alone does not name an image.  Two elements are the same
// image when id, feature counts and 64-bit hashes of the keypoint and
// descriptor bytes all agree.
struct ImageKey {
  uint32_t id = 0;
  int64_t nkp = 0, ndesc = 0;
  uint64_t hkp = 0, hdesc = 0;
  bool operator==(const ImageKey& o) const {
    return id == o.id && nkp == o.nkp && ndesc == o.ndesc && hkp == o.hkp && hdesc == o.hdesc;
  }
};
struct ImageKeyHash {
  size_t operator()(const ImageKey& k) const {
    return (size_t)(k.hdesc ^ (k.hkp * 0x9E3779B97F4A7C15ULL) ^ ((uint64_t)k.id << 17));
  }
};

// 64-bit content hash (the xxHash64 construction: four independent
// multiply-rotate lanes over 32-byte stripes, then a tail and an avalanche).
inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
uint64_t hash_bytes(const uint8_t* p, size_t n, uint64_t seed) {
  constexpr uint64_t P1 = 0x9E3779B185EBCA87ULL, P2 = 0xC2B2AE3D27D4EB4FULL,
                     P3 = 0x165667B19E3779F9ULL, P4 = 0x85EBCA77C2B2AE63ULL,
                     P5 = 0x27D4EB2F165667C5ULL;
  auto round = [](uint64_t acc, uint64_t w) { return rotl64(acc + w * P2, 31) * P1; };
  auto load = [](const uint8_t* q) {
    uint64_t w;
    std::memcpy(&w, q, 8);
    return w;
  };
  const uint8_t* const end = p + n;
  uint64_t h;
  if (n >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const uint8_t* const lim = end - 32;
    do {
      v1 = round(v1, load(p));
      v2 = round(v2, load(p + 8));
      v3 = round(v3, load(p + 16));
      v4 = round(v4, load(p + 24));
      p += 32;
    } while (p <= lim);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    for (uint64_t v : {v1, v2, v3, v4}) h = (h ^ round(0, v)) * P1 + P4;
  } else {
    h = seed + P5;
  }
  h += (uint64_t)n;
  for (; p + 8 <= end; p += 8) h = rotl64(h ^ round(0, load(p)), 27) * P1 + P4;
  for (; p < end; ++p) h = rotl64(h ^ ((uint64_t)*p * P5), 11) * P1;
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

// Content hash of a byte buffer of any size, computed in parallel: the
// buffer's kHashChunk-byte chunks are hashed independently (hash_bytes, seed
// mixed with the chunk index) and the hash of their hashes is the content
// hash (with the length).  Chunk tasks of many buffers run on a WorkerPool.
constexpr size_t kHashChunk = (size_t)256 << 10;
inline int64_t hash_chunks(size_t n) { return (int64_t)((n + kHashChunk - 1) / kHashChunk); }
inline uint64_t hash_chunk(const uint8_t* p, size_t n, int64_t k, uint64_t seed) {
  const size_t off = (size_t)k * kHashChunk;
  return hash_bytes(p + off, std::min(kHashChunk, n - off), seed + 0x9E3779B97F4A7C15ULL * (uint64_t)(k + 1));
}
inline uint64_t hash_combine_chunks(const uint64_t* h, int64_t m, size_t n, uint64_t seed) {
  return hash_bytes(reinterpret_cast<const uint8_t*>(h), (size_t)m * sizeof(uint64_t), seed ^ (uint64_t)n);
}

// Buffers of one execute() element (what Scanner hands over: the same
// buffers for an element that several stencils or calls share).
struct Src {
  const float* kp;
  int64_t nkp;
  const uint8_t* desc;
  int64_t ndesc;
  bool operator==(const Src& o) const {
    return kp == o.kp && nkp == o.nkp && desc == o.desc && ndesc == o.ndesc;
  }
};
struct SrcHash {
  size_t operator()(const Src& s) const {
    return std::hash<const void*>()(s.desc) ^ (std::hash<const void*>()(s.kp) * 31) ^
           (size_t)(s.nkp * 0x9E3779B97F4A7C15ULL) ^ (size_t)s.ndesc;
  }
};

// Sampled fingerprint of an element's bytes: 64 8-byte words at offsets
// i * stride (stride = ((n - 8) / 64) rounded down to a multiple of 8) and the
// last 8 bytes of each buffer, or the whole buffer when it is under 520 bytes.
// ~130 loads: cheap enough to check before the GPU run whether a buffer the
// previous call also handed over (same address and size) still holds the
// same image.  A recycled buffer that now holds another image differs in
// these words; only an in-place rewrite that leaves every sampled word alone
// gets past it, and the full content hash checked after the run catches that.
uint64_t sample_words(const uint8_t* p, size_t n, uint64_t h) {
  if (n < 520) return hash_bytes(p, n, h);
  const size_t stride = ((n - 8) / 64) & ~(size_t)7;
  auto mix = [](uint64_t a, uint64_t w) {
    a ^= w * 0x9E3779B185EBCA87ULL;
    return ((a << 29) | (a >> 35)) * 0xC2B2AE3D27D4EB4FULL;
  };
  for (size_t i = 0; i < 64; ++i) {
    uint64_t w;
    std::memcpy(&w, p + i * stride, 8);
    h = mix(h, w);
  }
  uint64_t w;
  std::memcpy(&w, p + n - 8, 8);
  return mix(h, w) ^ n;
}

struct SpecKey {
  ImageKey key;  // content key the buffers held in the previous call
  uint64_t fp;   // their sampled fingerprint then
};

// Pinned host result buffer: the DMA target of each batch's results.
struct PinnedOut {
  void* host = nullptr;
  void* dev = nullptr;  // its device address (launch_stage_upload reads the offsets there)
  size_t bytes = 0;
  int ensure(size_t need) {
    if (need <= bytes) return SCM_OK;
    release();
    const size_t want = need + need / 4 + 4096;
    if (hipHostMalloc(&host, want, hipHostMallocDefault) != hipSuccess) {
      host = nullptr;
      set_error("hipHostMalloc of " + std::to_string(want) + " bytes failed");
      return SCM_E_NOMEM;
    }
    if (hipHostGetDevicePointer(&dev, host, 0) != hipSuccess) {
      (void)hipHostFree(host);
      host = dev = nullptr;
      set_error("hipHostGetDevicePointer failed");
      return SCM_E_DEVICE;
    }
    bytes = want;
    return SCM_OK;
  }
  void release() {
    if (host) (void)hipHostFree(host);
    host = dev = nullptr;
    bytes = 0;
  }
};

// Diagnostics builds only (-DSCM_DIAG_HOST_TIMES, probes/build_*): host
// timestamps of one execute() call's steps, printed to stderr per call.
// With them, GPU times of the first batch's stage events from an event
// recorded on the matching stream at the call's start (g_hte, microseconds).
#ifdef SCM_DIAG_HOST_TIMES
std::chrono::steady_clock::time_point g_ht[16];
#define SCM_HT(k) (g_ht[k] = std::chrono::steady_clock::now())
hipEvent_t g_hte = nullptr;
float g_hte_us[4] = {0, 0, 0, 0};
#define SCM_HTE_RECORD(s) \
  do { \
    if (!g_hte) (void)hipEventCreate(&g_hte); \
    (void)hipEventRecord(g_hte, s); \
  } while (0)
#define SCM_HTE_READ(evs) \
  do { \
    for (int i_ = 0; i_ < 4; ++i_) { \
      float ms_ = -1.f; \
      (void)hipEventElapsedTime(&ms_, g_hte, (evs)[i_]); \
      g_hte_us[i_] = ms_ * 1000.f; \
    } \
  } while (0)
#else
#define SCM_HT(k) ((void)0)
#define SCM_HTE_RECORD(s) ((void)0)
#define SCM_HTE_READ(evs) ((void)0)
#endif

// One in-flight batch: device workspace, descriptor staging, results.
struct BatchSet {
  DevBuf rowaux, rlist;  // v2 finalize: row (best, second bound), row-recheck buckets
  // mdesc: the matcher's jobs, pair descriptors and match offsets, vdesc: the
  // gather and verification pair tables -- each one upload (one copy) of the
  // staging layout; d_* point into them
  DevBuf mdesc, rowres, colpart, m21, matches, counts, vdesc, xy1, xy2, scratch,
      snaps, masks, offsets, prof, xyf, dvout, dpack, dpmask, rst, samp, nmod, fcon,
      cnts, act, nact, mods, wsnap;
  MatchJob* d_jobs = nullptr;
  PairDesc* d_pairs = nullptr;
  int64_t* d_moff = nullptr;
  GatherPair* d_gpairs = nullptr;
  VerifyPair* d_vpairs = nullptr;
  // round buffers of the H LO-RANSAC (advanced beside F's, own PRNG stream)
  DevBuf h_rst, h_samp, h_nmod, h_fcon, h_cnts, h_act, h_nact, h_mods, h_wsnap;
  DevBuf ucnt, h_ucnt;  // split scoring: undecided points per model
  DevBuf wb, wstate, dtrial, h_wb, h_wstate, h_dtrial;  // window trial counts, PRNG states
  // odd-parity window buffers of small batches (speculative windows, launch_verify)
  DevBuf o_samp, o_nmod, o_fcon, o_mods, o_cnts, o_ucnt, o_wsnap, o_wb, o_wstate;
  DevBuf oh_samp, oh_nmod, oh_fcon, oh_mods, oh_cnts, oh_ucnt, oh_wsnap, oh_wb, oh_wstate;
  // their third parity (decoupled draws two windows ahead)
  DevBuf t_samp, t_nmod, t_fcon, t_mods, t_cnts, t_ucnt, t_wsnap, t_wb, t_wstate;
  DevBuf th_samp, th_nmod, th_fcon, th_mods, th_cnts, th_ucnt, th_wsnap, th_wb, th_wstate;
  DevBuf lo_slot[4], lo_data[4];  // small batches' parallel LO: (kind, parity) slots and their data
  hipStream_t rstream = nullptr;  // replay stream of speculative windows (another set's vstream)
  hipStream_t fstream = nullptr;  // early verify_final pass of small batches (the third set's)
  hipEvent_t wev[2 * kMaxVerifyWindows] = {};
  hipEvent_t dev[2 * kMaxVerifyWindows + 1] = {};  // decoupled draws (VerifySpec::draw_ev)
  hipEvent_t fev = nullptr;
  hipEvent_t spev = nullptr;  // the speculative watermark pass done (VerifySpec::spec_ev)
  HostBuf stage, vstage;
  PinnedOut out;
  size_t off_counts = 0, off_offsets = 0, off_vout = 0, off_matches = 0, off_masks = 0;
  // 0 match start, 1 tiles done, 2 finalize done, 3 counts on host (match
  // stream); 4 verify start, 5 verify done, 6 compaction done (verify stream)
  hipEvent_t ev[7] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  hipEvent_t sev[2 * kMaxVerifyWindows] = {};  // around each window's scoring kernels
  int nwin = 0;                                // windows of the last verification
  hipStream_t vstream = nullptr;  // verification stream of this set
  const ImageTable* table = nullptr;
  std::vector<PairSpec> specs;
  std::vector<int64_t> moff;  // first match slot of each pair
  int64_t P = 0, slots = 0, nprof = 0;
  bool verify = false;
  bool pending = false;  // stage 1 enqueued, results not collected
  bool posted = false;   // stage 2 enqueued
  bool matched = false;
  void release() {
    for (DevBuf* b : {&rowaux, &rlist, &mdesc, &rowres, &colpart, &m21, &matches, &counts, &vdesc,
                      &xy1, &xy2, &scratch, &snaps, &masks, &offsets, &prof, &xyf, &dvout,
                      &dpack, &dpmask, &rst, &samp, &nmod, &fcon, &cnts, &act, &nact,
                      &mods, &wsnap, &h_rst, &h_samp, &h_nmod, &h_fcon, &h_cnts, &h_act, &h_nact,
                      &h_mods, &h_wsnap, &ucnt, &h_ucnt, &wb, &wstate, &dtrial, &h_wb, &h_wstate,
                      &h_dtrial, &o_samp, &o_nmod, &o_fcon, &o_mods, &o_cnts, &o_ucnt, &o_wsnap,
                      &o_wb, &o_wstate, &oh_samp, &oh_nmod, &oh_fcon, &oh_mods, &oh_cnts, &oh_ucnt,
                      &oh_wsnap, &oh_wb, &oh_wstate, &t_samp, &t_nmod, &t_fcon, &t_mods, &t_cnts,
                      &t_ucnt, &t_wsnap, &t_wb, &t_wstate, &th_samp, &th_nmod, &th_fcon, &th_mods,
                      &th_cnts, &th_ucnt, &th_wsnap, &th_wb, &th_wstate, &lo_slot[0], &lo_slot[1], &lo_slot[2],
                      &lo_slot[3], &lo_data[0], &lo_data[1], &lo_data[2], &lo_data[3]})
      b->release();
    stage.release();
    vstage.release();
    out.release();
    for (auto& e : ev) {
      if (e) (void)hipEventDestroy(e);
      e = nullptr;
    }
    for (auto& e : sev) {
      if (e) (void)hipEventDestroy(e);
      e = nullptr;
    }
    for (auto& e : wev) {
      if (e) (void)hipEventDestroy(e);
      e = nullptr;
    }
    for (auto& e : dev) {
      if (e) (void)hipEventDestroy(e);
      e = nullptr;
    }
    if (fev) (void)hipEventDestroy(fev);
    fev = nullptr;
    if (spev) (void)hipEventDestroy(spev);
    spev = nullptr;
  }
};

// Collected results of one batch (views into the mapped buffer).
struct BatchView {
  int64_t P = 0;
  const int32_t* counts = nullptr;
  const int64_t* offsets = nullptr;
  const VerifyOut* vout = nullptr;  // P entries (verify runs only)
  const Match* matches = nullptr;   // pair p at offsets[p]
  const uint8_t* masks = nullptr;
};

}  // namespace
}  // namespace scm

using namespace scm;

struct scm_context {
  int device = 0;
  hipStream_t stream = nullptr;   // matching stream
  scm_matching_options opts;
  DevBuf lut;
  ImageTable table, scratch_table;
  bool table_loaded = false;
  // execute() image cache: the images of the previous call stay in HBM
  // (call_tab[call_cur], image key -> table index in call_map); the next
  // call's table reuses them by device-to-device copy and uploads only new
  // images.  Keyed by content (ImageKey), never by id alone.
  ImageTable call_tab[2];
  std::unordered_map<ImageKey, int32_t, ImageKeyHash> call_map[2];
  int call_cur = -1;
  int64_t call_reused = 0, call_uploaded = 0;  // images, cumulative (scm_stencil_stats)
  BatchSet sets[3];
  HostBuf h_stage;  // table upload staging
  int threads = 1;
  int64_t batch_pairs = kDefaultPairsPerBatch;  // SCM_BATCH_PAIRS overrides
  int64_t batch_bytes = 0;  // HBM budget of one batch set (SCM_BATCH_BYTES; 0 = from free HBM)
  bool match_bf16 = false;  // SCM_MATCH_BF16=1: bf16 MFMA matcher instead of i8
  bool serial = false;  // SCM_SERIAL=1: no overlap of the stages (diagnostics)
  bool score_split = true;  // H split scoring (rs_score_kernel<1> + exact recount), always
  double t_match = 0, t_final = 0, t_verify = 0, t_wall = 0;
  double t_run = 0, t_out = 0;     // last execute_batch: run_rows (GPU + its host steps), outputs
  double t_hash = 0, t_stage = 0;  // host time of the last execute_batch: content keys, table
  double t_score = 0;                  // scoring kernels (F + H) of the last run
  int64_t evals_f = 0, evals_h = 0;    // their (model, point) evaluations
  // small batches' speculative watermark decisions (VerifyOut::spec_check):
  // taken, recomputed and equal / different (SCM_DIAG_SPEC_CHECK), void
  int64_t spec_taken = 0, spec_equal = 0, spec_differ = 0, spec_void = 0;
  int64_t n_match_launches = 0;  // matcher kernel launches of the last table run
  // diagnostic phase profile of the verify kernel (SCM_PROFILE=1)
  bool profile = false;
  std::vector<uint64_t> prof_sum;
  std::vector<uint64_t> prof_worst;  // the pair with the most final-kernel cycles (slots 0-8)
  int64_t prof_pairs = 0;
  // raw matches of the last table run (scm_set_keep_matches)
  bool keep_matches = false;
  std::vector<std::pair<int64_t, int64_t>> keep_ranges;  // rows whose matches are kept
  bool kept(int64_t row) const {
    for (const auto& r : keep_ranges)
      if (row >= r.first && row < r.second) return true;
    return false;
  }
  int64_t last_begin = 0, last_end = 0;
  std::vector<std::vector<std::pair<int64_t, std::vector<Match>>>> last_matches;
  SiftState* sift = nullptr;  // SIFT extraction slots (scm_extract_frames), created on first use
  // Host workers: `pool` for a call's own host work (content keys of new
  // buffers, upload staging), `vpool` for the speculative key checks that run
  // while the GPU works (execute_rows).
  WorkerPool pool, vpool;
  // Content keys of the previous execute() call's element buffers.
  std::unordered_map<Src, SpecKey, SrcHash> spec_keys;
  int64_t spec_elems = 0, spec_rejected = 0, spec_retries = 0;  // scm_stencil_spec_stats
};

namespace {

// acosf LUT over [0, 2^18] built with the host libm: the exact float the
// reference computes as std::acos(std::min(kDistNorm * d, 1.0f)) in
// FindBestMatchesOneWay [upstream], SURVEY.md §8a "Ratio and distance tests".
void build_lut(std::vector<float>* lut) {
  lut->resize(kLutMax + 1);
  const float kDistNorm = 1.0f / (512.0f * 512.0f);
  for (uint32_t d = 0; d <= kLutMax; ++d)
    (*lut)[d] = std::acos(std::min(kDistNorm * (float)(int32_t)d, 1.0f));
}

double event_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0.0;
  return (double)ms;
}

template <typename F>
void parallel_for(int threads, int64_t n, F f) {
  if (threads <= 1 || n < 64) {
    for (int64_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::vector<std::thread> ts;
  const int T = (int)std::min<int64_t>(threads, n);
  const int64_t chunk = (n + T - 1) / T;
  for (int t = 0; t < T; ++t)
    ts.emplace_back([&, t] {
      const int64_t e = std::min(n, (t + 1) * chunk);
      for (int64_t i = t * chunk; i < e; ++i) f(i);
    });
  for (auto& th : ts) th.join();
}

int upload_table(scm_context* ctx, ImageTable* t, const std::vector<RowView>& rows,
                 bool with_desc, bool with_kp) {
  t->n = (int64_t)rows.size();
  t->ids.resize(t->n);
  t->nkp.resize(t->n);
  t->ndesc.resize(t->n);
  t->desc_row.resize(t->n);
  t->kp_off.resize(t->n);
  t->max_norm2.assign(t->n, 0);
  int64_t total_rows = 0, total_kp = 0;
  for (int64_t i = 0; i < t->n; ++i) {
    const RowView& r = rows[i];
    if (r.ndesc > INT32_MAX || r.nkp > INT32_MAX) {
      set_error("image has too many features");
      return SCM_E_INVALID;
    }
    t->ids[i] = r.id;
    t->nkp[i] = (int32_t)r.nkp;
    t->ndesc[i] = with_desc ? (int32_t)r.ndesc : 0;
    t->desc_row[i] = total_rows;
    t->kp_off[i] = total_kp;
    if (with_desc) total_rows += (r.ndesc + kDescRowAlign - 1) / kDescRowAlign * kDescRowAlign;
    if (with_kp) total_kp += r.nkp;
  }
  t->total_rows = total_rows;
  t->total_kp = total_kp;
  if (with_desc && total_rows > 0) {
    const size_t bytes = (size_t)total_rows * 128;
    SCM_TRY(ctx->h_stage.ensure(bytes));
    uint8_t* h = ctx->h_stage.as<uint8_t>();
    parallel_for(ctx->threads, t->n, [&](int64_t i) {
      const RowView& r = rows[i];
      uint8_t* dst = h + (size_t)t->desc_row[i] * 128;
      const size_t nb = (size_t)r.ndesc * 128;
      std::memcpy(dst, r.desc, nb);
      const size_t padded = (size_t)((r.ndesc + kDescRowAlign - 1) / kDescRowAlign * kDescRowAlign) * 128;
      std::memset(dst + nb, 0, padded - nb);
      uint64_t mx = 0;
      for (int64_t k = 0; k < r.ndesc; ++k) {
        const uint8_t* d = r.desc + k * 128;
        uint32_t s = 0;
        for (int j = 0; j < 128; ++j) s += (uint32_t)d[j] * d[j];
        mx = std::max<uint64_t>(mx, s);
      }
      t->max_norm2[i] = mx;
    });
    SCM_TRY(t->u8.ensure(bytes));
    SCM_HIP(hipMemcpyAsync(t->u8.ptr, h, bytes, hipMemcpyHostToDevice, ctx->stream));
    if (ctx->match_bf16) {
      SCM_TRY(t->desc.ensure(bytes * 2));
      SCM_HIP(launch_u8_to_bf16(t->u8.as<uint8_t>(), t->desc.as<uint16_t>(), (int64_t)bytes,
                                ctx->stream));
    } else {
      SCM_TRY(t->desc8.ensure(bytes));
      SCM_TRY(t->csum.ensure((size_t)total_rows * sizeof(int32_t)));
      SCM_HIP(launch_u8_to_i8(t->u8.as<uint8_t>(), t->desc8.as<uint8_t>(), t->csum.as<int32_t>(),
                              total_rows, ctx->stream));
    }
    SCM_HIP(hipStreamSynchronize(ctx->stream));
  }
  if (with_kp && total_kp > 0) {
    const size_t bytes = (size_t)total_kp * sizeof(float2);
    SCM_TRY(ctx->h_stage.ensure(bytes));
    float2* h = ctx->h_stage.as<float2>();
    for (int64_t i = 0; i < t->n; ++i) {
      const RowView& r = rows[i];
      for (int64_t k = 0; k < r.nkp; ++k)
        h[t->kp_off[i] + k] = make_float2(r.kp[6 * k], r.kp[6 * k + 1]);
    }
    SCM_TRY(t->kpxy.ensure(bytes));
    SCM_HIP(hipMemcpyAsync(t->kpxy.ptr, h, bytes, hipMemcpyHostToDevice, ctx->stream));
    SCM_HIP(hipStreamSynchronize(ctx->stream));
  }
  return SCM_OK;
}

// Content keys (ImageKey) of a set of elements, hashed chunk-parallel on a
// WorkerPool: plan(), task(t) for t in [0, ntasks()) (any order, any
// thread), then key(i) of elems[i].
struct KeyJob {
  static constexpr uint64_t kSeedKp = 0x6B70ULL, kSeedDesc = 0x64657363ULL;
  const std::vector<RowView>* rows = nullptr;
  std::vector<int64_t> elems;  // row indices
  std::vector<int64_t> off;    // first chunk of (element i, part: 0 keypoints / 1 descriptors)
  std::vector<uint64_t> ch;    // chunk hashes
  int64_t ntasks() const { return off.empty() ? 0 : off.back(); }
  void plan(const std::vector<RowView>& r, std::vector<int64_t> e) {
    rows = &r;
    elems = std::move(e);
    off.assign(2 * elems.size() + 1, 0);
    for (size_t i = 0; i < elems.size(); ++i) {
      const RowView& v = r[elems[i]];
      off[2 * i + 1] = off[2 * i] + hash_chunks((size_t)v.nkp * 24);
      off[2 * i + 2] = off[2 * i + 1] + hash_chunks((size_t)v.ndesc * 128);
    }
    ch.assign((size_t)ntasks(), 0);
  }
  void task(int64_t t) {
    const int64_t sl = (int64_t)(std::upper_bound(off.begin(), off.end(), t) - off.begin()) - 1;
    const RowView& v = (*rows)[elems[sl / 2]];
    const int64_t k = t - off[sl];
    ch[t] = sl % 2 == 0
                ? hash_chunk(reinterpret_cast<const uint8_t*>(v.kp), (size_t)v.nkp * 24, k, kSeedKp)
                : hash_chunk(v.desc, (size_t)v.ndesc * 128, k, kSeedDesc);
  }
  ImageKey key(size_t i) const {
    const RowView& v = (*rows)[elems[i]];
    ImageKey k;
    k.id = v.id;
    k.nkp = v.nkp;
    k.ndesc = v.ndesc;
    k.hkp = hash_combine_chunks(ch.data() + off[2 * i], off[2 * i + 1] - off[2 * i],
                                (size_t)v.nkp * 24, kSeedKp);
    k.hdesc = hash_combine_chunks(ch.data() + off[2 * i + 1], off[2 * i + 2] - off[2 * i + 1],
                                  (size_t)v.ndesc * 128, kSeedDesc);
    return k;
  }
};

inline bool same_content(const ImageKey& a, const ImageKey& b) {
  return a.nkp == b.nkp && a.ndesc == b.ndesc && a.hkp == b.hkp && a.hdesc == b.hdesc;
}

// Table of one execute() call over the call's unique images `rows` (content
// keys `keys`): images already resident in the previous call's table (same
// ImageKey) are copied device-to-device, the rest are staged, uploaded and
// converted in one tail range.  Layout: reused images first (in their old
// order, so consecutive ones coalesce into single copies), then new ones.
// (*idx)[i] = table index of rows[i]; (*uploaded)[i] = rows[i] was staged
// from its host bytes (not copied from the previous table).
int upload_call_table(scm_context* ctx, const std::vector<RowView>& rows,
                      const std::vector<ImageKey>& keys, std::vector<int32_t>* idx,
                      std::vector<char>* uploaded) {
  const int nxt = ctx->call_cur < 0 ? 0 : 1 - ctx->call_cur;
  const ImageTable* old = ctx->call_cur < 0 ? nullptr : &ctx->call_tab[ctx->call_cur];
  const std::unordered_map<ImageKey, int32_t, ImageKeyHash>* omap =
      ctx->call_cur < 0 ? nullptr : &ctx->call_map[ctx->call_cur];
  ImageTable* t = &ctx->call_tab[nxt];
  std::unordered_map<ImageKey, int32_t, ImageKeyHash>& nmap = ctx->call_map[nxt];
  nmap.clear();
  const int64_t n = (int64_t)rows.size();
  std::vector<int32_t> from(n, -1);  // old table index, or -1 (upload)
  std::vector<int64_t> reuse, fresh;
  for (int64_t i = 0; i < n; ++i) {
    const RowView& r = rows[i];
    if (r.ndesc > INT32_MAX || r.nkp > INT32_MAX) {
      set_error("image has too many features");
      return SCM_E_INVALID;
    }
    if (omap) {
      auto it = omap->find(keys[i]);
      if (it != omap->end()) from[i] = it->second;
    }
    (from[i] >= 0 ? reuse : fresh).push_back(i);
  }
  uploaded->assign(n, 0);
  for (int64_t i : fresh) (*uploaded)[i] = 1;
  std::stable_sort(reuse.begin(), reuse.end(),
                   [&](int64_t a, int64_t b) { return from[a] < from[b]; });
  std::vector<int64_t> order = reuse;
  order.insert(order.end(), fresh.begin(), fresh.end());
  t->n = n;
  t->ids.resize(n);
  t->nkp.resize(n);
  t->ndesc.resize(n);
  t->desc_row.resize(n);
  t->kp_off.resize(n);
  t->max_norm2.assign(n, 0);
  idx->assign(n, 0);
  int64_t total_rows = 0, total_kp = 0, tail_row = 0, tail_kp = 0;
  for (int64_t k = 0; k < n; ++k) {
    const int64_t i = order[k];
    const RowView& r = rows[i];
    if (k == (int64_t)reuse.size()) {
      tail_row = total_rows;
      tail_kp = total_kp;
    }
    (*idx)[i] = (int32_t)k;
    nmap[keys[i]] = (int32_t)k;
    t->ids[k] = r.id;
    t->nkp[k] = (int32_t)r.nkp;
    t->ndesc[k] = (int32_t)r.ndesc;
    t->desc_row[k] = total_rows;
    t->kp_off[k] = total_kp;
    if (from[i] >= 0) t->max_norm2[k] = old->max_norm2[from[i]];
    total_rows += (r.ndesc + kDescRowAlign - 1) / kDescRowAlign * kDescRowAlign;
    total_kp += r.nkp;
  }
  if (fresh.empty()) {
    tail_row = total_rows;
    tail_kp = total_kp;
  }
  t->total_rows = total_rows;
  t->total_kp = total_kp;
  const bool bf = ctx->match_bf16;
  if (total_rows > 0) {
    if (bf) SCM_TRY(t->desc.ensure((size_t)total_rows * 256));
    else {
      SCM_TRY(t->desc8.ensure((size_t)total_rows * 128));
      SCM_TRY(t->csum.ensure((size_t)total_rows * sizeof(int32_t)));
    }
  }
  if (total_kp > 0) SCM_TRY(t->kpxy.ensure((size_t)total_kp * sizeof(float2)));
  hipStream_t st = ctx->stream;
  // Reused images: coalesced device-to-device copies.
  for (size_t k = 0; k < reuse.size();) {
    size_t e = k + 1;
    while (e < reuse.size() && from[reuse[e]] == from[reuse[e - 1]] + 1) ++e;
    const int32_t o0 = from[reuse[k]], o1 = from[reuse[e - 1]];
    const int64_t orow = old->desc_row[o0];
    const int64_t nrow = old->desc_row[o1] - orow +
                         (old->ndesc[o1] + kDescRowAlign - 1) / kDescRowAlign * kDescRowAlign;
    const int64_t drow = t->desc_row[(size_t)k];
    if (nrow > 0) {
      if (bf)
        SCM_HIP(hipMemcpyAsync(t->desc.as<uint8_t>() + drow * 256, old->desc.as<uint8_t>() + orow * 256,
                               (size_t)nrow * 256, hipMemcpyDeviceToDevice, st));
      else {
        SCM_HIP(hipMemcpyAsync(t->desc8.as<uint8_t>() + drow * 128,
                               old->desc8.as<uint8_t>() + orow * 128, (size_t)nrow * 128,
                               hipMemcpyDeviceToDevice, st));
        SCM_HIP(hipMemcpyAsync(t->csum.as<int32_t>() + drow, old->csum.as<int32_t>() + orow,
                               (size_t)nrow * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
      }
    }
    const int64_t okp = old->kp_off[o0], nkp = old->kp_off[o1] + old->nkp[o1] - okp;
    if (nkp > 0)
      SCM_HIP(hipMemcpyAsync(t->kpxy.as<float2>() + t->kp_off[(size_t)k], old->kpxy.as<float2>() + okp,
                             (size_t)nkp * sizeof(float2), hipMemcpyDeviceToDevice, st));
    k = e;
  }
  // New images: one staged upload of the tail range (descriptors, then
  // keypoint xy), converted on the GPU like scm_table_load.
  const int64_t frows = total_rows - tail_row, fkp = total_kp - tail_kp;
  if (frows > 0 || fkp > 0) {
    const size_t dbytes = (size_t)frows * 128, kbytes = (size_t)fkp * sizeof(float2);
    const size_t koff = (dbytes + 255) / 256 * 256;
    SCM_TRY(ctx->h_stage.ensure(koff + kbytes));
    uint8_t* h = ctx->h_stage.as<uint8_t>();
    float2* hk = reinterpret_cast<float2*>(h + koff);
    const size_t nfresh = fresh.size(), k0 = reuse.size();
    // Tasks of kStageRows descriptor rows (a new image of 8192 features is
    // 8 tasks): copy into the staging buffer and the row norms' maximum; an
    // image's last task also pads its rows and converts its keypoints.
    constexpr int64_t kStageRows = 1024;
    std::vector<int64_t> tfirst(nfresh + 1, 0);
    for (size_t f = 0; f < nfresh; ++f) {
      const RowView& r = rows[order[k0 + f]];
      tfirst[f + 1] = tfirst[f] + std::max<int64_t>(1, (r.ndesc + kStageRows - 1) / kStageRows);
    }
    std::vector<uint64_t> tmax((size_t)tfirst[nfresh], 0);
    ctx->pool.run(tfirst[nfresh], [&](int64_t task) {
      const size_t f = (size_t)(std::upper_bound(tfirst.begin(), tfirst.end(), task) - tfirst.begin()) - 1;
      const int64_t k = (int64_t)(k0 + f);
      const RowView& r = rows[order[k]];
      uint8_t* dst = h + (size_t)(t->desc_row[k] - tail_row) * 128;
      const int64_t q0 = (task - tfirst[f]) * kStageRows, q1 = std::min(r.ndesc, q0 + kStageRows);
      if (q1 > q0) std::memcpy(dst + q0 * 128, r.desc + q0 * 128, (size_t)(q1 - q0) * 128);
      uint64_t mx = 0;
      for (int64_t q = q0; q < q1; ++q) {
        const uint8_t* d = r.desc + q * 128;
        uint32_t sq = 0;
        for (int j = 0; j < 128; ++j) sq += (uint32_t)d[j] * d[j];
        mx = std::max<uint64_t>(mx, sq);
      }
      tmax[task] = mx;
      if (task + 1 == tfirst[f + 1]) {
        const size_t nb = (size_t)r.ndesc * 128;
        const size_t padded =
            (size_t)((r.ndesc + kDescRowAlign - 1) / kDescRowAlign * kDescRowAlign) * 128;
        std::memset(dst + nb, 0, padded - nb);
        float2* kd = hk + (t->kp_off[k] - tail_kp);
        for (int64_t q = 0; q < r.nkp; ++q) kd[q] = make_float2(r.kp[6 * q], r.kp[6 * q + 1]);
      }
    });
    for (size_t f = 0; f < nfresh; ++f) {
      uint64_t mx = 0;
      for (int64_t q = tfirst[f]; q < tfirst[f + 1]; ++q) mx = std::max(mx, tmax[q]);
      t->max_norm2[k0 + f] = mx;
    }
    SCM_TRY(t->u8.ensure(koff + kbytes));
    SCM_HIP(hipMemcpyAsync(t->u8.ptr, h, koff + kbytes, hipMemcpyHostToDevice, st));
    if (frows > 0) {
      if (bf)
        SCM_HIP(launch_u8_to_bf16(t->u8.as<uint8_t>(), t->desc.as<uint16_t>() + tail_row * 128,
                                  (int64_t)dbytes, st));
      else
        SCM_HIP(launch_u8_to_i8(t->u8.as<uint8_t>(), t->desc8.as<uint8_t>() + tail_row * 128,
                                t->csum.as<int32_t>() + tail_row, frows, st));
    }
    if (fkp > 0)
      SCM_HIP(hipMemcpyAsync(t->kpxy.as<float2>() + tail_kp, t->u8.as<uint8_t>() + koff, kbytes,
                             hipMemcpyDeviceToDevice, st));
  }
  ctx->call_reused += (int64_t)reuse.size();
  ctx->call_uploaded += (int64_t)fresh.size();
  ctx->call_cur = nxt;  // the matching stream orders these copies before the call's kernels
  return SCM_OK;
}

// static_cast<size_t>(v) as gcc emits it on x86-64 (cvttsd2si, with the
// 2^63 offset branch for large values): -inf / negative -> 2^63, >= 2^64 and
// +inf -> 0, NaN -> 2^63.
uint64_t size_t_cast_x86(double v) {
  if (!(v < 9223372036854775808.0)) {
    if (!(v < 18446744073709551616.0)) return v == v ? 0 : 1ull << 63;
    return (uint64_t)(int64_t)(v - 9223372036854775808.0) ^ (1ull << 63);
  }
  if (!(v > -9223372036854775808.0)) return 1ull << 63;
  return (uint64_t)(int64_t)v;
}

// RANSAC::ComputeNumTrials [upstream optim/ransac.h] with the host libm, as
// the RANSAC constructor evaluates it for its max_num_trials cap (host only:
// the per-trial dynamic bound on the device uses geom::num_trials).
uint64_t num_trials_libm(uint64_t num_inliers, uint64_t num_samples, double confidence,
                         double multiplier, int kmin) {
  const double inlier_ratio = (double)num_inliers / (double)num_samples;
  const double nom = 1.0 - confidence;
  if (nom <= 0.0) return ~0ull;  // std::numeric_limits<size_t>::max()
  const double denom = 1.0 - std::pow(inlier_ratio, kmin);
  if (denom <= 0.0) return 1;
  return size_t_cast_x86(std::ceil(std::log(nom) / std::log(denom) * multiplier));
}

// `iteration` > 0: the k-th Estimate of TwoViewGeometry::EstimateMultiple
// (multiple_models), whose PRNG streams start from geom::iteration_seed.
VerifyParams make_params(const scm_matching_options& o, int iteration = 0) {
  VerifyParams p;
  std::memset(&p, 0, sizeof(p));
  const double max_error = (double)o.max_error;
  p.max_residual = max_error * max_error;
  p.confidence = o.confidence;
  p.dyn_num_trials_multiplier = o.dyn_num_trials_multiplier;
  p.max_H_inlier_ratio = o.max_H_inlier_ratio;
  p.watermark_min_inlier_ratio = o.watermark_min_inlier_ratio;
  p.watermark_border_size = o.watermark_border_size;
  p.min_num_trials = o.min_num_trials;
  p.min_num_inliers = o.min_num_inliers;
  p.detect_watermark = o.detect_watermark;
  p.base_seed = geom::iteration_seed(o.ransac_seed, (uint32_t)iteration);
  // RANSAC constructor: max_num_trials capped by ComputeNumTrials at the
  // assumed min_inlier_ratio over 1e5 samples [upstream optim/ransac.h],
  // evaluated with the host libm as the constructor does.
  auto cap = [&](double ratio, int kmin) {
    const uint64_t kNumSamples = 100000;
    const uint64_t dyn = num_trials_libm(size_t_cast_x86(ratio * (double)kNumSamples), kNumSamples,
                                         o.confidence, o.dyn_num_trials_multiplier, kmin);
    const uint64_t m = std::min<uint64_t>((uint64_t)std::max(0, o.max_num_trials), dyn);
    return (int32_t)std::min<uint64_t>(m, 0x7FFFFFFF);
  };
  p.max_trials_F = cap(o.min_inlier_ratio, 7);
  p.max_trials_H = cap(o.min_inlier_ratio, 4);
  p.max_trials_T = cap(o.watermark_min_inlier_ratio, 1);
  return p;
}

size_t align256(size_t x) { return (x + 255) / 256 * 256; }
size_t align16(size_t x) { return (x + 15) / 16 * 16; }

// Stream priorities: the verification streams (the longer stage, whose
// windows are short dependent kernels) run at high priority so that their
// launches are not queued behind the matcher's large grids (+1 % measured);
// the matching stream at the default (matcher-high measured equal on the
// table path and slower on the drop-in path, profiles/r02_o_*).
int stream_priority(bool high) {
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  return high ? hi : 0;
}

// XCD-aware job order.  Workgroups are dispatched round-robin over the 8
// XCDs (workgroup b -> XCD b mod 8), each XCD with its own L2.  The jobs of
// one pivot run (its row blocks, which all sweep the same neighbour
// descriptors; with the column split, of one column part) are kept on one XCD so that the neighbour tiles are fetched
// into that XCD's L2 once instead of once per XCD; the runs are spread over
// the XCDs by work (least-loaded first) and the queues interleaved, padding
// with empty jobs.
void xcd_order(std::vector<MatchJob>& jobs, const std::vector<PairDesc>& pds) {
  if (jobs.size() <= (size_t)kXcds) return;
  std::vector<std::vector<MatchJob>> q(kXcds);
  std::vector<double> load(kXcds, 0.0);
  for (size_t i = 0; i < jobs.size();) {
    size_t j = i;
    while (j < jobs.size() && jobs[j].a_row == jobs[i].a_row && jobs[j].pair0 == jobs[i].pair0 &&
           jobs[j].t0 == jobs[i].t0)
      ++j;
    double cols = 0.0;
    for (int32_t k = 0; k < jobs[i].npairs; ++k) cols += pds[jobs[i].pair0 + k].n2;
    if (jobs[i].t1 > 0)  // a column part
      cols = std::min<double>(cols, (double)(jobs[i].t1 - jobs[i].t0) * kTile8Cols);
    const int x = (int)(std::min_element(load.begin(), load.end()) - load.begin());
    load[x] += cols * (double)(j - i);
    q[x].insert(q[x].end(), jobs.begin() + i, jobs.begin() + j);
    i = j;
  }
  size_t len = 0;
  for (const auto& v : q) len = std::max(len, v.size());
  MatchJob empty;
  std::memset(&empty, 0, sizeof(empty));
  jobs.assign(len * kXcds, empty);
  for (int x = 0; x < kXcds; ++x)
    for (size_t k = 0; k < q[x].size(); ++k) jobs[k * kXcds + x] = q[x][k];
}

// Stage 1 of a batch, on the matching stream: upload the pair descriptors,
// run the tile + finalize kernels (or upload the given matches of the single
// pair specs[0]), and copy the match counts into the mapped result buffer.
// Buffers are laid out for the worst case (one match slot per pivot
// keypoint) so nothing waits for the counts.
int enqueue_match(scm_context* ctx, BatchSet& bs, const ImageTable& t,
                  const std::vector<PairSpec>& specs, const uint32_t* given,
                  const int32_t* given_counts) {
  const int64_t P = (int64_t)specs.size();
  bs.P = P;
  bs.verify = false;
  bs.matched = given == nullptr;
  bs.pending = false;
  bs.table = &t;
  bs.specs = specs;
  // Events 3 and 6 are waited for by the host before it reads pinned memory
  // (system-scope release); the others only time stages or order the
  // device's own streams (a device-scope release: no system-scope cache
  // writeback at each record, tens of microseconds on the small-batch path).
  for (int i = 0; i < 7; ++i)
    if (!bs.ev[i])
      SCM_HIP(hipEventCreateWithFlags(&bs.ev[i], i == 3 || i == 6 ? hipEventDefault
                                                                  : hipEventReleaseToDevice));
  if (P == 0) return SCM_OK;
  std::vector<PairDesc> pds(P);
  std::vector<MatchJob> jobs, jobs_clamp;
  struct Run {
    int32_t a, pair0, npairs;
    bool clamp;
  };
  std::vector<Run> runs;
  bs.moff.resize(P);
  int64_t rr = 0, cp = 0, m21 = 0, mo = 0, ax = 0, rlo = 0;
  const int32_t rpb = ctx->match_bf16 ? kRowsPerBlock : kRowsPerBlock8;  // pivot rows per job
  const int64_t want_jobs = 4 * kNumCUs;  // jobs of a batch that fills the GPU (below)
  // Column split (i8 matcher, small batches): with one pair per job a single
  // stencil (K - 1 pairs x 16 row blocks: 304 jobs) still leaves the last of
  // two rounds of jobs on 48 of the 256 CUs; cutting each pair's columns into
  // csplit parts (row segments of their own, merged by the finalize like the
  // 8192-column segments) gives ~4 rounds of shorter jobs.
  int32_t csplit = 1;
  if (!given && !ctx->match_bf16 && P <= verify_small_batch_pairs()) {
    int64_t pair_jobs = 0;
    for (int64_t k = 0; k < P; ++k)
      if (t.ndesc[specs[k].a] > 0 && t.ndesc[specs[k].b] > 0)
        pair_jobs += (t.ndesc[specs[k].a] + rpb - 1) / rpb;
    while (pair_jobs > 0 && csplit < kMaxColSplit && pair_jobs * csplit < want_jobs) csplit *= 2;
  }
  for (int64_t i = 0; i < P;) {
    const int32_t a = specs[i].a;
    int64_t j = i;
    while (j < P && specs[j].a == a) ++j;
    bool clamp = false;
    for (int64_t k = i; k < j; ++k) {
      // match slots of the pair: every pivot row, or the given list
      const int32_t slots = given ? std::max<int32_t>(given_counts[k], 1) : t.ndesc[a];
      const int32_t b = specs[k].b;
      PairDesc& pd = pds[k];
      std::memset(&pd, 0, sizeof(pd));
      pd.n1 = given ? 0 : t.ndesc[a];
      pd.n2 = given ? 0 : t.ndesc[b];
      pd.n2pad = (pd.n2 + kTile8Cols - 1) / kTile8Cols * kTile8Cols;  // whole 64-column tiles
      pd.nseg = (pd.n2 + kColsPerSeg - 1) / kColsPerSeg;
      pd.seg8_log2 = kSeg8Log2;
      if (csplit > 1) {
        // segments of 2^seg8_log2 tiles, at least ceil(tiles / csplit) each
        const int32_t nt = pd.n2pad / kTile8Cols, per = (nt + csplit - 1) / csplit;
        int32_t lg = 0;
        while (lg < kSeg8Log2 && (1 << lg) < per) ++lg;
        pd.seg8_log2 = lg;
        pd.nseg = (nt + (1 << lg) - 1) >> lg;
      }
      pd.nrb = (pd.n1 + rpb - 1) / rpb;
      pd.b_row = given ? 0 : t.desc_row[b];
      pd.a_row = given ? 0 : t.desc_row[a];
      pd.rowres_off = rr;
      pd.colpart_off = cp;
      pd.m21_off = m21;
      pd.match_off = mo;
      pd.aux_off = ax;
      pd.rlist_off = rlo;
      ax += pd.n1;
      rlo += 33 + (int64_t)pd.n1;
      bs.moff[k] = mo;
      rr += (int64_t)pd.nseg * pd.n1;
      cp += (int64_t)pd.nrb * pd.n2pad;
      m21 += pd.n2;
      mo += slots;
      if (!given) {
        // |a||b| < 2^19 for every row pair  <=>  max|a|^2 * max|b|^2 < 2^38.
        const unsigned __int128 prod = (unsigned __int128)t.max_norm2[a] * t.max_norm2[b];
        if (prod >= ((unsigned __int128)1 << 38)) clamp = true;
      }
    }
    for (int64_t k = i; k < j; ++k) pds[k].clamp = clamp ? 1 : 0;
    if (!given && t.ndesc[a] > 0) {
      // Runs of consecutive active pairs of this pivot (jobs are cut below).
      for (int64_t k = i; k < j;) {
        while (k < j && pds[k].n2 == 0) ++k;
        int64_t e = k;
        while (e < j && pds[e].n2 > 0) ++e;
        if (e > k) runs.push_back({a, (int32_t)k, (int32_t)(e - k), clamp});
        k = e;
      }
    }
    i = j;
  }
  // One job = one 512-row block of a pivot swept over a run of its pairs.  A
  // small batch (a single execute() stencil: K-1 pairs of one pivot = 16 row
  // blocks) would leave most of the 256 CUs idle, so runs are cut into
  // shorter runs until the batch has ~4 jobs per CU (a job over fewer pairs
  // re-reads nothing: every pair's columns are swept once per row block).
  {
    int64_t base_jobs = 0;
    for (const Run& r : runs) base_jobs += (t.ndesc[r.a] + rpb - 1) / rpb;
    for (const Run& r : runs) {
      const int32_t n1 = t.ndesc[r.a];
      const int32_t nrb = (n1 + rpb - 1) / rpb;
      auto add = [&](int32_t p0, int32_t np, int32_t t0, int32_t t1) {
        for (int32_t rb = 0; rb < nrb; ++rb) {
          MatchJob jb;
          jb.a_row = t.desc_row[r.a];
          jb.rb = rb;
          jb.n1 = n1;
          jb.pair0 = p0;
          jb.npairs = np;
          jb.t0 = t0;
          jb.t1 = t1;
          (r.clamp ? jobs_clamp : jobs).push_back(jb);
        }
      };
      if (csplit > 1) {  // one job per pair, row block and row segment
        for (int32_t k = r.pair0; k < r.pair0 + r.npairs; ++k) {
          const PairDesc& pd = pds[k];
          const int32_t nt = pd.n2pad / kTile8Cols;
          for (int32_t sg = 0; sg < pd.nseg; ++sg)
            add(k, 1, sg << pd.seg8_log2, std::min(nt, (sg + 1) << pd.seg8_log2));
        }
        continue;
      }
      int32_t parts = 1;
      if (base_jobs > 0 && base_jobs < want_jobs)
        parts = (int32_t)std::min<int64_t>(r.npairs, (want_jobs + base_jobs - 1) / base_jobs);
      for (int32_t q = 0; q < parts; ++q) {
        const int32_t p0 = r.pair0 + (int32_t)((int64_t)r.npairs * q / parts);
        const int32_t p1 = r.pair0 + (int32_t)((int64_t)r.npairs * (q + 1) / parts);
        if (p1 > p0) add(p0, p1 - p0, 0, 0);
      }
    }
  }
  bs.slots = mo;
  xcd_order(jobs, pds);
  xcd_order(jobs_clamp, pds);
  const int64_t nfast = (int64_t)jobs.size();
  jobs.insert(jobs.end(), jobs_clamp.begin(), jobs_clamp.end());
  const int64_t NJ = (int64_t)jobs.size();
  // ---- buffers.
  SCM_TRY(bs.rowres.ensure(std::max<int64_t>(rr, 1) * sizeof(uint2)));
  SCM_TRY(bs.colpart.ensure(std::max<int64_t>(cp, 1) * sizeof(uint2)));
  SCM_TRY(bs.m21.ensure(std::max<int64_t>(m21, 1) * sizeof(int32_t)));
  SCM_TRY(bs.rowaux.ensure(std::max<int64_t>(ax, 1) * sizeof(uint2)));
  SCM_TRY(bs.rlist.ensure(std::max<int64_t>(rlo, 1) * sizeof(int32_t)));
  SCM_TRY(bs.matches.ensure(std::max<int64_t>(mo, 1) * sizeof(uint2)));
  SCM_TRY(bs.masks.ensure(std::max<int64_t>(mo, 1)));
  SCM_TRY(bs.counts.ensure(P * sizeof(int32_t)));
  SCM_TRY(bs.offsets.ensure(align16((P + 1) * sizeof(int64_t))));
  bs.off_counts = 0;
  bs.off_offsets = align256(bs.off_counts + P * sizeof(int32_t));
  bs.off_vout = align256(bs.off_offsets + (P + 1) * sizeof(int64_t));
  bs.off_matches = align256(bs.off_vout + P * sizeof(VerifyOut));
  bs.off_masks = align256(bs.off_matches + mo * sizeof(uint2));
  SCM_TRY(bs.out.ensure(bs.off_masks + mo + 256));
  // ---- descriptor upload from pinned staging.
  const size_t s_pairs = align256(NJ * sizeof(MatchJob));
  const size_t s_mo = align256(s_pairs + P * sizeof(PairDesc));
  const size_t s_cnt = align256(s_mo + P * sizeof(int64_t));
  int64_t given_m = 0;  // given matches of all pairs (each list at its pair's slots)
  if (given)
    for (int64_t k = 0; k < P; ++k) given_m += given_counts[k];
  const size_t s_given = align256(s_cnt + P * sizeof(int32_t));
  const size_t s_end = s_given + (given ? (size_t)mo * sizeof(uint2) : 0);
  SCM_TRY(bs.stage.ensure(s_end));
  uint8_t* st = bs.stage.as<uint8_t>();
  if (NJ) std::memcpy(st, jobs.data(), NJ * sizeof(MatchJob));
  std::memcpy(st + s_pairs, pds.data(), P * sizeof(PairDesc));
  std::memcpy(st + s_mo, bs.moff.data(), P * sizeof(int64_t));
  // 64-row groups of the largest pivot (grid of match_recheck_g8_kernel)
  // and the widest neighbour (grid of match_colmerge_g8_kernel)
  int max_groups = 0, max_cols = 0;
  for (int64_t k = 0; k < P; ++k) {
    max_groups = std::max(max_groups, (pds[k].n1 + 63) / 64);
    max_cols = std::max(max_cols, pds[k].n2);
  }
  hipStream_t sm = ctx->stream;
  // jobs, pair descriptors and match offsets in one upload (one launch on the
  // small-batch critical path instead of three), by kernel on the matching
  // stream: as a copy-engine transfer it queued behind the previous batch's
  // result copies (another stream's, waiting for that batch's verification
  // chain), and the bench's last matcher started ~110 ms after its launch
  // (profiles/r06_ah)
  SCM_TRY(bs.mdesc.ensure(s_cnt));
  bs.d_jobs = reinterpret_cast<MatchJob*>(bs.mdesc.as<uint8_t>());
  bs.d_pairs = reinterpret_cast<PairDesc*>(bs.mdesc.as<uint8_t>() + s_pairs);
  bs.d_moff = reinterpret_cast<int64_t*>(bs.mdesc.as<uint8_t>() + s_mo);
  SCM_HIP(launch_stage_upload(bs.stage.dptr, bs.mdesc.ptr, align16(s_mo + P * sizeof(int64_t)), sm));
  if (given) {
    std::memcpy(st + s_cnt, given_counts, P * sizeof(int32_t));
    SCM_HIP(hipMemcpyAsync(bs.counts.ptr, st + s_cnt, P * sizeof(int32_t), hipMemcpyHostToDevice,
                           sm));
    if (given_m > 0) {
      uint2* gd = reinterpret_cast<uint2*>(st + s_given);
      int64_t src = 0;
      for (int64_t k = 0; k < P; ++k) {
        std::memcpy(gd + bs.moff[k], given + 2 * src, (size_t)given_counts[k] * sizeof(uint2));
        src += given_counts[k];
      }
      SCM_HIP(hipMemcpyAsync(bs.matches.ptr, st + s_given, (size_t)mo * sizeof(uint2),
                             hipMemcpyHostToDevice, sm));
    }
  }
  SCM_HIP(hipEventRecord(bs.ev[0], sm));
  if (!given)
    for (int clamp = 0; clamp < 2; ++clamp) {
      const MatchJob* jb = bs.d_jobs + (clamp ? nfast : 0);
      const int nj = (int)(clamp ? NJ - nfast : nfast);
      if (nj > 0) ctx->n_match_launches += 1;
      if (ctx->match_bf16)
        SCM_HIP(launch_match_tiles(t.desc.as<uint16_t>(), jb, nj, bs.d_pairs,
                                   bs.rowres.as<uint2>(), bs.colpart.as<uint2>(), clamp, sm));
      else
        SCM_HIP(launch_match_g8(t.desc8.as<uint8_t>(), t.csum.as<int32_t>(), jb, nj,
                                bs.d_pairs, bs.rowres.as<uint2>(),
                                bs.colpart.as<uint2>(), clamp, sm));
    }
  SCM_HIP(hipEventRecord(bs.ev[1], sm));
  // Finalize, the count read-back and (enqueue_verify) the verification run on
  // the set's own stream, so the matcher of the next batch follows this one on
  // the matching stream at once (the sets' buffers are disjoint; the set's
  // stream is idle: its previous batch was collected before this one began).
  hipStream_t sf = bs.vstream;
  SCM_HIP(hipStreamWaitEvent(sf, bs.ev[1], 0));
  if (!given && !ctx->match_bf16)
    SCM_HIP(launch_match_finalize_g8(bs.d_pairs, (int)P, bs.rowres.as<uint2>(),
                                     bs.colpart.as<uint2>(), bs.rowaux.as<uint2>(),
                                     bs.rlist.as<int32_t>(), t.desc8.as<uint8_t>(),
                                     t.csum.as<int32_t>(), ctx->lut.as<float>(),
                                     (float)ctx->opts.max_ratio, (float)ctx->opts.max_distance,
                                     ctx->opts.cross_check, bs.matches.as<uint2>(),
                                     bs.counts.as<int32_t>(), max_groups, max_cols, sf));
  else if (!given)
    SCM_HIP(launch_match_finalize(bs.d_pairs, (int)P, bs.rowres.as<uint2>(),
                                  bs.colpart.as<uint2>(), bs.m21.as<int32_t>(),
                                  ctx->lut.as<float>(), (float)ctx->opts.max_ratio,
                                  (float)ctx->opts.max_distance, ctx->opts.cross_check,
                                  ctx->match_bf16 ? 0 : 1,
                                  bs.matches.as<uint2>(), bs.counts.as<int32_t>(), sf));
  SCM_HIP(hipEventRecord(bs.ev[2], sf));
  uint8_t* outh = reinterpret_cast<uint8_t*>(bs.out.host);
  SCM_HIP(hipMemcpyAsync(outh + bs.off_counts, bs.counts.ptr, P * sizeof(int32_t),
                         hipMemcpyDeviceToHost, sf));
  SCM_HIP(hipEventRecord(bs.ev[3], sf));
  // The verification's zeroed state (TwoViewGeometry() outputs, empty active
  // lists), enqueued now: off the host's round trip on the counts.
  SCM_TRY(bs.dvout.ensure(P * sizeof(VerifyOut)));
  SCM_HIP(hipMemsetAsync(bs.dvout.ptr, 0, P * sizeof(VerifyOut), sf));
  SCM_TRY(bs.nact.ensure(3 * sizeof(int32_t)));
  SCM_TRY(bs.h_nact.ensure(3 * sizeof(int32_t)));
  SCM_HIP(hipMemsetAsync(bs.nact.ptr, 0, 3 * sizeof(int32_t), sf));
  SCM_HIP(hipMemsetAsync(bs.h_nact.ptr, 0, 3 * sizeof(int32_t), sf));
  bs.pending = true;
  return SCM_OK;
}

// Stage 2 of a batch, on the verification stream: waits (host side) for the
// batch's match counts, then verifies exactly the pairs the reference
// verifies (>= min_num_inliers matches, sequential_matching.cc:164-178 /
// EstimateUncalibrated), longest first so the launch tail is short, with the
// LDS sample buffer sized to the largest match count; finally compacts the
// matches and F-inlier masks into the mapped result buffer.
int enqueue_verify(scm_context* ctx, BatchSet& bs, bool verify, int iteration = 0) {
  bs.verify = verify;
  if (!bs.pending || bs.P == 0) return SCM_OK;
  const int64_t P = bs.P;
  const ImageTable& t = *bs.table;
  SCM_HT(5);
  SCM_HIP(hipEventSynchronize(bs.ev[3]));
  SCM_HT(6);
  SCM_HTE_READ(bs.ev);
  uint8_t* outh = reinterpret_cast<uint8_t*>(bs.out.host);
  const int32_t* counts = reinterpret_cast<const int32_t*>(outh + bs.off_counts);
  hipStream_t sv = bs.vstream;
  SCM_HIP(hipStreamWaitEvent(sv, bs.ev[3], 0));
  std::vector<int64_t> order;
  if (verify) {
    for (int64_t k = 0; k < P; ++k)
      if (counts[k] >= std::max(1, ctx->opts.min_num_inliers)) order.push_back(k);
    std::stable_sort(order.begin(), order.end(),
                     [&](int64_t x, int64_t y) { return counts[x] > counts[y]; });
  }
  // Packed output offsets (exclusive scan of the counts) on the host.
  int64_t* offs = reinterpret_cast<int64_t*>(outh + bs.off_offsets);
  int64_t total = 0;
  for (int64_t k = 0; k < P; ++k) {
    offs[k] = total;
    total += counts[k];
  }
  offs[P] = total;
  // The offsets go to the device now (by kernel, as every table upload of the
  // pipeline: launch_stage_upload), ahead of the verification chain.
  SCM_HIP(launch_stage_upload(reinterpret_cast<uint8_t*>(bs.out.dev) + bs.off_offsets,
                              bs.offsets.ptr, align16((P + 1) * sizeof(int64_t)), sv));
  const int64_t V = (int64_t)order.size();
  SCM_HIP(hipEventRecord(bs.ev[4], sv));
  if (verify) SCM_TRY(bs.dvout.ensure(P * sizeof(VerifyOut)));  // zeroed by enqueue_match
  if (V > 0) {
    std::vector<GatherPair> gps(V);
    std::vector<VerifyPair> vps(V);
    int64_t scr = 0;
    for (int64_t q = 0; q < V; ++q) {
      const int64_t k = order[q];
      const int32_t m = counts[k];
      GatherPair& g = gps[q];
      std::memset(&g, 0, sizeof(g));
      g.match_off = bs.moff[k];
      g.kp1_off = t.kp_off[bs.specs[k].a];
      g.kp2_off = t.kp_off[bs.specs[k].b];
      g.pts_off = bs.moff[k];
      g.m = m;
      g.cidx = -1;
      VerifyPair& v = vps[q];
      std::memset(&v, 0, sizeof(v));
      v.pts_off = 2 * bs.moff[k];
      v.scr_off = scr;
      v.mask_off = bs.moff[k];
      v.m = m;
      v.cidx = -1;
      v.id1 = t.ids[bs.specs[k].a];
      v.id2 = t.ids[bs.specs[k].b];
      v.out_idx = (int32_t)k;
      scr += verify_scratch_doubles(m);
    }
    const int max_m = counts[order[0]];
    SCM_TRY(bs.xy1.ensure(2 * std::max<int64_t>(bs.slots, 1) * sizeof(double)));
    SCM_TRY(bs.xy2.ensure(2 * std::max<int64_t>(bs.slots, 1) * sizeof(double)));
    SCM_TRY(bs.xyf.ensure(std::max<int64_t>(bs.slots, 1) * sizeof(float4)));
    SCM_TRY(bs.scratch.ensure(std::max<int64_t>(scr, 1) * sizeof(double)));
    SCM_TRY(bs.snaps.ensure(V * kVerifySnapWords * sizeof(uint32_t)));
    const size_t s_v = align256(V * sizeof(GatherPair));
    SCM_TRY(bs.vstage.ensure(align16(s_v + V * sizeof(VerifyPair))));
    uint8_t* st = bs.vstage.as<uint8_t>();
    std::memcpy(st, gps.data(), V * sizeof(GatherPair));
    std::memcpy(st + s_v, vps.data(), V * sizeof(VerifyPair));
    // both tables in one copy
    SCM_TRY(bs.vdesc.ensure(align16(s_v + V * sizeof(VerifyPair))));
    bs.d_gpairs = reinterpret_cast<GatherPair*>(bs.vdesc.as<uint8_t>());
    bs.d_vpairs = reinterpret_cast<VerifyPair*>(bs.vdesc.as<uint8_t>() + s_v);
    SCM_HIP(launch_stage_upload(bs.vstage.dptr, bs.vdesc.ptr, align16(s_v + V * sizeof(VerifyPair)), sv));
    SCM_HIP(launch_gather(bs.d_gpairs, (int)V, max_m, bs.matches.as<uint2>(),
                          t.kpxy.as<float2>(), bs.xy1.as<double>(), bs.xy2.as<double>(), nullptr,
                          bs.xyf.as<float4>(), sv));
    uint64_t* prof = nullptr;
    if (ctx->profile) {
      SCM_TRY(bs.prof.ensure(V * kVerifyProfSlots * sizeof(uint64_t)));
      SCM_HIP(hipMemsetAsync(bs.prof.ptr, 0, V * kVerifyProfSlots * sizeof(uint64_t), sv));
      prof = bs.prof.as<uint64_t>();
    }
    bs.nprof = V;
    SCM_HIP(hipEventRecord(bs.ev[4], sv));
    // Round buffers per kind (H: one model per hypothesis): the window
    // buffers of one parity, then the per-pair state.  Small batches take
    // windows of up to kMaxWindowSmall rounds (VerifyRoundBufs::wt).
    const int64_t wt = verify_small_batch((int)V, max_m) ? kWindowTrialsSmall : kWindowTrials;
    auto window_bufs = [&](DevBuf& samp, DevBuf& nmod, DevBuf& fcon, DevBuf& mods, DevBuf& cnts,
                           DevBuf& ucnt, DevBuf& wsnap, DevBuf& wb, DevBuf& wstate, bool split,
                           VerifyRoundBufs* rb) -> int {
      SCM_TRY(samp.ensure(V * wt * 8 * sizeof(uint32_t)));
      SCM_TRY(nmod.ensure(V * wt * sizeof(int32_t)));
      SCM_TRY(fcon.ensure(V * wt * 3 * 12 * sizeof(float)));
      SCM_TRY(mods.ensure(V * wt * 3 * 9 * sizeof(double)));
      SCM_TRY(cnts.ensure(V * wt * 3 * sizeof(uint32_t)));
      if (split) SCM_TRY(ucnt.ensure(V * wt * 3 * sizeof(uint32_t)));
      SCM_TRY(wsnap.ensure(V * 640 * sizeof(uint32_t)));  // window start states
      SCM_TRY(wb.ensure(V * sizeof(int32_t)));
      SCM_TRY(wstate.ensure(V * kVerifyStateWords * sizeof(uint32_t)));
      rb->samp = samp.as<uint32_t>();
      rb->nmod = nmod.as<int32_t>();
      rb->fcon = fcon.as<float>();
      rb->mods = mods.as<double>();
      rb->cnts = cnts.as<uint32_t>();
      rb->ucnt = split ? ucnt.as<uint32_t>() : nullptr;
      rb->wsnap = wsnap.as<uint32_t>();
      rb->wB = wb.as<int32_t>();
      rb->wstate = rb->pstate = wstate.as<uint32_t>();
      rb->wt = (int)wt;
      return SCM_OK;
    };
    auto round_bufs = [&](DevBuf& rst, DevBuf& samp, DevBuf& nmod, DevBuf& fcon, DevBuf& mods,
                          DevBuf& cnts, DevBuf& ucnt, DevBuf& wsnap, DevBuf& act, DevBuf& nact,
                          DevBuf& wb, DevBuf& wstate, DevBuf& dtrial, bool split,
                          VerifyRoundBufs* rb) -> int {
      SCM_TRY(rst.ensure(V * sizeof(RansacState)));
      SCM_TRY(window_bufs(samp, nmod, fcon, mods, cnts, ucnt, wsnap, wb, wstate, split, rb));
      SCM_TRY(act.ensure(3 * V * sizeof(int32_t)));
      SCM_TRY(nact.ensure(3 * sizeof(int32_t)));
      SCM_TRY(dtrial.ensure(V * sizeof(int32_t)));
      rb->rst = rst.as<RansacState>();
      for (int k = 0; k < 3; ++k) rb->act[k] = act.as<int32_t>() + k * V;
      rb->nact = nact.as<int32_t>();
      rb->dtrial = dtrial.as<int32_t>();
      return SCM_OK;
    };
    VerifyRoundBufs rbf, rbh;
    // Split scoring for H only: F runs mostly in its first windows, where the
    // best is still low and nearly every model would need the exact pass
    // (measured per step: F 35.4 + 8.3 ms split vs 40.8 ms one pass; H 138.3 +
    // 4.2 ms vs 153.1 ms).
    SCM_TRY(round_bufs(bs.rst, bs.samp, bs.nmod, bs.fcon, bs.mods, bs.cnts, bs.ucnt, bs.wsnap,
                       bs.act, bs.nact, bs.wb, bs.wstate, bs.dtrial, false, &rbf));
    SCM_TRY(round_bufs(bs.h_rst, bs.h_samp, bs.h_nmod, bs.h_fcon, bs.h_mods, bs.h_cnts,
                       bs.h_ucnt, bs.h_wsnap, bs.h_act, bs.h_nact, bs.h_wb, bs.h_wstate,
                       bs.h_dtrial, ctx->score_split, &rbh));
    if (!bs.sev[0])
      for (auto& e : bs.sev) SCM_HIP(hipEventCreateWithFlags(&e, hipEventReleaseToDevice));
    // Small batches (one Scanner stencil): odd-parity window buffers and a
    // replay stream, so that the next window's draws and scores overlap the
    // replay of this one.
    VerifySpec spec;
    spec.lists_zeroed = true;  // enqueue_match
    VerifyRoundBufs rbf1 = rbf, rbh1 = rbh, rbf2 = rbf, rbh2 = rbh;
    if (verify_small_batch((int)V, max_m)) {
      SCM_TRY(window_bufs(bs.o_samp, bs.o_nmod, bs.o_fcon, bs.o_mods, bs.o_cnts, bs.o_ucnt,
                          bs.o_wsnap, bs.o_wb, bs.o_wstate, false, &rbf1));
      SCM_TRY(window_bufs(bs.oh_samp, bs.oh_nmod, bs.oh_fcon, bs.oh_mods, bs.oh_cnts, bs.oh_ucnt,
                          bs.oh_wsnap, bs.oh_wb, bs.oh_wstate, ctx->score_split, &rbh1));
      // Parallel LO slots per kind and parity (rs_lo_chain2_kernel), when they
      // fit 1 GiB each; otherwise the replay runs every LO chain itself.
      const int64_t lo_stride = lo_slot_doubles(max_m);
      const int64_t lo_bytes = V * kLoSlots * lo_stride * (int64_t)sizeof(double);
      // SCM_PARALLEL_LO=0 (checks, read per call): every LO chain inline
      // (tests/test_gpu_stencil.py compares both forms with the oracle)
      const char* plo = getenv("SCM_PARALLEL_LO");
      const bool parallel_lo = !(plo && plo[0] == '0');
      if (parallel_lo && lo_bytes <= (int64_t(1) << 30)) {
        VerifyRoundBufs* lrb[4] = {&rbf, &rbf1, &rbh, &rbh1};
        for (int i = 0; i < 4; ++i) {
          SCM_TRY(bs.lo_slot[i].ensure(V * kLoSlots * sizeof(LoSlot)));
          SCM_TRY(bs.lo_data[i].ensure(lo_bytes));
          lrb[i]->lo = bs.lo_slot[i].as<LoSlot>();
          lrb[i]->lo_data = bs.lo_data[i].as<double>();
          lrb[i]->lo_stride = lo_stride;
        }
      }
      // The replay stream and the early-final stream are the other two batch
      // sets' verification streams: a process has few hardware queues
      // (GPU_MAX_HW_QUEUES, 4 by default) and streams beyond them share one,
      // serialising their work; these three are created on distinct queues.
      // (A small batch's neighbours have nothing pending on the drop-in path;
      // on the table path -- batch caps of <= 1,024 pairs, or a run's last
      // batch -- they may: sharing a stream with a pending batch only adds
      // ordering, never a cycle, since a batch waits only on its own events
      // and on work enqueued before it; tests/test_gpu_fullsize.py
      // test_k50_shape_many_batches runs several in flight.)
      const int si = (int)(&bs - ctx->sets);
      bs.rstream = ctx->sets[(si + 1) % 3].vstream;
      bs.fstream = ctx->sets[(si + 2) % 3].vstream;
      if (!bs.wev[0]) {
        for (auto& e : bs.wev)
          SCM_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventReleaseToDevice));
        for (auto& e : bs.dev)
          SCM_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventReleaseToDevice));
      }

      if (!bs.fev)
        SCM_HIP(hipEventCreateWithFlags(&bs.fev, hipEventDisableTiming | hipEventReleaseToDevice));
      if (!bs.spev)
        SCM_HIP(hipEventCreateWithFlags(&bs.spev, hipEventDisableTiming | hipEventReleaseToDevice));
      if (!ctx->serial) {
        spec.rb_f1 = &rbf1;
        spec.rb_h1 = &rbh1;
        spec.rstream = bs.rstream;
        spec.win_ev = bs.wev;
        spec.fstream = bs.fstream;
        spec.fin_ev = bs.fev;
        spec.spec_ev = bs.spev;
        // The windows' draws run ahead on the matching stream (a small
        // batch's matching is done before its verification starts; on the
        // early-final stream they held that pass back; in order on the scoring
        // stream: 3.74-3.77 vs 3.63-3.67 ms per call, profiles/r04_h, r04_j).
        {
          spec.dstream = ctx->stream;
          spec.draw_ev = bs.dev;
          // the third parity (no parallel-LO slots: only the first windows have them)
          SCM_TRY(window_bufs(bs.t_samp, bs.t_nmod, bs.t_fcon, bs.t_mods, bs.t_cnts, bs.t_ucnt,
                              bs.t_wsnap, bs.t_wb, bs.t_wstate, false, &rbf2));
          SCM_TRY(window_bufs(bs.th_samp, bs.th_nmod, bs.th_fcon, bs.th_mods, bs.th_cnts,
                              bs.th_ucnt, bs.th_wsnap, bs.th_wb, bs.th_wstate, ctx->score_split,
                              &rbh2));
          rbf2.lo = rbh2.lo = nullptr;
          rbf2.lo_data = rbh2.lo_data = nullptr;
          spec.rb_f2 = &rbf2;
          spec.rb_h2 = &rbh2;
        }
      }
    }
    const VerifyParams vparams = make_params(ctx->opts, iteration);
    SCM_HT(7);
    SCM_HIP(launch_verify(bs.d_vpairs, (int)V, max_m, bs.xy1.as<double>(),
                          bs.xy2.as<double>(), bs.scratch.as<double>(), bs.snaps.as<uint32_t>(),
                          bs.masks.as<uint8_t>(), bs.dvout.as<VerifyOut>(),
                          vparams, prof, nullptr, bs.xyf.as<float4>(), rbf, rbh,
                          sv, bs.sev, &bs.nwin, &spec));
  }
  SCM_HT(8);
  SCM_HIP(hipEventRecord(bs.ev[5], sv));
  // Compact matches + F-inlier masks in HBM, then DMA the results into the
  // pinned host buffer (counts are already there).
  SCM_TRY(bs.dpack.ensure(std::max<int64_t>(total, 1) * sizeof(uint2)));
  SCM_TRY(bs.dpmask.ensure(std::max<int64_t>(total, 1)));
  SCM_HIP(launch_compact(bs.counts.as<int32_t>(), (int)P, bs.offsets.as<int64_t>(),
                         bs.d_moff, bs.matches.as<uint2>(),
                         bs.masks.as<uint8_t>(), bs.dpack.as<uint2>(), bs.dpmask.as<uint8_t>(),
                         sv));
  if (total > 0) {
    SCM_HIP(hipMemcpyAsync(outh + bs.off_matches, bs.dpack.ptr, total * sizeof(uint2),
                           hipMemcpyDeviceToHost, sv));
    SCM_HIP(hipMemcpyAsync(outh + bs.off_masks, bs.dpmask.ptr, total, hipMemcpyDeviceToHost, sv));
  }
  if (verify)
    SCM_HIP(hipMemcpyAsync(outh + bs.off_vout, bs.dvout.ptr, P * sizeof(VerifyOut),
                           hipMemcpyDeviceToHost, sv));
  SCM_HIP(hipEventRecord(bs.ev[6], sv));
  bs.posted = true;
  return SCM_OK;
}

int collect_batch(scm_context* ctx, BatchSet& bs, BatchView* v) {
  *v = BatchView();
  v->P = bs.P;
  if (!bs.pending) return SCM_OK;
  if (!bs.posted) {
    set_error("internal: batch collected before its verification stage was enqueued");
    return SCM_E_STATE;
  }
  SCM_HT(10);
  SCM_HIP(hipEventSynchronize(bs.ev[6]));
  SCM_HT(11);
  bs.pending = bs.posted = false;
  if (bs.matched) {
    ctx->t_match += event_ms(bs.ev[0], bs.ev[1]);
    ctx->t_final += event_ms(bs.ev[1], bs.ev[2]);
  }
  if (bs.verify) ctx->t_verify += event_ms(bs.ev[4], bs.ev[5]);
  if (bs.verify) {
    for (int w = 0; w < bs.nwin; ++w) ctx->t_score += event_ms(bs.sev[2 * w], bs.sev[2 * w + 1]);
    bs.nwin = 0;
  }
  SCM_HT(14);
  const uint8_t* o = reinterpret_cast<const uint8_t*>(bs.out.host);
  v->counts = reinterpret_cast<const int32_t*>(o + bs.off_counts);
  v->offsets = reinterpret_cast<const int64_t*>(o + bs.off_offsets);
  v->vout = bs.verify ? reinterpret_cast<const VerifyOut*>(o + bs.off_vout) : nullptr;
  v->matches = reinterpret_cast<const Match*>(o + bs.off_matches);
  v->masks = o + bs.off_masks;
  if (v->vout)
    for (int64_t p = 0; p < bs.P; ++p) {
      ctx->evals_f += v->vout[p].f_evals;
      ctx->evals_h += v->vout[p].h_evals;
      const int32_t sc = v->vout[p].spec_check;
      ctx->spec_taken += sc == 3;
      ctx->spec_equal += sc == 1;
      ctx->spec_differ += sc == 2;
      ctx->spec_void += sc == 4;
    }
  if (ctx->profile && bs.verify && bs.nprof > 0) {
    std::vector<uint64_t> pr(bs.nprof * kVerifyProfSlots);
    SCM_HIP(hipMemcpy(pr.data(), bs.prof.ptr, pr.size() * sizeof(uint64_t),
                      hipMemcpyDeviceToHost));
    ctx->prof_sum.resize(kVerifyProfSlots, 0);
    ctx->prof_worst.resize(kVerifyProfSlots, 0);
    auto final_cycles = [](const uint64_t* x) {
      uint64_t t = 0;
      for (int j = 0; j < 9; ++j) t += x[j];
      return t;
    };
    for (int64_t k = 0; k < bs.nprof; ++k) {
      const uint64_t* x = pr.data() + k * kVerifyProfSlots;
      for (int j = 0; j < kVerifyProfSlots; ++j) ctx->prof_sum[j] += x[j];
      if (final_cycles(x) > final_cycles(ctx->prof_worst.data()))
        ctx->prof_worst.assign(x, x + kVerifyProfSlots);
    }
    ctx->prof_pairs += bs.nprof;
  }
  bs.nprof = 0;
  return SCM_OK;
}

// Both stages of one batch, then its results (single-pair / stencil calls).
int run_batch(scm_context* ctx, BatchSet& bs, const ImageTable& t,
              const std::vector<PairSpec>& specs, bool verify, const uint32_t* given,
              const int32_t* given_counts, BatchView* v, int iteration = 0) {
  SCM_TRY(enqueue_match(ctx, bs, t, specs, given, given_counts));
  SCM_TRY(enqueue_verify(ctx, bs, verify, iteration));
  return collect_batch(ctx, bs, v);
}

// Number of F inliers emitted for pair p (TwoViewGeometry() after the
// post-filter emits none, sequential_matching.cc:96-99).
int64_t inlier_count(const BatchView& v, int64_t p) {
  if (!v.vout || v.vout[p].config == 0) return 0;
  const uint8_t* m = v.masks + v.offsets[p];
  int64_t c = 0;
  for (int32_t i = 0; i < v.counts[p]; ++i) c += m[i] != 0;
  return c;
}

// Bytes of one TVG in the io.cc layout (io.cc:279-292): config, E, F, H,
// qvec, tvec, tri_angle, inlier count.
constexpr size_t kTvgFixed = 4 + 8 * 35 + 8;

uint8_t* write_tvg(uint8_t* d, const BatchView& v, int64_t p, int64_t ninl) {
  const VerifyOut* vo = v.vout ? &v.vout[p] : nullptr;
  const int32_t config = vo ? vo->config : 0;
  std::memcpy(d, &config, 4);
  d += 4;
  double blk[35];
  std::memset(blk, 0, sizeof(blk));
  if (vo && config != 0)
    for (int c = 0; c < 3; ++c)
      for (int r = 0; r < 3; ++r) {  // Eigen column-major
        blk[9 + 3 * c + r] = vo->F[3 * r + c];
        blk[18 + 3 * c + r] = vo->H[3 * r + c];
      }
  std::memcpy(d, blk, sizeof(blk));
  d += sizeof(blk);
  const uint64_t n = (uint64_t)ninl;
  std::memcpy(d, &n, 8);
  d += 8;
  if (ninl > 0) {
    // Branch-free compaction (the masks are data-dependent: a branch per match
    // mispredicts about every other time, ~8x slower): every match is stored
    // at the next output slot, which advances only past an inlier.  Up to the
    // last inlier L, the slot is always < ninl.
    const int64_t o = v.offsets[p];
    const uint8_t* mk = v.masks + o;
    const Match* mt = v.matches + o;
    int32_t last = v.counts[p] - 1;
    while (!mk[last]) --last;  // ninl > 0: an inlier exists
    int64_t w = 0;
    for (int32_t i = 0; i <= last; ++i) {
      std::memcpy(d + 8 * w, &mt[i], 8);
      w += mk[i] ? 1 : 0;
    }
    d += 8 * ninl;
  }
  return d;
}

// Growable malloc'd output (realloc of large blocks remaps, no copy).
struct Packed {
  uint8_t* data = nullptr;
  size_t size = 0, cap = 0;
  std::vector<int64_t> row_off;  // [ids_r, tvgs_r] per row, then the end
  bool reserve(size_t need) {
    if (!data) data = (uint8_t*)pool_take(&cap);  // recycled, already-mapped pages
    if (need <= cap) return true;
    const size_t want = std::max(need, cap + cap / 2);
    uint8_t* p = (uint8_t*)std::realloc(data, want);
    if (!p) return false;
    data = p;
    cap = want;
    return true;
  }
};

// Serialises one batch's output rows: row r's pairs are
// pairs_begin[r] .. pairs_begin[r + 1] of the batch.
int serialize_rows(scm_context* ctx, const BatchView& v, const std::vector<uint32_t>& pair_ids,
                   const std::vector<int64_t>& pairs_begin, Packed* out) {
  const int64_t nrows = (int64_t)pairs_begin.size() - 1;
  std::vector<int64_t> ninl(v.P);
  parallel_for(ctx->threads, v.P, [&](int64_t p) { ninl[p] = inlier_count(v, p); });
  std::vector<size_t> rstart(nrows + 1);
  size_t at = out->size;
  for (int64_t r = 0; r < nrows; ++r) {
    rstart[r] = at;
    const int64_t np = pairs_begin[r + 1] - pairs_begin[r];
    at += 8 + 4 * (size_t)np + 12;
    for (int64_t p = pairs_begin[r]; p < pairs_begin[r + 1]; ++p) at += kTvgFixed + 8 * ninl[p];
  }
  rstart[nrows] = at;
  if (!out->reserve(at)) {
    set_error("output allocation failed");
    return SCM_E_NOMEM;
  }
  parallel_for(ctx->threads, nrows, [&](int64_t r) {
    uint8_t* d = out->data + rstart[r];
    const int64_t pb = pairs_begin[r], pe = pairs_begin[r + 1];
    const uint64_t np = (uint64_t)(pe - pb);
    std::memcpy(d, &np, 8);  // createVectorBuffer<vector<image_t>> (io.cc:151-162)
    d += 8;
    for (int64_t p = pb; p < pe; ++p) {
      std::memcpy(d, &pair_ids[p], 4);
      d += 4;
    }
    // create_two_view_geometries_buffer (io.cc:256-297): total size, count.
    const uint64_t tb = (uint64_t)(rstart[r + 1] - rstart[r] - 8 - 4 * np);
    const int32_t cnt = (int32_t)np;
    std::memcpy(d, &tb, 8);
    std::memcpy(d + 8, &cnt, 4);
    d += 12;
    for (int64_t p = pb; p < pe; ++p) d = write_tvg(d, v, p, ninl[p]);
  });
  for (int64_t r = 0; r < nrows; ++r) {
    out->row_off.push_back((int64_t)rstart[r]);
    out->row_off.push_back((int64_t)(rstart[r] + 8 + 4 * (pairs_begin[r + 1] - pairs_begin[r])));
  }
  out->size = at;
  return SCM_OK;
}

// ---------------------------------------------------------------------------
// TwoViewGeometry::EstimateMultiple [upstream estimators/two_view_geometry.cc],
// taken by verifyTwoViewGeometry when multiple_models is set
// (sequential_matching.cc:94-96):
//   remaining = matches
//   loop: g = Estimate(remaining); stop if g.config == DEGENERATE;
//         keep g unless it is WATERMARK (Options::multiple_ignore_watermark,
//         COLMAP's default true; the op does not set it);
//         remaining = ExtractOutlierMatches(remaining, g.inlier_matches)
//   none kept -> DEGENERATE; one -> that geometry; more -> MULTIPLE with the
//   kept geometries' inlier matches concatenated (F, H left unset: zeros).
// The batch's own verification is the first Estimate; every later one runs
// for all still-active pairs of the batch together as a batch of given
// match lists on the same set, with the iteration's PRNG seeds
// (geom::iteration_seed).  One deviation: the reference loops forever when a
// non-degenerate Estimate removes no match (F failed, H succeeded); here the
// pair stops.
struct Geom {
  int32_t config = 0;
  double F[9] = {0}, H[9] = {0};
  std::vector<Match> inliers;
};

// The Estimate of pair p in view v on the match list `cur` (= the view's
// matches of p): appends the kept geometry and sets `cur` to the outliers;
// false when EstimateMultiple stops for the pair.
bool take_estimate(const scm_matching_options& o, const BatchView& v, int64_t p,
                   std::vector<Geom>* geoms, std::vector<Match>* cur) {
  const int32_t n = v.counts[p];
  const int32_t mni = o.min_num_inliers;
  if (!v.vout || n < std::max(1, mni)) return false;  // Estimate: DEGENERATE (too few)
  const VerifyOut& vo = v.vout[p];
  if (vo.raw_config == SCM_TVG_DEGENERATE || vo.raw_config == 0) return false;
  const Match* m = v.matches + v.offsets[p];
  const uint8_t* mk = v.masks + v.offsets[p];
  const bool f_ok = vo.f_inliers_raw >= 7;  // ExtractInlierMatches of a successful F report
  Geom g;
  g.config = vo.raw_config;
  std::memcpy(g.F, vo.F, sizeof(g.F));
  std::memcpy(g.H, vo.H, sizeof(g.H));
  std::vector<Match> out;
  for (int32_t i = 0; i < n; ++i) {
    if (f_ok && mk[i]) g.inliers.push_back(m[i]);
    else out.push_back(m[i]);
  }
  const bool removed = !g.inliers.empty();
  if (g.config != SCM_TVG_WATERMARK) geoms->push_back(std::move(g));
  cur->swap(out);
  // The oracle (verify_pair_multiple, oracle.cc) runs the next Estimate and
  // stops on its DEGENERATE result; stopping here when fewer than
  // min_num_inliers (or no) matches remain is the same decision only because
  // Estimate returns DEGENERATE for such a list before any RANSAC
  // (TwoViewGeometry::Estimate's size guard, oracle.cc verify_pair
  // `matches.size() < min_num_inliers`, and the `n < max(1, mni)` test at the
  // top of this function).  A change to that guard must change this stop.
  return removed && (int64_t)cur->size() >= std::max(1, mni);
}

int estimate_multiple(scm_context* ctx, BatchSet& bs, const BatchView& v0, std::vector<Tvg>* tvgs) {
  const int64_t P = v0.P;
  const ImageTable& t = *bs.table;
  const std::vector<PairSpec> specs = bs.specs;  // bs is reused by the later iterations
  std::vector<std::vector<Geom>> geoms(P);
  std::vector<std::vector<Match>> rem(P);
  std::vector<int64_t> active;
  for (int64_t p = 0; p < P; ++p)
    if (take_estimate(ctx->opts, v0, p, &geoms[p], &rem[p])) active.push_back(p);
  for (int it = 1; !active.empty(); ++it) {
    std::vector<PairSpec> sp;
    std::vector<int32_t> cnt;
    std::vector<Match> all;
    for (int64_t p : active) {
      sp.push_back(specs[p]);
      cnt.push_back((int32_t)rem[p].size());
      all.insert(all.end(), rem[p].begin(), rem[p].end());
    }
    BatchView v;
    SCM_TRY(run_batch(ctx, bs, t, sp, true, reinterpret_cast<const uint32_t*>(all.data()),
                      cnt.data(), &v, it));
    std::vector<int64_t> next;
    for (size_t q = 0; q < active.size(); ++q)
      if (take_estimate(ctx->opts, v, (int64_t)q, &geoms[active[q]], &rem[active[q]]))
        next.push_back(active[q]);
    active.swap(next);
  }
  tvgs->assign(P, Tvg());
  for (int64_t p = 0; p < P; ++p) {
    Tvg& tv = (*tvgs)[p];
    const std::vector<Geom>& g = geoms[p];
    if (g.size() == 1) {
      tv.config = g[0].config;
      std::memcpy(tv.F, g[0].F, sizeof(tv.F));
      std::memcpy(tv.H, g[0].H, sizeof(tv.H));
      tv.inlier_matches = g[0].inliers;
    } else if (g.size() > 1) {
      tv.config = SCM_TVG_MULTIPLE;
      for (const Geom& x : g) tv.inlier_matches.insert(tv.inlier_matches.end(), x.inliers.begin(),
                                                        x.inliers.end());
    } else {
      tv.config = SCM_TVG_DEGENERATE;  // none kept
    }
    // the op's post-filter (sequential_matching.cc:173-178)
    if ((int64_t)tv.inlier_matches.size() < (int64_t)ctx->opts.min_num_inliers) tv = Tvg();
  }
  return SCM_OK;
}

// serialize_rows for host geometries (the multiple_models path).
int serialize_rows_tvg(const std::vector<Tvg>& tv, const std::vector<uint32_t>& pair_ids,
                       const std::vector<int64_t>& pairs_begin, Packed* out) {
  const int64_t nrows = (int64_t)pairs_begin.size() - 1;
  for (int64_t r = 0; r < nrows; ++r) {
    const int64_t pb = pairs_begin[r], pe = pairs_begin[r + 1];
    const std::vector<uint8_t> a =
        id_list_bytes(std::vector<uint32_t>(pair_ids.begin() + pb, pair_ids.begin() + pe));
    const std::vector<uint8_t> b = tvg_list_bytes(std::vector<Tvg>(tv.begin() + pb, tv.begin() + pe));
    if (!out->reserve(out->size + a.size() + b.size())) {
      set_error("output allocation failed");
      return SCM_E_NOMEM;
    }
    out->row_off.push_back((int64_t)out->size);
    std::memcpy(out->data + out->size, a.data(), a.size());
    out->size += a.size();
    out->row_off.push_back((int64_t)out->size);
    std::memcpy(out->data + out->size, b.data(), b.size());
    out->size += b.size();
  }
  return SCM_OK;
}

int decode_rows(int64_t n, const scm_element* ids, const scm_element* kps,
                const scm_element* descs, std::vector<RowView>* rows) {
  if (n < 0 || (n > 0 && (!ids || !kps || !descs))) {
    set_error("invalid element arrays");
    return SCM_E_INVALID;
  }
  rows->resize(n);
  for (int64_t i = 0; i < n; ++i) SCM_TRY(decode_row(ids[i], kps[i], descs[i], &(*rows)[i]));
  for (int64_t i = 0; i < n; ++i)
    if ((*rows)[i].nkp < (*rows)[i].ndesc) {
      set_error("fewer keypoints than descriptors in row " + std::to_string(i));
      return SCM_E_INVALID;
    }
  return SCM_OK;
}

// Pair list of one output row: SequentialMatchingCPUKernel::execute's loop
// (sequential_matching.cc:139-146): stencil entries 1..K-1, skipping the
// pivot's own id and ids already paired.
void row_pairs(const std::vector<uint32_t>& stencil_ids, std::vector<int64_t>* sel) {
  sel->clear();
  std::vector<uint32_t> seen;
  for (size_t s = 1; s < stencil_ids.size(); ++s) {
    const uint32_t id2 = stencil_ids[s];
    if (id2 == stencil_ids[0] || std::count(seen.begin(), seen.end(), id2) > 0) continue;
    seen.push_back(id2);
    sel->push_back((int64_t)s);
  }
}

// Upper bound of the device workspace one pair takes in a batch set: the
// matcher's row / column partials and match slots (enqueue_match), and the
// verifier's points, scratch, window buffers and compaction output with every
// pivot keypoint matched (enqueue_verify).
// Round-buffer bytes per trial and kind: samples, model count, filter
// constants, models, counts (+ split counts).
constexpr int64_t kRoundTrialBytes = 8 * 4 + 4 + 3 * 12 * 4 + 3 * 9 * 8 + 2 * 3 * 4;

int64_t pair_workspace_bytes(int64_t n1, int64_t n2) {
  const int32_t rpb = kRowsPerBlock8 < kRowsPerBlock ? kRowsPerBlock8 : kRowsPerBlock;
  const int64_t nseg = (n2 + kColsPerSeg - 1) / kColsPerSeg;
  const int64_t nrb = (n1 + rpb - 1) / rpb;
  const int64_t n2pad = (n2 + kTile8Cols - 1) / kTile8Cols * kTile8Cols;
  const int64_t slots = std::max<int64_t>(n1, 1);
  const int64_t match = nseg * n1 * 8 + nrb * n2pad * 8 + n2 * 4 + slots * (8 + 1) +
                        n1 * 8 + (33 + n1) * 4;  // + v2 row aux and recheck buckets
  const int64_t verify_pts = slots * (16 + 16 + 16 + 8 + 1);  // xy1, xy2, xyf, dpack, dpmask
  const int64_t verify_pair = verify_scratch_doubles(slots) * 8 + kVerifySnapWords * 4 +
                              (int64_t)sizeof(RansacState) + (int64_t)sizeof(VerifyOut) +
                              2 * ((int64_t)kWindowTrials * kRoundTrialBytes + 640 * 4) +
                              256;  // F and H round buffers
  return match + verify_pts + verify_pair;
}

// Bytes per pair beyond pair_workspace_bytes' when a batch takes the
// small-batch kernels (enqueue_verify): windows of kWindowTrialsSmall trials
// in three parities, F and H (window starts, states and trial counts
// included), and the parallel-LO slots of both kinds and the first two
// parities (at most, for a pivot of n1 keypoints), and the row segments of
// the matcher's column split (enqueue_match).
int64_t small_batch_extra_bytes(int64_t n1) {
  return (int64_t)kMaxColSplit * n1 * 8 +
         2 * (3 * (int64_t)kWindowTrialsSmall - (int64_t)kWindowTrials) * kRoundTrialBytes +
         2 * 2 * (640 * 4 + kVerifyStateWords * 4 + 4) +
         4 * (int64_t)kLoSlots * (lo_slot_doubles(std::max<int64_t>(n1, 1)) * 8 + (int64_t)sizeof(LoSlot));
}

// Byte budget of one of the three batch sets: SCM_BATCH_BYTES, or a third of
// the free HBM plus what the sets already hold (reused), less a 2 GiB margin.
int64_t set_budget_bytes(scm_context* ctx) {
  if (ctx->batch_bytes > 0) return ctx->batch_bytes;
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return INT64_MAX;
  int64_t held = 0;
  for (const BatchSet& bs : ctx->sets)
    for (const DevBuf* b : {&bs.rowaux, &bs.rlist, &bs.mdesc, &bs.rowres, &bs.colpart, &bs.m21, &bs.matches,
                            &bs.counts, &bs.vdesc, &bs.xy1, &bs.xy2, &bs.scratch,
                            &bs.snaps, &bs.masks, &bs.offsets, &bs.prof, &bs.xyf,
                            &bs.dvout, &bs.dpack, &bs.dpmask, &bs.rst, &bs.samp, &bs.nmod,
                            &bs.fcon, &bs.cnts, &bs.act, &bs.nact, &bs.mods, &bs.wsnap,
                            &bs.h_rst, &bs.h_samp, &bs.h_nmod, &bs.h_fcon, &bs.h_cnts, &bs.h_act,
                            &bs.h_nact, &bs.h_mods, &bs.h_wsnap, &bs.ucnt, &bs.h_ucnt})
      held += (int64_t)b->bytes;
  const int64_t avail = (int64_t)free_b + held - ((int64_t)2 << 30);
  return std::max<int64_t>(avail / 3, (int64_t)64 << 20);
}

// One output row of a run: the pivot's table index and the table indices /
// image ids of the stencil entries it is paired with (execute()'s loop after
// the dedup, sequential_matching.cc:139-146).
struct RowPlan {
  int32_t pivot = 0;
  std::vector<int32_t> nb;
  std::vector<uint32_t> nb_ids;
};

// Runs output rows `plan` (pair lists over table t) through the pipelined
// batch machinery into one packed output.  keep_row0 >= 0 (table path):
// plan[i] is table row keep_row0 + i and the raw matches of the kept rows are
// recorded for scm_table_matches.
// Passes of a streamed run (run_rows with pass_rows > 0): pass k is plan rows
// [k * pass_rows, (k + 1) * pass_rows); `emit` receives each pass's packed rows
// (final row offset included) as soon as they are serialised, in order.
using PassEmit = std::function<int(int64_t, Packed&)>;
// Chunked runs (out == nullptr, pass_rows == 0): `emit` receives each batch's
// rows as its own packed output (first plan row index, then the rows), in row
// order, as soon as they are serialised.

int run_rows(scm_context* ctx, const ImageTable& t, const std::vector<RowPlan>& plan,
             int64_t keep_row0, Packed* out, int64_t pass_rows = 0,
             const PassEmit* emit = nullptr);

// Runs the sequential stencil over table rows [row_begin, row_end) through
// the pipelined batch machinery into one packed output.
int run_table(scm_context* ctx, int64_t overlap, int64_t row_begin, int64_t row_end,
              Packed* out, const PassEmit* chunk_emit = nullptr) {
  const ImageTable& t = ctx->table;
  std::vector<uint32_t> ids(overlap);
  std::vector<int64_t> rows(overlap), sel;
  // Pair lists of every row first (the stencil dedup of execute()).
  const int64_t nr = row_end - row_begin;
  std::vector<RowPlan> plan(nr);
  for (int64_t r = row_begin; r < row_end; ++r) {
    for (int64_t s = 0; s < overlap; ++s) {
      rows[s] = std::min(r + s, t.n - 1);  // stencil clamped at the table end
      ids[s] = t.ids[rows[s]];
    }
    row_pairs(ids, &sel);
    RowPlan& rp = plan[r - row_begin];
    rp.pivot = (int32_t)r;
    for (int64_t s : sel) {
      rp.nb.push_back((int32_t)rows[s]);
      rp.nb_ids.push_back(ids[s]);
    }
  }
  return run_rows(ctx, t, plan, row_begin, out, 0, chunk_emit);
}

int run_rows(scm_context* ctx, const ImageTable& t, const std::vector<RowPlan>& plan,
             int64_t keep_row0, Packed* out, int64_t pass_rows, const PassEmit* emit) {
  struct Batch {
    std::vector<PairSpec> specs;
    std::vector<uint32_t> pair_ids;
    std::vector<int64_t> pairs_begin;
    int64_t row0 = 0;  // plan index of the batch's first row
  };
  std::vector<Batch> batches;
  const int64_t nr = (int64_t)plan.size();
  const bool keep = keep_row0 >= 0 && ctx->keep_matches;
  const bool streamed = pass_rows > 0;
  // kept matches: the last pass's rows (every row of a single run)
  const int64_t keep_from = streamed ? nr - pass_rows : 0;
  const int64_t row_begin = keep_row0, row_end = keep_row0 + (nr - keep_from);
  // Batches of whole rows, closed at batch_pairs pairs or when the next row
  // would push the batch's device workspace past the per-set byte budget
  // (three sets are live at once).  A single row larger than the budget still
  // forms a batch of its own (its allocation fails loudly if HBM is short).
  // Measured on the bench workload: equal-size batches, short first / last
  // batches, and caps of 4,096-9,472 pairs were all slower than 8,192.
  const int64_t budget = set_budget_bytes(ctx);
  // (The remainder batch first instead of last measured slower, 44.4/44.5K vs
  // 47.4/47.6K pairs/s, profiles/r05_b_ab_*.)
  const int64_t first_cap = ctx->batch_pairs;
  // Scanner op calls (execute(): one packed output, no kept rows) that fit
  // one batch: cut into nb <= kOpCallBatches batches of about equal pairs
  // (whole rows), each of at least a small batch's pairs, so that each
  // batch's matching overlaps the previous batch's verification instead of
  // the call running its matcher and then its verification alone.  Op calls
  // of 256 stencils (4,864 pairs): 164.4 ms per call in one batch, 147.2 in
  // two, 136.9 in three; 64 stencils (1,216 pairs) stay one batch (49.2 vs
  // 50.8 in two); calls beyond one batch keep the table path's cut (two
  // equal batches at 512 stencils: no gain), profiles/r06_ao.
  std::vector<char> opens(nr, 0);  // rows that open a batch of their own
  if (keep_row0 < 0 && !streamed && !emit) {
    int64_t total = 0;
    for (const RowPlan& rp : plan) total += (int64_t)rp.nb.size();
    const int64_t nb = std::min<int64_t>(kOpCallBatches, total / verify_small_batch_pairs());
    if (nb >= 2 && total <= ctx->batch_pairs) {
      int64_t acc = 0, k = 1;
      for (int64_t i = 0; i < nr && k < nb; ++i) {
        if (acc > 0 && acc * nb >= k * total) {
          opens[i] = 1;
          ++k;
        }
        acc += (int64_t)plan[i].nb.size();
      }
    }
  }
  Batch cur;
  int64_t cur_bytes = 0, cur_small = 0;
  for (int64_t i = 0; i < nr; ++i) {
    const RowPlan& rp = plan[i];
    const int64_t np = (int64_t)rp.nb.size();
    int64_t row_bytes = 0;
    for (int32_t b : rp.nb) row_bytes += pair_workspace_bytes(t.ndesc[rp.pivot], t.ndesc[b]);
    const int64_t have = (int64_t)cur.specs.size();
    const int64_t cap = opens[i] ? have : batches.empty() ? first_cap : ctx->batch_pairs;
    // a batch small enough for the small-batch kernels holds their larger
    // round buffers and parallel-LO slots (enqueue_verify)
    const int64_t row_small = np * small_batch_extra_bytes(t.ndesc[rp.pivot]);
    const int64_t small_extra =
        have + np <= verify_small_batch_pairs() ? cur_small + row_small : 0;
    if (have > 0 && (have + np > cap || cur_bytes + row_bytes + small_extra > budget)) {
      cur.pairs_begin.push_back(have);
      batches.push_back(std::move(cur));
      cur = Batch();
      cur.row0 = i;
      cur_bytes = 0;
      cur_small = 0;
    }
    cur_bytes += row_bytes;
    cur_small += row_small;
    cur.pairs_begin.push_back((int64_t)cur.specs.size());
    for (size_t k = 0; k < rp.nb.size(); ++k) {
      cur.specs.push_back({rp.pivot, rp.nb[k]});
      cur.pair_ids.push_back(rp.nb_ids[k]);
    }
  }
  if (!cur.pairs_begin.empty()) {
    cur.pairs_begin.push_back((int64_t)cur.specs.size());
    batches.push_back(std::move(cur));
  }
  if (keep) {
    ctx->last_begin = row_begin;
    ctx->last_end = row_end;
    ctx->last_matches.assign(row_end - row_begin, {});
  }
  // Streamed runs: one output per pass; a batch may span a pass boundary, its
  // rows are serialised into the pass they belong to.
  const int64_t npass = streamed ? nr / pass_rows : 0;
  std::vector<Packed> packs(npass);
  // Passes not handed over when a run fails return their buffers (the
  // hand-over takes the data of the ones it emits).
  struct PacksGuard {
    std::vector<Packed>& v;
    ~PacksGuard() {
      for (Packed& p : v)
        if (p.data && !pool_give(p.data)) std::free(p.data);
    }
  } packs_guard{packs};
  std::vector<int64_t> rows_done(npass, 0);
  int64_t next_emit = 0;
  const bool chunked = !streamed && !out && emit;
  auto finish = [&](const Batch& b, BatchSet& bs) -> int {
    BatchView v;
    SCM_TRY(collect_batch(ctx, bs, &v));
    const int64_t nrows = (int64_t)b.pairs_begin.size() - 1;
    if (keep)
      for (int64_t r = 0; r < nrows; ++r) {
        if (b.row0 + r < keep_from) continue;
        for (int64_t p = b.pairs_begin[r]; p < b.pairs_begin[r + 1]; ++p) {
          const int64_t row = b.specs[p].a, o = v.offsets[p];
          if (!ctx->kept(row)) continue;
          ctx->last_matches[row - row_begin].push_back(
              {b.specs[p].b - row, std::vector<Match>(v.matches + o, v.matches + o + v.counts[p])});
        }
      }
    SCM_HT(15);
    std::vector<Tvg> tv;
    if (ctx->opts.multiple_models)  // the later Estimates reuse bs: v is consumed first
      SCM_TRY(estimate_multiple(ctx, bs, v, &tv));
    auto ser = [&](const std::vector<int64_t>& pb, Packed* o) {
      return ctx->opts.multiple_models ? serialize_rows_tvg(tv, b.pair_ids, pb, o)
                                       : serialize_rows(ctx, v, b.pair_ids, pb, o);
    };
    if (chunked) {
      Packed pk;
      int rc = ser(b.pairs_begin, &pk);
      if (rc == SCM_OK) {
        pk.row_off.push_back((int64_t)pk.size);
        rc = (*emit)(b.row0, pk);  // takes pk.data unless it fails
      }
      if (pk.data && !pool_give(pk.data)) std::free(pk.data);
      return rc;
    }
    if (!streamed) return ser(b.pairs_begin, out);
    for (int64_t r0 = 0; r0 < nrows;) {
      const int64_t pass = (b.row0 + r0) / pass_rows;
      const int64_t r1 = std::min(nrows, (pass + 1) * pass_rows - b.row0);
      const std::vector<int64_t> pb(b.pairs_begin.begin() + r0, b.pairs_begin.begin() + r1 + 1);
      SCM_TRY(ser(pb, &packs[pass]));
      rows_done[pass] += r1 - r0;
      r0 = r1;
    }
    while (next_emit < npass && rows_done[next_emit] == pass_rows) {
      Packed& pk = packs[next_emit];
      pk.row_off.push_back((int64_t)pk.size);
      SCM_TRY((*emit)(next_emit, pk));
      ++next_emit;
    }
    return SCM_OK;
  };
  if (!streamed && !chunked) out->row_off.reserve(2 * nr + 1);
  // Three buffer sets: at step k the GPU holds match(k) on the matching
  // stream and verify(k-1) (+ verify(k-2)) on the verification stream while
  // the host serialises batch k-3.
  const size_t B = batches.size();
  if (ctx->serial) {
    for (size_t k = 0; k < B; ++k) {
      BatchSet& bs = ctx->sets[k % 3];
      if (k >= 3) SCM_TRY(finish(batches[k - 3], bs));
      SCM_TRY(enqueue_match(ctx, bs, t, batches[k].specs, nullptr, nullptr));
      SCM_TRY(enqueue_verify(ctx, bs, true));
      if (bs.pending) SCM_HIP(hipStreamWaitEvent(ctx->stream, bs.ev[6], 0));
    }
  } else {
    for (size_t k = 0; k < B; ++k) {
      if (k >= 3) SCM_TRY(finish(batches[k - 3], ctx->sets[(k - 3) % 3]));
      SCM_HT(4);
      SCM_TRY(enqueue_match(ctx, ctx->sets[k % 3], t, batches[k].specs, nullptr, nullptr));
      if (k >= 1) SCM_TRY(enqueue_verify(ctx, ctx->sets[(k - 1) % 3], true));
    }
    if (B >= 1) SCM_TRY(enqueue_verify(ctx, ctx->sets[(B - 1) % 3], true));
    SCM_HT(9);
  }
  for (size_t k = B >= 3 ? B - 3 : 0; k < B; ++k) SCM_TRY(finish(batches[k], ctx->sets[k % 3]));
  if (!streamed && !chunked) out->row_off.push_back((int64_t)out->size);
  return SCM_OK;
}

// Drains any batch left in flight by an error path.
void drain(scm_context* ctx) {
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (BatchSet& bs : ctx->sets)
    if (bs.vstream) (void)hipStreamSynchronize(bs.vstream);
  for (BatchSet& bs : ctx->sets) bs.pending = bs.posted = false;
}

}  // namespace

// ===========================================================================
// C ABI.
// ===========================================================================
extern "C" {

int32_t scm_abi_version(void) { return SCM_ABI_VERSION; }

const char* scm_last_error(void) { return g_last_error.c_str(); }

int scm_context_create(int32_t device_index, const scm_matching_options* opts,
                       scm_context** out) {
  if (!out) {
    set_error("null context pointer");
    return SCM_E_INVALID;
  }
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    set_error("no HIP device visible (the MI355X stage has no CPU fallback)");
    return SCM_E_DEVICE;
  }
  if (device_index < 0 || device_index >= ndev) {
    set_error("device index out of range");
    return SCM_E_DEVICE;
  }
  hipDeviceProp_t prop;
  SCM_HIP(hipGetDeviceProperties(&prop, device_index));
  if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos) {
    set_error(std::string("device is ") + prop.gcnArchName + ", kernels are built for gfx950");
    return SCM_E_DEVICE;
  }
  scm_matching_options o;
  if (opts)
    o = *opts;
  else
    scm_default_options(&o);
  scm_context* ctx = new scm_context();
  ctx->device = device_index;
  ctx->opts = o;
  if (const char* e = std::getenv("SCM_PROFILE")) ctx->profile = e[0] == '1';
  int hw = (int)std::thread::hardware_concurrency();
  if (const char* e = std::getenv("OMP_NUM_THREADS")) hw = std::max(1, std::atoi(e));
  ctx->threads = std::max(1, std::min(16, hw));
  ctx->pool.start(ctx->threads - 1);
  ctx->vpool.start(std::max(1, ctx->threads - 1));
  if (const char* e = std::getenv("SCM_SERIAL")) ctx->serial = e[0] == '1';
  if (const char* e = std::getenv("SCM_BATCH_PAIRS"))
    ctx->batch_pairs = std::max<int64_t>(1, std::min<int64_t>(kMaxPairsPerBatch, std::atoll(e)));
  if (const char* e = std::getenv("SCM_BATCH_BYTES")) ctx->batch_bytes = std::max<int64_t>(1, std::atoll(e));
  if (const char* e = std::getenv("SCM_MATCH_BF16")) ctx->match_bf16 = e[0] == '1';
  // The i8 matcher tracks column top-2 by value only, which decides the
  // cross-check exactly when a tied column best fails the ratio test, i.e.
  // max_ratio <= 1 (match_kernels.hip, i8 section); otherwise the bf16 matcher
  // keeps the lowest-row tie rule with column keys.
  if ((float)o.max_ratio > 1.0f) ctx->match_bf16 = true;
  if (hipSetDevice(device_index) != hipSuccess ||
      hipStreamCreateWithPriority(&ctx->stream, hipStreamNonBlocking, stream_priority(false)) != hipSuccess ||
      hipStreamCreateWithPriority(&ctx->sets[0].vstream, hipStreamNonBlocking, stream_priority(true)) != hipSuccess ||
      hipStreamCreateWithPriority(&ctx->sets[1].vstream, hipStreamNonBlocking, stream_priority(true)) != hipSuccess ||
      hipStreamCreateWithPriority(&ctx->sets[2].vstream, hipStreamNonBlocking, stream_priority(true)) != hipSuccess) {
    scm_context_destroy(ctx);
    set_error("failed to create HIP streams");
    return SCM_E_DEVICE;
  }
  std::vector<float> lut;
  build_lut(&lut);
  if (ctx->lut.ensure(lut.size() * sizeof(float)) != SCM_OK ||
      hipMemcpy(ctx->lut.ptr, lut.data(), lut.size() * sizeof(float), hipMemcpyHostToDevice) !=
          hipSuccess) {
    set_error("failed to upload the acosf table");
    scm_context_destroy(ctx);
    return SCM_E_DEVICE;
  }
  *out = ctx;
  return SCM_OK;
}

void scm_context_destroy(scm_context* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  drain(ctx);
  sift_state_destroy(ctx->sift);
  ctx->sift = nullptr;
  if (ctx->profile && ctx->prof_pairs > 0) {
    static const char* names[] = {"sample",    "solve",   "score",  "cand_res", "seqsum",
                                  "lo_gather", "lo_est",  "lo_res", "other",    "n_batch",
                                  "n_cand",    "n_lo",    "n_trials", "n_points", "n_seqsum",
                                  "score_H", "n_hchunk", "n_hslow"};
    std::fprintf(stderr, "[scm verify profile] pairs=%lld (per pair: cycles / counts)\n",
                 (long long)ctx->prof_pairs);
    for (int j = 0; j < 18; ++j)
      std::fprintf(stderr, "  %-10s %14.1f   worst pair %12llu\n", names[j],
                   (double)ctx->prof_sum[j] / (double)ctx->prof_pairs,
                   (unsigned long long)ctx->prof_worst[j]);
    static const char* rnames[] = {"windows", "n_cand", "n_tie", "n_newbest", "n_lo_iter",
                                   "cyc_cand", "cyc_tie", "cyc_lo", "cyc_total", "trials"};
    for (int kind = 0; kind < 2; ++kind)
      for (int j = 0; j < 10; ++j)
        std::fprintf(stderr, "  replay %s %-10s %14.1f\n", kind ? "H" : "F", rnames[j],
                     (double)ctx->prof_sum[20 + 10 * kind + j] / (double)ctx->prof_pairs);
    for (int kind = 0; kind < 2; ++kind)
      std::fprintf(stderr, "  score %s chunk_models %14.1f slow %14.1f exact %14.1f item_cycles %14.1f\n",
                   kind ? "H" : "F", (double)ctx->prof_sum[80 + 4 * kind] / (double)ctx->prof_pairs,
                   (double)ctx->prof_sum[81 + 4 * kind] / (double)ctx->prof_pairs,
                   (double)ctx->prof_sum[82 + 4 * kind] / (double)ctx->prof_pairs,
                   (double)ctx->prof_sum[83 + 4 * kind] / (double)ctx->prof_pairs);
    static const char* snames[] = {"stage", "phaseA", "phaseB", "writeback", "targets"};
    for (int kind = 0; kind < 2; ++kind)
      for (int j = 0; j < 5; ++j)
        std::fprintf(stderr, "  shuffle %s %-10s %14.1f\n", kind ? "H" : "F", snames[j],
                     (double)ctx->prof_sum[60 + 5 * kind + j] / (double)ctx->prof_pairs);
    static const char* lnames[] = {"lo_gather", "lo_norm", "lo_ata", "lo_jacobi", "lo_resid",
                                   "lo_inliers", "lo_finish"};
    for (int kind = 0; kind < 2; ++kind)
      for (int j = 0; j < 7; ++j)
        std::fprintf(stderr, "  LO %s %-10s %14.1f\n", kind ? "H" : "F", lnames[j],
                     (double)ctx->prof_sum[40 + 10 * kind + j] / (double)ctx->prof_pairs);
  }
  ctx->table.release();
  ctx->scratch_table.release();
  ctx->call_tab[0].release();
  ctx->call_tab[1].release();
  ctx->lut.release();
  for (BatchSet& bs : ctx->sets) bs.release();
  ctx->h_stage.release();
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  for (BatchSet& bs : ctx->sets)
    if (bs.vstream) (void)hipStreamDestroy(bs.vstream);
  delete ctx;
}

int scm_match_pair(scm_context* ctx, const uint8_t* desc1, int64_t n1, const uint8_t* desc2,
                   int64_t n2, uint32_t* matches, int64_t cap, int64_t* num_matches) {
  if (!ctx || !num_matches || n1 < 0 || n2 < 0 || (n1 > 0 && !desc1) || (n2 > 0 && !desc2)) {
    set_error("invalid arguments");
    return SCM_E_INVALID;
  }
  SCM_HIP(hipSetDevice(ctx->device));
  std::vector<RowView> rows(2);
  rows[0].id = 1;
  rows[0].desc = desc1;
  rows[0].ndesc = n1;
  rows[1].id = 2;
  rows[1].desc = desc2;
  rows[1].ndesc = n2;
  SCM_TRY(upload_table(ctx, &ctx->scratch_table, rows, true, false));
  BatchSet& bs = ctx->sets[0];
  BatchView v;
  const int rc = run_batch(ctx, bs, ctx->scratch_table, {{0, 1}}, false, nullptr, nullptr, &v);
  if (rc != SCM_OK) {
    drain(ctx);
    return rc;
  }
  *num_matches = v.counts[0];
  if (v.counts[0] > cap) {
    set_error("match buffer too small");
    return SCM_E_CAPACITY;
  }
  if (v.counts[0] > 0) {
    if (!matches) {
      set_error("null match buffer");
      return SCM_E_INVALID;
    }
    std::memcpy(matches, v.matches + v.offsets[0], (size_t)v.counts[0] * sizeof(Match));
  }
  return SCM_OK;
}

int scm_verify_pair(scm_context* ctx, const float* kp1, int64_t n1, const float* kp2, int64_t n2,
                    const uint32_t* matches, int64_t num_matches, uint32_t image_id1,
                    uint32_t image_id2, scm_blob* tvg_out) {
  if (!ctx || !tvg_out || n1 < 0 || n2 < 0 || num_matches < 0 ||
      (num_matches > 0 && (!matches || !kp1 || !kp2))) {
    set_error("invalid arguments");
    return SCM_E_INVALID;
  }
  for (int64_t i = 0; i < num_matches; ++i)
    if ((int64_t)matches[2 * i] >= n1 || (int64_t)matches[2 * i + 1] >= n2) {
      set_error("match index out of range");
      return SCM_E_INVALID;
    }
  SCM_HIP(hipSetDevice(ctx->device));
  std::vector<RowView> rows(2);
  rows[0].id = image_id1;
  rows[0].kp = kp1;
  rows[0].nkp = n1;
  rows[1].id = image_id2;
  rows[1].kp = kp2;
  rows[1].nkp = n2;
  SCM_TRY(upload_table(ctx, &ctx->scratch_table, rows, false, true));
  BatchSet& bs = ctx->sets[0];
  BatchView v;
  const int32_t gm = (int32_t)num_matches;
  int rc = run_batch(ctx, bs, ctx->scratch_table, {{0, 1}}, true, matches, &gm, &v);
  if (rc == SCM_OK && ctx->opts.multiple_models) {
    std::vector<Tvg> tv;
    rc = estimate_multiple(ctx, bs, v, &tv);
    if (rc == SCM_OK) {
      std::vector<uint8_t> bytes;
      append_tvg(&bytes, tv[0]);
      return make_blob(bytes, tvg_out);
    }
  }
  if (rc != SCM_OK) {
    drain(ctx);
    return rc;
  }
  const int64_t ninl = inlier_count(v, 0);
  std::vector<uint8_t> bytes(kTvgFixed + 8 * ninl);
  write_tvg(bytes.data(), v, 0, ninl);
  return make_blob(bytes, tvg_out);
}

}  // extern "C"

namespace {

constexpr int kRetryKeys = 1;  // execute_rows: a speculated content key did not hold

// Sampled fingerprint of an element's keypoint and descriptor buffers.
uint64_t fingerprint(const RowView& r) {
  const uint64_t h = sample_words(reinterpret_cast<const uint8_t*>(r.kp), (size_t)r.nkp * 24, 0x6670ULL);
  return sample_words(r.desc, (size_t)r.ndesc * 128, h);
}

// One execute() call over decoded elements.  Content keys (ImageKey): element
// buffers the previous call also handed over take that call's keys
// speculatively and are re-hashed on ctx->vpool while the GPU runs; the
// results are returned only if every speculated key holds (else kRetryKeys,
// and the caller runs the call again with every key hashed first).  Buffers
// new to this call are hashed before anything is enqueued.
int execute_rows(scm_context* ctx, int64_t batch, int64_t stencil_size,
                 const std::vector<RowView>& rows, bool speculate, scm_blob* pair_image_ids_out,
                 scm_blob* tvgs_out) {
  const int64_t ne = batch * stencil_size;
  const auto h0 = std::chrono::steady_clock::now();
  SCM_HT(0);
  SCM_HTE_RECORD(ctx->stream);
  std::unordered_map<Src, int64_t, SrcHash> first;  // buffers -> first element
  std::vector<int64_t> of(ne), now_e, spec_e;
  for (int64_t e = 0; e < ne; ++e) {
    const RowView& r = rows[e];
    const Src src{r.kp, r.nkp, r.desc, r.ndesc};
    auto it = first.emplace(src, e).first;
    of[e] = it->second;
    if (it->second != e) continue;
    // Speculate only on buffers whose sampled words still match (a recycled
    // buffer that now holds another image is hashed now instead).
    auto sp = speculate ? ctx->spec_keys.find(src) : ctx->spec_keys.end();
    const bool spec = sp != ctx->spec_keys.end() && sp->second.fp == fingerprint(r);
    if (sp != ctx->spec_keys.end() && !spec) ++ctx->spec_rejected;
    (spec ? spec_e : now_e).push_back(e);
  }
  ctx->spec_elems += (int64_t)spec_e.size();
  std::vector<ImageKey> ekey(ne);
  KeyJob now_job;
  now_job.plan(rows, now_e);
  ctx->pool.run(now_job.ntasks(), [&](int64_t t) { now_job.task(t); });
  for (size_t i = 0; i < now_e.size(); ++i) ekey[now_e[i]] = now_job.key(i);
  for (int64_t e : spec_e) {
    const RowView& r = rows[e];
    ekey[e] = ctx->spec_keys[Src{r.kp, r.nkp, r.desc, r.ndesc}].key;
  }
  KeyJob spec_job;
  spec_job.plan(rows, spec_e);
  ctx->vpool.launch(spec_job.ntasks(), [&](int64_t t) { spec_job.task(t); });
  struct Join {
    WorkerPool& p;
    ~Join() { p.wait(); }
  } join{ctx->vpool};
  for (int64_t e = 0; e < ne; ++e) {
    ekey[e] = ekey[of[e]];
    ekey[e].id = rows[e].id;
  }
  const auto h1 = std::chrono::steady_clock::now();
  // Unique images of the call, by content (ImageKey): every element is
  // matched with its own bytes, as the reference decodes each stencil
  // element (sequential_matching.cc:115-122); an id that reappears with other
  // bytes is simply another image.
  std::unordered_map<ImageKey, int32_t, ImageKeyHash> uid;
  std::vector<RowView> uniq;
  std::vector<ImageKey> ukeys;
  std::vector<int32_t> elem_u(ne);
  for (int64_t e = 0; e < ne; ++e) {
    auto it = uid.find(ekey[e]);
    if (it == uid.end()) {
      it = uid.emplace(ekey[e], (int32_t)uniq.size()).first;
      uniq.push_back(rows[e]);
      ukeys.push_back(ekey[e]);
    }
    elem_u[e] = it->second;
  }
  const int64_t reused0 = ctx->call_reused, uploaded0 = ctx->call_uploaded;
  std::vector<int32_t> uidx;
  std::vector<char> uploaded;
  int rc = upload_call_table(ctx, uniq, ukeys, &uidx, &uploaded);
  if (rc != SCM_OK) {
    ctx->call_cur = -1;  // the cache may be half written
    drain(ctx);
    return rc;
  }
  ctx->t_hash = std::chrono::duration<double, std::milli>(h1 - h0).count();
  ctx->t_stage = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h1).count();
  const ImageTable& t = ctx->call_tab[ctx->call_cur];
  std::vector<RowPlan> plan(batch);
  std::vector<uint32_t> ids(stencil_size);
  std::vector<int64_t> sel;
  for (int64_t b = 0; b < batch; ++b) {
    for (int64_t s = 0; s < stencil_size; ++s) ids[s] = rows[b * stencil_size + s].id;
    row_pairs(ids, &sel);
    plan[b].pivot = uidx[elem_u[b * stencil_size]];
    for (int64_t s : sel) {
      plan[b].nb.push_back(uidx[elem_u[b * stencil_size + s]]);
      plan[b].nb_ids.push_back(ids[s]);
    }
  }
  ctx->t_match = ctx->t_final = ctx->t_verify = ctx->t_score = 0.0;
  ctx->evals_f = ctx->evals_h = 0;
  ctx->spec_taken = ctx->spec_equal = ctx->spec_differ = ctx->spec_void = 0;
  ctx->n_match_launches = 0;
  Packed pk;
  const auto h2 = std::chrono::steady_clock::now();
  SCM_HT(3);
  rc = run_rows(ctx, t, plan, -1, &pk);
  const auto h3 = std::chrono::steady_clock::now();
  SCM_HT(12);
  ctx->t_run = std::chrono::duration<double, std::milli>(h3 - h2).count();
  if (rc != SCM_OK) {
    drain(ctx);
    if (!pool_give(pk.data)) std::free(pk.data);
    return rc;
  }
  ctx->vpool.wait();
  bool held = true;
  for (size_t i = 0; i < spec_e.size(); ++i) held = held && same_content(spec_job.key(i), ekey[spec_e[i]]);
  if (!held) {
    // A buffer was rewritten in place since the previous call (its sampled
    // words unchanged): nothing of this run is returned and the call runs
    // again with every key hashed.  The image cache stays: an entry copied
    // from the previous table holds the bytes its key names.  Only an entry
    // staged from a wrong-keyed buffer (its key not resident) would name
    // other bytes, and those entries are dropped.
    if (!pool_give(pk.data)) std::free(pk.data);
    auto& cmap = ctx->call_map[ctx->call_cur];
    for (size_t i = 0; i < spec_e.size(); ++i) {
      const int32_t u = elem_u[spec_e[i]];
      if (uploaded[u] && !same_content(spec_job.key(i), ekey[spec_e[i]])) cmap.erase(ukeys[u]);
    }
    ctx->spec_keys.clear();
    ctx->call_reused = reused0;
    ctx->call_uploaded = uploaded0;
    ++ctx->spec_retries;
    return kRetryKeys;
  }
  ctx->spec_keys.clear();
  for (const auto& f : first) ctx->spec_keys[f.first] = SpecKey{ekey[f.second], fingerprint(rows[f.second])};
  // The output elements, one task per row on the worker pool (their fresh
  // pages' first touch and the copies in parallel).
  for (int64_t r = 0; r < batch; ++r) pair_image_ids_out[r] = tvgs_out[r] = scm_blob{nullptr, 0};
  std::atomic<bool> oom{false};
  ctx->pool.run(batch, [&](int64_t r) {
    const int64_t a = pk.row_off[2 * r], b = pk.row_off[2 * r + 1], c = pk.row_off[2 * r + 2];
    uint8_t* pa = (uint8_t*)std::malloc((size_t)std::max<int64_t>(b - a, 1));
    uint8_t* pb = (uint8_t*)std::malloc((size_t)std::max<int64_t>(c - b, 1));
    if (!pa || !pb) {
      std::free(pa);
      std::free(pb);
      oom.store(true);
      return;
    }
    std::memcpy(pa, pk.data + a, (size_t)(b - a));
    std::memcpy(pb, pk.data + b, (size_t)(c - b));
    pair_image_ids_out[r] = scm_blob{pa, (size_t)(b - a)};
    tvgs_out[r] = scm_blob{pb, (size_t)(c - b)};
  });
  if (!pool_give(pk.data)) std::free(pk.data);
  if (oom.load()) {
    for (int64_t r = 0; r < batch; ++r) {
      scm_blob_free(&pair_image_ids_out[r]);
      scm_blob_free(&tvgs_out[r]);
    }
    set_error("malloc failed");
    return SCM_E_NOMEM;
  }
  ctx->t_out = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h3).count();
#ifdef SCM_DIAG_HOST_TIMES
  SCM_HT(13);
  {
    static const int ks[] = {0, 3, 4, 5, 6, 7, 8, 9, 10, 11, 14, 15, 12, 13};
    std::string line = "[scm host us]";
    for (size_t i = 1; i < sizeof(ks) / sizeof(ks[0]); ++i)
      line += " " + std::to_string(ks[i]) + ":" +
              std::to_string((int)std::chrono::duration<double, std::micro>(g_ht[ks[i]] - g_ht[ks[0]]).count());
    line += " | gpu ev0-3 us";
    for (float u : g_hte_us) line += " " + std::to_string((int)u);
    fprintf(stderr, "%s\n", line.c_str());
  }
#endif
  return SCM_OK;
}

}  // namespace

extern "C" {

int scm_execute_batch(scm_context* ctx, int64_t batch, int64_t stencil_size,
                      const scm_element* image_ids, const scm_element* keypoints,
                      const scm_element* descriptors, scm_blob* pair_image_ids_out,
                      scm_blob* tvgs_out) {
  if (!ctx || batch < 0 || stencil_size < 1 || (batch > 0 && (!pair_image_ids_out || !tvgs_out))) {
    set_error("invalid arguments");
    return SCM_E_INVALID;
  }
  if (batch == 0) return SCM_OK;
  SCM_HIP(hipSetDevice(ctx->device));
  const int64_t ne = batch * stencil_size;
  std::vector<RowView> rows;
  SCM_TRY(decode_rows(ne, image_ids, keypoints, descriptors, &rows));
  const int rc = execute_rows(ctx, batch, stencil_size, rows, true, pair_image_ids_out, tvgs_out);
  if (rc != kRetryKeys) return rc;
  return execute_rows(ctx, batch, stencil_size, rows, false, pair_image_ids_out, tvgs_out);
}

int scm_execute_stencil(scm_context* ctx, int64_t stencil_size, const scm_element* image_ids,
                        const scm_element* keypoints, const scm_element* descriptors,
                        scm_blob* pair_image_ids_out, scm_blob* tvgs_out) {
  return scm_execute_batch(ctx, 1, stencil_size, image_ids, keypoints, descriptors,
                           pair_image_ids_out, tvgs_out);
}

int scm_stencil_stats(scm_context* ctx, int64_t* reused, int64_t* uploaded) {
  if (!ctx || !reused || !uploaded) {
    set_error("invalid arguments");
    return SCM_E_INVALID;
  }
  *reused = ctx->call_reused;
  *uploaded = ctx->call_uploaded;
  return SCM_OK;
}

int scm_stencil_spec_stats(scm_context* ctx, int64_t* speculated, int64_t* rejected,
                           int64_t* retried) {
  if (!ctx || !speculated || !rejected || !retried) {
    set_error("invalid arguments");
    return SCM_E_INVALID;
  }
  *speculated = ctx->spec_elems;
  *rejected = ctx->spec_rejected;
  *retried = ctx->spec_retries;
  return SCM_OK;
}

int scm_stencil_cache_clear(scm_context* ctx) {
  if (!ctx) {
    set_error("null context");
    return SCM_E_INVALID;
  }
  SCM_HIP(hipSetDevice(ctx->device));
  drain(ctx);
  ctx->call_cur = -1;
  for (int i = 0; i < 2; ++i) {
    ctx->call_tab[i].release();
    ctx->call_map[i].clear();
  }
  ctx->spec_keys.clear();
  return SCM_OK;
}

int scm_table_load(scm_context* ctx, int64_t num_rows, const scm_element* image_ids,
                   const scm_element* keypoints, const scm_element* descriptors) {
  if (!ctx) {
    set_error("null context");
    return SCM_E_INVALID;
  }
  SCM_HIP(hipSetDevice(ctx->device));
  std::vector<RowView> rows;
  SCM_TRY(decode_rows(num_rows, image_ids, keypoints, descriptors, &rows));
  ctx->table_loaded = false;
  SCM_TRY(upload_table(ctx, &ctx->table, rows, true, true));
  ctx->table_loaded = true;
  return SCM_OK;
}

static int table_run_common(scm_context* ctx, int64_t overlap, int64_t row_begin, int64_t row_end,
                            Packed* pk, const PassEmit* chunk_emit = nullptr) {
  if (!ctx->table_loaded) {
    set_error("scm_table_run before scm_table_load");
    return SCM_E_STATE;
  }
  if (overlap < 1 || row_begin < 0 || row_end > ctx->table.n || row_begin > row_end) {
    set_error("invalid row range / overlap");
    return SCM_E_INVALID;
  }
  SCM_HIP(hipSetDevice(ctx->device));
  ctx->t_match = ctx->t_final = ctx->t_verify = ctx->t_score = 0.0;
  ctx->evals_f = ctx->evals_h = 0;
  ctx->spec_taken = ctx->spec_equal = ctx->spec_differ = ctx->spec_void = 0;
  ctx->n_match_launches = 0;
  const auto w0 = std::chrono::steady_clock::now();
  const int rc = run_table(ctx, overlap, row_begin, row_end, pk, chunk_emit);
  if (rc != SCM_OK) drain(ctx);
  ctx->t_wall =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
  return rc;
}

int scm_table_run(scm_context* ctx, int64_t overlap, int64_t row_begin, int64_t row_end,
                  scm_blob* pair_image_ids_out, scm_blob* tvgs_out) {
  if (!ctx || ((!pair_image_ids_out || !tvgs_out) && row_end > row_begin)) {
    set_error("invalid arguments");
    return SCM_E_INVALID;
  }
  Packed pk;
  const int rc = table_run_common(ctx, overlap, row_begin, row_end, &pk);
  if (rc != SCM_OK) {
    if (!pool_give(pk.data)) std::free(pk.data);
    return rc;
  }
  const int64_t nrows = row_end - row_begin;
  for (int64_t r = 0; r < nrows; ++r) {
    const int64_t a = pk.row_off[2 * r], b = pk.row_off[2 * r + 1], c = pk.row_off[2 * r + 2];
    uint8_t* pa = (uint8_t*)std::malloc((size_t)(b - a));
    uint8_t* pb = (uint8_t*)std::malloc((size_t)(c - b));
    if (!pa || !pb) {
      std::free(pa);
      std::free(pb);
      for (int64_t q = 0; q < r; ++q) {
        scm_blob_free(&pair_image_ids_out[q]);
        scm_blob_free(&tvgs_out[q]);
      }
      if (!pool_give(pk.data)) std::free(pk.data);
      set_error("malloc failed");
      return SCM_E_NOMEM;
    }
    std::memcpy(pa, pk.data + a, (size_t)(b - a));
    std::memcpy(pb, pk.data + b, (size_t)(c - b));
    pair_image_ids_out[r] = scm_blob{pa, (size_t)(b - a)};
    tvgs_out[r] = scm_blob{pb, (size_t)(c - b)};
  }
  if (!pool_give(pk.data)) std::free(pk.data);
  return SCM_OK;
}

int scm_table_run_chunks(scm_context* ctx, int64_t overlap, int64_t row_begin, int64_t row_end,
                         scm_chunk_fn on_chunk, void* user) {
  if (!ctx || !on_chunk) {
    set_error("invalid arguments");
    return SCM_E_INVALID;
  }
  const PassEmit emit = [&](int64_t row0, Packed& pk) -> int {
    const int64_t nrows = ((int64_t)pk.row_off.size() - 1) / 2;
    scm_blob b{pk.data ? pk.data : (uint8_t*)std::malloc(1), pk.size};
    if (!b.data) {
      set_error("malloc failed");
      return SCM_E_NOMEM;
    }
    pk.data = nullptr;
    pk.size = pk.cap = 0;
    on_chunk(user, row_begin + row0, nrows, b.data, b.size, pk.row_off.data());
    return SCM_OK;
  };
  return table_run_common(ctx, overlap, row_begin, row_end, nullptr, &emit);
}

int scm_table_run_passes(scm_context* ctx, int64_t overlap, int64_t row_begin, int64_t row_end,
                         int64_t passes, scm_pass_fn on_pass, void* user) {
  if (!ctx || !on_pass || passes < 0) {
    set_error("invalid arguments");
    return SCM_E_INVALID;
  }
  if (!ctx->table_loaded) {
    set_error("scm_table_run_passes before scm_table_load");
    return SCM_E_STATE;
  }
  if (overlap < 1 || row_begin < 0 || row_end > ctx->table.n || row_begin > row_end) {
    set_error("invalid row range / overlap");
    return SCM_E_INVALID;
  }
  const int64_t n = row_end - row_begin;
  auto hand_over = [&](int64_t k, Packed& pk) -> int {
    scm_blob b{pk.data ? pk.data : (uint8_t*)std::malloc(1), pk.size};
    if (!b.data) {
      set_error("malloc failed");
      return SCM_E_NOMEM;
    }
    pk.data = nullptr;
    pk.size = pk.cap = 0;
    on_pass(user, k, b.data, b.size, pk.row_off.data());
    std::vector<int64_t>().swap(pk.row_off);
    return SCM_OK;
  };
  if (n == 0 || passes == 0) {
    for (int64_t k = 0; k < passes; ++k) {
      Packed pk;
      pk.row_off.push_back(0);
      SCM_TRY(hand_over(k, pk));
    }
    return SCM_OK;
  }
  SCM_HIP(hipSetDevice(ctx->device));
  ctx->t_match = ctx->t_final = ctx->t_verify = ctx->t_score = 0.0;
  ctx->evals_f = ctx->evals_h = 0;
  ctx->spec_taken = ctx->spec_equal = ctx->spec_differ = ctx->spec_void = 0;
  ctx->n_match_launches = 0;
  const auto w0 = std::chrono::steady_clock::now();
  // the stencil plan of the range (run_table), repeated `passes` times
  const ImageTable& t = ctx->table;
  std::vector<RowPlan> plan;
  plan.reserve((size_t)(n * passes));
  {
    std::vector<uint32_t> ids(overlap);
    std::vector<int64_t> rows(overlap), sel;
    for (int64_t r = row_begin; r < row_end; ++r) {
      for (int64_t s2 = 0; s2 < overlap; ++s2) {
        rows[s2] = std::min(r + s2, t.n - 1);
        ids[s2] = t.ids[rows[s2]];
      }
      row_pairs(ids, &sel);
      RowPlan rp;
      rp.pivot = (int32_t)r;
      for (int64_t s2 : sel) {
        rp.nb.push_back((int32_t)rows[s2]);
        rp.nb_ids.push_back(ids[s2]);
      }
      plan.push_back(std::move(rp));
    }
  }
  for (int64_t k = 1; k < passes; ++k)
    for (int64_t i = 0; i < n; ++i) plan.push_back(plan[i]);
  const PassEmit emit = hand_over;
  const int rc = run_rows(ctx, t, plan, row_begin, nullptr, n, &emit);
  if (rc != SCM_OK) drain(ctx);
  ctx->t_wall =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
  return rc;
}

int scm_table_run_packed(scm_context* ctx, int64_t overlap, int64_t row_begin, int64_t row_end,
                         scm_blob* rows_out, int64_t* row_offsets) {
  if (!ctx || !rows_out || !row_offsets) {
    set_error("invalid arguments");
    return SCM_E_INVALID;
  }
  Packed pk;
  const int rc = table_run_common(ctx, overlap, row_begin, row_end, &pk);
  if (rc != SCM_OK) {
    std::free(pk.data);
    return rc;
  }
  std::memcpy(row_offsets, pk.row_off.data(), pk.row_off.size() * sizeof(int64_t));
  rows_out->data = pk.data ? pk.data : (uint8_t*)std::malloc(1);
  rows_out->size = pk.size;
  return SCM_OK;
}

int scm_extract_frames(scm_context* ctx, int64_t n, const uint64_t* image_ids,
                       const scm_frame* frames, scm_blob* keypoints_out,
                       scm_blob* descriptors_out, scm_blob* cameras_out) {
  if (!ctx) {
    set_error("null context");
    return SCM_E_INVALID;
  }
  // the slots run on the context's four streams (one hardware queue each:
  // streams beyond GPU_MAX_HW_QUEUES share one and serialise, 418 vs 570
  // frames/s)
  const hipStream_t lent[kSiftSlotStreams] = {ctx->stream, ctx->sets[0].vstream,
                                              ctx->sets[1].vstream, ctx->sets[2].vstream};
  return sift_extract_frames(&ctx->sift, ctx->device, lent, n,
                             image_ids, frames, keypoints_out, descriptors_out, cameras_out);
}

int scm_set_serial(scm_context* ctx, int32_t serial) {
  if (!ctx) {
    set_error("null context");
    return SCM_E_INVALID;
  }
  ctx->serial = serial != 0;
  return SCM_OK;
}

int scm_set_keep_matches(scm_context* ctx, int32_t keep) {
  if (!ctx) {
    set_error("null context");
    return SCM_E_INVALID;
  }
  ctx->keep_matches = keep != 0;
  ctx->keep_ranges.assign(1, {0, INT64_MAX});
  if (!keep) ctx->last_matches.clear();
  return SCM_OK;
}

int scm_set_keep_matches_range(scm_context* ctx, int64_t row_begin, int64_t row_end) {
  if (!ctx || row_begin < 0 || row_end < row_begin) {
    set_error("invalid arguments");
    return SCM_E_INVALID;
  }
  ctx->keep_matches = row_end > row_begin;
  ctx->keep_ranges.assign(1, {row_begin, row_end});
  if (!ctx->keep_matches) ctx->last_matches.clear();
  return SCM_OK;
}

int scm_add_keep_matches_range(scm_context* ctx, int64_t row_begin, int64_t row_end) {
  if (!ctx || row_begin < 0 || row_end < row_begin) {
    set_error("invalid arguments");
    return SCM_E_INVALID;
  }
  if (row_end > row_begin) {
    if (!ctx->keep_matches) ctx->keep_ranges.clear();
    ctx->keep_ranges.push_back({row_begin, row_end});
    ctx->keep_matches = true;
  }
  return SCM_OK;
}

int scm_table_matches(scm_context* ctx, int64_t row, int64_t offset, uint32_t* matches,
                      int64_t cap, int64_t* num_matches) {
  if (!ctx || !num_matches) {
    set_error("invalid arguments");
    return SCM_E_INVALID;
  }
  if (!ctx->keep_matches) {
    set_error("call scm_set_keep_matches(ctx, 1) before scm_table_run");
    return SCM_E_STATE;
  }
  if (row < ctx->last_begin || row >= ctx->last_end || !ctx->kept(row) ||
      ctx->last_matches.size() != (size_t)(ctx->last_end - ctx->last_begin)) {
    set_error("row outside the last scm_table_run");
    return SCM_E_INVALID;
  }
  for (const auto& e : ctx->last_matches[row - ctx->last_begin]) {
    if (e.first != offset) continue;
    *num_matches = (int64_t)e.second.size();
    if (*num_matches > cap) {
      set_error("match buffer too small");
      return SCM_E_CAPACITY;
    }
    if (*num_matches > 0) {
      if (!matches) {
        set_error("null match buffer");
        return SCM_E_INVALID;
      }
      std::memcpy(matches, e.second.data(), e.second.size() * sizeof(Match));
    }
    return SCM_OK;
  }
  set_error("no pair (row, row + offset) in the last run");
  return SCM_E_INVALID;
}

int scm_table_timings(scm_context* ctx, double* t, int32_t n) {
  if (!ctx || !t) {
    set_error("invalid arguments");
    return SCM_E_INVALID;
  }
  const double v[16] = {ctx->t_match, ctx->t_final, ctx->t_verify, ctx->t_wall,
                        (double)ctx->n_match_launches, ctx->t_score, (double)ctx->evals_f,
                        (double)ctx->evals_h, ctx->t_hash, ctx->t_stage, ctx->t_run, ctx->t_out,
                        (double)ctx->spec_taken, (double)ctx->spec_equal, (double)ctx->spec_differ,
                        (double)ctx->spec_void};
  for (int32_t i = 0; i < n && i < 16; ++i) t[i] = v[i];
  return SCM_OK;
}

}  // extern "C"
