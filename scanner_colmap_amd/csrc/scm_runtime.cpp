// Host runtime of the MI355X sequential-matching stage: implements the C ABI
// of include/scm.h on top of the two HIP kernels (match_kernels.hip,
// verify_kernels.hip).  Mirrors SequentialMatchingCPUKernel
// (reference integration/op_cpp/sequential_matching.cc:27-205): one context
// = one kernel instance bound to one device with its own stream and HBM
// workspace; execute() over a stencil, or the batched table path that keeps
// every descriptor resident in HBM and runs all pairs of a row range in
// large launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "geom_solvers.h"
#include "scm_internal.h"
#include "verify_kernels.h"

namespace scm {

thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

namespace {

constexpr int64_t kMaxPairsPerBatch = 4096;

struct ImageTable {
  int64_t n = 0;
  std::vector<uint32_t> ids;
  std::vector<int32_t> nkp, ndesc;
  std::vector<int64_t> desc_row;  // first (padded) bf16 descriptor row
  std::vector<int64_t> kp_off;    // first float2 keypoint
  std::vector<uint64_t> max_norm2;
  int64_t total_rows = 0, total_kp = 0;
  DevBuf desc;   // uint16 bf16 [total_rows][128]
  DevBuf kpxy;   // float2 [total_kp]
  DevBuf u8;     // upload staging
  void release() {
    desc.release();
    kpxy.release();
    u8.release();
  }
};

struct PairSpec {
  int32_t a, b;  // image indices in the table
};

struct PairResult {
  std::vector<Match> matches;
  VerifyOut vo;
  std::vector<uint8_t> mask;
};

}  // namespace
}  // namespace scm

using namespace scm;

struct scm_context {
  int device = 0;
  hipStream_t stream = nullptr;
  scm_matching_options opts;
  std::vector<float> lut_host;
  DevBuf lut;
  ImageTable table, scratch_table;
  bool table_loaded = false;
  // matcher workspace
  DevBuf d_jobs, d_pairs, d_rowres, d_colpart, d_m21, d_matches, d_counts;
  // verification workspace
  DevBuf d_gpairs, d_vpairs, d_xy1, d_xy2, d_packed, d_scratch, d_idx, d_masks, d_vout;
  HostBuf h_stage;
  // diagnostic phase profile of the verify kernel (SCM_PROFILE=1)
  bool profile = false;
  DevBuf d_prof;
  std::vector<uint64_t> prof_sum;
  int64_t prof_pairs = 0;
  hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  double t_match = 0, t_final = 0, t_verify = 0, t_wall = 0;
  // last table run, for scm_table_matches
  int64_t last_begin = 0, last_end = 0, last_overlap = 0;
  std::vector<std::vector<std::pair<int64_t, std::vector<Match>>>> last_matches;
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
    if (with_desc) total_rows += (r.ndesc + 31) / 32 * 32;
    if (with_kp) total_kp += r.nkp;
  }
  t->total_rows = total_rows;
  t->total_kp = total_kp;
  if (with_desc && total_rows > 0) {
    const size_t bytes = (size_t)total_rows * 128;
    SCM_TRY(ctx->h_stage.ensure(bytes));
    uint8_t* h = ctx->h_stage.as<uint8_t>();
    for (int64_t i = 0; i < t->n; ++i) {
      const RowView& r = rows[i];
      uint8_t* dst = h + (size_t)t->desc_row[i] * 128;
      const size_t nb = (size_t)r.ndesc * 128;
      std::memcpy(dst, r.desc, nb);
      const size_t padded = (size_t)((r.ndesc + 31) / 32 * 32) * 128;
      std::memset(dst + nb, 0, padded - nb);
      uint64_t mx = 0;
      for (int64_t k = 0; k < r.ndesc; ++k) {
        const uint8_t* d = r.desc + k * 128;
        uint32_t s = 0;
        for (int j = 0; j < 128; ++j) s += (uint32_t)d[j] * d[j];
        mx = std::max<uint64_t>(mx, s);
      }
      t->max_norm2[i] = mx;
    }
    SCM_TRY(t->u8.ensure(bytes));
    SCM_TRY(t->desc.ensure(bytes * 2));
    SCM_HIP(hipMemcpyAsync(t->u8.ptr, h, bytes, hipMemcpyHostToDevice, ctx->stream));
    SCM_HIP(launch_u8_to_bf16(t->u8.as<uint8_t>(), t->desc.as<uint16_t>(), (int64_t)bytes,
                              ctx->stream));
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

VerifyParams make_params(const scm_matching_options& o) {
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
  p.base_seed = o.ransac_seed;
  // RANSAC constructor: max_num_trials capped by ComputeNumTrials at the
  // assumed min_inlier_ratio over 1e5 samples [upstream optim/ransac.h].
  auto cap = [&](double ratio, int kmin) {
    const uint64_t kNumSamples = 100000;
    const uint64_t dyn = geom::num_trials((uint64_t)(ratio * (double)kNumSamples), kNumSamples,
                                          o.confidence, o.dyn_num_trials_multiplier, kmin);
    const uint64_t m = std::min<uint64_t>((uint64_t)std::max(0, o.max_num_trials), dyn);
    return (int32_t)std::min<uint64_t>(m, 0x7FFFFFFF);
  };
  p.max_trials_F = cap(o.min_inlier_ratio, 7);
  p.max_trials_H = cap(o.min_inlier_ratio, 4);
  p.max_trials_T = cap(o.watermark_min_inlier_ratio, 1);
  return p;
}

double event_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0.0;
  return (double)ms;
}

// Descriptor matching of the given pairs (pairs of one pivot consecutive).
// Leaves per-pair matches on the device at PairDesc.match_off and counts in
// d_counts; returns host copies of both descriptors arrays for the verifier.
int match_stage(scm_context* ctx, const ImageTable& t, const std::vector<PairSpec>& specs,
                std::vector<PairDesc>* pds_out, std::vector<int32_t>* counts_out) {
  const int64_t P = (int64_t)specs.size();
  std::vector<PairDesc> pds(P);
  std::vector<MatchJob> jobs_fast, jobs_clamp;
  int64_t rr = 0, cp = 0, m21 = 0, mo = 0;
  std::vector<char> active(P, 0);
  // Active pairs are packed first so the finalize grid covers exactly them.
  std::vector<int64_t> order;
  for (int64_t i = 0; i < P; ++i)
    if (t.ndesc[specs[i].a] > 0 && t.ndesc[specs[i].b] > 0) active[i] = 1;
  int64_t i = 0;
  std::vector<PairDesc> packed;
  std::vector<int64_t> packed_src;
  while (i < P) {
    const int32_t a = specs[i].a;
    int64_t j = i;
    while (j < P && specs[j].a == a) ++j;
    const int32_t pair0 = (int32_t)packed.size();
    bool clamp = false;
    int32_t np = 0;
    for (int64_t k = i; k < j; ++k) {
      if (!active[k]) continue;
      const int32_t b = specs[k].b;
      PairDesc pd;
      std::memset(&pd, 0, sizeof(pd));
      pd.n1 = t.ndesc[a];
      pd.n2 = t.ndesc[b];
      pd.n2pad = (pd.n2 + 31) / 32 * 32;
      pd.nseg = (pd.n2 + kColsPerSeg - 1) / kColsPerSeg;
      pd.nrb = (pd.n1 + kRowsPerBlock - 1) / kRowsPerBlock;
      pd.b_row = t.desc_row[b];
      pd.rowres_off = rr;
      pd.colpart_off = cp;
      pd.m21_off = m21;
      pd.match_off = mo;
      rr += (int64_t)pd.nseg * pd.n1;
      cp += (int64_t)pd.nrb * pd.n2pad;
      m21 += pd.n2;
      mo += pd.n1;
      // |a||b| < 2^19 for every row pair  <=>  max|a|^2 * max|b|^2 < 2^38.
      const unsigned __int128 prod = (unsigned __int128)t.max_norm2[a] * t.max_norm2[b];
      if (prod >= ((unsigned __int128)1 << 38)) clamp = true;
      packed.push_back(pd);
      packed_src.push_back(k);
      ++np;
    }
    if (np > 0) {
      const int32_t n1 = t.ndesc[a];
      const int32_t nrb = (n1 + kRowsPerBlock - 1) / kRowsPerBlock;
      for (int32_t rb = 0; rb < nrb; ++rb) {
        MatchJob jb;
        jb.a_row = t.desc_row[a];
        jb.rb = rb;
        jb.n1 = n1;
        jb.pair0 = pair0;
        jb.npairs = np;
        (clamp ? jobs_clamp : jobs_fast).push_back(jb);
      }
    }
    i = j;
  }
  const int64_t PA = (int64_t)packed.size();
  pds_out->assign(P, PairDesc());
  counts_out->assign(P, 0);
  for (int64_t k = 0; k < PA; ++k) (*pds_out)[packed_src[k]] = packed[k];
  if (PA == 0) return SCM_OK;
  const int64_t nj = (int64_t)(jobs_fast.size() + jobs_clamp.size());
  SCM_TRY(ctx->d_jobs.ensure(nj * sizeof(MatchJob)));
  SCM_TRY(ctx->d_pairs.ensure(PA * sizeof(PairDesc)));
  SCM_TRY(ctx->d_rowres.ensure(std::max<int64_t>(rr, 1) * sizeof(uint2)));
  SCM_TRY(ctx->d_colpart.ensure(std::max<int64_t>(cp, 1) * sizeof(uint2)));
  SCM_TRY(ctx->d_m21.ensure(std::max<int64_t>(m21, 1) * sizeof(int32_t)));
  SCM_TRY(ctx->d_matches.ensure(std::max<int64_t>(mo, 1) * sizeof(uint2)));
  SCM_TRY(ctx->d_counts.ensure(PA * sizeof(int32_t)));
  std::vector<MatchJob> jobs(jobs_fast);
  jobs.insert(jobs.end(), jobs_clamp.begin(), jobs_clamp.end());
  SCM_HIP(hipMemcpyAsync(ctx->d_jobs.ptr, jobs.data(), nj * sizeof(MatchJob),
                         hipMemcpyHostToDevice, ctx->stream));
  SCM_HIP(hipMemcpyAsync(ctx->d_pairs.ptr, packed.data(), PA * sizeof(PairDesc),
                         hipMemcpyHostToDevice, ctx->stream));
  SCM_HIP(hipEventRecord(ctx->ev[0], ctx->stream));
  SCM_HIP(launch_match_tiles(t.desc.as<uint16_t>(), ctx->d_jobs.as<MatchJob>(),
                             (int)jobs_fast.size(), ctx->d_pairs.as<PairDesc>(),
                             ctx->d_rowres.as<uint2>(), ctx->d_colpart.as<uint2>(), false,
                             ctx->stream));
  SCM_HIP(launch_match_tiles(t.desc.as<uint16_t>(), ctx->d_jobs.as<MatchJob>() + jobs_fast.size(),
                             (int)jobs_clamp.size(), ctx->d_pairs.as<PairDesc>(),
                             ctx->d_rowres.as<uint2>(), ctx->d_colpart.as<uint2>(), true,
                             ctx->stream));
  SCM_HIP(hipEventRecord(ctx->ev[1], ctx->stream));
  SCM_HIP(launch_match_finalize(ctx->d_pairs.as<PairDesc>(), (int)PA, ctx->d_rowres.as<uint2>(),
                                ctx->d_colpart.as<uint2>(), ctx->d_m21.as<int32_t>(),
                                ctx->lut.as<float>(), (float)ctx->opts.max_ratio,
                                (float)ctx->opts.max_distance, ctx->opts.cross_check,
                                ctx->d_matches.as<uint2>(), ctx->d_counts.as<int32_t>(),
                                ctx->stream));
  SCM_HIP(hipEventRecord(ctx->ev[2], ctx->stream));
  std::vector<int32_t> cnt(PA);
  SCM_HIP(hipMemcpyAsync(cnt.data(), ctx->d_counts.ptr, PA * sizeof(int32_t),
                         hipMemcpyDeviceToHost, ctx->stream));
  SCM_HIP(hipStreamSynchronize(ctx->stream));
  ctx->t_match += event_ms(ctx->ev[0], ctx->ev[1]);
  ctx->t_final += event_ms(ctx->ev[1], ctx->ev[2]);
  for (int64_t k = 0; k < PA; ++k) (*counts_out)[packed_src[k]] = cnt[k];
  return SCM_OK;
}

// Geometry of the given pairs from matches already on the device
// (d_matches at pds[i].match_off, counts[i] entries); fills results.
int verify_stage(scm_context* ctx, const ImageTable& t, const std::vector<PairSpec>& specs,
                 const std::vector<PairDesc>& pds, const std::vector<int32_t>& counts,
                 bool verify, std::vector<PairResult>* results) {
  const int64_t P = (int64_t)specs.size();
  results->assign(P, PairResult());
  std::vector<GatherPair> gp;
  std::vector<VerifyPair> vp;
  std::vector<int64_t> vsrc, gsrc;
  int64_t pts = 0, scr = 0;
  int max_m = 0;
  for (int64_t i = 0; i < P; ++i) {
    const int32_t m = counts[i];
    if (m <= 0) continue;
    if (m > kMaxVerifyMatches) {
      set_error("more than 65535 matches in one pair");
      return SCM_E_INVALID;
    }
    GatherPair g;
    std::memset(&g, 0, sizeof(g));
    g.match_off = pds[i].match_off;
    g.kp1_off = t.kp_off[specs[i].a];
    g.kp2_off = t.kp_off[specs[i].b];
    g.pts_off = pts;
    g.m = m;
    gp.push_back(g);
    gsrc.push_back(i);
    if (verify && m >= ctx->opts.min_num_inliers) {
      VerifyPair v;
      std::memset(&v, 0, sizeof(v));
      v.pts_off = 2 * pts;
      v.scr_off = scr;
      v.mask_off = pts;
      v.m = m;
      v.id1 = t.ids[specs[i].a];
      v.id2 = t.ids[specs[i].b];
      vp.push_back(v);
      vsrc.push_back(i);
      scr += 10 * (int64_t)m + kVerifyModelDoubles;
      max_m = std::max(max_m, m);
    }
    pts += m;
  }
  if (gp.empty()) return SCM_OK;
  const int64_t G = (int64_t)gp.size(), V = (int64_t)vp.size();
  SCM_TRY(ctx->d_gpairs.ensure(G * sizeof(GatherPair)));
  SCM_TRY(ctx->d_xy1.ensure(2 * pts * sizeof(double)));
  SCM_TRY(ctx->d_xy2.ensure(2 * pts * sizeof(double)));
  SCM_TRY(ctx->d_packed.ensure(pts * sizeof(uint2)));
  SCM_TRY(ctx->d_masks.ensure(pts));
  SCM_HIP(hipMemcpyAsync(ctx->d_gpairs.ptr, gp.data(), G * sizeof(GatherPair),
                         hipMemcpyHostToDevice, ctx->stream));
  SCM_HIP(launch_gather(ctx->d_gpairs.as<GatherPair>(), (int)G, ctx->d_matches.as<uint2>(),
                        t.kpxy.as<float2>(), ctx->d_xy1.as<double>(), ctx->d_xy2.as<double>(),
                        ctx->d_packed.as<uint2>(), ctx->stream));
  std::vector<VerifyOut> vout(V);
  if (V > 0) {
    SCM_TRY(ctx->d_vpairs.ensure(V * sizeof(VerifyPair)));
    SCM_TRY(ctx->d_scratch.ensure(std::max<int64_t>(scr, 1) * sizeof(double)));
    SCM_TRY(ctx->d_idx.ensure(V * 640 * sizeof(uint32_t)));
    SCM_TRY(ctx->d_vout.ensure(V * sizeof(VerifyOut)));
    SCM_HIP(hipMemcpyAsync(ctx->d_vpairs.ptr, vp.data(), V * sizeof(VerifyPair),
                           hipMemcpyHostToDevice, ctx->stream));
    const VerifyParams params = make_params(ctx->opts);
    SCM_HIP(hipEventRecord(ctx->ev[3], ctx->stream));
    uint64_t* prof = nullptr;
    if (ctx->profile) {
      SCM_TRY(ctx->d_prof.ensure(V * kVerifyProfSlots * sizeof(uint64_t)));
      SCM_HIP(hipMemsetAsync(ctx->d_prof.ptr, 0, V * kVerifyProfSlots * sizeof(uint64_t),
                             ctx->stream));
      prof = ctx->d_prof.as<uint64_t>();
    }
    SCM_HIP(launch_verify(ctx->d_vpairs.as<VerifyPair>(), (int)V, max_m, ctx->d_xy1.as<double>(),
                          ctx->d_xy2.as<double>(), ctx->d_scratch.as<double>(),
                          ctx->d_idx.as<uint32_t>(), ctx->d_masks.as<uint8_t>(),
                          ctx->d_vout.as<VerifyOut>(), params, prof, ctx->stream));
    SCM_HIP(hipEventRecord(ctx->ev[4], ctx->stream));
    SCM_HIP(hipMemcpyAsync(vout.data(), ctx->d_vout.ptr, V * sizeof(VerifyOut),
                           hipMemcpyDeviceToHost, ctx->stream));
  }
  std::vector<Match> packed(pts);
  std::vector<uint8_t> masks(pts);
  SCM_HIP(hipMemcpyAsync(packed.data(), ctx->d_packed.ptr, pts * sizeof(uint2),
                         hipMemcpyDeviceToHost, ctx->stream));
  SCM_HIP(hipMemcpyAsync(masks.data(), ctx->d_masks.ptr, pts, hipMemcpyDeviceToHost,
                         ctx->stream));
  SCM_HIP(hipStreamSynchronize(ctx->stream));
  if (V > 0) ctx->t_verify += event_ms(ctx->ev[3], ctx->ev[4]);
  if (V > 0 && ctx->profile) {
    std::vector<uint64_t> pr(V * kVerifyProfSlots);
    SCM_HIP(hipMemcpy(pr.data(), ctx->d_prof.ptr, pr.size() * sizeof(uint64_t),
                      hipMemcpyDeviceToHost));
    ctx->prof_sum.resize(kVerifyProfSlots, 0);
    for (int64_t k = 0; k < V; ++k)
      for (int j = 0; j < kVerifyProfSlots; ++j) ctx->prof_sum[j] += pr[k * kVerifyProfSlots + j];
    ctx->prof_pairs += V;
  }
  for (int64_t k = 0; k < G; ++k) {
    PairResult& r = (*results)[gsrc[k]];
    r.matches.assign(packed.begin() + gp[k].pts_off, packed.begin() + gp[k].pts_off + gp[k].m);
  }
  for (int64_t k = 0; k < V; ++k) {
    PairResult& r = (*results)[vsrc[k]];
    r.vo = vout[k];
    r.mask.assign(masks.begin() + vp[k].mask_off, masks.begin() + vp[k].mask_off + vp[k].m);
  }
  return SCM_OK;
}

Tvg to_tvg(const PairResult& r) {
  Tvg t;
  t.config = r.vo.config;
  if (t.config == 0) return t;  // TwoViewGeometry()
  for (int i = 0; i < 9; ++i) {
    t.F[i] = r.vo.F[i];
    t.H[i] = r.vo.H[i];
  }
  for (size_t i = 0; i < r.mask.size(); ++i)
    if (r.mask[i]) t.inlier_matches.push_back(r.matches[i]);
  return t;
}

int run_pairs(scm_context* ctx, const ImageTable& t, const std::vector<PairSpec>& specs,
              bool verify, std::vector<PairResult>* results) {
  std::vector<PairDesc> pds;
  std::vector<int32_t> counts;
  SCM_TRY(match_stage(ctx, t, specs, &pds, &counts));
  return verify_stage(ctx, t, specs, pds, counts, verify, results);
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
  if (opts) o = *opts;
  else scm_default_options(&o);
  if (o.multiple_models) {
    set_error("multiple_models (TwoViewGeometry::EstimateMultiple) is not supported");
    return SCM_E_INVALID;
  }
  scm_context* ctx = new scm_context();
  ctx->device = device_index;
  ctx->opts = o;
  if (const char* e = std::getenv("SCM_PROFILE")) ctx->profile = e[0] == '1';
  if (hipSetDevice(device_index) != hipSuccess ||
      hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    set_error("failed to create HIP stream");
    delete ctx;
    return SCM_E_DEVICE;
  }
  for (auto& e : ctx->ev) (void)hipEventCreate(&e);
  build_lut(&ctx->lut_host);
  if (ctx->lut.ensure(ctx->lut_host.size() * sizeof(float)) != SCM_OK ||
      hipMemcpy(ctx->lut.ptr, ctx->lut_host.data(), ctx->lut_host.size() * sizeof(float),
                hipMemcpyHostToDevice) != hipSuccess) {
    set_error("failed to upload the acosf table");
    scm_context_destroy(ctx);
    return SCM_E_DEVICE;
  }
  *out = ctx;
  return SCM_OK;
}

void scm_context_destroy(scm_context* ctx) {
  if (!ctx) return;
  if (ctx->profile && ctx->prof_pairs > 0) {
    static const char* names[] = {"sample", "solve", "score", "cand_res", "seqsum", "lo_gather",
                                  "lo_est", "lo_res", "other", "n_batch", "n_cand", "n_lo",
                                  "n_trials", "n_points", "n_seqsum", "-"};
    std::fprintf(stderr, "[scm verify profile] pairs=%lld (per pair: cycles / counts)\n",
                 (long long)ctx->prof_pairs);
    for (int j = 0; j < 15; ++j)
      std::fprintf(stderr, "  %-10s %14.1f\n", names[j],
                   (double)ctx->prof_sum[j] / (double)ctx->prof_pairs);
  }
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  ctx->table.release();
  ctx->scratch_table.release();
  for (DevBuf* b : {&ctx->lut, &ctx->d_jobs, &ctx->d_pairs, &ctx->d_rowres, &ctx->d_colpart,
                    &ctx->d_m21, &ctx->d_matches, &ctx->d_counts, &ctx->d_gpairs, &ctx->d_vpairs,
                    &ctx->d_xy1, &ctx->d_xy2, &ctx->d_packed, &ctx->d_scratch, &ctx->d_idx,
                    &ctx->d_masks, &ctx->d_vout, &ctx->d_prof})
    b->release();
  ctx->h_stage.release();
  for (auto& e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
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
  rows[0].id = 1; rows[0].desc = desc1; rows[0].ndesc = n1;
  rows[1].id = 2; rows[1].desc = desc2; rows[1].ndesc = n2;
  SCM_TRY(upload_table(ctx, &ctx->scratch_table, rows, true, false));
  std::vector<PairSpec> specs = {{0, 1}};
  std::vector<PairDesc> pds;
  std::vector<int32_t> counts;
  SCM_TRY(match_stage(ctx, ctx->scratch_table, specs, &pds, &counts));
  *num_matches = counts[0];
  if (counts[0] > cap) {
    set_error("match buffer too small");
    return SCM_E_CAPACITY;
  }
  if (counts[0] > 0) {
    if (!matches) {
      set_error("null match buffer");
      return SCM_E_INVALID;
    }
    SCM_HIP(hipMemcpy(matches, ctx->d_matches.as<uint2>() + pds[0].match_off,
                      (size_t)counts[0] * sizeof(uint2), hipMemcpyDeviceToHost));
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
  rows[0].id = image_id1; rows[0].kp = kp1; rows[0].nkp = n1;
  rows[1].id = image_id2; rows[1].kp = kp2; rows[1].nkp = n2;
  SCM_TRY(upload_table(ctx, &ctx->scratch_table, rows, false, true));
  std::vector<PairSpec> specs = {{0, 1}};
  std::vector<PairDesc> pds(1);
  std::memset(&pds[0], 0, sizeof(PairDesc));
  std::vector<int32_t> counts = {(int32_t)num_matches};
  SCM_TRY(ctx->d_matches.ensure(std::max<int64_t>(num_matches, 1) * sizeof(uint2)));
  if (num_matches > 0)
    SCM_HIP(hipMemcpy(ctx->d_matches.ptr, matches, (size_t)num_matches * sizeof(uint2),
                      hipMemcpyHostToDevice));
  std::vector<PairResult> res;
  SCM_TRY(verify_stage(ctx, ctx->scratch_table, specs, pds, counts, true, &res));
  std::vector<uint8_t> bytes;
  append_tvg(&bytes, to_tvg(res[0]));
  return make_blob(bytes, tvg_out);
}

int scm_execute_stencil(scm_context* ctx, int64_t stencil_size, const scm_element* image_ids,
                        const scm_element* keypoints, const scm_element* descriptors,
                        scm_blob* pair_image_ids_out, scm_blob* tvgs_out) {
  if (!ctx || stencil_size < 1 || !pair_image_ids_out || !tvgs_out) {
    set_error("invalid arguments");
    return SCM_E_INVALID;
  }
  SCM_HIP(hipSetDevice(ctx->device));
  std::vector<RowView> rows;
  SCM_TRY(decode_rows(stencil_size, image_ids, keypoints, descriptors, &rows));
  std::vector<uint32_t> ids(stencil_size);
  for (int64_t i = 0; i < stencil_size; ++i) ids[i] = rows[i].id;
  std::vector<int64_t> sel;
  row_pairs(ids, &sel);
  SCM_TRY(upload_table(ctx, &ctx->scratch_table, rows, true, true));
  std::vector<PairSpec> specs;
  for (int64_t s : sel) specs.push_back({0, (int32_t)s});
  std::vector<PairResult> res;
  SCM_TRY(run_pairs(ctx, ctx->scratch_table, specs, true, &res));
  std::vector<uint32_t> pair_ids;
  std::vector<Tvg> tvgs;
  for (size_t k = 0; k < sel.size(); ++k) {
    pair_ids.push_back(ids[sel[k]]);
    tvgs.push_back(to_tvg(res[k]));
  }
  SCM_TRY(make_blob(id_list_bytes(pair_ids), pair_image_ids_out));
  return make_blob(tvg_list_bytes(tvgs), tvgs_out);
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

int scm_table_run(scm_context* ctx, int64_t overlap, int64_t row_begin, int64_t row_end,
                  scm_blob* pair_image_ids_out, scm_blob* tvgs_out) {
  if (!ctx || !pair_image_ids_out || !tvgs_out) {
    set_error("invalid arguments");
    return SCM_E_INVALID;
  }
  if (!ctx->table_loaded) {
    set_error("scm_table_run before scm_table_load");
    return SCM_E_STATE;
  }
  const ImageTable& t = ctx->table;
  if (overlap < 1 || row_begin < 0 || row_end > t.n || row_begin > row_end) {
    set_error("invalid row range / overlap");
    return SCM_E_INVALID;
  }
  SCM_HIP(hipSetDevice(ctx->device));
  hipEvent_t w0 = ctx->ev[5];
  SCM_HIP(hipEventRecord(w0, ctx->stream));
  ctx->t_match = ctx->t_final = ctx->t_verify = 0.0;
  const int64_t nrows = row_end - row_begin;
  ctx->last_begin = row_begin;
  ctx->last_end = row_end;
  ctx->last_overlap = overlap;
  ctx->last_matches.assign(nrows, {});
  std::vector<std::vector<int64_t>> row_sel(nrows);  // neighbour table rows per output row
  for (int64_t r = row_begin; r < row_end; ++r) {
    std::vector<uint32_t> ids(overlap);
    std::vector<int64_t> rows(overlap);
    for (int64_t s = 0; s < overlap; ++s) {
      rows[s] = std::min(r + s, t.n - 1);  // stencil clamped at the table end
      ids[s] = t.ids[rows[s]];
    }
    std::vector<int64_t> sel;
    row_pairs(ids, &sel);
    for (int64_t s : sel) row_sel[r - row_begin].push_back(rows[s]);
  }
  std::vector<std::vector<Tvg>> tvgs(nrows);
  std::vector<std::vector<uint32_t>> pids(nrows);
  int64_t r = row_begin;
  while (r < row_end) {
    std::vector<PairSpec> specs;
    std::vector<std::pair<int64_t, int64_t>> where;  // (output row, neighbour row)
    while (r < row_end && (specs.empty() ||
                           (int64_t)(specs.size() + row_sel[r - row_begin].size()) <= kMaxPairsPerBatch)) {
      for (int64_t nb : row_sel[r - row_begin]) {
        specs.push_back({(int32_t)r, (int32_t)nb});
        where.push_back({r, nb});
      }
      ++r;
    }
    std::vector<PairResult> res;
    SCM_TRY(run_pairs(ctx, t, specs, true, &res));
    for (size_t k = 0; k < specs.size(); ++k) {
      const int64_t orow = where[k].first - row_begin;
      pids[orow].push_back(t.ids[where[k].second]);
      tvgs[orow].push_back(to_tvg(res[k]));
      ctx->last_matches[orow].push_back({where[k].second - where[k].first, std::move(res[k].matches)});
    }
  }
  for (int64_t k = 0; k < nrows; ++k) {
    SCM_TRY(make_blob(id_list_bytes(pids[k]), &pair_image_ids_out[k]));
    SCM_TRY(make_blob(tvg_list_bytes(tvgs[k]), &tvgs_out[k]));
  }
  SCM_HIP(hipEventRecord(ctx->ev[4], ctx->stream));
  SCM_HIP(hipEventSynchronize(ctx->ev[4]));
  ctx->t_wall = event_ms(w0, ctx->ev[4]);
  return SCM_OK;
}

int scm_table_matches(scm_context* ctx, int64_t row, int64_t offset, uint32_t* matches,
                      int64_t cap, int64_t* num_matches) {
  if (!ctx || !num_matches) {
    set_error("invalid arguments");
    return SCM_E_INVALID;
  }
  if (row < ctx->last_begin || row >= ctx->last_end) {
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
    if (*num_matches > 0) std::memcpy(matches, e.second.data(), e.second.size() * sizeof(Match));
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
  const double v[4] = {ctx->t_match, ctx->t_final, ctx->t_verify, ctx->t_wall};
  for (int32_t i = 0; i < n && i < 4; ++i) t[i] = v[i];
  return SCM_OK;
}

}  // extern "C"
