// io.cc byte formats (reference integration/op_cpp/io.cc) and the proto2
// decoding of SequentialMatchingArgs (reference colmap.proto:6-65,
// sequential_matching.cc:36-76) for the product library.
#include <malloc.h>

#include <cstdlib>
#include <mutex>
#include <string>

#include "geom_solvers.h"
#include "scm_internal.h"

namespace scm {

namespace {
template <typename T>
void put(std::vector<uint8_t>* b, const T& v) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
  b->insert(b->end(), p, p + sizeof(T));
}
}  // namespace

// Input row decoders:
//   read_single_from_element<image_t>       io.cc:67-69  (low 4 bytes of the size_t id)
//   read_vector_from_element<FeatureKeypoints> io.cc:115-147 (size_t n, n x 24 B)
//   read_matrix_from_element<FeatureDescriptors> io.cc:180-194 (size_t rows, cols, u8)
int decode_row(const scm_element& id, const scm_element& kp, const scm_element& desc,
               RowView* out) {
  if (!id.buffer || !kp.buffer || !desc.buffer) {
    set_error("null element buffer");
    return SCM_E_INVALID;
  }
  if (id.size < 4 || kp.size < 8 || desc.size < 16) {
    set_error("element too small");
    return SCM_E_INVALID;
  }
  std::memcpy(&out->id, id.buffer, 4);
  uint64_t n = 0;
  std::memcpy(&n, kp.buffer, 8);
  if (n > (kp.size - 8) / 24) {
    set_error("keypoints element shorter than its size prefix");
    return SCM_E_INVALID;
  }
  out->nkp = (int64_t)n;
  out->kp = reinterpret_cast<const float*>(kp.buffer + 8);
  uint64_t rows = 0, cols = 0;
  std::memcpy(&rows, desc.buffer, 8);
  std::memcpy(&cols, desc.buffer + 8, 8);
  if (cols != 128) {
    set_error("descriptor matrix must have 128 columns");
    return SCM_E_INVALID;
  }
  if (rows > (desc.size - 16) / 128) {
    set_error("descriptors element shorter than its shape prefix");
    return SCM_E_INVALID;
  }
  out->ndesc = (int64_t)rows;
  out->desc = desc.buffer + 16;
  return SCM_OK;
}

// One TwoViewGeometry as create_two_view_geometries_buffer writes it
// (io.cc:279-292): int config, E, F, H (Eigen column-major), qvec[4],
// tvec[3], tri_angle, size_t n, n x {uint32, uint32}.  E / qvec / tvec are
// never assigned on the uncalibrated path; they are written as zeros.
void append_tvg(std::vector<uint8_t>* b, const Tvg& t) {
  put<int32_t>(b, t.config);
  for (int i = 0; i < 9; ++i) put<double>(b, 0.0);
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) put<double>(b, t.F[3 * r + c]);
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) put<double>(b, t.H[3 * r + c]);
  for (int i = 0; i < 7; ++i) put<double>(b, 0.0);
  put<double>(b, t.tri_angle);
  put<uint64_t>(b, (uint64_t)t.inlier_matches.size());
  const uint8_t* p = reinterpret_cast<const uint8_t*>(t.inlier_matches.data());
  b->insert(b->end(), p, p + t.inlier_matches.size() * sizeof(Match));
}

// create_two_view_geometries_buffer (io.cc:256-297).
std::vector<uint8_t> tvg_list_bytes(const std::vector<Tvg>& list) {
  std::vector<uint8_t> body;
  for (const Tvg& t : list) append_tvg(&body, t);
  std::vector<uint8_t> b;
  b.reserve(12 + body.size());
  put<uint64_t>(&b, (uint64_t)(sizeof(uint64_t) + sizeof(int32_t) + body.size()));
  put<int32_t>(&b, (int32_t)list.size());
  b.insert(b.end(), body.begin(), body.end());
  return b;
}

// createVectorBuffer<vector<image_t>> (io.cc:151-162).
std::vector<uint8_t> id_list_bytes(const std::vector<uint32_t>& ids) {
  std::vector<uint8_t> b;
  put<uint64_t>(&b, (uint64_t)ids.size());
  for (uint32_t id : ids) put<uint32_t>(&b, id);
  return b;
}

int make_blob(const std::vector<uint8_t>& bytes, scm_blob* out) {
  if (!out) {
    set_error("null output blob");
    return SCM_E_INVALID;
  }
  out->data = (uint8_t*)std::malloc(bytes.empty() ? 1 : bytes.size());
  if (!out->data) {
    set_error("malloc failed");
    return SCM_E_NOMEM;
  }
  if (!bytes.empty()) std::memcpy(out->data, bytes.data(), bytes.size());
  out->size = bytes.size();
  return SCM_OK;
}

}  // namespace scm

// ---------------------------------------------------------------------------
// Options.
// ---------------------------------------------------------------------------
extern "C" void scm_default_options(scm_matching_options* o) {
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

namespace {

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  uint64_t varint() {
    uint64_t v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      if (p >= end) { ok = false; return 0; }
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7F) << shift;
      if (!(b & 0x80)) return v;
    }
    ok = false;
    return 0;
  }
  template <typename T> T fixed() {
    T v{};
    if (end - p < (ptrdiff_t)sizeof(T)) { ok = false; return v; }
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  bool skip(int wt) {
    switch (wt) {
      case 0: varint(); return ok;
      case 1: if (end - p < 8) return ok = false; p += 8; return true;
      case 2: { const uint64_t n = varint(); if (!ok || (uint64_t)(end - p) < n) return ok = false; p += n; return true; }
      case 5: if (end - p < 4) return ok = false; p += 4; return true;
      default: return ok = false;
    }
  }
};

bool parse_sift_args(const uint8_t* b, size_t n, scm_matching_options* o) {
  Reader r{b, b + n};
  while (r.ok && r.p < r.end) {
    const uint64_t tag = r.varint();
    if (!r.ok) break;
    const int field = (int)(tag >> 3), wt = (int)(tag & 7);
    switch (field) {
      case 1: if (wt != 0) return false; o->use_gpu = r.varint() != 0; break;
      case 2: {
        if (wt != 2) return false;
        const uint64_t len = r.varint();
        if (!r.ok || (uint64_t)(r.end - r.p) < len) return false;
        o->gpu_index = (int32_t)std::atoi(std::string((const char*)r.p, (size_t)len).c_str());
        r.p += len;
        break;
      }
      case 3: if (wt != 1) return false; o->max_ratio = r.fixed<double>(); break;
      case 4: if (wt != 1) return false; o->max_distance = r.fixed<double>(); break;
      case 5: if (wt != 0) return false; o->cross_check = r.varint() != 0; break;
      case 6: if (wt != 0) return false; o->max_num_matches = (int32_t)r.varint(); break;
      case 7: if (wt != 5) return false; o->max_error = r.fixed<float>(); break;
      case 8: if (wt != 1) return false; o->confidence = r.fixed<double>(); break;
      case 9: if (wt != 0) return false; o->min_num_trials = (int32_t)r.varint(); break;
      case 10: if (wt != 0) return false; o->max_num_trials = (int32_t)r.varint(); break;
      case 11: if (wt != 1) return false; o->min_inlier_ratio = r.fixed<double>(); break;
      case 12: if (wt != 0) return false; o->min_num_inliers = (int32_t)r.varint(); break;
      case 13: if (wt != 0) return false; o->multiple_models = r.varint() != 0; break;
      case 14: if (wt != 0) return false; o->guided_matching = r.varint() != 0; break;
      default: if (!r.skip(wt)) return false;
    }
  }
  return r.ok;
}

}  // namespace

// SequentialMatchingArgs::ParseFromArray + parseConfigs
// (sequential_matching.cc:36-76): proto2 wire format, unknown fields skipped,
// absent fields keep their defaults.
extern "C" int scm_parse_args(const uint8_t* bytes, size_t size, scm_matching_options* o) {
  scm_default_options(o);
  if (size == 0) return SCM_OK;
  if (!bytes) {
    scm::set_error("null args buffer");
    return SCM_E_INVALID;
  }
  Reader r{bytes, bytes + size};
  while (r.ok && r.p < r.end) {
    const uint64_t tag = r.varint();
    if (!r.ok) break;
    const int field = (int)(tag >> 3), wt = (int)(tag & 7);
    switch (field) {
      case 1: if (wt != 0) goto bad; o->loop_detection = r.varint() != 0; break;
      case 2: if (wt != 0) goto bad; o->overlap = (int32_t)r.varint(); break;
      case 3: if (wt != 0) goto bad; o->quadratic_overlap = r.varint() != 0; break;
      case 4: {
        if (wt != 2) goto bad;
        const uint64_t len = r.varint();
        if (!r.ok || (uint64_t)(r.end - r.p) < len) goto bad;
        if (!parse_sift_args(r.p, (size_t)len, o)) goto bad;
        r.p += len;
        break;
      }
      default: if (!r.skip(wt)) goto bad;
    }
  }
  if (r.ok) return SCM_OK;
bad:
  scm::set_error("malformed SequentialMatchingArgs bytes");
  return SCM_E_INVALID;
}

extern "C" uint32_t scm_pair_seed(uint32_t base, uint32_t id1, uint32_t id2) {
  return scm::geom::pair_seed(base, id1, id2);
}

// Recycled output buffers: a packed table-run result is hundreds of MB, and
// the first touch of freshly mapped pages costs the host ~50 ms per step.
// scm_blob_free parks up to two large blocks here and the next packed run
// writes into one of them (its pages are already mapped).
namespace scm {
namespace {
std::mutex g_pool_mu;
void* g_pool[2] = {nullptr, nullptr};
constexpr size_t kPoolMin = 16u << 20;
}  // namespace

void* pool_take(size_t* cap) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  int best = -1;
  for (int i = 0; i < 2; ++i)
    if (g_pool[i] && (best < 0 || malloc_usable_size(g_pool[i]) > malloc_usable_size(g_pool[best])))
      best = i;
  if (best < 0) return nullptr;
  void* p = g_pool[best];
  g_pool[best] = nullptr;
  *cap = malloc_usable_size(p);
  return p;
}

bool pool_give(void* p) {
  if (!p || malloc_usable_size(p) < kPoolMin) return false;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (int i = 0; i < 2; ++i)
    if (!g_pool[i]) {
      g_pool[i] = p;
      return true;
    }
  return false;
}
}  // namespace scm

extern "C" void scm_blob_free(scm_blob* b) {
  if (!b) return;
  if (!scm::pool_give(b->data)) std::free(b->data);
  b->data = nullptr;
  b->size = 0;
}
