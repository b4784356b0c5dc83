// Host side of the GPU SIFT extraction: the
// SiftExtractionKernel::execute replacement (reference
// integration/op_cpp/extraction_op.cc:70-121) behind scm_extract_frames.
//
// Per frame: upload (pinned staging), grey + 2x upsampling, the six Gaussian
// levels of each of the 4 octaves, detection / refinement and gradients per
// octave, then orientations and descriptors of every octave's keypoints in one
// launch each (sift_kernels.hip), then the counts and the features come back
// and the host writes the three io.cc elements: COLMAP's DoG-level selection
// of max_num_features (ExtractSiftFeaturesCPU keeps the coarsest levels whose
// keypoint count first exceeds it), FeatureKeypoint(x, y, scale, orientation)
// with the host libm's cosf / sinf, and the extractCamera SIMPLE_RADIAL camera.
// Frames rotate over a few image slots, each with its own stream and HBM
// workspace, so consecutive frames overlap (upload, kernels, read-back).
// A frame larger than max_image_size is first reduced as resizeBitmap does
// (extraction_op.cc:28-39): grey bytes, FreeImage's bilinear rescale by
// 3200 / max(w, h) (host-built weight tables, one GPU pass per axis), then the
// same pipeline on the smaller grey image.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>

#include "scm_internal.h"
#include "sift_kernels.h"

namespace scm {

namespace {

constexpr int kMaxImageSize = 3200;  // SiftExtractionOptions::max_image_size
constexpr int kMaxNumFeatures = 8192;
constexpr double kPeakThreshold = 0.02 / 3;
constexpr double kEdgeThreshold = 10.0;
constexpr int kSlots = kSiftSlotStreams;

struct Slot {
  hipStream_t st = nullptr;
  DevBuf frame, ws, counts, rs, rtab;  // rs: grey + rescale images; rtab: weight tables
  HostBuf pin_in, pin_cnt, pin_out, pin_rtab;
  int rtab_w = 0, rtab_h = 0;  // source size the uploaded tables are for
  SiftDev dev{};
  int64_t nel_cap = 0;  // first-octave pixels the workspace holds
  int64_t cap_scale = 1;  // candidate / keypoint / feature capacities x this (grown on overflow)
  bool caps_at_bound = false;  // every capacity at its hard per-frame bound (no overflow possible)
  int64_t pending = -1; // frame index whose results are in flight
  int w = 0, h = 0;
};

template <typename T>
T* carve(uint8_t*& p, size_t n) {
  T* r = reinterpret_cast<T*>(p);
  p += (n * sizeof(T) + 255) & ~(size_t)255;
  return r;
}

}  // namespace

struct SiftState {
  int device = 0;
  // initial candidate / keypoint / feature capacities (0: sized by the
  // frame); SCM_SIFT_CAPS=c,k,f sets them (tests: force the overflow path)
  int caps[3] = {0, 0, 0};
  DevBuf consts;
  SiftConsts c{};
  int widths[6] = {0, 0, 0, 0, 0, 0};
  Slot slots[kSlots];
  bool own_streams = false;  // slot streams created here (else the context's, borrowed)
};

void sift_state_destroy(SiftState* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  for (Slot& sl : s->slots) {
    if (sl.st) {
      (void)hipStreamSynchronize(sl.st);
      if (s->own_streams) (void)hipStreamDestroy(sl.st);
    }
    sl.frame.release();
    sl.rs.release();
    sl.rtab.release();
    sl.pin_rtab.release();
    sl.ws.release();
    sl.counts.release();
    sl.pin_in.release();
    sl.pin_cnt.release();
    sl.pin_out.release();
  }
  s->consts.release();
  delete s;
}

namespace {

// _vl_sift_smooth's taps for one sigma (host libm exp, as the reference).
int gauss_taps(double sigma, float* g) {
  const int W = std::max((int)std::ceil(4.0 * sigma), 1);
  float acc = 0;
  for (int j = 0; j < 2 * W + 1; ++j) {
    const float d = ((float)(j - W)) / ((float)sigma);
    g[j] = (float)std::exp(-0.5 * (d * d));
    acc += g[j];
  }
  for (int j = 0; j < 2 * W + 1; ++j) g[j] /= acc;
  return W;
}

int init_state(SiftState* s, const hipStream_t* streams) {
  // VLFeat: sigmak = 2^(1/S), sigma0 = 1.6 sigmak, dsigma0 = sigma0 sqrt(1 - 1/sigmak^2),
  // first level of the first octave: sd = sqrt(sa^2 - sb^2), sa = sigma0 sigmak^-1,
  // sb = 0.5 * 2^1; level s: dsigma0 sigmak^s.
  const double sigmak = std::pow(2.0, 1.0 / 3), sigma0 = 1.6 * sigmak;
  const double dsigma0 = sigma0 * std::sqrt(1.0 - 1.0 / (sigmak * sigmak));
  std::vector<float> taps(6 * kSiftMaxTaps, 0.0f);
  const double sa = sigma0 * std::pow(sigmak, -1), sb = 0.5 * std::pow(2.0, 1);
  s->widths[0] = gauss_taps(std::sqrt(sa * sa - sb * sb), taps.data());
  for (int l = 0; l < 5; ++l)
    s->widths[1 + l] = gauss_taps(dsigma0 * std::pow(sigmak, l), taps.data() + (1 + l) * kSiftMaxTaps);
  double expn[257];
  for (int k = 0; k < 257; ++k) expn[k] = std::exp(-(double)k * (25.0 / 256));
  const size_t tb = taps.size() * sizeof(float), wb = 256, eb = sizeof(expn);
  SCM_TRY(s->consts.ensure(tb + wb + eb));
  uint8_t* base = s->consts.as<uint8_t>();
  s->c.taps = reinterpret_cast<float*>(base);
  s->c.widths = reinterpret_cast<int32_t*>(base + tb);
  s->c.expn = reinterpret_cast<double*>(base + tb + wb);
  SCM_HIP(hipMemcpy(s->c.taps, taps.data(), tb, hipMemcpyHostToDevice));
  SCM_HIP(hipMemcpy(s->c.widths, s->widths, sizeof(s->widths), hipMemcpyHostToDevice));
  SCM_HIP(hipMemcpy(s->c.expn, expn, eb, hipMemcpyHostToDevice));
  // The slots run on the context's streams when it lends them: each of those
  // has a hardware queue of its own, while streams created past
  // GPU_MAX_HW_QUEUES share queues, and frames on one queue serialise.
  s->own_streams = streams == nullptr;
  for (int i = 0; i < kSlots; ++i) {
    if (streams) s->slots[i].st = streams[i];
    else SCM_HIP(hipStreamCreateWithFlags(&s->slots[i].st, hipStreamNonBlocking));
  }
  return SCM_OK;
}

// resizeBitmap's target size: scale 3200 / max(w, h), sizes truncated.
void fit_size(int w, int h, int* nw, int* nh) {
  *nw = w;
  *nh = h;
  if (w > kMaxImageSize || h > kMaxImageSize) {
    const double scale = (double)kMaxImageSize / std::max(w, h);
    *nw = (int)(w * scale);
    *nh = (int)(h * scale);
  }
}

// FreeImage 3.17 CWeightsTable of CBilinearFilter (width 1) for a src -> dst
// line: per destination pixel (left, count) and count normalised weights
// (padded to win, the window size table_layout also computes).  Returns win.
int bilinear_table(int dst, int src, std::vector<int32_t>* hdr, std::vector<double>* wt) {
  const double scale = double(dst) / double(src);
  const double width = scale < 1.0 ? 1.0 / scale : 1.0, fscale = scale < 1.0 ? scale : 1.0;
  const int win = 2 * (int)std::ceil(width) + 1;
  const double offset = 0.5 / scale;
  hdr->assign(2 * (size_t)dst, 0);
  wt->assign((size_t)dst * win, 0.0);
  for (int u = 0; u < dst; ++u) {
    const double center = (double)u / scale + offset;
    const int lo = std::max(0, (int)(center - width + 0.5));
    const int hi = std::min((int)(center + width + 0.5), src);
    double* w = wt->data() + (size_t)u * win;
    double total = 0;
    for (int i = lo; i < hi; ++i) {
      const double x = std::fabs(fscale * ((double)i + 0.5 - center));
      w[i - lo] = fscale * (x < 1.0 ? 1.0 - x : 0.0);
      total += w[i - lo];
    }
    if (total > 0 && total != 1)
      for (int i = lo; i < hi; ++i) w[i - lo] /= total;
    int right = hi;
    while (right > lo && w[right - lo - 1] == 0) --right;  // trailing null weights
    (*hdr)[2 * (size_t)u] = lo;
    (*hdr)[2 * (size_t)u + 1] = right - lo;
  }
  return win;
}

// Workspace of a slot for a frame whose first octave has nel pixels (2w x 2h).
// Capacities: candidates of one octave, the frame's refined keypoints (every
// octave's) and their features (<= 2 orientations each), times the slot's
// cap_scale, which grows whenever a frame overflows them (the frame is then
// extracted again: the reference has no capacity limit,
// extraction_op.cc:71-120).
int ensure_slot(const SiftState* s, Slot& sl, int w, int h) {
  const int64_t ow = 2 * (int64_t)w, oh = 2 * (int64_t)h, nel = ow * oh;
  if (nel <= sl.nel_cap && sl.dev.cnt) return SCM_OK;
  const int64_t sc = sl.cap_scale;
  const int64_t c0 = s->caps[0] ? s->caps[0] : std::min<int64_t>(std::max<int64_t>(65536, nel / 16), 1 << 22);
  const int64_t k0 = s->caps[1] ? s->caps[1] : std::min<int64_t>(c0, 1 << 18);
  const int64_t f0 = s->caps[2] ? s->caps[2] : 2 * k0;
  // every octave pixel of the 3 detection levels is at most one candidate
  const int cand_cap = (int)std::min<int64_t>({c0 * sc, 3 * nel + 64, INT32_MAX});
  // every octave's keypoints: at most 3 per pixel of each octave (<= 4 nel in all)
  const int key_cap = (int)std::min<int64_t>({k0 * sc, 4 * nel + 64, INT32_MAX});
  const int feat_cap = (int)std::min<int64_t>({f0 * sc, 4 * (int64_t)key_cap, INT32_MAX});
  // every octave's gradient planes stay until the frame's describe launches
  // (octave sizes nel, nel / 4, <= nel / 16, <= nel / 64)
  const size_t ngrad = 3 * ((size_t)nel + nel / 4 + nel / 16 + nel / 64 + 64);
  const size_t bytes = 12 * (size_t)nel * 4 + ngrad * 8 + 4 * 256 +
                       2 * (3 * (size_t)oh + 1) * 4 +
                       (size_t)cand_cap * (16 + 32 + 8) +
                       (size_t)key_cap * (32 + 4 + 16 + 4) +
                       (size_t)feat_cap * (16 + 512 + 128 + 4) + 64 * 256;
  SCM_TRY(sl.ws.ensure(bytes));
  SCM_TRY(sl.counts.ensure(sizeof(SiftCounts)));
  uint8_t* p = sl.ws.as<uint8_t>();
  SiftDev& d = sl.dev;
  d.levels = carve<float>(p, kSiftLevels * (size_t)nel);
  d.temp = carve<float>(p, (size_t)nel);
  d.dog = carve<float>(p, kSiftDogLevels * (size_t)nel);
  d.grad = carve<float2>(p, ngrad);
  d.rowcnt = carve<int32_t>(p, 3 * (size_t)oh + 1);
  d.rowoff = carve<int32_t>(p, 3 * (size_t)oh + 1);
  d.cand = carve<SiftCand>(p, cand_cap);
  d.ktmp = carve<SiftKey>(p, cand_cap);
  d.flag = carve<int32_t>(p, cand_cap);
  d.foff = carve<int32_t>(p, cand_cap);
  d.keys = carve<SiftKey>(p, key_cap);
  d.nori = carve<int32_t>(p, key_cap);
  d.ang = carve<double>(p, 2 * (size_t)key_cap);
  d.koff = carve<int32_t>(p, key_cap);
  d.feat = carve<SiftFeat>(p, feat_cap);
  d.descf = carve<float>(p, 128 * (size_t)feat_cap);
  d.desc = carve<uint8_t>(p, 128 * (size_t)feat_cap);
  d.stale = carve<int32_t>(p, feat_cap);
  d.cnt = sl.counts.as<SiftCounts>();
  d.cand_cap = cand_cap;
  d.key_cap = key_cap;
  d.feat_cap = feat_cap;
  if ((size_t)(p - sl.ws.as<uint8_t>()) > sl.ws.bytes) {
    set_error("sift workspace layout exceeds its allocation");
    return SCM_E_INVALID;
  }
  sl.nel_cap = nel;
  sl.caps_at_bound = cand_cap == std::min<int64_t>(INT32_MAX, 3 * nel + 64) &&
                     key_cap == std::min<int64_t>(INT32_MAX, 4 * nel + 64) &&
                     feat_cap == std::min<int64_t>(INT32_MAX, 4 * (int64_t)key_cap);
  return SCM_OK;
}

// Byte offsets of the rescale tables in Slot::rtab for an nw x nh target:
// horizontal (left, count) pairs, vertical pairs, horizontal weights,
// vertical weights.
struct TableLayout {
  int winh, winv;
  size_t o1, o2, o3, bytes;
};

TableLayout table_layout(int w, int h, int nw, int nh) {
  auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
  auto win = [](int dst, int src) {
    const double scale = double(dst) / double(src);
    return 2 * (int)std::ceil(scale < 1.0 ? 1.0 / scale : 1.0) + 1;
  };
  TableLayout L;
  L.winh = win(nw, w);
  L.winv = win(nh, h);
  L.o1 = up(2 * (size_t)nw * 4);
  L.o2 = L.o1 + up(2 * (size_t)nh * 4);
  L.o3 = L.o2 + up((size_t)nw * L.winh * 8);
  L.bytes = L.o3 + (size_t)nh * L.winv * 8;
  return L;
}

// resizeBitmap on the GPU: grey bytes of the frame in slot.frame, then the
// two bilinear passes (xy or yx: FreeImage filters first along the axis that
// gives the smaller intermediate); the nw x nh grey image ends in *out.
// The slot's stream is idle here (its previous frame was harvested).
int enqueue_rescale(Slot& sl, int w, int h, int ch, int nw, int nh, const uint8_t** out) {
  hipStream_t st = sl.st;
  const TableLayout L = table_layout(w, h, nw, nh);
  if (sl.rtab_w != w || sl.rtab_h != h) {  // weight tables for this source size
    std::vector<int32_t> hh, hv;
    std::vector<double> wh, wv;
    bilinear_table(nw, w, &hh, &wh);
    bilinear_table(nh, h, &hv, &wv);
    SCM_TRY(sl.pin_rtab.ensure(L.bytes));
    SCM_TRY(sl.rtab.ensure(L.bytes));
    uint8_t* p = sl.pin_rtab.as<uint8_t>();
    std::memcpy(p, hh.data(), hh.size() * 4);
    std::memcpy(p + L.o1, hv.data(), hv.size() * 4);
    std::memcpy(p + L.o2, wh.data(), wh.size() * 8);
    std::memcpy(p + L.o3, wv.data(), wv.size() * 8);
    SCM_HIP(hipMemcpyAsync(sl.rtab.ptr, p, L.bytes, hipMemcpyHostToDevice, st));
    sl.rtab_w = w;
    sl.rtab_h = h;
  }
  const uint8_t* tb = sl.rtab.as<uint8_t>();
  const int2* hh = reinterpret_cast<const int2*>(tb);
  const int2* hv = reinterpret_cast<const int2*>(tb + L.o1);
  const double* wh = reinterpret_cast<const double*>(tb + L.o2);
  const double* wv = reinterpret_cast<const double*>(tb + L.o3);
  const bool xy = (int64_t)nw * h <= (int64_t)nh * w;
  auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t g = (size_t)w * h, t = xy ? (size_t)nw * h : (size_t)w * nh, o = (size_t)nw * nh;
  SCM_TRY(sl.rs.ensure(up(g) + up(t) + o));
  uint8_t* grey = sl.rs.as<uint8_t>();
  uint8_t* tmp = grey + up(g);
  uint8_t* res = tmp + up(t);
  SCM_HIP(sift_grey(sl.frame.as<uint8_t>(), w, h, ch, grey, st));
  if (xy) {
    SCM_HIP(sift_rescale_rows(grey, w, h, tmp, nw, hh, wh, L.winh, st));
    SCM_HIP(sift_rescale_cols(tmp, nw, h, res, nh, hv, wv, L.winv, st));
  } else {
    SCM_HIP(sift_rescale_cols(grey, w, h, tmp, nh, hv, wv, L.winv, st));
    SCM_HIP(sift_rescale_rows(tmp, w, nh, res, nw, hh, wh, L.winh, st));
  }
  *out = res;
  return SCM_OK;
}

int enqueue_frame(SiftState* s, Slot& sl, const scm_frame& f) {
  const int fw = f.width, fh = f.height;
  int w, h;
  fit_size(fw, fh, &w, &h);
  int ch = f.channels;
  SCM_TRY(ensure_slot(s, sl, std::max(w, 1), std::max(h, 1)));
  const size_t fb = (size_t)fw * fh * ch;
  SCM_TRY(sl.pin_in.ensure(fb));
  SCM_TRY(sl.frame.ensure(fb));
  hipStream_t st = sl.st;
  std::memcpy(sl.pin_in.ptr, f.data, fb);
  SCM_HIP(hipMemcpyAsync(sl.frame.ptr, sl.pin_in.ptr, fb, hipMemcpyHostToDevice, st));
  SCM_HIP(hipMemsetAsync(sl.dev.cnt, 0, sizeof(SiftCounts), st));
  const uint8_t* src = sl.frame.as<uint8_t>();
  if (w != fw || h != fh) {
    SCM_TRY(enqueue_rescale(sl, fw, fh, ch, w, h, &src));
    ch = 1;
  }
  SiftDev& d = sl.dev;
  SiftOctaves oct{};
  float2* grad = d.grad;
  int ow = 2 * w, oh = 2 * h, pw = 0, ph = 0;  // this octave's and the previous octave's size
  // A frame of any size >= 1 x 1 runs, as VLFeat's filter does: octaves too
  // small for an interior pixel detect nothing, and an octave with no pixel
  // (width or height >> o == 0) ends the octaves -- VLFeat still steps
  // through it, on empty images.  (A rescale to a zero size leaves no octave.)
  for (int o = -1; o < kSiftOctaves - 1 && w > 0 && h > 0; ++o) {
    if (o >= 0) {  // VLFeat octave size: width >> o (width << 1 for o = -1)
      pw = ow;
      ph = oh;
      ow = w >> o;
      oh = h >> o;
      if (ow == 0 || oh == 0) break;
    }
    const size_t so = (size_t)ow * oh;
    if (o == -1) {
      SCM_HIP(sift_upsample(src, w, h, ch, d.temp, st));
      SCM_HIP(sift_smooth(d.temp, d.levels, d.dog, nullptr, ow, oh, s->c, 0, s->widths[0], st));
    } else {
      // copy_and_downsample of level s_best = 2 (index 3) of the previous
      // octave: every other pixel; no extra smoothing (sa == sb).  The source
      // [3 pw ph, 4 pw ph) lies past the destination [0, ow oh).
      SCM_HIP(sift_downsample(d.levels + 3 * (size_t)pw * ph, pw, d.levels, ow, oh, st));
    }
    for (int l = 1; l < kSiftLevels; ++l)
      SCM_HIP(sift_smooth(d.levels + (l - 1) * so, d.levels + l * so, d.temp,
                          d.dog + (l - 1) * so, ow, oh, s->c, l, s->widths[l], st));
    SCM_HIP(sift_octave_detect(d, s->c, ow, oh, o, kPeakThreshold, kEdgeThreshold, st));
    SCM_HIP(sift_octave_gradient(d, grad, ow, oh, st));
    oct.grad[o + 1] = grad;
    oct.w[o + 1] = ow;
    oct.h[o + 1] = oh;
    grad += 3 * so;
  }
  // orientations and descriptors of every octave's keypoints at once
  SCM_HIP(sift_describe(d, s->c, oct, st));
  SCM_HIP(sift_fixup(d, st));
  SCM_TRY(sl.pin_cnt.ensure(sizeof(SiftCounts)));
  SCM_HIP(hipMemcpyAsync(sl.pin_cnt.ptr, d.cnt, sizeof(SiftCounts), hipMemcpyDeviceToHost, st));
  sl.w = w;
  sl.h = h;
  return SCM_OK;
}

template <typename T>
void put(std::vector<uint8_t>* b, const T& v) {
  const uint8_t* q = reinterpret_cast<const uint8_t*>(&v);
  b->insert(b->end(), q, q + sizeof(T));
}

// Wait for a slot's frame and write its three elements; *overflow (and
// nothing written) when the frame exceeded the slot's capacities.
int harvest(Slot& sl, uint64_t image_id, scm_blob* kp_out, scm_blob* desc_out, scm_blob* cam_out,
            bool* overflow) {
  SCM_HIP(hipStreamSynchronize(sl.st));
  const SiftCounts cnt = *sl.pin_cnt.as<SiftCounts>();
  *overflow = cnt.overflow != 0;
  if (*overflow) return SCM_OK;
  const int nf = cnt.nfeat;
  // COLMAP: keep the coarsest DoG levels; the level whose keypoints first push
  // the count past max_num_features is kept whole.
  int first_keep = 0, acc = 0;
  for (int l = kSiftOctaves * 3 - 1; l >= 0; --l) {
    if (cnt.level_keys[l] == 0) continue;  // no such level in COLMAP's list
    acc += cnt.level_keys[l];
    if (acc > kMaxNumFeatures) {
      first_keep = l;
      break;
    }
  }
  int start = 0;
  for (int l = 0; l < first_keep; ++l) start += cnt.level_feats[l];
  const int n = nf - start;
  const size_t fbytes = (size_t)nf * sizeof(SiftFeat), dbytes = (size_t)nf * 128;
  SCM_TRY(sl.pin_out.ensure(fbytes + dbytes + 64));
  if (nf > 0) {
    SCM_HIP(hipMemcpyAsync(sl.pin_out.ptr, sl.dev.feat, fbytes, hipMemcpyDeviceToHost, sl.st));
    SCM_HIP(hipMemcpyAsync(sl.pin_out.as<uint8_t>() + fbytes, sl.dev.desc, dbytes,
                           hipMemcpyDeviceToHost, sl.st));
    SCM_HIP(hipStreamSynchronize(sl.st));
  }
  const SiftFeat* feat = sl.pin_out.as<SiftFeat>() + start;
  const uint8_t* desc = sl.pin_out.as<uint8_t>() + fbytes + (size_t)start * 128;
  std::vector<uint8_t> kb, db, cb;
  kb.reserve(8 + 24 * (size_t)n);
  put(&kb, (uint64_t)n);
  for (int i = 0; i < n; ++i) {
    const SiftFeat& f = feat[i];
    const float sc = f.scale, ori = f.orientation;
    const float kp[6] = {f.x, f.y, sc * std::cos(ori), -sc * std::sin(ori + 0.0f),
                         sc * std::sin(ori), sc * std::cos(ori + 0.0f)};
    for (float v : kp) put(&kb, v);
  }
  db.reserve(16 + 128 * (size_t)n);
  put(&db, (uint64_t)n);
  put(&db, (uint64_t)128);
  db.insert(db.end(), desc, desc + 128 * (size_t)n);
  // create_camera_buffer (io.cc:307-333) of extractCamera's SIMPLE_RADIAL camera.
  const double focal = 1.2 * std::max(sl.w, sl.h);
  const double params[4] = {focal, sl.w / 2.0, sl.h / 2.0, 0.0};
  put(&cb, (uint64_t)(8 + 4 + 4 + 8 + 8 + 1 + 8 + 4 * 8));
  put(&cb, (uint32_t)image_id);
  put(&cb, (int32_t)2);
  put(&cb, (uint64_t)sl.w);
  put(&cb, (uint64_t)sl.h);
  put(&cb, (uint8_t)0);
  put(&cb, (uint64_t)4);
  for (double p : params) put(&cb, p);
  SCM_TRY(make_blob(kb, kp_out));
  SCM_TRY(make_blob(db, desc_out));
  SCM_TRY(make_blob(cb, cam_out));
  return SCM_OK;
}

}  // namespace

// Harvest of slot sl's frame j; on overflow the slot's capacities grow 4x and
// the frame is extracted again (synchronously) until it fits.  The capacities
// reach their hard bounds (ensure_slot: one candidate per detection-level
// pixel, three keypoints per octave pixel, four features per keypoint) after
// at most ~12 regrowths; an overflow at those bounds is an internal error.
// The enlarged workspace stays with the slot (it is reused by later frames).
int harvest_or_regrow(SiftState* s, Slot& sl, int64_t j, const uint64_t* ids,
                      const scm_frame* frames, scm_blob* kp_out, scm_blob* desc_out,
                      scm_blob* cam_out) {
  for (int regrow = 0;; ++regrow) {
    bool overflow = false;
    SCM_TRY(harvest(sl, ids[j], &kp_out[j], &desc_out[j], &cam_out[j], &overflow));
    if (!overflow) return SCM_OK;
    if (sl.caps_at_bound || regrow >= 16) {
      set_error("scm_extract_frames: frame " + std::to_string(j) +
                " overflows the SIFT capacities at their upper bounds");
      return SCM_E_CAPACITY;
    }
    sl.cap_scale = std::min<int64_t>(sl.cap_scale * 4, (int64_t)1 << 40);
    sl.nel_cap = 0;  // re-layout the workspace with the larger capacities
    SCM_TRY(enqueue_frame(s, sl, frames[j]));
  }
}

int sift_extract_frames(SiftState** state, int device, const hipStream_t* streams, int64_t n,
                        const uint64_t* ids, const scm_frame* frames, scm_blob* kp_out,
                        scm_blob* desc_out, scm_blob* cam_out) {
  if (n < 0 || (n > 0 && (!ids || !frames || !kp_out || !desc_out || !cam_out))) {
    set_error("scm_extract_frames: null argument");
    return SCM_E_INVALID;
  }
  for (int64_t i = 0; i < n; ++i) {
    const scm_frame& f = frames[i];
    if (!f.data || !(f.channels == 1 || f.channels == 3 || f.channels == 4) || f.width < 1 ||
        f.height < 1) {
      set_error("scm_extract_frames: frame " + std::to_string(i) +
                " is not a non-empty frame of 1, 3 or 4 channels");
      return SCM_E_INVALID;
    }
  }
  SCM_HIP(hipSetDevice(device));
  if (!*state) {
    std::unique_ptr<SiftState> s(new SiftState());
    s->device = device;
    if (const char* e = std::getenv("SCM_SIFT_CAPS"))
      std::sscanf(e, "%d,%d,%d", &s->caps[0], &s->caps[1], &s->caps[2]);
    SCM_TRY(init_state(s.get(), streams));
    *state = s.release();
  }
  SiftState* s = *state;
  for (Slot& sl : s->slots) sl.pending = -1;
  for (int64_t i = 0; i < n; ++i) kp_out[i] = desc_out[i] = cam_out[i] = scm_blob{nullptr, 0};
  int rc = SCM_OK;
  for (int64_t i = 0; i < n && rc == SCM_OK; ++i) {
    Slot& sl = s->slots[i % kSlots];
    if (sl.pending >= 0) {
      const int64_t j = sl.pending;
      sl.pending = -1;
      rc = harvest_or_regrow(s, sl, j, ids, frames, kp_out, desc_out, cam_out);
      if (rc != SCM_OK) break;
    }
    rc = enqueue_frame(s, sl, frames[i]);
    if (rc == SCM_OK) sl.pending = i;
  }
  // Every slot still holding a frame is drained, on error too (its stream
  // finishes before the caller's buffers can go away).
  for (int64_t i = std::max<int64_t>(0, n - kSlots); i < n; ++i) {
    Slot& sl = s->slots[i % kSlots];
    if (sl.pending == i) {
      sl.pending = -1;
      if (rc == SCM_OK) rc = harvest_or_regrow(s, sl, i, ids, frames, kp_out, desc_out, cam_out);
    }
  }
  for (Slot& sl : s->slots) {
    if (sl.st) (void)hipStreamSynchronize(sl.st);
    sl.pending = -1;
  }
  if (rc != SCM_OK)  // no partial output: free what earlier frames produced
    for (int64_t i = 0; i < n; ++i) {
      scm_blob_free(&kp_out[i]);
      scm_blob_free(&desc_out[i]);
      scm_blob_free(&cam_out[i]);
    }
  return rc;
}

}  // namespace scm
