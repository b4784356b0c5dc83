// GPU SIFT extraction: the producer of the
// `extraction` table the matcher reads.  Kernels in sift_kernels.hip,
// orchestration in scm_sift.cpp.  Replaces SiftExtractionKernel::execute
// (reference integration/op_cpp/extraction_op.cc:70-121) ->
// colmap::ExtractSiftFeaturesCPU -> VLFeat vl/sift.c.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace scm {

constexpr int kSiftLevels = 6;       // s = s_min .. s_max = -1 .. 4 (octave_resolution 3)
constexpr int kSiftDogLevels = 5;    // DoG s = -1 .. 3
constexpr int kSiftOctaves = 4;      // octaves -1 .. 2 (first_octave -1, num_octaves 4)
constexpr int kSiftMaxTaps = 2 * 13 + 1;  // widest smoothing kernel (sigma 3.09 -> W = 13)

struct SiftCand {  // DoG extremum (detection order s, y, x)
  int32_t x, y, s, pad;
};

struct SiftKey {  // VlSiftKeypoint after refinement
  float x, y, s, sigma;  // x, y, sigma in input-image pixels (VLFeat convention)
  int32_t ix, iy, is, o;
};

struct SiftFeat {  // one (keypoint, orientation): COLMAP FeatureKeypoint parameters
  float x, y, scale, orientation;  // x + 0.5f, y + 0.5f
};

// Device counters of one image.
struct SiftCounts {
  int32_t ncand;                         // candidates of the current octave
  int32_t nkey;                          // refined keypoints so far (all octaves, <= key_cap)
  int32_t nfeat;                         // features so far (all octaves)
  int32_t nstale;                        // features whose descriptor VLFeat leaves unwritten
  int32_t overflow;                      // a capacity was exceeded
  int32_t keys_run;                      // refined keypoints so far (uncapped)
  int32_t pad[2];
  int32_t level_keys[kSiftOctaves * 3];  // keypoints per (octave, is) DoG level
  int32_t level_feats[kSiftOctaves * 3]; // features per level
};

// One image slot's device workspace (sizes for the first octave).
struct SiftDev {
  float* levels;   // kSiftLevels x (ow x oh)
  float* temp;     // ow x oh
  float* dog;      // kSiftDogLevels x (ow x oh)
  float2* grad;    // per octave 3 x (its w x h): (modulus, angle) of levels s = 0 .. 2
  int32_t* rowcnt; // 3 x oh per-row candidate counts, then exclusive offsets
  int32_t* rowoff;
  SiftCand* cand;  // cand_cap
  SiftKey* ktmp;   // cand_cap (refinement output slots)
  int32_t* flag;   // cand_cap
  int32_t* foff;   // cand_cap
  SiftKey* keys;   // key_cap (every octave's, in octave order)
  int32_t* nori;   // key_cap (orientations used, <= 2)
  double* ang;     // 2 x key_cap
  int32_t* koff;   // key_cap (feature offset of each keypoint)
  SiftFeat* feat;  // feat_cap
  float* descf;    // feat_cap x 128 (L1-rooted floats, VLFeat bin order)
  uint8_t* desc;   // feat_cap x 128 (u8, UBC order)
  int32_t* stale;  // feat_cap
  SiftCounts* cnt;
  int32_t cand_cap, key_cap, feat_cap;
};

// The octaves' gradient planes, for the orientation and descriptor launches
// that cover every octave's keypoints at once (indexed by octave + 1).
struct SiftOctaves {
  const float2* grad[kSiftOctaves];
  int32_t w[kSiftOctaves], h[kSiftOctaves];
};

// Host-built constants: smoothing taps (index 0: the first octave's s_min
// level, 1 + s: level s = 0 .. 4; each kSiftMaxTaps floats, W in widths[])
// and the fast_expn table (vl/mathop.h: exp(-k 25 / 256), k = 0 .. 256).
struct SiftConsts {
  float* taps;      // 6 x kSiftMaxTaps
  int32_t* widths;  // 6
  double* expn;     // 257
};

// Frames above max_image_size: grey bytes, then FreeImage's bilinear rescale
// one axis at a time (weight tables built on the host, scm_sift.cpp).
hipError_t sift_grey(const uint8_t* frame, int w, int h, int ch, uint8_t* out, hipStream_t st);
hipError_t sift_rescale_rows(const uint8_t* src, int sw, int rows, uint8_t* dst, int dw,
                             const int2* hdr, const double* wt, int win, hipStream_t st);
hipError_t sift_rescale_cols(const uint8_t* src, int cols, int sh, uint8_t* dst, int dh,
                             const int2* hdr, const double* wt, int win, hipStream_t st);
hipError_t sift_upsample(const uint8_t* frame, int w, int h, int ch, float* out, hipStream_t st);
// One Gaussian level out = smooth(in) (in != out; tmp: a w x h scratch plane),
// and when dog is given the DoG level dog = out - in.
hipError_t sift_smooth(const float* in, float* out, float* tmp, float* dog, int w, int h,
                       const SiftConsts& c, int tap_set, int W, hipStream_t st);
hipError_t sift_downsample(const float* in, int w_in, float* out, int w, int h, hipStream_t st);
hipError_t sift_octave_detect(const SiftDev& d, const SiftConsts& c, int w, int h, int octave,
                              double peak_thresh, double edge_thresh, hipStream_t st);
// update_gradient of an octave's levels s = 0 .. 2 into grad (3 x w x h).
hipError_t sift_octave_gradient(const SiftDev& d, float2* grad, int w, int h, hipStream_t st);
// Orientations and descriptors of every octave's keypoints, one launch each.
hipError_t sift_describe(const SiftDev& d, const SiftConsts& c, const SiftOctaves& oct,
                         hipStream_t st);
hipError_t sift_fixup(const SiftDev& d, hipStream_t st);

}  // namespace scm
