// CPU oracle of the SIFT extraction op.
//
// TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg, always as the checker / the timed CPU
// baseline; the product path (scanner_colmap_amd/csrc/sift_kernels.hip,
// scm_sift.cpp) never links or calls it.
//
// Restates, sequentially and operation for operation, what the reference op
// SiftExtractionKernel::execute (integration/op_cpp/extraction_op.cc:70-121)
// computes through its un-vendored dependencies:
//   * FreeImage_ConvertFromRawBits + Bitmap::CloneAsGrey (:79-86): the frame's
//     bytes are taken as FreeImage's in-memory B, G, R order (the raw-bits
//     call copies them as they are), grey = (BYTE)(0.2126F R + 0.7152F G +
//     0.0722F B + 0.5F) (FreeImage 3.17 Utilities.h LUMA_REC709 / GREY), i.e.
//     frame channel 2 is weighted as red and channel 0 as blue;
//   * resizeBitmap (:28-39): a grey image larger than max_image_size (3200) in
//     either dimension is scaled by 3200 / max(w, h) (new sizes truncated) with
//     Bitmap::Rescale -> FreeImage_Rescale(FILTER_BILINEAR) (FreeImage 3.17
//     Resize.cpp: CWeightsTable of CBilinearFilter, one 8-bit pass per axis in
//     FreeImage's bottom-up scanline order, xy or yx by the smaller
//     intermediate, fp64 sums rounded to BYTE after each pass) -- restated from
//     FreeImage's published source (not vendored in the reference);
//   * colmap::ExtractSiftFeaturesCPU (COLMAP 3.4 src/feature/sift.cc) with the
//     default SiftExtractionOptions (max_num_features 8192, first_octave -1,
//     num_octaves 4, octave_resolution 3, peak_threshold 0.02 / 3,
//     edge_threshold 10, max_num_orientations 2, L1_ROOT), which drives the
//     VLFeat covariant SIFT filter (vl/sift.c as vendored by COLMAP:
//     vl_sift_new, vl_sift_process_first_octave / _next_octave, _vl_sift_smooth
//     with vl_imconvcol_vf, vl_sift_detect, update_gradient,
//     vl_sift_calc_keypoint_orientations, vl_sift_calc_keypoint_descriptor,
//     vl/mathop.h fast_expn, vl_fast_atan2_f, vl_fast_sqrt_f, vl_mod_2pi_f),
//     then L1RootNormalizeFeatureDescriptors, FeatureDescriptorsToUnsignedByte,
//     the DoG-level selection of max_num_features and
//     TransformVLFeatToUBCFeatureDescriptors;
//   * extractCamera (:41-64): SIMPLE_RADIAL (model id 2), f = 1.2 max(w, h),
//     principal point (w / 2, h / 2), k = 0, no prior focal length (a
//     raw-bits bitmap carries no EXIF), camera id = image id;
//   * the io.cc writers of the three outputs (write_vector_to_element,
//     write_matrix_to_element, write_camera_to_element io.cc:307-335).
// PARITY UNPINNED: FreeImage, VLFeat and COLMAP are absent from this
// container and the reference holds no fixtures; the restatement is pinned by
// known-answer tests (tests/test_oracle_sift.py).
//
// Quirk reproduced: vl_sift_calc_keypoint_descriptor returns without writing
// when the keypoint's row is the octave's last (yi >= h - 1, stricter than the
// orientation check), and COLMAP then re-normalises the descriptor buffer of
// the previous keypoint (L1-root of an L1-rooted vector); the very first
// buffer is uninitialised in the reference, zeros here.
// Third-party algorithms restated (test oracle): VLFeat's SIFT (vl/sift.c,
// vl/mathop.h; A. Vedaldi and B. Fulkerson, BSD licence) and FreeImage 3.17's
// bilinear rescale (Resize.cpp; FreeImage Public License), as COLMAP 3.4 calls
// them -- written from their published algorithms, no source copied.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/scm.h"

namespace {

constexpr double kPi = 3.141592653589793;  // VL_PI
constexpr float kEpsF = 1.19209290E-07F;   // VL_EPSILON_F
constexpr double kEpsD = 2.220446049250313e-16;  // VL_EPSILON_D

struct SiftOpts {  // colmap::SiftExtractionOptions defaults (COLMAP 3.4)
  int max_image_size = 3200;
  int max_num_features = 8192;
  int first_octave = -1;
  int num_octaves = 4;
  int octave_resolution = 3;
  double peak_threshold = 0.02 / 3;
  double edge_threshold = 10.0;
  int max_num_orientations = 2;
};

// vl/mathop.h
float fast_resqrt_f(float x) {
  union {
    float x;
    int32_t i;
  } u;
  const float xhalf = 0.5F * x;
  u.x = x;
  u.i = 0x5f3759df - (u.i >> 1);
  u.x = u.x * (1.5F - xhalf * u.x * u.x);
  u.x = u.x * (1.5F - xhalf * u.x * u.x);
  return u.x;
}
float fast_sqrt_f(float x) { return (x < 1e-8) ? 0 : x * fast_resqrt_f(x); }
float fast_atan2_f(float y, float x) {
  const float c3 = 0.1821F, c1 = 0.9675F;
  const float abs_y = std::fabs(y) + kEpsF;
  float angle, r;
  if (x >= 0) {
    r = (x - abs_y) / (x + abs_y);
    angle = (float)(kPi / 4);
  } else {
    r = (x + abs_y) / (abs_y - x);
    angle = (float)(3 * kPi / 4);
  }
  angle += (c3 * r * r - c1) * r;
  return (y < 0) ? -angle : angle;
}
float mod_2pi_f(float x) {
  while (x > (float)(2 * kPi)) x -= (float)(2 * kPi);
  while (x < 0.0F) x += (float)(2 * kPi);
  return x;
}
constexpr int kExpnSz = 256;
constexpr double kExpnMax = 25.0;
struct ExpnTab {
  double t[kExpnSz + 1];
  ExpnTab() {
    for (int k = 0; k < kExpnSz + 1; ++k) t[k] = std::exp(-(double)k * (kExpnMax / kExpnSz));
  }
};
const ExpnTab& expn_tab() {
  static const ExpnTab tab;
  return tab;
}
double fast_expn(double x) {
  if (x > kExpnMax) return 0.0;
  x *= kExpnSz / kExpnMax;
  const int i = (int)std::floor(x);
  const double r = x - i;
  const double a = expn_tab().t[i], b = expn_tab().t[i + 1];
  return a + r * (b - a);
}

// _vl_sift_smooth's kernel: width max(ceil(4 sigma), 1), taps exp(-d^2 / 2)
// with d = (j - W) / sigma in float, normalised by their float sum.
std::vector<float> gauss_taps(double sigma) {
  const int W = std::max((int)std::ceil(4.0 * sigma), 1);
  std::vector<float> g(2 * W + 1);
  float acc = 0;
  for (int j = 0; j < 2 * W + 1; ++j) {
    const float d = ((float)(j - W)) / ((float)sigma);
    g[j] = (float)std::exp(-0.5 * (d * d));
    acc += g[j];
  }
  for (int j = 0; j < 2 * W + 1; ++j) g[j] /= acc;
  return g;
}

// vl_imconvcol_vf with VL_PAD_BY_CONTINUITY | VL_TRANSPOSE: out(y) = sum over
// p = y - W .. y + W ascending of in(clamp(p)) * g[W + y - p], float
// multiply then add; the vertical pass runs first, then the horizontal one.
void smooth(const float* in, float* out, float* tmp, int w, int h, const std::vector<float>& g) {
  const int W = ((int)g.size() - 1) / 2;
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      float acc = 0;
      for (int p = y - W; p <= y + W; ++p) {
        const int pc = std::min(std::max(p, 0), h - 1);
        acc += in[(size_t)pc * w + x] * g[W + y - p];
      }
      tmp[(size_t)y * w + x] = acc;
    }
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      float acc = 0;
      for (int p = x - W; p <= x + W; ++p) {
        const int pc = std::min(std::max(p, 0), w - 1);
        acc += tmp[(size_t)y * w + pc] * g[W + x - p];
      }
      out[(size_t)y * w + x] = acc;
    }
}

// Gradient and Hessian of the DoG at a sample (vl_sift_refine_keypoints,
// VLFeat sift.c): at() reads vl_sift_pix (float), so the sums and
// differences round in float; only the products with the double literals
// (0.5, 2.0, 0.25) widen to double (C's usual arithmetic conversions).
// D = Dx, Dy, Ds, Dxx, Dyy, Dss, Dxy, Dxs, Dys.
static void refine_terms(const float* pt, ptrdiff_t yo, ptrdiff_t so, double* D) {
  auto at = [&](int ax, int ay, int as) -> float { return *(pt + ax + ay * yo + as * so); };
  D[0] = 0.5 * (at(1, 0, 0) - at(-1, 0, 0));
  D[1] = 0.5 * (at(0, 1, 0) - at(0, -1, 0));
  D[2] = 0.5 * (at(0, 0, 1) - at(0, 0, -1));
  D[3] = (at(1, 0, 0) + at(-1, 0, 0) - 2.0 * at(0, 0, 0));
  D[4] = (at(0, 1, 0) + at(0, -1, 0) - 2.0 * at(0, 0, 0));
  D[5] = (at(0, 0, 1) + at(0, 0, -1) - 2.0 * at(0, 0, 0));
  D[6] = 0.25 * (at(1, 1, 0) + at(-1, -1, 0) - at(-1, 1, 0) - at(1, -1, 0));
  D[7] = 0.25 * (at(1, 0, 1) + at(-1, 0, -1) - at(-1, 0, 1) - at(1, 0, -1));
  D[8] = 0.25 * (at(0, 1, 1) + at(0, -1, -1) - at(0, -1, 1) - at(0, 1, -1));
}

struct Keypoint {  // VlSiftKeypoint
  int o, ix, iy, is;
  float x, y, s, sigma;
};

// The VLFeat filter state for one image (vl_sift_new + the processing calls).
struct Sift {
  int width, height, O, S, o_min, s_min, s_max, o_cur;
  double sigma0, sigmak, sigman, dsigma0, peak_thresh, edge_thresh;
  int ow = 0, oh = 0;
  std::vector<float> octave, temp, dog, grad;
  int grad_o;
  std::vector<Keypoint> keys;

  Sift(int w, int h, int noct, int nlev, int omin)
      : width(w), height(h), O(noct), S(nlev), o_min(omin), s_min(-1), s_max(nlev + 1),
        o_cur(omin) {
    const int wmax = omin < 0 ? w << -omin : w >> omin, hmax = omin < 0 ? h << -omin : h >> omin;
    const size_t nel = (size_t)wmax * hmax;
    temp.resize(nel);
    octave.resize(nel * (s_max - s_min + 1));
    dog.resize(nel * (s_max - s_min));
    grad.resize(nel * 2 * (s_max - s_min));
    sigman = 0.5;
    sigmak = std::pow(2.0, 1.0 / nlev);
    sigma0 = 1.6 * sigmak;
    dsigma0 = sigma0 * std::sqrt(1.0 - 1.0 / (sigmak * sigmak));
    grad_o = omin - 1;
  }
  float* level(int s) { return octave.data() + (size_t)ow * oh * (s - s_min); }
  static int shl(int x, int n) { return n >= 0 ? x << n : x >> -n; }

  // copy_and_upsample_rows twice: x first, then y; mid = 0.5 * (a + b).
  void upsample(const float* im) {
    const int w = width, h = height;
    std::vector<float> t((size_t)2 * w * h);
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        const float a = im[(size_t)y * w + x];
        const float b = im[(size_t)y * w + std::min(x + 1, w - 1)];
        t[(size_t)y * 2 * w + 2 * x] = a;
        t[(size_t)y * 2 * w + 2 * x + 1] = x + 1 < w ? (float)(0.5 * (a + b)) : a;
      }
    float* o = level(s_min);
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < 2 * w; ++x) {
        const float a = t[(size_t)y * 2 * w + x];
        const float b = t[(size_t)std::min(y + 1, h - 1) * 2 * w + x];
        o[(size_t)(2 * y) * 2 * w + x] = a;
        o[(size_t)(2 * y + 1) * 2 * w + x] = y + 1 < h ? (float)(0.5 * (a + b)) : a;
      }
  }
  void fill_levels() {
    for (int s = s_min + 1; s <= s_max; ++s) {
      const double sd = dsigma0 * std::pow(sigmak, s);
      smooth(level(s - 1), level(s), temp.data(), ow, oh, gauss_taps(sd));
    }
  }
  // vl_sift_process_first_octave (first_octave = -1 only: one doubling).
  void first_octave(const float* im) {
    o_cur = o_min;
    keys.clear();
    ow = shl(width, -o_cur);
    oh = shl(height, -o_cur);
    upsample(im);
    const double sa = sigma0 * std::pow(sigmak, s_min);
    const double sb = sigman * std::pow(2.0, -o_min);
    if (sa > sb) {
      const double sd = std::sqrt(sa * sa - sb * sb);
      smooth(level(s_min), level(s_min), temp.data(), ow, oh, gauss_taps(sd));
    }
    fill_levels();
  }
  // vl_sift_process_next_octave: level s_best = min(s_min + S, s_max) of the
  // current octave, every other pixel (copy_and_downsample with d = 2);
  // sa == sb for these options, so no extra smoothing.
  bool next_octave() {
    if (o_cur == o_min + O - 1) return false;
    const int s_best = std::min(s_min + S, s_max);
    const int w = ow, h = oh;
    std::vector<float> src(level(s_best), level(s_best) + (size_t)w * h);
    o_cur += 1;
    keys.clear();
    ow = shl(width, -o_cur);
    oh = shl(height, -o_cur);
    float* dst = level(s_min);
    for (int y = 0; y < oh; ++y)
      for (int x = 0; x < ow; ++x) dst[(size_t)y * ow + x] = src[(size_t)(2 * y) * w + 2 * x];
    const double sa = sigma0 * std::pow(sigmak, (double)s_min);
    const double sb = sigma0 * std::pow(sigmak, (double)(s_best - S));
    if (sa > sb) {
      const double sd = std::sqrt(sa * sa - sb * sb);
      smooth(level(s_min), level(s_min), temp.data(), ow, oh, gauss_taps(sd));
    }
    fill_levels();
    return true;
  }

  // vl_sift_detect: DoG, 26-neighbour strict extrema with |v| >= 0.8 tp in
  // scan order (s, y, x), then refinement (<= 5 Newton steps, Gauss
  // elimination with partial pivoting) and the peak / edge / bounds tests.
  void detect() {
    const int w = ow, h = oh;
    const size_t so = (size_t)w * h;
    const double tp = peak_thresh, te = edge_thresh;
    const double xper = std::pow(2.0, o_cur);
    for (int s = s_min; s <= s_max - 1; ++s) {
      const float* a = level(s);
      const float* b = level(s + 1);
      float* d = dog.data() + so * (s - s_min);
      for (size_t i = 0; i < so; ++i) d[i] = b[i] - a[i];
    }
    keys.clear();
    for (int s = s_min + 1; s <= s_max - 2; ++s)
      for (int y = 1; y < h - 1; ++y)
        for (int x = 1; x < w - 1; ++x) {
          const float* pt = dog.data() + so * (s - s_min) + (size_t)y * w + x;
          const float v = *pt;
          bool mx = v >= 0.8 * tp, mn = v <= -0.8 * tp;
          for (int ds = -1; ds <= 1 && (mx || mn); ++ds)
            for (int dy = -1; dy <= 1; ++dy)
              for (int dx = -1; dx <= 1; ++dx) {
                if (!ds && !dy && !dx) continue;
                const float u = *(pt + (ptrdiff_t)ds * (ptrdiff_t)so + (ptrdiff_t)dy * w + dx);
                mx = mx && v > u;
                mn = mn && v < u;
              }
          if (mx || mn) keys.push_back(Keypoint{0, x, y, s, 0, 0, 0, 0});
        }
    std::vector<Keypoint> good;
    for (const Keypoint& kc : keys) {
      int x = kc.ix, y = kc.iy;
      const int s = kc.is;
      double Dx = 0, Dy = 0, Ds = 0, Dxx = 0, Dyy = 0, Dss = 0, Dxy = 0, Dxs = 0, Dys = 0;
      double A[9], b[3];
      int dx = 0, dy = 0;
      const float* pt = nullptr;
      for (int iter = 0; iter < 5; ++iter) {
        x += dx;
        y += dy;
        pt = dog.data() + (size_t)x + (size_t)y * w + so * (s - s_min);
        double D[9];
        refine_terms(pt, w, (ptrdiff_t)so, D);
        Dx = D[0]; Dy = D[1]; Ds = D[2];
        Dxx = D[3]; Dyy = D[4]; Dss = D[5];
        Dxy = D[6]; Dxs = D[7]; Dys = D[8];
        // A column-major: A[i + 3 j]
        A[0] = Dxx; A[4] = Dyy; A[8] = Dss;
        A[3] = A[1] = Dxy;
        A[6] = A[2] = Dxs;
        A[7] = A[5] = Dys;
        b[0] = -Dx; b[1] = -Dy; b[2] = -Ds;
        for (int j = 0; j < 3; ++j) {
          double maxa = 0, maxabsa = 0;
          int maxi = -1;
          for (int i = j; i < 3; ++i) {
            const double av = A[i + 3 * j], absa = std::fabs(av);
            if (absa > maxabsa) {
              maxa = av;
              maxabsa = absa;
              maxi = i;
            }
          }
          if (maxabsa < 1e-10f) {
            b[0] = b[1] = b[2] = 0;
            break;
          }
          const int i = maxi;
          for (int jj = j; jj < 3; ++jj) {
            const double t = A[i + 3 * jj];
            A[i + 3 * jj] = A[j + 3 * jj];
            A[j + 3 * jj] = t;
            A[j + 3 * jj] /= maxa;
          }
          const double t = b[j];
          b[j] = b[i];
          b[i] = t;
          b[j] /= maxa;
          for (int ii = j + 1; ii < 3; ++ii) {
            const double xx = A[ii + 3 * j];
            for (int jj = j; jj < 3; ++jj) A[ii + 3 * jj] -= xx * A[j + 3 * jj];
            b[ii] -= xx * b[j];
          }
        }
        for (int i = 2; i > 0; --i) {
          const double xx = b[i];
          for (int ii = i - 1; ii >= 0; --ii) b[ii] -= xx * A[ii + 3 * i];
        }
        dx = ((b[0] > 0.6 && x < w - 2) ? 1 : 0) + ((b[0] < -0.6 && x > 1) ? -1 : 0);
        dy = ((b[1] > 0.6 && y < h - 2) ? 1 : 0) + ((b[1] < -0.6 && y > 1) ? -1 : 0);
        if (dx == 0 && dy == 0) break;
      }
      const double val = *pt + 0.5 * (Dx * b[0] + Dy * b[1] + Ds * b[2]);
      const double score = (Dxx + Dyy) * (Dxx + Dyy) / (Dxx * Dyy - Dxy * Dxy);
      const double xn = x + b[0], yn = y + b[1], sn = s + b[2];
      const bool ok = std::fabs(val) > tp && score < (te + 1) * (te + 1) / te && score >= 0 &&
                      std::fabs(b[0]) < 1.5 && std::fabs(b[1]) < 1.5 && std::fabs(b[2]) < 1.5 &&
                      xn >= 0 && xn <= w - 1 && yn >= 0 && yn <= h - 1 && sn >= s_min &&
                      sn <= s_max;
      if (ok) {
        Keypoint k;
        k.o = o_cur;
        k.ix = x;
        k.iy = y;
        k.is = s;
        k.s = (float)sn;
        k.x = (float)(xn * xper);
        k.y = (float)(yn * xper);
        k.sigma = (float)(sigma0 * std::pow(2.0, sn / S) * xper);
        good.push_back(k);
      }
    }
    keys.swap(good);
  }

  // update_gradient: per level s = s_min + 1 .. s_max - 2, (modulus, angle)
  // with one-sided differences on the border rows / columns.
  void update_gradient() {
    if (grad_o == o_cur) return;
    const int w = ow, h = oh;
    const size_t so = (size_t)w * h;
    for (int s = s_min + 1; s <= s_max - 2; ++s) {
      const float* src = level(s);
      float* g = grad.data() + 2 * so * (s - s_min - 1);
      for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
          const float* p = src + (size_t)y * w + x;
          float gx, gy;
          if (x == 0) gx = p[1] - p[0];
          else if (x == w - 1) gx = p[0] - p[-1];
          else gx = (float)(0.5 * (p[1] - p[-1]));
          if (y == 0) gy = p[w] - p[0];
          else if (y == h - 1) gy = p[0] - p[-w];
          else gy = (float)(0.5 * (p[w] - p[-w]));
          const size_t i = 2 * ((size_t)y * w + x);
          g[i] = fast_sqrt_f(gx * gx + gy * gy);
          g[i + 1] = mod_2pi_f((float)(fast_atan2_f(gy, gx) + 2 * kPi));
        }
    }
    grad_o = o_cur;
  }

  int orientations(double angles[4], const Keypoint& k) {
    const double winf = 1.5;
    const double xper = std::pow(2.0, o_cur);
    const int w = ow, h = oh;
    const int xo = 2, yo = 2 * w;
    const size_t so = 2 * (size_t)w * h;
    const double x = k.x / xper, y = k.y / xper, sigma = k.sigma / xper;
    const int xi = (int)(x + 0.5), yi = (int)(y + 0.5), si = k.is;
    const double sigmaw = winf * sigma;
    const int W = std::max((int)std::floor(3.0 * sigmaw), 1);
    constexpr int nbins = 36;
    double hist[nbins];
    if (k.o != o_cur) return 0;
    if (xi < 0 || xi > w - 1 || yi < 0 || yi > h - 1 || si < s_min + 1 || si > s_max - 2) return 0;
    update_gradient();
    std::memset(hist, 0, sizeof(hist));
    const float* pt = grad.data() + xo * xi + (size_t)yo * yi + so * (si - s_min - 1);
    for (int ys = std::max(-W, -yi); ys <= std::min(W, h - 1 - yi); ++ys)
      for (int xs = std::max(-W, -xi); xs <= std::min(W, w - 1 - xi); ++xs) {
        const double dx = (double)(xi + xs) - x, dy = (double)(yi + ys) - y;
        const double r2 = dx * dx + dy * dy;
        if (r2 >= W * W + 0.6) continue;
        const double wgt = fast_expn(r2 / (2 * sigmaw * sigmaw));
        const double mod = *(pt + xs * xo + (ptrdiff_t)ys * yo);
        const double ang = *(pt + xs * xo + (ptrdiff_t)ys * yo + 1);
        const int bin = (int)std::floor(nbins * ang / (2 * kPi));
        hist[bin % nbins] += mod * wgt;
      }
    for (int iter = 0; iter < 6; ++iter) {
      double prev = hist[nbins - 1];
      const double first = hist[0];
      int i;
      for (i = 0; i < nbins - 1; ++i) {
        const double nh = (prev + hist[i] + hist[(i + 1) % nbins]) / 3.0;
        prev = hist[i];
        hist[i] = nh;
      }
      hist[i] = (prev + hist[i] + first) / 3.0;
    }
    double maxh = 0;
    for (int i = 0; i < nbins; ++i) maxh = std::max(maxh, hist[i]);
    int n = 0;
    for (int i = 0; i < nbins; ++i) {
      const double h0 = hist[i], hm = hist[(i - 1 + nbins) % nbins], hp = hist[(i + 1 + nbins) % nbins];
      if (h0 > 0.8 * maxh && h0 > hm && h0 > hp) {
        const double di = -0.5 * (hp - hm) / (hp + hm - 2 * h0);
        angles[n++] = 2 * kPi * (i + di + 0.5) / nbins;
        if (n == 4) break;
      }
    }
    return n;
  }

  // Returns false (buffer untouched) on the reference's early exit.
  bool descriptor(float* descr, const Keypoint& k, double angle0) {
    constexpr int NBP = 4, NBO = 8;
    const double magnif = 3.0;
    const double xper = std::pow(2.0, o_cur);
    const int w = ow, h = oh;
    const int xo = 2, yo = 2 * w;
    const size_t so = 2 * (size_t)w * h;
    const double x = k.x / xper, y = k.y / xper, sigma = k.sigma / xper;
    const int xi = (int)(x + 0.5), yi = (int)(y + 0.5), si = k.is;
    const double st0 = std::sin(angle0), ct0 = std::cos(angle0);
    const double SBP = magnif * sigma + kEpsD;
    const int W = (int)std::floor(std::sqrt(2.0) * SBP * (NBP + 1) / 2.0 + 0.5);
    const int binto = 1, binyo = NBO * NBP, binxo = NBO;
    if (k.o != o_cur || xi < 0 || xi >= w || yi < 0 || yi >= h - 1 || si < s_min + 1 ||
        si > s_max - 2)
      return false;
    update_gradient();
    std::memset(descr, 0, sizeof(float) * NBO * NBP * NBP);
    const float* pt = grad.data() + xi * xo + (size_t)yi * yo + (si - s_min - 1) * so;
    float* dpt = descr + (NBP / 2) * binyo + (NBP / 2) * binxo;
    for (int dyi = std::max(-W, 1 - yi); dyi <= std::min(W, h - yi - 2); ++dyi)
      for (int dxi = std::max(-W, 1 - xi); dxi <= std::min(W, w - xi - 2); ++dxi) {
        const float mod = *(pt + dxi * xo + (ptrdiff_t)dyi * yo);
        const float angle = *(pt + dxi * xo + (ptrdiff_t)dyi * yo + 1);
        const float theta = mod_2pi_f((float)(angle - angle0));
        const float dx = (float)(xi + dxi - x);
        const float dy = (float)(yi + dyi - y);
        const float nx = (float)((ct0 * dx + st0 * dy) / SBP);
        const float ny = (float)((-st0 * dx + ct0 * dy) / SBP);
        const float nt = (float)(NBO * theta / (2 * kPi));
        const float wsigma = (float)(NBP / 2);
        const float win = (float)fast_expn((nx * nx + ny * ny) / (2.0 * wsigma * wsigma));
        const int binx = (int)std::floor((float)(nx - 0.5));
        const int biny = (int)std::floor((float)(ny - 0.5));
        const int bint = (int)std::floor(nt);
        const float rbinx = (float)(nx - (binx + 0.5));
        const float rbiny = (float)(ny - (biny + 0.5));
        const float rbint = nt - bint;
        for (int dbinx = 0; dbinx < 2; ++dbinx)
          for (int dbiny = 0; dbiny < 2; ++dbiny)
            for (int dbint = 0; dbint < 2; ++dbint)
              if (binx + dbinx >= -(NBP / 2) && binx + dbinx < (NBP / 2) &&
                  biny + dbiny >= -(NBP / 2) && biny + dbiny < (NBP / 2)) {
                const float weight = win * mod * std::fabs(1 - dbinx - rbinx) *
                                     std::fabs(1 - dbiny - rbiny) * std::fabs(1 - dbint - rbint);
                *(dpt + ((bint + dbint) % NBO) * binto + (biny + dbiny) * binyo +
                  (binx + dbinx) * binxo) += weight;
              }
      }
    auto normalize = [&]() {
      float norm = 0;
      for (int i = 0; i < 128; ++i) norm += descr[i] * descr[i];
      norm = fast_sqrt_f(norm) + kEpsF;
      for (int i = 0; i < 128; ++i) descr[i] /= norm;
    };
    normalize();
    for (int i = 0; i < 128; ++i)
      if (descr[i] > 0.2) descr[i] = 0.2;
    normalize();
    return true;
  }
};

// COLMAP L1RootNormalizeFeatureDescriptors (row L1 norm in index order, then
// elementwise sqrt).
void l1_root(float* d) {
  float norm = 0;
  for (int i = 0; i < 128; ++i) norm += std::fabs(d[i]);
  for (int i = 0; i < 128; ++i) d[i] = d[i] / norm;
  for (int i = 0; i < 128; ++i) d[i] = std::sqrt(d[i]);
}

// FeatureDescriptorsToUnsignedByte + TransformVLFeatToUBCFeatureDescriptors
// (orientation bins of each spatial cell reordered k -> q[k]).
void to_ubc_u8(const float* d, uint8_t* out) {
  static const int q[8] = {0, 7, 6, 5, 4, 3, 2, 1};
  for (int c = 0; c < 16; ++c)
    for (int k = 0; k < 8; ++k) {
      const float v = std::round(512.0f * d[8 * c + k]);
      out[8 * c + q[k]] = (uint8_t)std::min(255.0f, std::max(0.0f, v));
    }
}

struct Feature {
  float kp[6];
  uint8_t desc[128];
};

// Grey conversion of the op (FreeImage BGR memory order, LUMA_REC709 + 0.5).
void frame_to_grey(const uint8_t* frame, int w, int h, int ch, std::vector<uint8_t>* g) {
  g->resize((size_t)w * h);
  for (size_t i = 0; i < (size_t)w * h; ++i) {
    const uint8_t* p = frame + i * ch;
    if (ch == 1) {
      (*g)[i] = p[0];
    } else {
      const float r = p[2], gg = p[1], b = p[0];
      (*g)[i] = (uint8_t)(0.2126F * r + 0.7152F * gg + 0.0722F * b + 0.5F);
    }
  }
}

// FreeImage 3.17 CWeightsTable (Resize.cpp) of CBilinearFilter (width 1) for
// a src -> dst line: per destination pixel the source range [left, left +
// cnt) and its normalised weights.
struct RescaleTable {
  std::vector<int> left, cnt;
  std::vector<std::vector<double>> w;
};

RescaleTable rescale_table(int dst, int src) {
  RescaleTable t;
  const double filter_width = 1.0;
  const double scale = double(dst) / double(src);
  double width, fscale;
  if (scale < 1.0) {
    width = filter_width / scale;
    fscale = scale;
  } else {
    width = filter_width;
    fscale = 1.0;
  }
  const double offset = 0.5 / scale;
  for (int u = 0; u < dst; ++u) {
    const double center = (double)u / scale + offset;
    const int lo = std::max(0, (int)(center - width + 0.5));
    const int hi = std::min((int)(center + width + 0.5), src);
    std::vector<double> w;
    double total = 0;
    for (int i = lo; i < hi; ++i) {
      const double x = std::fabs(fscale * ((double)i + 0.5 - center));
      const double weight = fscale * (x < filter_width ? filter_width - x : 0.0);
      w.push_back(weight);
      total += weight;
    }
    if (total > 0 && total != 1)
      for (double& x : w) x /= total;
    int right = hi;
    while (right > lo && w[right - lo - 1] == 0) --right;  // trailing null weights
    w.resize(right - lo);
    t.left.push_back(lo);
    t.cnt.push_back(right - lo);
    t.w.push_back(w);
  }
  return t;
}

inline uint8_t to_byte(double v) { return (uint8_t)std::min(std::max((int)(v + 0.5), 0), 255); }

// FreeImage_Rescale(FILTER_BILINEAR) of an 8-bit grey image (top-down rows
// here; FreeImage's scanline j is row h - 1 - j, which the vertical pass's
// weight table indexes).
void rescale_grey(const std::vector<uint8_t>& g, int w, int h, int nw, int nh,
                  std::vector<uint8_t>* out) {
  const RescaleTable th = rescale_table(nw, w), tv = rescale_table(nh, h);
  auto horiz = [&](const std::vector<uint8_t>& src, int rows, std::vector<uint8_t>* dst) {
    dst->assign((size_t)nw * rows, 0);
    for (int y = 0; y < rows; ++y)
      for (int x = 0; x < nw; ++x) {
        double v = 0;
        for (int i = 0; i < th.cnt[x]; ++i)
          v += th.w[x][i] * (double)src[(size_t)y * w + th.left[x] + i];
        (*dst)[(size_t)y * nw + x] = to_byte(v);
      }
  };
  auto vert = [&](const std::vector<uint8_t>& src, int cols, std::vector<uint8_t>* dst) {
    dst->assign((size_t)cols * nh, 0);
    for (int r = 0; r < nh; ++r) {
      const int u = nh - 1 - r;  // destination scanline
      for (int x = 0; x < cols; ++x) {
        double v = 0;
        for (int i = 0; i < tv.cnt[u]; ++i)
          v += tv.w[u][i] * (double)src[(size_t)(h - 1 - (tv.left[u] + i)) * cols + x];
        (*dst)[(size_t)r * cols + x] = to_byte(v);
      }
    }
  };
  std::vector<uint8_t> tmp;
  if ((int64_t)nw * h <= (int64_t)nh * w) {  // xy: the smaller intermediate
    horiz(g, h, &tmp);
    vert(tmp, nw, out);
  } else {
    vert(g, w, &tmp);
    horiz(tmp, nh, out);
  }
}

// resizeBitmap (extraction_op.cc:28-39): the new size, or (w, h) when the
// image fits.
void fit_size(int w, int h, int max_size, int* nw, int* nh) {
  *nw = w;
  *nh = h;
  if (w > max_size || h > max_size) {
    const double scale = (double)max_size / std::max(w, h);
    *nw = (int)(w * scale);
    *nh = (int)(h * scale);
  }
}

// colmap::ExtractSiftFeaturesCPU.
void extract(const std::vector<uint8_t>& grey, int w, int h, const SiftOpts& o,
             std::vector<Feature>* out, std::vector<int>* level_sizes) {
  Sift sift(w, h, o.num_octaves, o.octave_resolution, o.first_octave);
  sift.peak_thresh = o.peak_threshold;
  sift.edge_thresh = o.edge_threshold;
  std::vector<float> im((size_t)w * h);
  for (size_t i = 0; i < im.size(); ++i) im[i] = (float)grey[i] / 255.0f;
  std::vector<int> level_num;                       // keypoints per DoG level
  std::vector<std::vector<Feature>> level_feats;    // with orientations
  float desc[128];
  std::memset(desc, 0, sizeof(desc));
  bool first = true;
  while (true) {
    if (first) {
      sift.first_octave(im.data());
      first = false;
    } else if (!sift.next_octave()) {
      break;
    }
    sift.detect();
    const std::vector<Keypoint> keys = sift.keys;
    int prev_level = -1;
    for (const Keypoint& k : keys) {
      if (k.is != prev_level) {
        level_num.push_back(0);
        level_feats.emplace_back();
      }
      level_num.back() += 1;
      prev_level = k.is;
      double angles[4];
      const int na = sift.orientations(angles, k);
      const int nu = std::min(na, o.max_num_orientations);
      for (int a = 0; a < nu; ++a) {
        Feature f;
        const float ori = (float)angles[a];
        const float x = k.x + 0.5f, y = k.y + 0.5f, sc = k.sigma;
        f.kp[0] = x;
        f.kp[1] = y;
        f.kp[2] = sc * std::cos(ori);
        f.kp[3] = -sc * std::sin(ori + 0.0f);
        f.kp[4] = sc * std::sin(ori);
        f.kp[5] = sc * std::cos(ori + 0.0f);
        sift.descriptor(desc, k, angles[a]);
        l1_root(desc);
        to_ubc_u8(desc, f.desc);
        level_feats.back().push_back(f);
      }
    }
  }
  int first_keep = 0, nf = 0;
  for (int i = (int)level_feats.size() - 1; i >= 0; --i) {
    nf += level_num[i];
    if (nf > o.max_num_features) {
      first_keep = i;
      break;
    }
  }
  out->clear();
  if (level_sizes) level_sizes->clear();
  for (size_t i = (size_t)first_keep; i < level_feats.size(); ++i) {
    out->insert(out->end(), level_feats[i].begin(), level_feats[i].end());
    if (level_sizes) level_sizes->push_back((int)level_feats[i].size());
  }
}

template <typename T>
void put(std::vector<uint8_t>* b, const T& v) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
  b->insert(b->end(), p, p + sizeof(T));
}

uint8_t* to_heap(const std::vector<uint8_t>& v, size_t* n) {
  *n = v.size();
  uint8_t* p = (uint8_t*)std::malloc(std::max<size_t>(1, v.size()));
  if (!v.empty()) std::memcpy(p, v.data(), v.size());
  return p;
}

}  // namespace

extern "C" {

// Test hook: refine_terms on a 3 x 3 x 3 float patch p[s][y][x] (centre
// p[1][1][1]) -> the nine derivative terms.
void oracle_sift_refine_terms(const float* p27, double* out9) {
  refine_terms(p27 + 13, 3, 9, out9);
}


// SiftExtractionKernel::execute for one frame (height x width x channels
// bytes, row-major; channels 1, 3 or 4): the keypoints, descriptors and
// camera elements (io.cc byte layouts), library-allocated (oracle_free).
int oracle_sift_extract(const uint8_t* frame, int32_t width, int32_t height, int32_t channels,
                        uint64_t image_id, uint8_t** kp_out, size_t* kp_size, uint8_t** desc_out,
                        size_t* desc_size, uint8_t** cam_out, size_t* cam_size) {
  const SiftOpts o;
  // any size >= 1 x 1, as VLFeat (vl_sift_new / vl_sift_process_*_octave put no
  // floor on it: octaves of an image that small simply have no interior
  // pixels, so no keypoints, and the op still emits its three elements)
  if (!frame || width < 1 || height < 1 || !(channels == 1 || channels == 3 || channels == 4))
    return SCM_E_INVALID;
  std::vector<uint8_t> grey;
  frame_to_grey(frame, width, height, channels, &grey);
  int nw, nh;
  fit_size(width, height, o.max_image_size, &nw, &nh);
  if (nw != width || nh != height) {
    std::vector<uint8_t> small;
    rescale_grey(grey, width, height, nw, nh, &small);
    grey.swap(small);
    width = nw;
    height = nh;
  }
  std::vector<Feature> f;
  extract(grey, width, height, o, &f, nullptr);
  std::vector<uint8_t> kb, db, cb;
  put(&kb, (uint64_t)f.size());
  for (const Feature& x : f)
    for (int j = 0; j < 6; ++j) put(&kb, x.kp[j]);
  put(&db, (uint64_t)f.size());
  put(&db, (uint64_t)128);
  for (const Feature& x : f) db.insert(db.end(), x.desc, x.desc + 128);
  // create_camera_buffer (io.cc:307-333): total, camera_id (u32), model_id
  // (int), width, height (size_t), prior_focal_length (bool), num_params,
  // params (double).
  const double focal = 1.2 * std::max(width, height);
  const double params[4] = {focal, width / 2.0, height / 2.0, 0.0};
  const uint64_t total = 8 + 4 + 4 + 8 + 8 + 1 + 8 + 4 * 8;
  put(&cb, total);
  put(&cb, (uint32_t)image_id);
  put(&cb, (int32_t)2);  // SIMPLE_RADIAL
  put(&cb, (uint64_t)width);
  put(&cb, (uint64_t)height);
  put(&cb, (uint8_t)0);
  put(&cb, (uint64_t)4);
  for (double p : params) put(&cb, p);
  *kp_out = to_heap(kb, kp_size);
  *desc_out = to_heap(db, desc_size);
  *cam_out = to_heap(cb, cam_size);
  return SCM_OK;
}

// Diagnostics for the tests: grey image, and the Gaussian scale space of one
// octave (levels s_min .. s_max, each oct_w x oct_h floats) of a grey image.
int oracle_sift_grey(const uint8_t* frame, int32_t width, int32_t height, int32_t channels,
                     uint8_t* out) {
  std::vector<uint8_t> g;
  frame_to_grey(frame, width, height, channels, &g);
  std::memcpy(out, g.data(), g.size());
  return SCM_OK;
}

// Diagnostics for the tests: FreeImage_Rescale(FILTER_BILINEAR) of an 8-bit
// grey image (top-down rows) to nw x nh, and the op's fitted size.
int oracle_sift_rescale(const uint8_t* grey, int32_t width, int32_t height, int32_t nw, int32_t nh,
                        uint8_t* out) {
  if (!grey || width < 1 || height < 1 || nw < 1 || nh < 1) return SCM_E_INVALID;
  std::vector<uint8_t> g(grey, grey + (size_t)width * height), r;
  rescale_grey(g, width, height, nw, nh, &r);
  std::memcpy(out, r.data(), r.size());
  return SCM_OK;
}

int oracle_sift_fit_size(int32_t width, int32_t height, int32_t* nw, int32_t* nh) {
  fit_size(width, height, SiftOpts().max_image_size, nw, nh);
  return SCM_OK;
}

int oracle_sift_octave(const uint8_t* grey, int32_t width, int32_t height, int32_t octave,
                       float* out, int32_t* ow, int32_t* oh) {
  const SiftOpts o;
  Sift sift(width, height, o.num_octaves, o.octave_resolution, o.first_octave);
  std::vector<float> im((size_t)width * height);
  for (size_t i = 0; i < im.size(); ++i) im[i] = (float)grey[i] / 255.0f;
  sift.first_octave(im.data());
  for (int k = o.first_octave; k < octave; ++k)
    if (!sift.next_octave()) return SCM_E_INVALID;
  *ow = sift.ow;
  *oh = sift.oh;
  if (out)
    std::memcpy(out, sift.level(sift.s_min),
                sizeof(float) * (size_t)sift.ow * sift.oh * (sift.s_max - sift.s_min + 1));
  return SCM_OK;
}

// Keypoints of one image before the level selection, as rows of
// (octave, is, ix, iy, x, y, sigma, orientation count); returns the count.
int64_t oracle_sift_keypoints(const uint8_t* grey, int32_t width, int32_t height, double* out,
                              int64_t cap) {
  const SiftOpts o;
  Sift sift(width, height, o.num_octaves, o.octave_resolution, o.first_octave);
  sift.peak_thresh = o.peak_threshold;
  sift.edge_thresh = o.edge_threshold;
  std::vector<float> im((size_t)width * height);
  for (size_t i = 0; i < im.size(); ++i) im[i] = (float)grey[i] / 255.0f;
  int64_t n = 0;
  bool first = true;
  while (true) {
    if (first) {
      sift.first_octave(im.data());
      first = false;
    } else if (!sift.next_octave()) {
      break;
    }
    sift.detect();
    for (const Keypoint& k : sift.keys) {
      double ang[4];
      const int na = sift.orientations(ang, k);
      if (n < cap) {
        double* r = out + 8 * n;
        r[0] = k.o; r[1] = k.is; r[2] = k.ix; r[3] = k.iy;
        r[4] = k.x; r[5] = k.y; r[6] = k.sigma; r[7] = na;
      }
      ++n;
    }
  }
  return n;
}

// vl/mathop.h helpers, for known-answer tests.
float oracle_fast_atan2_f(float y, float x) { return fast_atan2_f(y, x); }
float oracle_fast_sqrt_f(float x) { return fast_sqrt_f(x); }
double oracle_fast_expn(double x) { return fast_expn(x); }
int32_t oracle_gauss_taps(double sigma, float* out, int32_t cap) {
  const std::vector<float> g = gauss_taps(sigma);
  for (int i = 0; i < (int)g.size() && i < cap; ++i) out[i] = g[i];
  return (int32_t)g.size();
}

}  // extern "C"
