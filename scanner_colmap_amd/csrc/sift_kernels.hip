// GPU SIFT extraction kernels.
//
// Replaces SiftExtractionKernel::execute (reference
// integration/op_cpp/extraction_op.cc:70-121): the op's grey conversion, then
// colmap::ExtractSiftFeaturesCPU, i.e. the VLFeat covariant SIFT filter
// (vl/sift.c) with COLMAP's default SiftExtractionOptions (first_octave -1,
// 4 octaves, 3 levels, peak 0.02 / 3, edge 10, 2 orientations, L1-root).
// Every floating-point value follows the reference's operation sequence
// (built with -ffp-contract=off; the same sequence as oracle/sift_oracle.cc),
// so the keypoints and descriptors are the oracle's bit for bit:
//   * Gaussian smoothing: vl_imconvcol_vf's sum over the window in ascending
//     source order (multiply, then add, float), vertical pass first, edge
//     samples repeated (VL_PAD_BY_CONTINUITY); both passes and the DoG
//     difference in one kernel per level (smooth_vh_kernel: the input window
//     and the intermediate tile in LDS, register-blocked runs of outputs);
//   * detection in VLFeat's scan order (s, y, x) by per-row counts, one
//     exclusive scan and an ordered write (ballot prefix within each wave);
//   * refinement one thread per candidate; orientation histograms and
//     descriptors one wave per keypoint (and orientation), over every
//     octave's keypoints in one launch each: the window's samples are
//     prepared 64 at a time (one per lane), written into a zero-filled
//     bin-major LDS table, and each histogram bin is owned by one lane, which
//     adds its row in VLFeat's sample order -- the reference's serial float /
//     double sums, bit for bit, with 64-way parallelism per keypoint.
// Layout: one image slot holds the first octave's six levels (the largest),
// later octaves reuse the same buffers at their smaller size; the gradient
// planes of every octave stay until the frame's describe launches.
// Third-party algorithms restated here (bit-exactness needs their constants
// and operation order): VLFeat's SIFT (vl/sift.c, vl/mathop.h; A. Vedaldi and
// B. Fulkerson, BSD licence) and FreeImage 3.17's bilinear rescale
// (Source/FreeImageToolkit/Resize.cpp; FreeImage Public License), as COLMAP
// 3.4 calls them.  The code is written from their published algorithms; no
// source of theirs is copied.
#include "sift_kernels.h"

namespace scm {
namespace {

constexpr double kPi = 3.141592653589793;        // VL_PI
constexpr float kEpsF = 1.19209290E-07F;         // VL_EPSILON_F
constexpr double kEpsD = 2.220446049250313e-16;  // VL_EPSILON_D
constexpr int kSMin = -1, kSMax = 4, kS = 3;
constexpr int kVTile = 64;   // vertical pass: 64 columns x 64 rows per block
constexpr int kHTile = 1024; // horizontal pass: 1024 outputs of a row per block
constexpr int kGrid = 2048;  // grid-stride kernels over device-side counts

// The op's grey value (FreeImage B, G, R memory order; LUMA_REC709 + 0.5).
__device__ __forceinline__ uint8_t grey_u8_at(const uint8_t* f, int w, int ch, int y, int x) {
  const uint8_t* p = f + ((size_t)y * w + x) * ch;
  if (ch == 1) return p[0];
  const float r = p[2], gg = p[1], b = p[0];
  return (uint8_t)(0.2126F * r + 0.7152F * gg + 0.0722F * b + 0.5F);
}

// ... as the float the SIFT filter reads (grey / 255.0f).
__device__ __forceinline__ float grey_at(const uint8_t* f, int w, int ch, int y, int x) {
  return (float)grey_u8_at(f, w, ch, y, x) / 255.0f;
}

// Grey image of a frame larger than max_image_size (the input of the rescale).
__global__ void grey_kernel(const uint8_t* __restrict__ f, int w, int h, int ch,
                            uint8_t* __restrict__ out) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x < w) out[(size_t)y * w + x] = grey_u8_at(f, w, ch, y, x);
}

// FreeImage_Rescale(FILTER_BILINEAR) of the 8-bit grey bitmap (resizeBitmap,
// extraction_op.cc:28-39), one axis per launch: each output pixel is the fp64
// sum, in ascending source order, of the CWeightsTable weights times the
// source bytes, rounded to BYTE ((int)(v + 0.5), clamped) -- FreeImage 3.17
// Resize.cpp's 8-bit horizontalFilter / verticalFilter.  The vertical table is
// indexed in FreeImage's bottom-up scanline order (scanline j = row h - 1 - j).
__device__ __forceinline__ uint8_t rescale_byte(double v) {
  const int i = (int)(v + 0.5);
  return (uint8_t)(i < 0 ? 0 : (i > 255 ? 255 : i));
}

__global__ void rescale_rows_kernel(const uint8_t* __restrict__ src, int sw,
                                    uint8_t* __restrict__ dst, int dw,
                                    const int2* __restrict__ hdr, const double* __restrict__ wt,
                                    int win) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= dw) return;
  const int2 lc = hdr[x];
  const uint8_t* s = src + (size_t)y * sw + lc.x;
  const double* wx = wt + (size_t)x * win;
  double v = 0.0;
  for (int i = 0; i < lc.y; ++i) v += wx[i] * (double)s[i];
  dst[(size_t)y * dw + x] = rescale_byte(v);
}

__global__ void rescale_cols_kernel(const uint8_t* __restrict__ src, int w, int sh,
                                    uint8_t* __restrict__ dst, int dh,
                                    const int2* __restrict__ hdr, const double* __restrict__ wt,
                                    int win) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, r = blockIdx.y;
  if (x >= w) return;
  const int u = dh - 1 - r;  // destination scanline
  const int2 lc = hdr[u];
  const double* wu = wt + (size_t)u * win;
  double v = 0.0;
  for (int i = 0; i < lc.y; ++i) v += wu[i] * (double)src[(size_t)(sh - 1 - (lc.x + i)) * w + x];
  dst[(size_t)r * w + x] = rescale_byte(v);
}

// copy_and_upsample_rows twice (x first, then y): out is 2w x 2h.
__global__ void upsample_kernel(const uint8_t* __restrict__ f, int w, int h, int ch,
                                float* __restrict__ out) {
  const int X = blockIdx.x * blockDim.x + threadIdx.x, Y = blockIdx.y;
  if (X >= 2 * w) return;
  const int i = X >> 1;
  auto row_up = [&](int yy) -> float {
    const float a = grey_at(f, w, ch, yy, i);
    if ((X & 1) == 0 || i + 1 >= w) return a;
    return (a + grey_at(f, w, ch, yy, i + 1)) * 0.5f;
  };
  const int y = Y >> 1;
  const float a = row_up(y);
  float v = a;
  if ((Y & 1) && y + 1 < h) v = (a + row_up(y + 1)) * 0.5f;
  out[(size_t)Y * 2 * w + X] = v;
}

__global__ __launch_bounds__(256) void smooth_v_kernel(const float* __restrict__ in,
                                                       float* __restrict__ out, int w, int h,
                                                       const float* __restrict__ taps, int W) {
  __shared__ float tile[(kVTile + kSiftMaxTaps - 1) * kVTile];
  __shared__ float g[kSiftMaxTaps];
  const int tx = threadIdx.x & (kVTile - 1), ty = threadIdx.x / kVTile;
  const int x = blockIdx.x * kVTile + tx;
  const int y0 = blockIdx.y * kVTile;
  if ((int)threadIdx.x < 2 * W + 1) g[threadIdx.x] = taps[threadIdx.x];
  const int nrows = min(kVTile, h - y0) + 2 * W;
  for (int r = ty; r < nrows; r += 256 / kVTile) {
    const int p = min(max(y0 - W + r, 0), h - 1);
    tile[r * kVTile + tx] = x < w ? in[(size_t)p * w + x] : 0.0f;
  }
  __syncthreads();
  if (x >= w) return;
  for (int yl = ty; yl < kVTile; yl += 256 / kVTile) {
    const int y = y0 + yl;
    if (y >= h) break;
    float acc = 0.0f;
    for (int k = 0; k <= 2 * W; ++k) acc += tile[(yl + k) * kVTile + tx] * g[2 * W - k];
    out[(size_t)y * w + x] = acc;
  }
}

__global__ __launch_bounds__(256) void smooth_h_kernel(const float* __restrict__ in,
                                                       float* __restrict__ out, int w, int h,
                                                       const float* __restrict__ taps, int W) {
  __shared__ float row[kHTile + kSiftMaxTaps - 1];
  __shared__ float g[kSiftMaxTaps];
  const int y = blockIdx.y, x0 = blockIdx.x * kHTile;
  if ((int)threadIdx.x < 2 * W + 1) g[threadIdx.x] = taps[threadIdx.x];
  const float* src = in + (size_t)y * w;
  const int n = min(kHTile, w - x0) + 2 * W;
  for (int i = threadIdx.x; i < n; i += 256) row[i] = src[min(max(x0 - W + i, 0), w - 1)];
  __syncthreads();
  for (int xl = threadIdx.x; xl < kHTile; xl += 256) {
    const int x = x0 + xl;
    if (x >= w) break;
    float acc = 0.0f;
    for (int k = 0; k <= 2 * W; ++k) acc += row[xl + k] * g[2 * W - k];
    out[(size_t)y * w + x] = acc;
  }
}

// The same two passes fused for the widths the filter uses (W = 5, 7, 8, 10,
// 13): one workgroup per 64 x 64 output tile stages the (64 + 2W)^2 input
// window (edges clamped) in LDS, runs the vertical pass over the window's
// 64 + 2W columns (kSmoothVR rows per thread), then -- in the same LDS, once
// the window is consumed -- the horizontal pass (kSmoothR outputs per
// thread), and writes the level plus, when dog is given, the DoG level
// out - in (the difference dog_kernel took; the centre inputs are kept in
// registers).  Each thread's outputs come from a run of samples in
// registers, taps in scalar registers: every output is the same
// multiply-then-add sequence in ascending source order as the two-kernel
// path, and the intermediate level never goes to HBM.  in and out must differ
// (the window is read while other tiles write).  The horizontal pass reads
// lane = row (odd pitch: no bank conflicts); results leave through LDS for
// coalesced stores.
constexpr int kSmoothR = 16, kSmoothVR = 32;

template <int W>
__global__ __launch_bounds__(256) void smooth_vh_kernel(const float* __restrict__ in,
                                                        float* __restrict__ out,
                                                        float* __restrict__ dog, int w, int h,
                                                        const float* __restrict__ taps) {
  constexpr int N = 2 * W + 1, R = kSmoothR, VR = kSmoothVR, C = 64 + 2 * W;  // window side
  constexpr int PM = C | 1;  // pitch of the intermediate and output tiles (odd)
  static_assert(64 * PM <= C * C, "the intermediate tile reuses the window's LDS");
  __shared__ float lds[C * C];
  const int x0 = blockIdx.x * 64, y0 = blockIdx.y * 64;
  const int tid = threadIdx.x;
  for (int i = tid; i < C * C; i += 256) {
    const int r = i / C, c = i - r * C;
    const int yy = min(max(y0 - W + r, 0), h - 1), xx = min(max(x0 - W + c, 0), w - 1);
    lds[i] = in[(size_t)yy * w + xx];
  }
  float g[N];
#pragma unroll
  for (int k = 0; k < N; ++k) g[k] = taps[k];
  __syncthreads();
  float ctr[16];  // the inputs at this thread's 16 output pixels (tile element tid + 256 m)
  if (dog) {
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int i = tid + 256 * m;
      ctr[m] = lds[((i >> 6) + W) * C + (i & 63) + W];
    }
  }
  // vertical pass: column c, rows yl0 .. yl0 + VR - 1 of the tile
  const bool vt = tid < C * (64 / VR);
  const int c = tid % C, yl0 = (tid / C) * VR;
  float vacc[VR];
  if (vt) {
    float v[VR + 2 * W];
#pragma unroll
    for (int j = 0; j < VR + 2 * W; ++j) v[j] = lds[(yl0 + j) * C + c];
#pragma unroll
    for (int r = 0; r < VR; ++r) vacc[r] = 0.0f;
#pragma unroll
    for (int k = 0; k < N; ++k)
#pragma unroll
      for (int r = 0; r < VR; ++r) vacc[r] += v[r + k] * g[2 * W - k];
  }
  __syncthreads();
  if (vt) {
#pragma unroll
    for (int r = 0; r < VR; ++r) lds[(yl0 + r) * PM + c] = vacc[r];
  }
  __syncthreads();
  // horizontal pass: row, outputs xs .. xs + R - 1
  const int row = tid & 63, xs = (tid >> 6) * R;
  float acc[R];
  {
    float v[R + 2 * W];
#pragma unroll
    for (int j = 0; j < R + 2 * W; ++j) v[j] = lds[row * PM + xs + j];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.0f;
#pragma unroll
    for (int k = 0; k < N; ++k)
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] += v[r + k] * g[2 * W - k];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) lds[row * PM + xs + r] = acc[r];
  __syncthreads();
  const int nr = min(64, h - y0), nc = min(64, w - x0);
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int i = tid + 256 * m, r = i >> 6, cc = i & 63;
    if (r < nr && cc < nc) {
      const float o = lds[r * PM + cc];
      const size_t at = (size_t)(y0 + r) * w + x0 + cc;
      out[at] = o;
      if (dog) dog[at] = o - ctr[m];
    }
  }
}

// DoG level of the two-kernel path: dog = a - b.
__global__ void sub_kernel(const float* __restrict__ a, const float* __restrict__ b,
                           float* __restrict__ dog, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    dog[i] = a[i] - b[i];
}

__global__ void downsample_kernel(const float* __restrict__ in, int w_in, float* __restrict__ out,
                                  int w, int h) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x < w) out[(size_t)y * w + x] = in[(size_t)(2 * y) * w_in + 2 * x];
}

// vl_sift_detect's 26-neighbour strict extremum test at DoG level s.
__device__ __forceinline__ bool is_extremum(const float* __restrict__ dog, int w, size_t so, int x,
                                            int y, int s, double tp) {
  const float* pt = dog + so * (size_t)(s - kSMin) + (size_t)y * w + x;
  const float v = *pt;
  bool mx = v >= 0.8 * tp, mn = v <= -0.8 * tp;
  if (!(mx || mn)) return false;
  for (int ds = -1; ds <= 1; ++ds)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        if (!ds && !dy && !dx) continue;
        const float u = *(pt + (ptrdiff_t)ds * (ptrdiff_t)so + (ptrdiff_t)dy * w + dx);
        mx = mx && v > u;
        mn = mn && v < u;
      }
  return mx || mn;
}

// Extrema per (level l = s, row y): grid (h, 3).
__global__ __launch_bounds__(256) void detect_count_kernel(const float* __restrict__ dog, int w,
                                                           int h, double tp,
                                                           int32_t* __restrict__ rowcnt) {
  __shared__ int c;
  const int y = blockIdx.x, s = blockIdx.y;
  if (threadIdx.x == 0) c = 0;
  __syncthreads();
  int mine = 0;
  if (y >= 1 && y < h - 1)
    for (int x = 1 + threadIdx.x; x < w - 1; x += 256)
      mine += is_extremum(dog, w, (size_t)w * h, x, y, s, tp);
  if (mine) atomicAdd(&c, mine);
  __syncthreads();
  if (threadIdx.x == 0) rowcnt[s * h + y] = c;
}

// The extrema of one (level, row) in x order at rowoff[level h + row].
__global__ __launch_bounds__(256) void detect_write_kernel(const float* __restrict__ dog, int w,
                                                           int h, double tp,
                                                           const int32_t* __restrict__ rowoff,
                                                           SiftCand* __restrict__ cand, int cap) {
  __shared__ int wsum[4];
  const int y = blockIdx.x, s = blockIdx.y;
  if (y < 1 || y >= h - 1) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int base = rowoff[s * h + y];
  for (int x0 = 1; x0 < w - 1; x0 += 256) {
    const int x = x0 + threadIdx.x;
    const bool f = x < w - 1 && is_extremum(dog, w, (size_t)w * h, x, y, s, tp);
    const uint64_t b = __ballot(f);
    if (lane == 0) wsum[wave] = __popcll(b);
    __syncthreads();
    int off = 0;
    for (int k = 0; k < wave; ++k) off += wsum[k];
    const int tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (f) {
      const int idx = base + off + __popcll(b & ((1ull << lane) - 1ull));
      if (idx < cap) cand[idx] = SiftCand{x, y, s, 0};
    }
    base += tot;
    __syncthreads();
  }
}

// Exclusive scan of n = (n_dev ? *n_dev : n_const) counts, one workgroup;
// out[i] = base + prefix with base = (acc ? *acc : 0); *total = sum,
// *acc = base + sum.
__global__ __launch_bounds__(1024) void scan_kernel(const int32_t* __restrict__ in,
                                                    int32_t* __restrict__ out,
                                                    const int32_t* __restrict__ n_dev, int n_const,
                                                    int cap, int32_t* __restrict__ total,
                                                    int32_t* __restrict__ acc) {
  __shared__ int buf[1024];
  const int tid = threadIdx.x;
  const int n = min(n_dev ? *n_dev : n_const, cap);
  const int base = acc ? *acc : 0;
  int run = base;
  for (int c0 = 0; c0 < n; c0 += 1024) {
    const int v = c0 + tid < n ? in[c0 + tid] : 0;
    buf[tid] = v;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
      const int t = tid >= d ? buf[tid - d] : 0;
      __syncthreads();
      buf[tid] += t;
      __syncthreads();
    }
    if (c0 + tid < n) out[c0 + tid] = run + buf[tid] - v;
    run += buf[1023];
    __syncthreads();
  }
  if (tid == 0) {
    if (total) *total = run - base;
    if (acc) *acc = run;
  }
}

__global__ void set_count_kernel(SiftCounts* cnt, const int32_t* __restrict__ tot, int which,
                                 int cap) {
  const int v = *tot;
  if (v > cap) cnt->overflow = 1;
  if (which == 0) cnt->ncand = min(v, cap);
  else cnt->nkey = min(v, cap);
}

// Keypoint refinement of vl_sift_detect (quadratic fit, <= 5 moves, Gauss
// elimination with partial pivoting, peak / edge / bounds tests).
__global__ __launch_bounds__(64) void refine_kernel(const float* __restrict__ dog, int w, int h,
                                                    const SiftCand* __restrict__ cand,
                                                    const SiftCounts* __restrict__ cnt,
                                                    SiftKey* __restrict__ out,
                                                    int32_t* __restrict__ flag, double tp,
                                                    double te, double sigma0, int octave) {
  const int n = cnt->ncand;
  const size_t so = (size_t)w * h;
  const double xper = ldexp(1.0, octave);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const SiftCand c = cand[i];
    int x = c.x, y = c.y;
    const int s = c.s;
    double Dx = 0, Dy = 0, Ds = 0, Dxx = 0, Dyy = 0, Dss = 0, Dxy = 0, Dxs = 0, Dys = 0;
    double A[9], b[3];
    int dx = 0, dy = 0;
    const float* pt = nullptr;
    for (int iter = 0; iter < 5; ++iter) {
      x += dx;
      y += dy;
      pt = dog + (size_t)x + (size_t)y * w + so * (size_t)(s - kSMin);
// VLFeat's at() reads vl_sift_pix (float): sums and differences of samples
// round in float, and only the products with the double literals (0.5, 2.0,
// 0.25) widen to double -- C's usual arithmetic conversions, kept here.
#define AT(ax, ay, as) (*(pt + (ax) + (ptrdiff_t)(ay) * w + (ptrdiff_t)(as) * (ptrdiff_t)so))
      Dx = 0.5 * (AT(1, 0, 0) - AT(-1, 0, 0));
      Dy = 0.5 * (AT(0, 1, 0) - AT(0, -1, 0));
      Ds = 0.5 * (AT(0, 0, 1) - AT(0, 0, -1));
      Dxx = (AT(1, 0, 0) + AT(-1, 0, 0) - 2.0 * AT(0, 0, 0));
      Dyy = (AT(0, 1, 0) + AT(0, -1, 0) - 2.0 * AT(0, 0, 0));
      Dss = (AT(0, 0, 1) + AT(0, 0, -1) - 2.0 * AT(0, 0, 0));
      Dxy = 0.25 * (AT(1, 1, 0) + AT(-1, -1, 0) - AT(-1, 1, 0) - AT(1, -1, 0));
      Dxs = 0.25 * (AT(1, 0, 1) + AT(-1, 0, -1) - AT(-1, 0, 1) - AT(1, 0, -1));
      Dys = 0.25 * (AT(0, 1, 1) + AT(0, -1, -1) - AT(0, -1, 1) - AT(0, 1, -1));
#undef AT
      A[0] = Dxx; A[4] = Dyy; A[8] = Dss;
      A[3] = A[1] = Dxy;
      A[6] = A[2] = Dxs;
      A[7] = A[5] = Dys;
      b[0] = -Dx; b[1] = -Dy; b[2] = -Ds;
      for (int j = 0; j < 3; ++j) {
        double maxa = 0, maxabsa = 0;
        int maxi = -1;
        for (int ii = j; ii < 3; ++ii) {
          const double av = A[ii + 3 * j], absa = fabs(av);
          if (absa > maxabsa) {
            maxa = av;
            maxabsa = absa;
            maxi = ii;
          }
        }
        if (maxabsa < 1e-10f) {
          b[0] = b[1] = b[2] = 0;
          break;
        }
        const int r = maxi;
        for (int jj = j; jj < 3; ++jj) {
          const double t = A[r + 3 * jj];
          A[r + 3 * jj] = A[j + 3 * jj];
          A[j + 3 * jj] = t;
          A[j + 3 * jj] /= maxa;
        }
        const double t = b[j];
        b[j] = b[r];
        b[r] = t;
        b[j] /= maxa;
        for (int ii = j + 1; ii < 3; ++ii) {
          const double xx = A[ii + 3 * j];
          for (int jj = j; jj < 3; ++jj) A[ii + 3 * jj] -= xx * A[j + 3 * jj];
          b[ii] -= xx * b[j];
        }
      }
      for (int ii = 2; ii > 0; --ii) {
        const double xx = b[ii];
        for (int k = ii - 1; k >= 0; --k) b[k] -= xx * A[k + 3 * ii];
      }
      dx = ((b[0] > 0.6 && x < w - 2) ? 1 : 0) + ((b[0] < -0.6 && x > 1) ? -1 : 0);
      dy = ((b[1] > 0.6 && y < h - 2) ? 1 : 0) + ((b[1] < -0.6 && y > 1) ? -1 : 0);
      if (dx == 0 && dy == 0) break;
    }
    const double val = (double)*pt + 0.5 * (Dx * b[0] + Dy * b[1] + Ds * b[2]);
    const double score = (Dxx + Dyy) * (Dxx + Dyy) / (Dxx * Dyy - Dxy * Dxy);
    const double xn = x + b[0], yn = y + b[1], sn = s + b[2];
    const bool ok = fabs(val) > tp && score < (te + 1) * (te + 1) / te && score >= 0 &&
                    fabs(b[0]) < 1.5 && fabs(b[1]) < 1.5 && fabs(b[2]) < 1.5 && xn >= 0 &&
                    xn <= w - 1 && yn >= 0 && yn <= h - 1 && sn >= kSMin && sn <= kSMax;
    flag[i] = ok ? 1 : 0;
    if (ok) {
      SiftKey k;
      k.o = octave;
      k.ix = x;
      k.iy = y;
      k.is = s;
      k.s = (float)sn;
      k.x = (float)(xn * xper);
      k.y = (float)(yn * xper);
      k.sigma = (float)(sigma0 * pow(2.0, sn / kS) * xper);
      out[i] = k;
    }
  }
}

__global__ void compact_keys_kernel(const SiftKey* __restrict__ ktmp, const int32_t* __restrict__ flag,
                                    const int32_t* __restrict__ off, SiftCounts* __restrict__ cnt,
                                    SiftKey* __restrict__ keys, int cap, int octave) {
  const int n = cnt->ncand;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    if (flag[i]) {
      const int j = off[i];
      if (j < cap) {
        keys[j] = ktmp[i];
        atomicAdd(&cnt->level_keys[(octave + 1) * 3 + ktmp[i].is], 1);
      }
    }
}

// vl/mathop.h
__device__ __forceinline__ float fast_resqrt_f(float x) {
  const float xhalf = 0.5F * x;
  float y = __int_as_float(0x5f3759df - (__float_as_int(x) >> 1));
  y = y * (1.5F - xhalf * y * y);
  y = y * (1.5F - xhalf * y * y);
  return y;
}
__device__ __forceinline__ float fast_sqrt_f(float x) { return (x < 1e-8) ? 0 : x * fast_resqrt_f(x); }
__device__ __forceinline__ float fast_atan2_f(float y, float x) {
  const float c3 = 0.1821F, c1 = 0.9675F;
  const float abs_y = fabsf(y) + kEpsF;
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
__device__ __forceinline__ float mod_2pi_f(float x) {
  while (x > (float)(2 * kPi)) x -= (float)(2 * kPi);
  while (x < 0.0F) x += (float)(2 * kPi);
  return x;
}
__device__ __forceinline__ double fast_expn(const double* __restrict__ tab, double x) {
  if (x > 25.0) return 0.0;
  x *= 256 / 25.0;
  const int i = (int)floor(x);
  const double r = x - i;
  const double a = tab[i], b = tab[i + 1];
  return a + r * (b - a);
}

// update_gradient for levels s = 0 .. 2: (modulus, angle in [0, 2 pi]).
__global__ void gradient_kernel(const float* __restrict__ lev, float2* __restrict__ grad, int w,
                                int h) {
  const size_t so = (size_t)w * h;
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, l = blockIdx.z;
  if (x >= w) return;
  const float* p = lev + so * (size_t)(l + 1) + (size_t)y * w + x;
  float gx, gy;
  if (x == 0) gx = p[1] - p[0];
  else if (x == w - 1) gx = p[0] - p[-1];
  else gx = (p[1] - p[-1]) * 0.5f;
  if (y == 0) gy = p[w] - p[0];
  else if (y == h - 1) gy = p[0] - p[-w];
  else gy = (p[w] - p[-w]) * 0.5f;
  grad[so * l + (size_t)y * w + x] =
      make_float2(fast_sqrt_f(gx * gx + gy * gy), mod_2pi_f((float)(fast_atan2_f(gy, gx) + 2 * kPi)));
}

// vl_sift_calc_keypoint_orientations, one wave per keypoint.  The window's
// samples are visited 64 at a time in VLFeat's (ys, xs) order: lane j
// prepares sample j of the chunk (mod * wgt) and writes it into column j of
// its bin's row of a zero-filled bin-major LDS table; lane b < 36 then adds
// row b over all 64 columns in order.  Each sample reaches one bin and every
// value is >= +0, so the added zeros leave the double sums unchanged -- the
// serial histogram's additions in its order.  The six smoothing passes read
// only the previous pass's bins (new[b] = (old[b-1] + old[b] + old[b+1]) / 3,
// circular), so lane b computes bin b; the peaks are the first two set bits
// of a ballot in bin order (VLFeat keeps up to 4, COLMAP uses 2).
constexpr int kOriRow = 66;  // doubles per bin row (64 samples + pad)

__global__ __launch_bounds__(64) void orient_kernel(SiftOctaves oct,
                                                    const SiftKey* __restrict__ keys,
                                                    SiftCounts* __restrict__ cnt,
                                                    int32_t* __restrict__ nori,
                                                    double* __restrict__ ang,
                                                    const double* __restrict__ expn) {
  constexpr int nbins = 36;
  __shared__ __attribute__((aligned(16))) double s_v[nbins * kOriRow];
  __shared__ double s_expn[257];
  __shared__ double hist[nbins];
  const int lane = threadIdx.x;
  for (int b = lane; b < nbins * kOriRow; b += 64) s_v[b] = 0.0;
  for (int b = lane; b < 257; b += 64) s_expn[b] = expn[b];
  __syncthreads();
  const int n = cnt->nkey;
  const double2* row = reinterpret_cast<const double2*>(s_v + min(lane, nbins - 1) * kOriRow);
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    const SiftKey k = keys[i];
    const int octave = k.o, w = oct.w[octave + 1], h = oct.h[octave + 1];
    const float2* __restrict__ grad = oct.grad[octave + 1];
    const double xper = ldexp(1.0, octave);
    const size_t so = (size_t)w * h;
    const double x = k.x / xper, y = k.y / xper, sigma = k.sigma / xper;
    const int xi = (int)(x + 0.5), yi = (int)(y + 0.5), si = k.is;
    const double sigmaw = 1.5 * sigma;
    const int W = max((int)floor(3.0 * sigmaw), 1);
    const bool valid =
        !(xi < 0 || xi > w - 1 || yi < 0 || yi > h - 1 || si < kSMin + 1 || si > kSMax - 2);
    int nu = 0;
    double out0 = 0.0, out1 = 0.0;
    if (valid) {
      const int ys0 = max(-W, -yi), ys1 = min(W, h - 1 - yi);
      const int xs0 = max(-W, -xi), xs1 = min(W, w - 1 - xi);
      const int ncols = xs1 - xs0 + 1, total = (ys1 - ys0 + 1) * ncols;
      const float2* pt = grad + so * (size_t)(si - kSMin - 1) + (size_t)yi * w + xi;
      double acc = 0.0;
      for (int t0 = 0; t0 < total; t0 += 64) {
        const int t = t0 + lane;
        int p = -1;
        if (t < total) {
          const int ys = ys0 + t / ncols, xs = xs0 + t % ncols;
          const double dx = (double)(xi + xs) - x, dy = (double)(yi + ys) - y;
          const double r2 = dx * dx + dy * dy;
          if (r2 < W * W + 0.6) {
            const double wgt = fast_expn(s_expn, r2 / (2 * sigmaw * sigmaw));
            const float2 g = pt[xs + (ptrdiff_t)ys * w];
            const double mod = g.x, an = g.y;
            const int bin = (int)floor(nbins * an / (2 * kPi)) % nbins;
            p = bin * kOriRow + lane;
            s_v[p] = mod * wgt;
          }
        }
        __syncthreads();
        if (lane < nbins) {
#pragma unroll
          for (int q = 0; q < 32; ++q) {
            const double2 u = row[q];
            acc += u.x;
            acc += u.y;
          }
        }
        __syncthreads();
        if (p >= 0) s_v[p] = 0.0;
      }
      // six smoothing passes, bin b on lane b
      double hb = acc;
      for (int iter = 0; iter < 6; ++iter) {
        if (lane < nbins) hist[lane] = hb;
        __syncthreads();
        if (lane < nbins) {
          const double hm = hist[(lane + nbins - 1) % nbins], hp = hist[(lane + 1) % nbins];
          hb = (hm + hb + hp) / 3.0;
        }
        __syncthreads();
      }
      if (lane < nbins) hist[lane] = hb;
      __syncthreads();
      double maxh = 0;
      for (int b = 0; b < nbins; ++b) maxh = fmax(maxh, hist[b]);
      bool peak = false;
      double th = 0.0;
      if (lane < nbins) {
        const double h0 = hb, hm = hist[(lane + nbins - 1) % nbins], hp = hist[(lane + 1) % nbins];
        if (h0 > 0.8 * maxh && h0 > hm && h0 > hp) {
          const double di = -0.5 * (hp - hm) / (hp + hm - 2 * h0);
          th = 2 * kPi * (lane + di + 0.5) / nbins;
          peak = true;
        }
      }
      uint64_t m = __ballot(peak);
      if (m) {
        out0 = __shfl(th, __builtin_ctzll(m));
        m &= m - 1;
        nu = 1;
        if (m) {
          out1 = __shfl(th, __builtin_ctzll(m));
          nu = 2;
        }
      }
      __syncthreads();
    }
    if (lane == 0) {
      nori[i] = nu;
      ang[2 * i] = out0;
      ang[2 * i + 1] = out1;
      if (nu) atomicAdd(&cnt->level_feats[(octave + 1) * 3 + si], nu);
    }
  }
}

// The descriptor tail of one feature by one wave, bins b = lane and lane + 64
// in a0 / a1 (VLFeat bin order): normalise, truncate at 0.2, normalise
// (vl_sift_calc_keypoint_descriptor), then COLMAP's L1-root, x512 rounding
// with TruncateCast and the UBC orientation-bin order.  The sums run serially
// in bin order on lane 0 (the reference's float sums), the elementwise steps
// on every lane.
__device__ void descriptor_finish(float a0, float a1, float* __restrict__ sh, float* __restrict__ df,
                                  uint8_t* __restrict__ out) {
  const int lane = threadIdx.x;
  for (int pass = 0; pass < 2; ++pass) {
    sh[lane] = a0;
    sh[lane + 64] = a1;
    __syncthreads();
    if (lane == 0) {
      float norm = 0;
      for (int b = 0; b < 128; ++b) norm += sh[b] * sh[b];
      sh[128] = fast_sqrt_f(norm) + kEpsF;
    }
    __syncthreads();
    const float norm = sh[128];
    a0 /= norm;
    a1 /= norm;
    if (pass == 0) {
      if (a0 > 0.2) a0 = 0.2f;
      if (a1 > 0.2) a1 = 0.2f;
    }
    __syncthreads();
  }
  sh[lane] = a0;
  sh[lane + 64] = a1;
  __syncthreads();
  if (lane == 0) {
    float norm = 0;
    for (int b = 0; b < 128; ++b) norm += fabsf(sh[b]);
    sh[128] = norm;
  }
  __syncthreads();
  const float l1 = sh[128];
  float v[2] = {sqrtf(a0 / l1), sqrtf(a1 / l1)};
  for (int q = 0; q < 2; ++q) {
    const int b = lane + 64 * q;
    df[b] = v[q];
    const float r = roundf(512.0f * v[q]);
    const float lo = (0.0f < r) ? r : 0.0f;        // std::max(0.0f, r)
    const float hi = (lo < 255.0f) ? lo : 255.0f;  // std::min(255.0f, lo)
    out[(b & ~7) + ((8 - (b & 7)) & 7)] = (uint8_t)hi;
  }
  __syncthreads();
}

// vl_sift_calc_keypoint_descriptor + the COLMAP conversions, one wave per
// (keypoint, orientation).  The sample rectangle is visited 64 samples at a
// time in VLFeat's (dyi, dxi) order: lane j prepares sample j of the chunk
// and keeps its (up to 8) bin weights.  The samples that reach a bin keep
// their order as columns 0 .. k-1 (ballot rank), 32 at a time: each writes
// its weights into its column of a bin-major LDS table whose other entries
// are zero, and lane L adds rows L and L + 64 over the used columns in order.
// A sample reaches a bin through at most one corner and every weight is >= +0
// (win * mod * |.| * |.| * |.|), so the added zeros leave the sums unchanged:
// every bin sees VLFeat's float additions in VLFeat's order.  Rows of
// kDescRow floats are read as float2 (34: the 32 lanes of a read fall on
// distinct bank pairs); the writers zero their entries again after each pass,
// and unused corners write to a dummy slot (no branches).  20 KB of LDS per
// wave: 2 waves per SIMD.
constexpr int kDescRow = 34;

__global__ __launch_bounds__(64) void descriptor_kernel(
    SiftOctaves oct, const SiftKey* __restrict__ keys, SiftCounts* __restrict__ cnt,
    const int32_t* __restrict__ nori, const double* __restrict__ ang,
    const int32_t* __restrict__ koff, SiftFeat* __restrict__ feat, float* __restrict__ descf,
    uint8_t* __restrict__ desc, int32_t* __restrict__ stale, const double* __restrict__ expn,
    int feat_cap) {
  constexpr int NBP = 4, NBO = 8;
  constexpr int kDummy = 128 * kDescRow;  // 32 dummy floats, then the finish's 129
  __shared__ __attribute__((aligned(16))) float s_v[128 * kDescRow + 32 + 129];
  __shared__ double s_expn[257];
  float* sh = s_v + kDummy + 32;
  const int lane = threadIdx.x;
  for (int b = lane; b < 128 * kDescRow; b += 64) s_v[b] = 0.0f;
  for (int b = lane; b < 257; b += 64) s_expn[b] = expn[b];
  __syncthreads();
  const int n = cnt->nkey;
  const float2* r0 = reinterpret_cast<const float2*>(s_v + lane * kDescRow);
  const float2* r1 = reinterpret_cast<const float2*>(s_v + (lane + 64) * kDescRow);
  for (int it = blockIdx.x; it < 2 * n; it += gridDim.x) {
    const int i = it >> 1, o = it & 1;
    if (o >= nori[i]) continue;
    const SiftKey k = keys[i];
    const int fi = koff[i] + o;
    if (fi >= feat_cap) {
      if (lane == 0) cnt->overflow = 1;
      continue;
    }
    const double angle0 = ang[2 * i + o];
    if (lane == 0) feat[fi] = SiftFeat{k.x + 0.5f, k.y + 0.5f, k.sigma, (float)angle0};
    const int w = oct.w[k.o + 1], h = oct.h[k.o + 1];
    const float2* __restrict__ grad = oct.grad[k.o + 1];
    const double xper = ldexp(1.0, k.o);
    const size_t so = (size_t)w * h;
    const double x = k.x / xper, y = k.y / xper, sigma = k.sigma / xper;
    const int xi = (int)(x + 0.5), yi = (int)(y + 0.5), si = k.is;
    if (xi < 0 || xi >= w || yi < 0 || yi >= h - 1 || si < kSMin + 1 || si > kSMax - 2) {
      // vl_sift_calc_keypoint_descriptor returns before writing: COLMAP
      // re-normalises the previous descriptor's buffer (fixup_kernel)
      if (lane == 0) {
        stale[fi] = 1;
        atomicAdd(&cnt->nstale, 1);
      }
      continue;
    }
    if (lane == 0) stale[fi] = 0;
    const double st0 = sin(angle0), ct0 = cos(angle0);
    const double SBP = 3.0 * sigma + kEpsD;
    const int W = (int)floor(sqrt(2.0) * SBP * (NBP + 1) / 2.0 + 0.5);
    const int dy0 = max(-W, 1 - yi), dy1 = min(W, h - yi - 2);
    const int dx0 = max(-W, 1 - xi), dx1 = min(W, w - xi - 2);
    const int ncols = dx1 - dx0 + 1, nrows = max(dy1 - dy0 + 1, 0);
    const float2* pt = grad + so * (size_t)(si - kSMin - 1) + (size_t)yi * w + xi;
    float a0 = 0.0f, a1 = 0.0f;
    // Only samples that can reach the 4 x 4 grid are visited: per row of the
    // rectangle, the dxi interval where |nx| and |ny| <= 2.5 (binx =
    // floor(nx - 0.5) in -3 .. 1, likewise biny), widened by a pixel on each
    // side and clipped to the rectangle.  Every skipped sample reaches no bin
    // and the visited ones keep VLFeat's (dyi, dxi) order.  Row r's
    // (first dxi - dx0) << 16 | length sits in rtab (the finish's scratch).
    int* rtab = reinterpret_cast<int*>(sh);
    const bool rag = nrows <= 129;
    int total = 0;
    if (ncols > 0 && nrows > 0) {
      if (rag) {
        const double B = 2.5 * SBP * (1.0 + 1e-6) + 1e-3;
        for (int rr = lane; rr < nrows; rr += 64) {
          const double dy = (double)(yi + dy0 + rr) - y;
          double lo = -1e6, hi = 1e6;  // dx = xi + dxi - x
          // |ct0 dx + st0 dy| <= B and |-st0 dx + ct0 dy| <= B
          const double ca[2] = {ct0, -st0}, cb[2] = {st0 * dy, ct0 * dy};
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            if (fabs(ca[e]) < 1e-9) {
              if (fabs(cb[e]) > B) hi = -1e6;
            } else {
              const double u = (-B - cb[e]) / ca[e], v = (B - cb[e]) / ca[e];
              lo = fmax(lo, fmin(u, v));
              hi = fmin(hi, fmax(u, v));
            }
          }
          int l = dx0, len = 0;
          if (lo <= hi) {
            l = max(dx0, (int)floor(lo + x - xi) - 1);
            len = max(0, min(dx1, (int)ceil(hi + x - xi) + 1) - l + 1);
          }
          rtab[rr] = ((l - dx0) << 16) | len;
          total += len;
        }
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) total += __shfl_xor(total, m);
      } else {
        total = ncols * nrows;
      }
    }
    __syncthreads();
    auto row_len = [&](int r) { return rag ? (rtab[r] & 0xFFFF) : ncols; };
    auto row_lo = [&](int r) { return rag ? dx0 + (rtab[r] >> 16) : dx0; };
    // the lane's sample t = t0 + lane as (row, column), stepped by 64 per
    // chunk; the next chunk's gradient is loaded while this chunk is summed
    int r = 0, c = lane;
    auto advance = [&]() {
      while (r < nrows && c >= row_len(r)) {
        c -= row_len(r);
        ++r;
      }
    };
    if (total > 0) advance();
    float2 gn = make_float2(0.0f, 0.0f);
    if (total > 0 && r < nrows) gn = pt[row_lo(r) + c + (ptrdiff_t)(dy0 + r) * w];
    for (int t0 = 0; t0 < total; t0 += 64) {
      const bool valid = r < nrows;
      const int dyi = dy0 + r, dxi = valid ? row_lo(r) + c : dx0;
      const float2 g = gn;
      c += 64;
      advance();
      gn = r < nrows ? pt[row_lo(r) + c + (ptrdiff_t)(dy0 + r) * w] : make_float2(0.0f, 0.0f);
      // every lane prepares its sample (lanes past the rectangle's end see a
      // zero gradient and reach nothing)
      float wv[8];
      int row[8];  // LDS row offset of the corner's bin, -1 outside the 4 x 4 grid
      const float mod = g.x, angle = g.y;
      const float theta = mod_2pi_f((float)(angle - angle0));
      const float dx = (float)(xi + dxi - x);
      const float dy = (float)(yi + dyi - y);
      const float nx = (float)((ct0 * dx + st0 * dy) / SBP);
      const float ny = (float)((-st0 * dx + ct0 * dy) / SBP);
      const float nt = (float)(NBO * theta / (2 * kPi));
      const float wsigma = 2.0f;
      const float win = (float)fast_expn(s_expn, (nx * nx + ny * ny) / (2.0 * wsigma * wsigma));
      const int binx = (int)floorf((float)(nx - 0.5));
      const int biny = (int)floorf((float)(ny - 0.5));
      const int bint = (int)floorf(nt);  // 0 .. 8: nt is in [0, 8]
      const float wm = win * mod;
      const float rx = (float)(nx - (binx + 0.5));
      const float ry = (float)(ny - (biny + 0.5));
      const float rt = nt - bint;
      bool reach = false;
#pragma unroll
      for (int dbinx = 0; dbinx < 2; ++dbinx)
#pragma unroll
        for (int dbiny = 0; dbiny < 2; ++dbiny)
#pragma unroll
          for (int dbint = 0; dbint < 2; ++dbint) {
            const int c = dbinx * 4 + dbiny * 2 + dbint;
            const int bx = binx + dbinx + NBP / 2, by = biny + dbiny + NBP / 2;
            const bool in = valid && (unsigned)bx < (unsigned)NBP && (unsigned)by < (unsigned)NBP;
            wv[c] = wm * fabsf(1 - dbinx - rx) * fabsf(1 - dbiny - ry) * fabsf(1 - dbint - rt);
            row[c] = in ? __mul24(((bint + dbint) & (NBO - 1)) + by * NBO * NBP + bx * NBO, kDescRow)
                        : -1;
            reach |= in;
          }
      // the reaching samples as columns 0 .. k-1 in sample order
      const uint64_t rm = __ballot(reach);
      const int kk = __popcll(rm);
      const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(rm >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)rm, 0));
      for (int c0 = 0; c0 < kk; c0 += 32) {
        const bool mine = reach && rank >= c0 && rank < c0 + 32;
        const int colp = rank - c0;
        int pos[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          pos[c] = (mine && row[c] >= 0) ? row[c] + colp : kDummy + (lane & 31);
          s_v[pos[c]] = wv[c];
        }
        __syncthreads();
        const int ng = min(kk - c0, 32);  // columns of this pass
        for (int q = 0; q < ng; q += 8) {
          float2 u[4], v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            u[e] = r0[q / 2 + e];
            v[e] = r1[q / 2 + e];
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            a0 += u[e].x;
            a1 += v[e].x;
            a0 += u[e].y;
            a1 += v[e].y;
          }
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < 8; ++c) s_v[pos[c]] = 0.0f;
      }
    }
    descriptor_finish(a0, a1, sh, descf + (size_t)fi * 128, desc + (size_t)fi * 128);
  }
}

// The unwritten descriptors in feature order: each is the L1-root of the
// previous feature's (float) buffer, the first one's of zeros.  The wave
// finds them 64 flags at a time; lane 0 recomputes each in order.
__global__ void fixup_kernel(const SiftCounts* __restrict__ cnt, const int32_t* __restrict__ stale,
                             float* __restrict__ descf, uint8_t* __restrict__ desc, int feat_cap) {
  if (cnt->nstale == 0) return;
  const int lane = threadIdx.x;
  const int n = min(cnt->nfeat, feat_cap);
  for (int base = 0; base < n; base += 64) {
    uint64_t m = __ballot(base + lane < n && stale[base + lane]);
    if (lane == 0)
      while (m) {
        const int i = base + __builtin_ctzll(m);
        m &= m - 1;
        float* d = descf + (size_t)i * 128;
        for (int b = 0; b < 128; ++b) d[b] = i ? d[b - 128] : 0.0f;
        float norm = 0;
        for (int b = 0; b < 128; ++b) norm += fabsf(d[b]);
        for (int b = 0; b < 128; ++b) d[b] = sqrtf(d[b] / norm);
        for (int b = 0; b < 128; ++b) {
          const float r = roundf(512.0f * d[b]);
          const float lo = (0.0f < r) ? r : 0.0f;
          const float hi = (lo < 255.0f) ? lo : 255.0f;
          desc[(size_t)i * 128 + (b & ~7) + ((8 - (b & 7)) & 7)] = (uint8_t)hi;
        }
      }
  }
}

int blocks_for(size_t n, int t) { return (int)((n + t - 1) / t); }

}  // namespace

hipError_t sift_upsample(const uint8_t* frame, int w, int h, int ch, float* out, hipStream_t st) {
  dim3 grid(blocks_for(2 * (size_t)w, 256), 2 * h);
  upsample_kernel<<<grid, 256, 0, st>>>(frame, w, h, ch, out);
  return hipGetLastError();
}

hipError_t sift_grey(const uint8_t* frame, int w, int h, int ch, uint8_t* out, hipStream_t st) {
  grey_kernel<<<dim3(blocks_for(w, 256), h), 256, 0, st>>>(frame, w, h, ch, out);
  return hipGetLastError();
}

hipError_t sift_rescale_rows(const uint8_t* src, int sw, int rows, uint8_t* dst, int dw,
                             const int2* hdr, const double* wt, int win, hipStream_t st) {
  rescale_rows_kernel<<<dim3(blocks_for(dw, 256), rows), 256, 0, st>>>(src, sw, dst, dw, hdr, wt,
                                                                       win);
  return hipGetLastError();
}

hipError_t sift_rescale_cols(const uint8_t* src, int cols, int sh, uint8_t* dst, int dh,
                             const int2* hdr, const double* wt, int win, hipStream_t st) {
  rescale_cols_kernel<<<dim3(blocks_for(cols, 256), dh), 256, 0, st>>>(src, cols, sh, dst, dh, hdr,
                                                                       wt, win);
  return hipGetLastError();
}

hipError_t sift_smooth(const float* in, float* out, float* tmp, float* dog, int w, int h,
                       const SiftConsts& c, int tap_set, int W, hipStream_t st) {
  const float* taps = c.taps + tap_set * kSiftMaxTaps;
  const dim3 tiles(blocks_for(w, 64), blocks_for(h, 64));
  switch (W) {
#define SCM_SMOOTH_CASE(WW)                                                       \
  case WW:                                                                        \
    smooth_vh_kernel<WW><<<tiles, 256, 0, st>>>(in, out, dog, w, h, taps);        \
    return hipGetLastError();
    SCM_SMOOTH_CASE(5)
    SCM_SMOOTH_CASE(7)
    SCM_SMOOTH_CASE(8)
    SCM_SMOOTH_CASE(10)
    SCM_SMOOTH_CASE(13)
#undef SCM_SMOOTH_CASE
    default:
      break;
  }
  smooth_v_kernel<<<dim3(blocks_for(w, kVTile), blocks_for(h, kVTile)), 256, 0, st>>>(in, tmp, w, h,
                                                                                     taps, W);
  smooth_h_kernel<<<dim3(blocks_for(w, kHTile), h), 256, 0, st>>>(tmp, out, w, h, taps, W);
  if (dog) {
    const size_t n = (size_t)w * h;
    sub_kernel<<<min(4096, blocks_for(n, 256)), 256, 0, st>>>(out, in, dog, n);
  }
  return hipGetLastError();
}

hipError_t sift_downsample(const float* in, int w_in, float* out, int w, int h, hipStream_t st) {
  downsample_kernel<<<dim3(blocks_for(w, 256), h), 256, 0, st>>>(in, w_in, out, w, h);
  return hipGetLastError();
}

hipError_t sift_octave_detect(const SiftDev& d, const SiftConsts& c, int w, int h, int octave,
                              double tp, double te, hipStream_t st) {
  (void)c;  // the DoG levels come from sift_smooth
  detect_count_kernel<<<dim3(h, 3), 256, 0, st>>>(d.dog, w, h, tp, d.rowcnt);
  // rowoff[3h] = total (the candidate count), written by the scan's total
  scan_kernel<<<1, 1024, 0, st>>>(d.rowcnt, d.rowoff, nullptr, 3 * h, 3 * h, d.rowoff + 3 * h,
                                  nullptr);
  set_count_kernel<<<1, 1, 0, st>>>(d.cnt, d.rowoff + 3 * h, 0, d.cand_cap);
  detect_write_kernel<<<dim3(h, 3), 256, 0, st>>>(d.dog, w, h, tp, d.rowoff, d.cand, d.cand_cap);
  const double sigma0 = 1.6 * pow(2.0, 1.0 / kS);
  refine_kernel<<<kGrid, 64, 0, st>>>(d.dog, w, h, d.cand, d.cnt, d.ktmp, d.flag, tp, te, sigma0,
                                      octave);
  // positions in the frame's key list: after the earlier octaves' keypoints
  scan_kernel<<<1, 1024, 0, st>>>(d.flag, d.foff, &d.cnt->ncand, 0, d.cand_cap, d.rowcnt,
                                  &d.cnt->keys_run);
  set_count_kernel<<<1, 1, 0, st>>>(d.cnt, &d.cnt->keys_run, 1, d.key_cap);
  compact_keys_kernel<<<kGrid, 64, 0, st>>>(d.ktmp, d.flag, d.foff, d.cnt, d.keys, d.key_cap,
                                            octave);
  return hipGetLastError();
}

hipError_t sift_octave_gradient(const SiftDev& d, float2* grad, int w, int h, hipStream_t st) {
  gradient_kernel<<<dim3(blocks_for(w, 256), h, 3), 256, 0, st>>>(d.levels, grad, w, h);
  return hipGetLastError();
}

hipError_t sift_describe(const SiftDev& d, const SiftConsts& c, const SiftOctaves& oct,
                         hipStream_t st) {
  orient_kernel<<<4 * kGrid, 64, 0, st>>>(oct, d.keys, d.cnt, d.nori, d.ang, c.expn);
  scan_kernel<<<1, 1024, 0, st>>>(d.nori, d.koff, &d.cnt->nkey, 0, d.key_cap, nullptr,
                                  &d.cnt->nfeat);
  descriptor_kernel<<<4 * kGrid, 64, 0, st>>>(oct, d.keys, d.cnt, d.nori, d.ang, d.koff, d.feat,
                                              d.descf, d.desc, d.stale, c.expn, d.feat_cap);
  return hipGetLastError();
}

hipError_t sift_fixup(const SiftDev& d, hipStream_t st) {
  fixup_kernel<<<1, 64, 0, st>>>(d.cnt, d.stale, d.descf, d.desc, d.feat_cap);
  return hipGetLastError();
}

}  // namespace scm
