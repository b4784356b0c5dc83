// Diagnostics (not product): the H split pass of rs_score_kernel (points not
// surely outside, per model) in three forms, on a realistic point / model
// mix, 512-point work items x 64 models:
//   VAR 0: the product's packed-fp32 loop (score_h_notout_n, 4 models per
//          iteration, 11 v_pk_fma per point pair and model, ballot counts);
//   VAR 1: the three affine forms q_k of 8 models x 32 points on one
//          v_mfma_f32_32x32x2_f32 (rows 8k + model, K = (s0, s1), the constant
//          terms as the C operand), w / lhs / diff on packed VALU, per-model
//          ballot counts (lane halves popcounted separately);
//   VAR 2: as 1, counts per lane (v_cmp + v_addc), reduced once per model tile.
// Prints time per (model, point) evaluation and checks that the three count
// the same points up to the filter's rounding band.
// Build: hipcc -O3 -ffp-contract=off --offload-arch=gfx950 probes/hsplit_bench.hip -o probes/build/hsplit_bench
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kPch = 8;             // points per lane (product kScorePch)
constexpr int kChunk = 64 * kPch;   // 512 points per work item
constexpr int kModels = 64;         // one round of hypotheses

#define PKFMA_BB(d, a, b, c, SA, SC)                                                     \
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[" #SA ",0," #SC "] op_sel_hi:[" #SA ",1," #SC "]" \
      : "=v"(d) : "v"(a), "v"(b), "v"(c))
#define PKFMA_BV(d, a, b, c, SA)                                                   \
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[" #SA ",0,0] op_sel_hi:[" #SA ",1,1]"  \
      : "=v"(d) : "v"(a), "v"(b), "v"(c))

struct HFilt {
  f32x2 p01, p23, p45, p67, p8m;
};

__device__ __forceinline__ f32x2 h_filter_pair(const HFilt& f, f32x2 s0, f32x2 s1, f32x2 d0, f32x2 d1) {
  f32x2 t0, t1, t2, q0, q1, q2;
  PKFMA_BB(t0, f.p01, s1, f.p23, 1, 0);
  PKFMA_BB(t1, f.p45, s1, f.p45, 0, 1);
  PKFMA_BB(t2, f.p67, s1, f.p8m, 1, 0);
  PKFMA_BV(q0, f.p01, s0, t0, 0);
  PKFMA_BV(q1, f.p23, s0, t1, 1);
  PKFMA_BV(q2, f.p67, s0, t2, 0);
  const f32x2 w0 = __builtin_elementwise_fma(d0, q2, -q0);
  const f32x2 w1 = __builtin_elementwise_fma(d1, q2, -q1);
  const f32x2 lhs = __builtin_elementwise_fma(w0, w0, w1 * w1);
  return __builtin_elementwise_fma(-q2, q2, lhs);
}

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

// w = e q2 + q (e = -d'): one packed FMA with e broadcast from dword SA of pair E.
#define PKFMA_EB(d, e, q2, q, SA)                                                  \
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[" #SA ",0,0] op_sel_hi:[" #SA ",1,1]"  \
      : "=v"(d) : "v"(e), "v"(q2), "v"(q))

template <int VAR>
__global__ __launch_bounds__(64) void kern(const float4* __restrict__ pts, const float* __restrict__ cons,
                                           int nitems, int reps, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float lc[kModels][12];
  const int lane = threadIdx.x;
  for (int i = lane; i < kModels * 12; i += 64) (&lc[0][0])[i] = cons[i];
  __syncthreads();
  for (int item = blockIdx.x; item < nitems; item += gridDim.x) {
    const float4* p = pts + (size_t)item * kChunk;
    uint32_t u0 = 0;  // lane t: count of model t
    if (VAR == 0) {
      f32x2 x0[kPch / 2], x1[kPch / 2], y0[kPch / 2], y1[kPch / 2];
#pragma unroll
      for (int qq = 0; qq < kPch / 2; ++qq) {
        const float4 v0 = p[(2 * qq) * 64 + lane], v1 = p[(2 * qq + 1) * 64 + lane];
        x0[qq] = f32x2{v0.x, v1.x};
        x1[qq] = f32x2{v0.y, v1.y};
        y0[qq] = f32x2{v0.z, v1.z};
        y1[qq] = f32x2{v0.w, v1.w};
      }
      for (int rep = 0; rep < reps; ++rep)
        for (int t = 0; t < kModels; t += 4) {
          HFilt f[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) f[k] = h_filter_load(&lc[t + k][0]);
          int c[4] = {0, 0, 0, 0};
#pragma unroll
          for (int q = 0; q < kPch / 2; ++q) {
            f32x2 d[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = h_filter_pair(f[k], x0[q], x1[q], y0[q], y1[q]);
#pragma unroll
            for (int k = 0; k < 4; ++k)
              c[k] += __popcll(__ballot(d[k].x <= f[k].p8m.y)) + __popcll(__ballot(d[k].y <= f[k].p8m.y));
          }
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (lane == t + k) u0 += (uint32_t)c[k];
        }
    } else {
      constexpr int NT = 8;  // point tiles of 32 per pass (two passes per 512-point item)
      const int r = lane & 31, h = lane >> 5;
      for (int half = 0; half < kChunk / (32 * NT); ++half) {
        float bv[NT];
        f32x2 E[NT];  // (-d0', -d1') of the lane's point
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const float4 v = p[32 * (NT * half + j) + r];
          bv[j] = h ? v.y : v.x;
          E[j] = f32x2{-v.z, -v.w};
        }
        for (int rep = 0; rep < reps; ++rep)
          for (int mt = 0; mt < kModels / 8; ++mt) {
            // A: row r = 8k + m holds coefficient h of form k of model m
            const int krow = r >> 3;
            const float a = krow < 3 ? lc[mt * 8 + (r & 7)][3 * krow + h] : 0.0f;
            f32x16 cm;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int k = i >> 2;
              cm[i] = k < 3 ? lc[mt * 8 + 4 * h + (i & 3)][3 * k + 2] : 0.0f;
            }
            const f32x2 M01 = f32x2{lc[mt * 8 + 4 * h][9], lc[mt * 8 + 4 * h + 1][9]};
            const f32x2 M23 = f32x2{lc[mt * 8 + 4 * h + 2][9], lc[mt * 8 + 4 * h + 3][9]};
            uint32_t clo[4] = {0, 0, 0, 0}, chi[4] = {0, 0, 0, 0};
            uint32_t vc[4] = {0, 0, 0, 0};
            f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv[0], cm, 0, 0, 0);
#pragma unroll
            for (int j = 0; j < NT; ++j) {
              const f32x16 cur = acc;
              if (j + 1 < NT) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv[j + 1], cm, 0, 0, 0);
#pragma unroll
              for (int cp = 0; cp < 2; ++cp) {
                const f32x2 q0 = f32x2{cur[2 * cp], cur[2 * cp + 1]};
                const f32x2 q1 = f32x2{cur[4 + 2 * cp], cur[5 + 2 * cp]};
                const f32x2 q2 = f32x2{cur[8 + 2 * cp], cur[9 + 2 * cp]};
                f32x2 w0, w1;
                PKFMA_EB(w0, E[j], q2, q0, 0);
                PKFMA_EB(w1, E[j], q2, q1, 1);
                const f32x2 lhs = __builtin_elementwise_fma(w0, w0, w1 * w1);
                const f32x2 nd = __builtin_elementwise_fma(q2, q2, -lhs);  // -diff
                const f32x2 M = cp ? M23 : M01;
                if (VAR == 1) {
                  const uint64_t bx = __ballot(nd.x >= -M.x), by = __ballot(nd.y >= -M.y);
                  clo[2 * cp] += __builtin_popcount((uint32_t)bx);
                  chi[2 * cp] += __builtin_popcount((uint32_t)(bx >> 32));
                  clo[2 * cp + 1] += __builtin_popcount((uint32_t)by);
                  chi[2 * cp + 1] += __builtin_popcount((uint32_t)(by >> 32));
                } else {
                  // sign(fl(nd + M)) = sign(nd + M) exactly: count the sign bits
                  // of the points outside (nd + M < 0), subtract at the end
                  const f32x2 sm = nd + M;
                  vc[2 * cp] += __float_as_uint(sm.x) >> 31;
                  vc[2 * cp + 1] += __float_as_uint(sm.y) >> 31;
                }
              }
            }
            if (VAR == 2) {
#pragma unroll
              for (int c = 0; c < 4; ++c) {
                uint32_t v = vc[c];
#pragma unroll
                for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
                clo[c] = 32 * NT - __builtin_amdgcn_readlane(v, 0);
                chi[c] = 32 * NT - __builtin_amdgcn_readlane(v, 32);
              }
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              if (lane == mt * 8 + c) u0 += clo[c];
              if (lane == mt * 8 + 4 + c) u0 += chi[c];
            }
          }
      }
    }
    out[(size_t)item * 64 + lane] = u0;
  }
}

int main() {
  const int nitems = 32768, reps = 4;
  const double S = 2000.0, maxr = 16.0;
  std::mt19937 g(7);
  std::uniform_real_distribution<double> U(0.0, S);
  std::normal_distribution<double> N(0.0, 1.0);
  const double H0[9] = {1.02, 0.01, 15.0, -0.01, 0.99, -8.0, 1e-5, 2e-6, 1.0};
  std::vector<float4> hp((size_t)nitems * kChunk);
  const double r = 1.0 / sqrt(maxr);
  const float rf = (float)r;
  for (auto& q : hp) {
    const double x = U(g), y = U(g);
    double dx, dy;
    if (g() % 100 < 15) {
      const double w = H0[6] * x + H0[7] * y + H0[8];
      dx = (H0[0] * x + H0[1] * y + H0[2]) / w + N(g) * 2.0;
      dy = (H0[3] * x + H0[4] * y + H0[5]) / w + N(g) * 2.0;
    } else {
      dx = U(g);
      dy = U(g);
    }
    q = make_float4((float)x, (float)y, (float)dx * rf, (float)dy * rf);
  }
  // models: H0 perturbed (counts from ~0 to ~15 %), filter constants as h_filter_consts
  std::vector<float> hc(kModels * 12);
  const double u = 0x1p-24;
  for (int m = 0; m < kModels; ++m) {
    double H[9];
    const double sc = pow(10.0, -4.0 + 3.0 * (m % 16) / 15.0);
    for (int j = 0; j < 9; ++j) H[j] = H0[j] * (1.0 + sc * N(g));
    double Hs[9];
    for (int j = 0; j < 6; ++j) Hs[j] = H[j] * r;
    for (int j = 6; j < 9; ++j) Hs[j] = H[j];
    const double A0 = (fabs(Hs[0]) + fabs(Hs[1])) * S + fabs(Hs[2]);
    const double A1 = (fabs(Hs[3]) + fabs(Hs[4])) * S + fabs(Hs[5]);
    const double A2 = (fabs(Hs[6]) + fabs(Hs[7])) * S + fabs(Hs[8]);
    const double al0 = 3.01 * u * A0, al1 = 3.01 * u * A1, al2 = 3.01 * u * A2;
    const double b = S * r * (1.0001 * al2 + 2.02 * u * A2) + fmax(al0, al1);
    const double E = (2.85 * b + 2.0 * al2) * A2 + 6.1 * b * b + al2 * al2 + 5.2 * u * A2 * A2;
    for (int j = 0; j < 9; ++j) hc[m * 12 + j] = (float)Hs[j];
    hc[m * 12 + 9] = (float)(1.5 * E + 1e-30);
  }
  float4* dp;
  float* dc;
  uint32_t* dout[3];
  hipMalloc(&dp, hp.size() * 16);
  hipMalloc(&dc, hc.size() * 4);
  for (int v = 0; v < 3; ++v) hipMalloc(&dout[v], (size_t)nitems * 64 * 4);
  hipMemcpy(dp, hp.data(), hp.size() * 16, hipMemcpyHostToDevice);
  hipMemcpy(dc, hc.data(), hc.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](auto kfn, const char* name, uint32_t* o) {
    hipLaunchKernelGGL(kfn, dim3(8192), dim3(64), 0, 0, dp, dc, nitems, reps, o);
    hipEventRecord(a);
    hipLaunchKernelGGL(kfn, dim3(8192), dim3(64), 0, 0, dp, dc, nitems, reps, o);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double ev = (double)nitems * kChunk * kModels * reps;
    printf("%-34s %8.3f ms  %.4f ns/1k-eval  %.3f cycles/eval/SIMD @2.4GHz\n", name, ms,
           ms * 1e9 / ev, ms * 1e-3 * 1024 * 2.4e9 / ev);
  };
  for (int rep = 0; rep < 2; ++rep) {
    run(kern<0>, "VALU split pass (product)", dout[0]);
    run(kern<1>, "MFMA q + ballot counts", dout[1]);
    run(kern<2>, "MFMA q + per-lane counts", dout[2]);
  }
  std::vector<uint32_t> h[3];
  for (int v = 0; v < 3; ++v) {
    h[v].resize((size_t)nitems * 64);
    hipMemcpy(h[v].data(), dout[v], h[v].size() * 4, hipMemcpyDeviceToHost);
  }
  for (int v = 1; v < 3; ++v) {
    long long tot0 = 0, totv = 0, maxd = 0, ndiff = 0;
    for (size_t i = 0; i < h[0].size(); ++i) {
      tot0 += h[0][i];
      totv += h[v][i];
      const long long d = llabs((long long)h[v][i] - (long long)h[0][i]);
      maxd = d > maxd ? d : maxd;
      ndiff += d != 0;
    }
    printf("VAR %d vs 0: total %lld vs %lld (%.3f %% inside-or-undecided), %lld counts differ, max |diff| %lld\n",
           v, totv, tot0, 100.0 * tot0 / ((double)nitems * kChunk * kModels * reps), ndiff, maxd);
  }
  return 0;
}
