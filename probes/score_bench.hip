// Diagnostics (not product): throughput of the packed-fp32 homography inlier
// filter loop of rs_score_kernel under variations of its structure.
// usage: ./score_bench   (prints ns per 512-point chunk-model per variant)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
typedef __attribute__((ext_vector_type(2))) float f32x2;
struct HF { float h[9], a0, a2, mr; };

__device__ __forceinline__ float uf(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }

template <int VAR>
__global__ __launch_bounds__(64) void kern(const float4* pts, const float* cons, int nmodels, int reps, uint32_t* out) {
  __shared__ float lc[64][12];
  const int lane = threadIdx.x;
  for (int i = lane; i < 64 * 12; i += 64) (&lc[0][0])[i] = cons[i];
  __syncthreads();
  f32x2 s0[4], s1[4], d0[4], d1[4];
  const float4* p = pts + blockIdx.x * 512;
  for (int q = 0; q < 4; ++q) {
    float4 a = p[128 * q + lane], b = p[128 * q + 64 + lane];
    s0[q] = f32x2{a.x, b.x}; s1[q] = f32x2{a.y, b.y}; d0[q] = f32x2{a.z, b.z}; d1[q] = f32x2{a.w, b.w};
  }
  uint32_t acc = 0, accv = 0;
  for (int r = 0; r < reps; ++r) {
    for (int m = 0; m < nmodels; ++m) {
      HF f;
      if (VAR == 2) {  // constants without LDS / readfirstlane
        for (int j = 0; j < 9; ++j) f.h[j] = 0.001f * (j + 1) + 1e-7f * m;
        f.a0 = 0.5f; f.a2 = 1e-4f; f.mr = 16.f;
      } else if (VAR == 4) {  // constants stay in VGPRs (no readfirstlane)
        const float4 c0 = reinterpret_cast<const float4*>(&lc[m][0])[0];
        const float4 c1 = reinterpret_cast<const float4*>(&lc[m][0])[1];
        const float4 c2 = reinterpret_cast<const float4*>(&lc[m][0])[2];
        f.h[0] = c0.x; f.h[1] = c0.y; f.h[2] = c0.z; f.h[3] = c0.w;
        f.h[4] = c1.x; f.h[5] = c1.y; f.h[6] = c1.z; f.h[7] = c1.w;
        f.h[8] = c2.x; f.a0 = c2.y; f.a2 = c2.z; f.mr = 16.f;
      } else {
        const float4 c0 = reinterpret_cast<const float4*>(&lc[m][0])[0];
        const float4 c1 = reinterpret_cast<const float4*>(&lc[m][0])[1];
        const float4 c2 = reinterpret_cast<const float4*>(&lc[m][0])[2];
        f.h[0] = uf(c0.x); f.h[1] = uf(c0.y); f.h[2] = uf(c0.z); f.h[3] = uf(c0.w);
        f.h[4] = uf(c1.x); f.h[5] = uf(c1.y); f.h[6] = uf(c1.z); f.h[7] = uf(c1.w);
        f.h[8] = uf(c2.x); f.a0 = uf(c2.y); f.a2 = uf(c2.z); f.mr = 16.f;
      }
      int cnt = 0;
      uint64_t any = 0;
      uint32_t vc = 0;
      if (VAR == 3) {  // scalar fp32 (no packed math)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const float S0 = hh ? s0[q].y : s0[q].x, S1 = hh ? s1[q].y : s1[q].x;
            const float D0 = hh ? d0[q].y : d0[q].x, D1 = hh ? d1[q].y : d1[q].x;
            const float Q0 = __builtin_fmaf(f.h[0], S0, __builtin_fmaf(f.h[1], S1, f.h[2]));
            const float Q1 = __builtin_fmaf(f.h[3], S0, __builtin_fmaf(f.h[4], S1, f.h[5]));
            const float Q2 = __builtin_fmaf(f.h[6], S0, __builtin_fmaf(f.h[7], S1, f.h[8]));
            const float W0 = __builtin_fmaf(D0, Q2, -Q0), W1 = __builtin_fmaf(D1, Q2, -Q1);
            const float L = __builtin_fmaf(W0, W0, W1 * W1);
            const float T = Q2 * Q2;
            const float lo = __builtin_fmaf(T, f.mr, -f.a0), hi = __builtin_fmaf(T, f.a2, f.a0);
            cnt += __popcll(__ballot(L <= lo));
            any |= ~(__ballot(L <= lo) | __ballot(L > hi));
          }
        }
      } else
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x2 q0 = __builtin_elementwise_fma(f32x2(f.h[0]), s0[q], __builtin_elementwise_fma(f32x2(f.h[1]), s1[q], f32x2(f.h[2])));
        const f32x2 q1 = __builtin_elementwise_fma(f32x2(f.h[3]), s0[q], __builtin_elementwise_fma(f32x2(f.h[4]), s1[q], f32x2(f.h[5])));
        const f32x2 q2 = __builtin_elementwise_fma(f32x2(f.h[6]), s0[q], __builtin_elementwise_fma(f32x2(f.h[7]), s1[q], f32x2(f.h[8])));
        const f32x2 w0 = __builtin_elementwise_fma(d0[q], q2, -q0);
        const f32x2 w1 = __builtin_elementwise_fma(d1[q], q2, -q1);
        const f32x2 lhs = __builtin_elementwise_fma(w0, w0, w1 * w1);
        const f32x2 rhs = f32x2(f.mr) * (q2 * q2);
        const f32x2 mg = __builtin_elementwise_fma(f32x2(f.a2), rhs, f32x2(f.a0));
        const f32x2 diff = lhs - rhs;
        if (VAR == 1) {  // per-lane VALU counting, no ballots
          vc += (diff.x <= -mg.x) + (diff.y <= -mg.y);
          vc += ((fabsf(diff.x) <= mg.x) | (fabsf(diff.y) <= mg.y)) << 16;
        } else {
          cnt += __popcll(__ballot(diff.x <= -mg.x)) + __popcll(__ballot(diff.y <= -mg.y));
          any |= __ballot(fabsf(diff.x) <= mg.x) | __ballot(fabsf(diff.y) <= mg.y);
        }
      }
      if (VAR == 1) accv += vc;
      else { acc += (lane == (m & 63)) ? cnt : 0; if (any) acc ^= 1; }
    }
  }
  out[blockIdx.x * 64 + lane] = acc + accv;
}

int main() {
  const int nblk = 8192 * 4, nmodels = 64, reps = 4;
  std::vector<float4> hp(nblk * 512);
  for (size_t i = 0; i < hp.size(); ++i) hp[i] = make_float4((i * 37) % 1920, (i * 91) % 1080, (i * 53) % 1920, (i * 17) % 1080);
  std::vector<float> hc(64 * 12);
  for (int m = 0; m < 64; ++m) for (int j = 0; j < 12; ++j) hc[m * 12 + j] = j < 9 ? 0.001f * (j + 1) + 1e-7f * m : (j == 9 ? 0.5f : 1e-4f);
  float4* dp; float* dc; uint32_t* dout;
  hipMalloc(&dp, hp.size() * 16); hipMalloc(&dc, hc.size() * 4); hipMalloc(&dout, nblk * 64 * 4);
  hipMemcpy(dp, hp.data(), hp.size() * 16, hipMemcpyHostToDevice);
  hipMemcpy(dc, hc.data(), hc.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  auto run = [&](auto kfn, const char* name) {
    hipLaunchKernelGGL(kfn, dim3(nblk), dim3(64), 0, 0, dp, dc, nmodels, reps, dout);
    hipEventRecord(a);
    hipLaunchKernelGGL(kfn, dim3(nblk), dim3(64), 0, 0, dp, dc, nmodels, reps, dout);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    double cm = (double)nblk * nmodels * reps;
    printf("%-28s %8.3f ms  %.3f ns/chunk-model  %.1f chunk-models/us/SIMD-equiv -> %.0f cycles/chunk-model/SIMD @2.4GHz\n", name, ms, ms * 1e6 / cm, cm / (ms * 1e3), ms * 1e-3 * 1024 * 2.4e9 / cm);
  };
  run(kern<0>, "ballot+LDS consts");
  run(kern<1>, "VALU count");
  run(kern<2>, "no LDS consts");
  run(kern<3>, "scalar fp32 lo/hi");
  run(kern<4>, "VGPR consts");
  return 0;
}
