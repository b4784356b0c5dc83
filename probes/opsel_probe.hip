// Diagnostics (not product): packed-fp32 homography filter with constants
// broadcast by op_sel from their LDS float4 (no v_mov pairs) vs the splat
// form of verify_kernels.hip h_filter_pair: bitwise equality and timing.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
typedef __attribute__((ext_vector_type(2))) float f32x2;

// d = a[sel_a] * b + c[sel_c] per half, a/c broadcast from one dword of the pair
#define PKFMA_BB(d, a, b, c, sa, sc) \
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[" #sa ",0," #sc "] op_sel_hi:[" #sa ",1," #sc "]" \
               : "=v"(d) : "v"(a), "v"(b), "v"(c))
#define PKFMA_BV(d, a, b, c, sa) \
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[" #sa ",0,0] op_sel_hi:[" #sa ",1,1]" \
               : "=v"(d) : "v"(a), "v"(b), "v"(c))

struct HF { float h[9], a0, a2, mr; };

__device__ __forceinline__ void ref_pair(const HF& f, f32x2 s0, f32x2 s1, f32x2 d0, f32x2 d1, f32x2* diff, f32x2* mg) {
  const f32x2 q0 = __builtin_elementwise_fma(f32x2(f.h[0]), s0, __builtin_elementwise_fma(f32x2(f.h[1]), s1, f32x2(f.h[2])));
  const f32x2 q1 = __builtin_elementwise_fma(f32x2(f.h[3]), s0, __builtin_elementwise_fma(f32x2(f.h[4]), s1, f32x2(f.h[5])));
  const f32x2 q2 = __builtin_elementwise_fma(f32x2(f.h[6]), s0, __builtin_elementwise_fma(f32x2(f.h[7]), s1, f32x2(f.h[8])));
  const f32x2 w0 = __builtin_elementwise_fma(d0, q2, -q0);
  const f32x2 w1 = __builtin_elementwise_fma(d1, q2, -q1);
  const f32x2 lhs = __builtin_elementwise_fma(w0, w0, w1 * w1);
  const f32x2 rhs = f32x2(f.mr) * (q2 * q2);
  *mg = __builtin_elementwise_fma(f32x2(f.a2), rhs, f32x2(f.a0));
  *diff = lhs - rhs;
}

// P01 = (h0,h1), P23 = (h2,h3), P45 = (h4,h5), P67 = (h6,h7), P8a = (h8,a0), Pa2 = (a2, -)
__device__ __forceinline__ void opsel_pair(f32x2 P01, f32x2 P23, f32x2 P45, f32x2 P67, f32x2 P8a, f32x2 Pa2,
                                           f32x2 mr2, f32x2 s0, f32x2 s1, f32x2 d0, f32x2 d1, f32x2* diff, f32x2* mg) {
  f32x2 t0, t1, t2, q0, q1, q2;
  PKFMA_BB(t0, P01, s1, P23, 1, 0);   // h1 s1 + h2
  PKFMA_BB(t1, P45, s1, P45, 0, 1);   // h4 s1 + h5
  PKFMA_BB(t2, P67, s1, P8a, 1, 0);   // h7 s1 + h8
  PKFMA_BV(q0, P01, s0, t0, 0);       // h0 s0 + .
  PKFMA_BV(q1, P23, s0, t1, 1);       // h3 s0 + .
  PKFMA_BV(q2, P67, s0, t2, 0);       // h6 s0 + .
  const f32x2 w0 = __builtin_elementwise_fma(d0, q2, -q0);
  const f32x2 w1 = __builtin_elementwise_fma(d1, q2, -q1);
  const f32x2 lhs = __builtin_elementwise_fma(w0, w0, w1 * w1);
  const f32x2 rhs = mr2 * (q2 * q2);
  f32x2 m;
  PKFMA_BB(m, Pa2, rhs, P8a, 0, 1);   // a2 rhs + a0
  *mg = m;
  *diff = lhs - rhs;
}

template <int V>
__global__ __launch_bounds__(64) void kern(const float4* pts, const float* cons, int nmodels, int reps, uint32_t* out, float* dump) {
  __shared__ __attribute__((aligned(16))) float lc[64][12];
  const int lane = threadIdx.x;
  for (int i = lane; i < 64 * 12; i += 64) (&lc[0][0])[i] = cons[i];
  __syncthreads();
  f32x2 s0[4], s1[4], d0[4], d1[4];
  const float4* p = pts + blockIdx.x * 512;
  for (int q = 0; q < 4; ++q) {
    float4 a = p[128 * q + lane], b = p[128 * q + 64 + lane];
    s0[q] = f32x2{a.x, b.x}; s1[q] = f32x2{a.y, b.y}; d0[q] = f32x2{a.z, b.z}; d1[q] = f32x2{a.w, b.w};
  }
  const f32x2 mr2 = f32x2(16.0f);
  uint32_t acc = 0;
  for (int r = 0; r < reps; ++r) {
    for (int m = 0; m < nmodels; ++m) {
      const float4 c0 = reinterpret_cast<const float4*>(&lc[m][0])[0];
      const float4 c1 = reinterpret_cast<const float4*>(&lc[m][0])[1];
      const float4 c2 = reinterpret_cast<const float4*>(&lc[m][0])[2];
      int cnt = 0;
      uint64_t any = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x2 diff, mg;
        if (V == 0) {
          HF f;
          f.h[0] = c0.x; f.h[1] = c0.y; f.h[2] = c0.z; f.h[3] = c0.w;
          f.h[4] = c1.x; f.h[5] = c1.y; f.h[6] = c1.z; f.h[7] = c1.w;
          f.h[8] = c2.x; f.a0 = c2.y; f.a2 = c2.z; f.mr = 16.f;
          ref_pair(f, s0[q], s1[q], d0[q], d1[q], &diff, &mg);
        } else {
          opsel_pair(f32x2{c0.x, c0.y}, f32x2{c0.z, c0.w}, f32x2{c1.x, c1.y}, f32x2{c1.z, c1.w},
                     f32x2{c2.x, c2.y}, f32x2{c2.z, c2.w}, mr2, s0[q], s1[q], d0[q], d1[q], &diff, &mg);
        }
        if (dump && r == 0) {
          float* o = dump + ((((size_t)blockIdx.x * nmodels + m) * 4 + q) * 64 + lane) * 4;
          o[0] = diff.x; o[1] = diff.y; o[2] = mg.x; o[3] = mg.y;
        }
        const uint64_t i0 = __ballot(diff.x < -mg.x), i1 = __ballot(diff.y < -mg.y);
        any |= __ballot(fabsf(diff.x) <= mg.x) | __ballot(fabsf(diff.y) <= mg.y);
        cnt += __popcll(i0) + __popcll(i1);
      }
      acc += cnt + (any ? 1 : 0);
    }
  }
  if (lane == 0) out[blockIdx.x] = acc;
}

int main() {
  const int nblk = 4096, nm = 64, reps = 4;
  std::vector<float4> hp(nblk * 512);
  uint32_t st = 12345;
  auto rnd = [&]() { st = st * 1664525u + 1013904223u; return (st >> 8) * (1.0f / 16777216.0f); };
  for (auto& v : hp) v = make_float4(rnd() * 1000, rnd() * 800, rnd() * 1000, rnd() * 800);
  std::vector<float> hc(64 * 12);
  for (int m = 0; m < 64; ++m) {
    float* c = &hc[m * 12];
    c[0] = 1 + 0.01f * rnd(); c[1] = 0.01f * rnd(); c[2] = 10 * rnd();
    c[3] = 0.01f * rnd(); c[4] = 1 + 0.01f * rnd(); c[5] = 10 * rnd();
    c[6] = 1e-5f * rnd(); c[7] = 1e-5f * rnd(); c[8] = 1.0f;
    c[9] = 0.5f * rnd(); c[10] = 1e-4f; c[11] = 0;
  }
  float4* dp; float* dc; uint32_t* dout; float *dd0, *dd1;
  const size_t nd = (size_t)64 * nm * 4 * 64 * 4;  // dump only first 64 blocks
  hipMalloc(&dp, hp.size() * 16); hipMalloc(&dc, hc.size() * 4); hipMalloc(&dout, nblk * 4);
  hipMalloc(&dd0, nd * 4); hipMalloc(&dd1, nd * 4);
  hipMemcpy(dp, hp.data(), hp.size() * 16, hipMemcpyHostToDevice);
  hipMemcpy(dc, hc.data(), hc.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(kern<0>, dim3(64), dim3(64), 0, 0, dp, dc, nm, 1, dout, dd0);
  hipLaunchKernelGGL(kern<1>, dim3(64), dim3(64), 0, 0, dp, dc, nm, 1, dout, dd1);
  hipDeviceSynchronize();
  std::vector<uint32_t> a(nd), b(nd);
  hipMemcpy(a.data(), dd0, nd * 4, hipMemcpyDeviceToHost);
  hipMemcpy(b.data(), dd1, nd * 4, hipMemcpyDeviceToHost);
  size_t diffs = 0;
  for (size_t i = 0; i < nd; ++i) diffs += a[i] != b[i];
  printf("bitwise differences: %zu of %zu\n", diffs, nd);
  for (int v = 0; v < 2; ++v) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int w = 0; w < 2; ++w) {
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(kern<0>, dim3(nblk), dim3(64), 0, 0, dp, dc, nm, reps, dout, (float*)nullptr);
      else hipLaunchKernelGGL(kern<1>, dim3(nblk), dim3(64), 0, 0, dp, dc, nm, reps, dout, (float*)nullptr);
      hipEventRecord(e1); hipEventSynchronize(e1);
    }
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%s %.3f ms  %.1f ns per 512-point chunk-model (whole GPU)\n", v ? "opsel" : "splat", ms, ms * 1e6 / ((double)nblk * nm * reps));
  }
  return 0;
}
