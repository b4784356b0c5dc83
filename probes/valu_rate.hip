// Diagnostics (not product): per-SIMD issue cost of the matcher epilogue's
// VALU instructions alone and beside bf16 MFMAs, 1 or 2 waves per SIMD.
// Cycles from s_memtime (shader clock) per wave; one workgroup per CU (LDS).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int kIter = 2048;

#define MED3(d, a, b) asm volatile("v_med3_u32 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b))
#define MAXU(d, a) asm volatile("v_max_u32 %0, %1, %0" : "+v"(d) : "v"(a))
#define LSHLOR(d, a, s) asm volatile("v_lshl_or_b32 %0, %1, 9, %2" : "=v"(d) : "v"(a), "s"(s))
#define ADDU(d, a) asm volatile("v_add_u32 %0, %1, %0" : "+v"(d) : "v"(a))
#define FMAF(d, a) asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(d) : "v"(a))
#define PKFMA(d, a) asm volatile("v_pk_fma_f32 %0, %1, %1, %0" : "+v"(d) : "v"(a))
#define FMA64(d, a) asm volatile("v_fma_f64 %0, %1, %1, %0" : "+v"(d) : "v"(a))
#define LSHLADD64(d, a, s) asm volatile("v_lshl_add_u64 %0, %1, 8, %2" : "=v"(d) : "v"(a), "v"(s))
#define LSHLADD32(d, a, s) asm volatile("v_lshl_add_u32 %0, %1, 8, %2" : "=v"(d) : "v"(a), "v"(s))
#define MAX3U(d, a, b) asm volatile("v_max3_u32 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b))
#define CMPF(a, b) asm volatile("v_cmp_le_f32 vcc, %0, %1" : : "v"(a), "v"(b) : "vcc")

// MODE: 0 max, 1 med3, 2 lshl_or, 3 add, 4 mfma only, 5 mfma + NV valu (epilogue mix) per mfma,
//       6 mfma + NV valu, two independent chains
template <int MODE, int NV>
__global__ __launch_bounds__(1024) void rate_kernel(uint32_t* out, long long* cyc, uint32_t seed) {
  extern __shared__ uint8_t lds[];
  uint32_t x[16];
  for (int i = 0; i < 16; ++i) x[i] = seed * (threadIdx.x + i);
  const uint32_t y = seed ^ threadIdx.x, z = seed + 7;
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (short)(threadIdx.x + i); b[i] = (short)(seed + i); }
  f32x16 acc0 = {}, acc1 = {};
  lds[threadIdx.x] = 0;
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIter; ++it) {
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) MAXU(x[i], y);
    } else if (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 16; ++i) MED3(x[i], y, z);
    } else if (MODE == 2) {
#pragma unroll
      for (int i = 0; i < 16; ++i) { uint32_t t; LSHLOR(t, x[i], z); x[i] = t; }
    } else if (MODE == 3) {
#pragma unroll
      for (int i = 0; i < 16; ++i) ADDU(x[i], y);
    } else if (MODE == 7) {
#pragma unroll
      for (int i = 0; i < 16; ++i) FMAF(x[i], y);
    } else if (MODE == 8) {
      typedef __attribute__((ext_vector_type(2))) float f2;
      f2* xp = reinterpret_cast<f2*>(x);
      f2 yy = {__uint_as_float(y), __uint_as_float(z)};
#pragma unroll
      for (int i = 0; i < 8; ++i) PKFMA(xp[i], yy);
    } else if (MODE == 9) {
      double* xd = reinterpret_cast<double*>(x);
      double yd = (double)y;
#pragma unroll
      for (int i = 0; i < 8; ++i) FMA64(xd[i], yd);
    } else if (MODE == 10) {
#pragma unroll
      for (int i = 0; i < 16; ++i) CMPF(x[i], y);
    } else if (MODE == 11) {
      uint64_t* xq = reinterpret_cast<uint64_t*>(x);
      const uint64_t kq = ((uint64_t)z << 32) | z;
#pragma unroll
      for (int i = 0; i < 8; ++i) { uint64_t t; LSHLADD64(t, xq[i], kq); xq[i] = t; }
    } else if (MODE == 12) {
#pragma unroll
      for (int i = 0; i < 16; ++i) { uint32_t t; LSHLADD32(t, x[i], z); x[i] = t; }
    } else if (MODE == 13) {
#pragma unroll
      for (int i = 0; i < 16; ++i) MAX3U(x[i], y, z);
    } else if (MODE == 4) {
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc0, 0, 0, 0);
    } else if (MODE == 5) {
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc0, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        if (i % 5 == 0) { uint32_t t; LSHLOR(t, x[i & 15], z); x[(i + 1) & 15] ^= 0; x[i & 15] = t; }
        else if (i % 5 == 1 || i % 5 == 3) MED3(x[i & 15], y, z);
        else MAXU(x[i & 15], y);
      }
    } else if (MODE == 6) {
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc0, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < NV / 2; ++i) MED3(x[i & 15], y, z);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, acc1, 0, 0, 0);
#pragma unroll
      for (int i = NV / 2; i < NV; ++i) MED3(x[i & 15], y, z);
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t s = 0;
  for (int i = 0; i < 16; ++i) s += x[i] + __float_as_uint(acc0[i]) + __float_as_uint(acc1[i]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s + lds[threadIdx.x ^ 1];
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int MODE, int NV>
void run(const char* name, int threads, double ops_per_iter) {
  const int blocks = 256;
  uint32_t* out;
  long long* cyc;
  hipMalloc(&out, blocks * threads * 4);
  hipMalloc(&cyc, blocks * (threads / 64) * 8);
  const size_t lds = 96 * 1024;  // one workgroup per CU
  hipFuncSetAttribute((const void*)rate_kernel<MODE, NV>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL((rate_kernel<MODE, NV>), dim3(blocks), dim3(threads), lds, 0, out, cyc, 3u);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL((rate_kernel<MODE, NV>), dim3(blocks), dim3(threads), lds, 0, out, cyc, 5u);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const int nw = blocks * threads / 64;
  long long* h = new long long[nw];
  hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < nw; ++i) avg += h[i];
  avg /= nw;
  const int wps = threads / 256;  // waves per SIMD (one workgroup per CU)
  printf("%-28s waves/SIMD %d  cycles/iter/wave %.1f  per-SIMD cycles per op %.2f  (%.3f ms)\n", name,
         wps, avg / kIter, avg / kIter / (ops_per_iter * wps), ms);
  delete[] h;
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int threads : {256, 512}) {
    run<11, 0>("v_lshl_add_u64 x8", threads, 8);
    run<12, 0>("v_lshl_add_u32 x16", threads, 16);
    run<13, 0>("v_max3_u32 x16", threads, 16);
  }
  for (int threads : {256, 512, 1024}) {
    run<7, 0>("v_fma_f32 x16", threads, 16);
    run<8, 0>("v_pk_fma_f32 x8", threads, 8);
    run<9, 0>("v_fma_f64 x8", threads, 8);
    run<10, 0>("v_cmp_le_f32 x16", threads, 16);
    run<0, 0>("v_max_u32 x16", threads, 16);
    run<1, 0>("v_med3_u32 x16", threads, 16);
    run<2, 0>("v_lshl_or_b32 x16", threads, 16);
    run<3, 0>("v_add_u32 x16", threads, 16);
    run<4, 0>("mfma 32x32x16 (dep chain)", threads, 1);
    run<5, 0>("mfma + 0 valu", threads, 1);
    run<5, 5>("mfma + 5 valu", threads, 1);
    run<5, 10>("mfma + 10 valu", threads, 1);
    run<5, 20>("mfma + 20 valu", threads, 1);
    run<6, 20>("2 chains, mfma + 10 valu", threads, 2);
  }
  return 0;
}
