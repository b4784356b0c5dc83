// Diagnostics (not product): does the matcher's tile run faster at four waves
// per SIMD?  Two models of match_g8_kernel's tile work on random operands
// (the clock depends on the data), B fragments read from LDS every tile as in
// the kernel (ring stages, the kernel's XOR swizzle), no DMA, no barriers:
//   W64: 512-thread workgroups, waves of 64 rows (two row sub-tiles), two waves
//        per SIMD (the shipped structure: 16 MFMAs and 8 fragment reads per
//        wave and tile);
//   W32: 1024-thread workgroups, waves of 32 rows (one row sub-tile), four
//        waves per SIMD within 128 VGPRs (8 MFMAs and 8 fragment reads per
//        wave and tile).
// Per element the same epilogue: rows one v_lshl_add_u64 per two elements and
// one v_max3 folding the tile's two column sub-tiles, columns a max3 tree and
// a permlane32 fold.  One workgroup per CU (LDS).  Prints TOP/s.
// Build: hipcc -O3 --offload-arch=gfx950 probes/mfma_model4.hip -o probes/build/mfma_model4
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef unsigned long long u64;

constexpr int kTiles = 2048;  // tiles per wave
constexpr int kStages = 16;
constexpr int kTileBytes = 8192;

__device__ __forceinline__ uint32_t max3u(uint32_t a, uint32_t b, uint32_t c) {
  return max(max(a, b), c);
}
__device__ __forceinline__ u64 add_pair_u64(u64 x, u64 k, uint32_t dep) {
  u64 d;
  asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(d) : "v"(x), "v"(k), "v"(dep));
  return d;
}
__device__ __forceinline__ int sw8(int col, int c) { return col * 128 + ((c ^ ((col >> 1) & 7)) << 4); }

// One sub-tile chain, its column max and its row values.
__device__ __forceinline__ void subtile(const i32x4 (&a)[4], const i32x4 (&b)[4], const i32x16& ra,
                                        u64 kq, uint32_t& cm, uint32_t (&kv)[16]) {
  i32x16 acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[0], b[0], ra, 0, 0, 0);
#pragma unroll
  for (int q = 1; q < 4; ++q) acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[q], b[q], acc, 0, 0, 0);
  uint32_t m = max3u((uint32_t)acc[0], (uint32_t)acc[1], (uint32_t)acc[2]);
#pragma unroll
  for (int i = 3; i < 15; i += 2) m = max3u(m, (uint32_t)acc[i], (uint32_t)acc[i + 1]);
  m = max(m, (uint32_t)acc[15]);
  cm = m;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const u64 k = add_pair_u64(((u64)(uint32_t)acc[2 * i + 1] << 32) | (uint32_t)acc[2 * i], kq, m);
    kv[2 * i] = (uint32_t)k;
    kv[2 * i + 1] = (uint32_t)(k >> 32);
  }
}

template <int ROWS>  // 64: two row sub-tiles per wave; 32: one
__global__ __launch_bounds__(ROWS == 64 ? 512 : 1024) void model_kernel(const i32x4* __restrict__ src,
                                                                      uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[160 * 1024 - 64];
  constexpr int S = ROWS / 32;
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  for (int i = threadIdx.x; i < kStages * kTileBytes / 16; i += blockDim.x)
    reinterpret_cast<i32x4*>(lds)[i] = src[(blockIdx.x * 4096 + i) & 0xFFFFF];
  __syncthreads();
  i32x4 a[S][4];
  i32x16 ra[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
#pragma unroll
    for (int q = 0; q < 4; ++q) a[s][q] = src[(tid * 8 + 4 * s + q) & 0xFFFFF];
#pragma unroll
    for (int i = 0; i < 16; ++i) ra[s][i] = src[(tid * 7 + 16 * s + i) & 0xFFFFF][0] & 0xFFFF;
  }
  uint32_t b1r[S][16] = {};
  uint32_t sink = 0;
  for (int t = 0; t < kTiles; ++t) {
    const uint8_t* tile = lds + (t % kStages) * kTileBytes;
    const u64 kq = ((u64)(uint32_t)t << 32) | (uint32_t)(t * 3);
    i32x4 b[2][4];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q) b[c][q] = *reinterpret_cast<const i32x4*>(tile + sw8(32 * c + r, 4 * h + q));
    uint32_t cm[2][S];
    uint32_t k0[S][16];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int s = 0; s < S; ++s) {
        uint32_t kv[16];
        subtile(a[s], b[c], ra[s], kq, cm[c][s], kv);
        if (c == 0) {
#pragma unroll
          for (int i = 0; i < 16; ++i) k0[s][i] = kv[i];
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i) b1r[s][i] = max3u(b1r[s][i], kv[i], k0[s][i]);
        }
      }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      uint32_t mm = cm[c][0];
#pragma unroll
      for (int s = 1; s < S; ++s) mm = max(mm, cm[c][s]);
      const auto sw = __builtin_amdgcn_permlane32_swap(mm, mm, false, false);
      sink += max((uint32_t)sw[0], (uint32_t)sw[1]);
    }
  }
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int i = 0; i < 16; ++i) sink ^= b1r[s][i];
  out[tid] = sink;
}

template <int ROWS>
static void run(const i32x4* src, uint32_t* out) {
  const int threads = ROWS == 64 ? 512 : 1024;
  const int blocks = 256 * 2;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  model_kernel<ROWS><<<blocks, threads>>>(src, out);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  model_kernel<ROWS><<<blocks, threads>>>(src, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  // ops: every workgroup covers 512 rows x 64 columns x 128 K x 2 per tile
  const double ops = (double)blocks * kTiles * 512.0 * 64.0 * 128.0 * 2.0;
  printf("model W%d (%d waves/SIMD): %.3f ms, %.1f TOP/s (%.3f of 5000)\n", ROWS, ROWS == 64 ? 2 : 4, ms,
         ops / (ms * 1e-3) / 1e12, ops / (ms * 1e-3) / 1e12 / 5000.0);
}

int main() {
  const size_t n = 1 << 20;
  i32x4* src;
  uint32_t* out;
  hipMalloc(&src, n * sizeof(i32x4));
  i32x4* h = (i32x4*)malloc(n * sizeof(i32x4));
  srand(1);
  for (size_t i = 0; i < n; ++i)
    for (int k = 0; k < 4; ++k) h[i][k] = (rand() << 16) ^ rand();
  hipMemcpy(src, h, n * sizeof(i32x4), hipMemcpyHostToDevice);
  hipMalloc(&out, (size_t)512 * 1024 * sizeof(uint32_t));
  for (int rep = 0; rep < 3; ++rep) {
    run<64>(src, out);
    run<32>(src, out);
  }
  return 0;
}
