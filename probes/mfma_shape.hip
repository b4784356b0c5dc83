// Diagnostics (not product): chip-wide i8 MFMA throughput of the two gfx950
// shapes the matcher could use, v_mfma_i32_32x32x32_i8 and
// v_mfma_i32_16x16x64_i8, on random operands (power, hence the clock, depends
// on the data), 8 waves per CU, every CU busy.  Prints TOP/s and the
// effective shader clock (s_memtime cycles per wave / wall time).
// Build: hipcc -O3 --offload-arch=gfx950 probes/mfma_shape.hip -o probes/build/mfma_shape
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr int kIter = 4096;

// MODE 0: 32x32x32, 4 accumulators (16 MFMAs per iteration: a 64-row x 64-col tile, K = 128)
// MODE 1: 16x16x64, 16 accumulators (32 MFMAs per iteration: the same tile and K)
template <int MODE>
__global__ __launch_bounds__(512) void shape_kernel(const i32x4* __restrict__ src, int* out,
                                                    long long* cyc) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  i32x4 a[4], b[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    a[q] = src[(tid * 8 + q) & 0xFFFFF];
    b[q] = src[(tid * 8 + 4 + q) & 0xFFFFF];
  }
  const long long t0 = __builtin_amdgcn_s_memtime();
  int sink = 0;
  if (MODE == 0) {
    i32x16 acc[4] = {};
    for (int it = 0; it < kIter; ++it) {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          acc[s] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[(q + s) & 3], b[q], acc[s], 0, 0, 0);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < 16; ++i) sink ^= acc[s][i];
  } else {
    i32x4 acc[16] = {};
    for (int it = 0; it < kIter; ++it) {
#pragma unroll
      for (int s = 0; s < 16; ++s)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          acc[s] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[(2 * q + s) & 3], b[(s + q) & 3],
                                                         acc[s], 0, 0, 0);
    }
#pragma unroll
    for (int s = 0; s < 16; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) sink ^= acc[s][i];
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[tid] = sink;
  if ((threadIdx.x & 63) == 0) cyc[tid >> 6] = t1 - t0;
}

typedef unsigned long long u64;
__device__ __forceinline__ u64 add_pair_u64(u64 x, u64 k, uint32_t dep) {
  u64 d;
  asm volatile("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(d) : "v"(x), "v"(k), "v"(dep));
  return d;
}
__device__ __forceinline__ uint32_t max3u(uint32_t a, uint32_t b, uint32_t c) { return max(max(a, b), c); }

// The matcher's tile with a representative epilogue, operands in registers:
// MODE 2: 32x32x32 (4 chains of 4 per 64x64 tile): per sub-tile the column
//   max tree, 8 v_lshl_add_u64 row values, row state max3, a permlane32 fold
//   of the column maxima per column sub-tile;
// MODE 3: 16x16x64 (16 chains of 2): per sub-tile 2 v_lshl_add_u64, row state
//   max3 per column pair, column maxima over the 4 row sub-tiles folded over
//   the four 16-lane groups (permlane16 + permlane32 swaps).
template <int MODE>
__global__ __launch_bounds__(512) void tile_kernel(const i32x4* __restrict__ src, uint32_t* out,
                                                   long long* cyc) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  i32x4 a[8], b[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    a[q] = src[(tid * 16 + q) & 0xFFFFF];
    b[q] = src[(tid * 16 + 8 + q) & 0xFFFFF];
  }
  const u64 kq = ((u64)(uint32_t)src[tid & 0xFFFF][0] << 32) | (uint32_t)src[tid & 0xFFFF][1];
  const long long t0 = __builtin_amdgcn_s_memtime();
  uint32_t sink = 0;
  if (MODE == 2) {
    uint32_t b1r[2][16] = {};
    i32x16 ra = {};
    for (int it = 0; it < kIter / 2; ++it) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        uint32_t cm[2];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          i32x16 acc = ra;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[4 * s2 + q], b[(4 * c + q + it) & 7], acc, 0, 0, 0);
          uint32_t m = 0;
#pragma unroll
          for (int i = 0; i < 16; i += 2) m = max3u(m, (uint32_t)acc[i], (uint32_t)acc[i + 1]);
          cm[s2] = m;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const u64 k = add_pair_u64(((u64)(uint32_t)acc[2 * i + 1] << 32) | (uint32_t)acc[2 * i], kq, m);
            b1r[s2][2 * i] = max(b1r[s2][2 * i], (uint32_t)k);
            b1r[s2][2 * i + 1] = max(b1r[s2][2 * i + 1], (uint32_t)(k >> 32));
          }
        }
        const uint32_t mm = max(cm[0], cm[1]);
        const auto sw = __builtin_amdgcn_permlane32_swap(mm, mm, false, false);
        sink += max((uint32_t)sw[0], (uint32_t)sw[1]);
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 16; ++i) sink ^= b1r[s2][i];
  } else {
    uint32_t b1r[4][4] = {};
    i32x4 ra = {};
    for (int it = 0; it < kIter / 2; ++it) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        uint32_t cm = 0;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          i32x4 acc = ra;
#pragma unroll
          for (int q = 0; q < 2; ++q)
            acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[2 * s4 + q], b[(2 * c + q + it) & 7], acc, 0, 0, 0);
          cm = max3u(cm, max3u((uint32_t)acc[0], (uint32_t)acc[1], (uint32_t)acc[2]), (uint32_t)acc[3]);
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const u64 k = add_pair_u64(((u64)(uint32_t)acc[2 * i + 1] << 32) | (uint32_t)acc[2 * i], kq, cm);
            b1r[s4][2 * i] = max(b1r[s4][2 * i], (uint32_t)k);
            b1r[s4][2 * i + 1] = max(b1r[s4][2 * i + 1], (uint32_t)(k >> 32));
          }
        }
        const auto s16 = __builtin_amdgcn_permlane16_swap(cm, cm, false, false);
        const uint32_t m1 = max((uint32_t)s16[0], (uint32_t)s16[1]);
        const auto s32 = __builtin_amdgcn_permlane32_swap(m1, m1, false, false);
        sink += max((uint32_t)s32[0], (uint32_t)s32[1]);
      }
    }
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int i = 0; i < 4; ++i) sink ^= b1r[s4][i];
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[tid] = sink;
  if ((threadIdx.x & 63) == 0) cyc[tid >> 6] = t1 - t0;
}

// The 32x32x32 tile as match_g8_kernel does it (rows: v_lshl_add_u64 values,
// one v_max3 per row folding the tile's two column sub-tiles; columns: max
// tree per sub-tile, permlane32 fold per column sub-tile), and (DIGIT) the
// digit-block form: a fifth MFMA per chain adds the column sum, so rows fold
// accumulators directly (no v_lshl_add_u64).  One workgroup per CU (a 160 KB
// LDS allocation): two waves per SIMD, as in the matcher.
template <bool DIGIT>
__global__ __launch_bounds__(512) void g8_model_kernel(const i32x4* __restrict__ src, uint32_t* out,
                                                       long long* cyc) {
  __shared__ uint8_t pad[160 * 1024 - 64];
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid == 1 << 30) pad[threadIdx.x] = 0;  // keeps the allocation
  i32x4 a[8], b[8], dg[2];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    a[q] = src[(tid * 16 + q) & 0xFFFFF];
    b[q] = src[(tid * 16 + 8 + q) & 0xFFFFF];
  }
  dg[0] = src[(tid * 3) & 0xFFFFF];
  dg[1] = src[(tid * 5) & 0xFFFFF];
  const i32x4 wneg = {(int)0x80808080u, (int)0x80808080u, (int)0x80808080u, (int)0x80808080u};
  const u64 kq = ((u64)(uint32_t)src[tid & 0xFFFF][0] << 32) | (uint32_t)src[tid & 0xFFFF][1];
  const long long t0 = __builtin_amdgcn_s_memtime();
  uint32_t sink = 0;
  uint32_t b1r[2][16] = {};
  i32x16 ra2[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int i = 0; i < 16; ++i) ra2[s2][i] = src[(tid * 7 + 16 * s2 + i) & 0xFFFFF][0] & 0xFFFF;
  for (int it = 0; it < kIter / 2; ++it) {
    uint32_t k0[2][16];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      uint32_t cm[2];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        i32x16 acc = ra2[s2];
        if (DIGIT) acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(wneg, dg[c], acc, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[4 * s2 + q], b[4 * c + q], acc, 0, 0, 0);
        uint32_t m = max3u((uint32_t)acc[0], (uint32_t)acc[1], (uint32_t)acc[2]);
#pragma unroll
        for (int i = 3; i < 15; i += 2) m = max3u(m, (uint32_t)acc[i], (uint32_t)acc[i + 1]);
        m = max(m, (uint32_t)acc[15]);
        cm[s2] = m;
        uint32_t kv[16];
        if (DIGIT) {
#pragma unroll
          for (int i = 0; i < 16; ++i) kv[i] = (uint32_t)acc[i];
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const u64 k = add_pair_u64(((u64)(uint32_t)acc[2 * i + 1] << 32) | (uint32_t)acc[2 * i], kq, m);
            kv[2 * i] = (uint32_t)k;
            kv[2 * i + 1] = (uint32_t)(k >> 32);
          }
        }
        if (c == 0) {
#pragma unroll
          for (int i = 0; i < 16; ++i) k0[s2][i] = kv[i];
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i) b1r[s2][i] = max3u(b1r[s2][i], kv[i], k0[s2][i]);
        }
      }
      const uint32_t mm = max(cm[0], cm[1]);
      const auto sw = __builtin_amdgcn_permlane32_swap(mm, mm, false, false);
      sink += max((uint32_t)sw[0], (uint32_t)sw[1]);
    }
    ra2[it & 1][0] += 1;  // loop-carried: the chains cannot be hoisted
  }
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int i = 0; i < 16; ++i) sink ^= b1r[s2][i];
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[tid] = sink;
  if ((threadIdx.x & 63) == 0) cyc[tid >> 6] = t1 - t0;
}

template <int MODE>
static void run(const i32x4* src, int* out, long long* cyc, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto launch = [&]() {
    if (MODE < 2) shape_kernel<MODE><<<blocks, 512>>>(src, out, cyc);
    else if (MODE < 4) tile_kernel<MODE><<<blocks, 512>>>(src, (uint32_t*)out, cyc);
    else g8_model_kernel<MODE == 5><<<blocks, 512>>>(src, (uint32_t*)out, cyc);
  };
  launch();  // warm
  hipDeviceSynchronize();
  hipEventRecord(e0);
  launch();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const int waves = blocks * 8;
  long long* h = (long long*)malloc(waves * sizeof(long long));
  hipMemcpy(h, cyc, waves * sizeof(long long), hipMemcpyDeviceToHost);
  double mean = 0;
  for (int i = 0; i < waves; ++i) mean += (double)h[i];
  mean /= waves;
  free(h);
  // ops per wave per iteration: 64 rows x 64 cols x 128 K x 2
  const double ops = (double)waves * (MODE < 2 ? kIter : kIter / 2) * 64.0 * 64.0 * 128.0 * 2.0;
  // s_memtime ticks at a fixed 100 MHz reference on gfx950? report cycles as counted
  const char* names[6] = {"32x32x32_i8", "16x16x64_i8", "32x32x32_i8 + epilogue", "16x16x64_i8 + epilogue",
                          "g8 model (2 waves/SIMD)", "g8 model + digit-block MFMA"};
  printf("%s: %.3f ms, %.1f TOP/s (%.3f of 5000), wave ticks %.0f, ticks/ms %.0f\n",
         names[MODE], ms, ops / (ms * 1e-3) / 1e12,
         ops / (ms * 1e-3) / 1e12 / 5000.0, mean, mean / ms);
}

int main() {
  const size_t n = 1 << 20;
  i32x4* src;
  int* out;
  long long* cyc;
  hipMalloc(&src, n * sizeof(i32x4));
  i32x4* h = (i32x4*)malloc(n * sizeof(i32x4));
  srand(1);
  for (size_t i = 0; i < n; ++i)
    for (int k = 0; k < 4; ++k) h[i][k] = (rand() << 16) ^ rand();
  hipMemcpy(src, h, n * sizeof(i32x4), hipMemcpyHostToDevice);
  const int blocks = 256 * 4;
  hipMalloc(&out, (size_t)blocks * 512 * sizeof(int));
  hipMalloc(&cyc, (size_t)blocks * 8 * sizeof(long long));
  for (int rep = 0; rep < 2; ++rep) {
    run<0>(src, out, cyc, blocks);
    run<1>(src, out, cyc, blocks);
    run<2>(src, out, cyc, blocks);
    run<3>(src, out, cyc, blocks);
    run<4>(src, out, cyc, blocks / 2);
    run<5>(src, out, cyc, blocks / 2);
  }
  return 0;
}
