// Probe: exactness of bf16 MFMA 32x32x16 for u8-valued operands with a 2^23
// accumulator offset, and IEEE-exactness of fp64 div/sqrt on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cmath>
#include <cstring>
typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__global__ void tile_kernel(const uint16_t* A, const uint16_t* B, uint32_t* out) {
  int l = threadIdx.x; int r = l & 31, h = l >> 5;
  f32x16 c; for (int i = 0; i < 16; ++i) c[i] = 8388608.0f;
  f32x16 acc;
  const bf16x8* a = (const bf16x8*)(A + r * 128 + h * 64);
  const bf16x8* b = (const bf16x8*)(B + r * 128 + h * 64);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], c, 0, 0, 0);
  for (int s = 1; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[s], b[s], acc, 0, 0, 0);
  for (int i = 0; i < 16; ++i) {
    int row = (i & 3) + 8 * (i >> 2) + 4 * h;
    out[row * 32 + r] = __float_as_uint(acc[i]);
  }
}
__global__ void f64_kernel(const double* x, const double* y, double* q, double* s, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { q[i] = x[i] / y[i]; s[i] = sqrt(fabs(x[i])); }
}
static uint16_t bf(uint8_t v) { float f = (float)v; uint32_t u; memcpy(&u, &f, 4); return (uint16_t)(u >> 16); }
int main() {
  int bad = 0;
  for (int trial = 0; trial < 4; ++trial) {
    uint8_t a8[32 * 128], b8[32 * 128];
    for (int i = 0; i < 32 * 128; ++i) {
      a8[i] = trial == 0 ? 255 : (trial == 1 ? (rand() & 255) : (trial == 2 ? (rand() % 40) : (uint8_t)(255 - (rand() & 1))));
      b8[i] = trial == 0 ? 255 : (trial == 1 ? (rand() & 255) : (trial == 2 ? (rand() % 40) : (uint8_t)(255 - (rand() & 3))));
    }
    uint16_t a[32 * 128], b[32 * 128];
    for (int i = 0; i < 32 * 128; ++i) { a[i] = bf(a8[i]); b[i] = bf(b8[i]); }
    uint16_t *dA, *dB; uint32_t* dO; uint32_t o[1024];
    hipMalloc(&dA, sizeof a); hipMalloc(&dB, sizeof b); hipMalloc(&dO, 4096);
    hipMemcpy(dA, a, sizeof a, hipMemcpyHostToDevice); hipMemcpy(dB, b, sizeof b, hipMemcpyHostToDevice);
    tile_kernel<<<1, 64>>>(dA, dB, dO);
    hipMemcpy(o, dO, 4096, hipMemcpyDeviceToHost);
    int nbad = 0;
    for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) {
      int64_t ref = 0; for (int k = 0; k < 128; ++k) ref += a8[i * 128 + k] * b8[j * 128 + k];
      uint32_t got = o[i * 32 + j] - 0x4B000000u;
      if (got != ref) { if (nbad < 4) printf("trial %d mismatch (%d,%d) got %u ref %ld bits %08x\n", trial, i, j, got, (long)ref, o[i*32+j]); nbad++; }
    }
    printf("mfma trial %d: %d mismatches (e.g. S[0][0]=%u)\n", trial, nbad, o[0] - 0x4B000000u);
    bad += nbad;
  }
  const int n = 1 << 20;
  double *x = (double*)malloc(n * 8), *y = (double*)malloc(n * 8), *q = (double*)malloc(n * 8), *s = (double*)malloc(n * 8);
  srand(7);
  for (int i = 0; i < n; ++i) {
    uint64_t u = ((uint64_t)rand() << 33) ^ ((uint64_t)rand() << 11) ^ rand(); 
    uint64_t v = ((uint64_t)rand() << 33) ^ ((uint64_t)rand() << 11) ^ rand();
    // random doubles in a broad exponent range
    u = (u & 0x800FFFFFFFFFFFFFull) | ((uint64_t)(1023 - 60 + (rand() % 120)) << 52);
    v = (v & 0x800FFFFFFFFFFFFFull) | ((uint64_t)(1023 - 60 + (rand() % 120)) << 52);
    memcpy(&x[i], &u, 8); memcpy(&y[i], &v, 8);
  }
  double *dx, *dy, *dq, *ds;
  hipMalloc(&dx, n * 8); hipMalloc(&dy, n * 8); hipMalloc(&dq, n * 8); hipMalloc(&ds, n * 8);
  hipMemcpy(dx, x, n * 8, hipMemcpyHostToDevice); hipMemcpy(dy, y, n * 8, hipMemcpyHostToDevice);
  f64_kernel<<<n / 256, 256>>>(dx, dy, dq, ds, n);
  hipMemcpy(q, dq, n * 8, hipMemcpyDeviceToHost); hipMemcpy(s, ds, n * 8, hipMemcpyDeviceToHost);
  int bq = 0, bs = 0;
  for (int i = 0; i < n; ++i) {
    volatile double rq = x[i] / y[i]; volatile double rs = std::sqrt(std::fabs(x[i]));
    if (memcmp((const void*)&rq, &q[i], 8)) bq++;
    if (memcmp((const void*)&rs, &s[i], 8)) bs++;
  }
  printf("f64 div mismatches %d / %d, sqrt mismatches %d / %d\n", bq, n, bs, n);
  printf("RESULT %s\n", (bad == 0 && bq == 0 && bs == 0) ? "PASS" : "FAIL");
  return 0;
}
