// Kernel 1 of the sequential-matching stage: brute-force SIFT descriptor
// similarity on bf16 MFMA with a fused, bit-exact two-way top-2 reduction,
// plus the finalize kernel (ratio / distance tests, cross-check, ordered
// compaction).
//
// Replaces colmap::MatchSiftFeaturesCPU as called from
// SequentialMatchingCPUKernel::execute (reference
// integration/op_cpp/sequential_matching.cc:154-155), i.e. the upstream
// ComputeSiftDistanceMatrix + FindBestMatchesOneWay x2 + FindBestMatches
// (SURVEY.md §8a a5-a7).  The int32 N1 x N2 matrix is never materialised.
//
// Exactness (SURVEY.md §8a "Exactness facts"):
//  * u8 descriptors are exact in bf16; each MFMA chain starts from an
//    accumulator tuple holding 2^23, so every partial sum is an integer in
//    [2^23, 2^24) — exact in f32 — and the f32 bit pattern of the result is
//    0x4B000000 | dot (dot <= 128*255^2 < 2^23).  Verified on gfx950
//    (probes/probe_mfma.hip, including all-255 operands).
//  * Ordering keys are 32-bit: key = (dot << 13) | 13 index bits, where the
//    index bits are [row code i (4 bits) | spare | tile index t (8 bits)].
//    Fast variant: the pivot's bf16 operand is pre-scaled by 16 (exact) and
//    the accumulator of register i starts at 2^23 + (15 - i), so the MFMA
//    result bits are 0x4B000000 | dot << 4 | (15 - i) and ONE v_lshl_or_b32
//    (acc << 9 | t-bits from an SGPR) forms the key.  This needs dot < 2^19
//    for every pair of rows, which the host guarantees from exact squared
//    norms (|a||b| < 2^19; RootSIFT u8 descriptors have |a|^2 ~ 2^18).
//  * Otherwise the CLAMP variant (unscaled operand, accumulator 2^23) uses
//    min(dot, 2^18), which changes no output: acosf(min(d * 2^-18, 1)) is 0
//    for every d >= 2^18, so any (best, second) >= 2^18 fails the ratio test
//    and a unique best above 2^18 keeps its index.
//  * max(key) = largest dot, lowest index among ties (FindBestMatchesOneWay
//    keeps the first maximum; equal values fall to "second"); the running
//    second is med3(key, best, second).  Both merges are associative, so the
//    tile-parallel reduction equals the sequential scan bit for bit.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "match_kernels.h"

namespace scm {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

__device__ __forceinline__ uint32_t merge_second(uint32_t b1a, uint32_t b2a,
                                                 uint32_t b1b, uint32_t b2b) {
  const uint32_t lo = min(b1a, b1b) & ~kIdxMask;
  return max(max(b2a, b2b), lo);
}

constexpr int kStages = 3;

__device__ __forceinline__ void load_bfrag(const uint8_t* bt, int r, int h, bf16x8 (&bfrag)[8]) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int ch = (h * 8 + q) ^ (r & 15);
    bfrag[q] = *reinterpret_cast<const bf16x8*>(bt + r * 256 + (ch << 4));
  }
}

// One 32 x 32 sub-tile over K = 128: an 8-MFMA accumulation chain.
__device__ __forceinline__ f32x16 chain(const bf16x8 (&a)[8], const bf16x8 (&b)[8],
                                        const f32x16& cinit) {
  f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], cinit, 0, 0, 0);
#pragma unroll
  for (int q = 1; q < 8; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[q], b[q], acc, 0, 0, 0);
  return acc;
}

// The same chain, refilling each B fragment with the next tile's as soon as
// its last MFMA has been issued: the next tile's LDS reads are in flight for
// the whole epilogue instead of stalling the next chain (no extra VGPRs).
__device__ __forceinline__ f32x16 chain_refill(const bf16x8 (&a)[8], bf16x8 (&b)[8],
                                               const f32x16& cinit, const uint8_t* bt_next,
                                               int r, int h) {
  f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], cinit, 0, 0, 0);
  b[0] = *reinterpret_cast<const bf16x8*>(bt_next + r * 256 + (((h * 8 + 0) ^ (r & 15)) << 4));
#pragma unroll
  for (int q = 1; q < 8; ++q) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[q], b[q], acc, 0, 0, 0);
    b[q] = *reinterpret_cast<const bf16x8*>(bt_next + r * 256 + (((h * 8 + q) ^ (r & 15)) << 4));
  }
  return acc;
}

// Keys of one finished sub-tile: row top-2 state update; returns the
// sub-tile's column partial (best two keys of the lane's column, re-keyed
// with the row inside the workgroup).
// Top-2 of three unique keys: (max, median).
__device__ __forceinline__ uint2 top2_of3(uint32_t a, uint32_t b, uint32_t c) {
  return make_uint2(max(max(a, b), c), med3_u32(a, b, c));
}

// Merge of three top-2 pairs: best = max of the bests; second = max(median
// of the bests, largest second) -- a second can only beat the median of the
// bests when it belongs to the overall best's pair.
__device__ __forceinline__ uint2 merge3(uint2 a, uint2 b, uint2 c) {
  return make_uint2(max(max(a.x, b.x), c.x), max(med3_u32(a.x, b.x, c.x), max(max(a.y, b.y), c.y)));
}

template <bool CLAMP>
__device__ __forceinline__ uint2 subtile_epilogue(const f32x16& acc, uint32_t tbits,
                                                  uint32_t (&b1r)[16], uint32_t (&b2r)[16],
                                                  uint32_t row_base) {
#ifdef SCM_DIAG_MATCH_SKELETON
  // diagnostics only: MFMA + LDS + staging skeleton, results discarded
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) x ^= __float_as_uint(acc[i]);
  b1r[0] ^= x;
  return make_uint2(x, x);
#endif
  uint32_t key[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t bits = __float_as_uint(acc[i]);
    if (CLAMP)
      key[i] = (min(bits, 0x4B040000u) << 13) | tbits | ((uint32_t)(15 - i) << 9);
    else
      key[i] = (bits << 9) | tbits;
    b2r[i] = med3_u32(key[i], b1r[i], b2r[i]);
    b1r[i] = max(b1r[i], key[i]);
  }
  // Column top-2 of the lane's 16 keys (unique: the row code differs) as a
  // 3-input tree: 21 ops instead of 32 for the streaming update.
  const uint2 p0 = top2_of3(key[0], key[1], key[2]);
  const uint2 p1 = top2_of3(key[3], key[4], key[5]);
  const uint2 p2 = top2_of3(key[6], key[7], key[8]);
  const uint2 p3 = top2_of3(key[9], key[10], key[11]);
  const uint2 p4 = top2_of3(key[12], key[13], key[14]);
  const uint2 l0 = merge3(p0, p1, p2);
  const uint2 l1 = make_uint2(max(max(p3.x, p4.x), key[15]),
                              max(med3_u32(p3.x, p4.x, key[15]), max(p3.y, p4.y)));
  const uint32_t b1c = max(l0.x, l1.x);
  const uint32_t b2c = max(max(min(l0.x, l1.x), l0.y), l1.y);
  const uint32_t ii = 15u - ((b1c >> 9) & 15u);
  const uint32_t row_in_blk = row_base + (ii & 3u) + 8u * (ii >> 2);
  return make_uint2((b1c & ~kIdxMask) | (kIdxMask - row_in_blk), b2c & ~kIdxMask);
}

// One workgroup = one MatchJob = 512 rows of the pivot image (8 waves x 64
// rows, two 32-row MFMA sub-tiles per wave, A fragments register-resident)
// swept against every column of every neighbour image of the job, 32 columns
// per LDS tile.  Per element (fast variant): 1 v_lshl_or (key) + 2 row-state
// ops + ~1.3 column-state ops (3-input tree).
//
// Software pipeline (per wave, sub-tile granularity): the MFMA chain of
// sub-tile (t, 1) runs while the epilogue of (t, 0) executes, and the chain of
// (t + 1, 0) while the epilogue of (t, 1) executes, so the matrix core and
// the vector ALU overlap inside every wave with only two accumulators.  B
// tiles rotate through three LDS buffers (tile t+2 is staged while t+1 is
// read); one barrier per tile.  The loop body is branch-free: past the last
// tile of a segment the chain runs on a clamped tile and is discarded.
template <bool CLAMP>
__global__ __launch_bounds__(kMatchThreads, 1) void match_tiles_kernel(
    const uint16_t* __restrict__ desc,        // bf16 table, [rows][128]
    const MatchJob* __restrict__ jobs,
    const PairDesc* __restrict__ pairs,
    uint2* __restrict__ rowres,               // per pair [nseg][n1]
    uint2* __restrict__ colpart) {            // per pair [nrb][n2pad]
  __shared__ __attribute__((aligned(16))) uint8_t lds[kStages * kTileBytes + 2 * kMatchWaves * 32 * 8];
  uint2* colscratch = reinterpret_cast<uint2*>(lds + kStages * kTileBytes);

  const MatchJob job = jobs[blockIdx.x];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r = lane & 31;
  const int h = lane >> 5;

  // ---- A fragments: rows rb*512 + wave*64 + 32*s + r, 16-B chunks h*8+q.
  bf16x8 afrag[2][8];
  {
    const int64_t a_base = job.a_row;  // first table row of the pivot image
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int row = job.rb * kRowsPerBlock + wave * 64 + 32 * s + r;
      const bool ok = row < job.n1;
      const uint4* src = reinterpret_cast<const uint4*>(desc + (a_base + (ok ? row : 0)) * 128) + h * 8;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        uint4 v = ok ? src[q] : make_uint4(0, 0, 0, 0);
        if (!CLAMP) {  // x16: +4 on the bf16 exponent of every non-zero element
          uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const uint32_t lo = w[e] & 0xFFFFu, hi = w[e] >> 16;
            w[e] = (lo ? lo + 0x200u : 0u) | ((hi ? hi + 0x200u : 0u) << 16);
          }
          v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        afrag[s][q] = *reinterpret_cast<bf16x8*>(&v);
      }
    }
  }
  f32x16 cinit;
#pragma unroll
  for (int i = 0; i < 16; ++i) cinit[i] = CLAMP ? 8388608.0f : 8388608.0f + (float)(15 - i);
  const uint32_t row_base0 = (uint32_t)wave * 64u + 4u * (uint32_t)h;

  // Staging role of this thread: one 16-B chunk of the 8 KiB B tile.
  const int st_col = tid >> 4;    // 0..31
  const int st_chunk = tid & 15;  // 0..15
  const int st_lds = st_col * 256 + ((st_chunk ^ (st_col & 15)) << 4);

  for (int p = 0; p < job.npairs; ++p) {
    const PairDesc pd = pairs[job.pair0 + p];
    const int ntiles_total = (pd.n2 + 31) >> 5;
    uint2* colp = colpart + pd.colpart_off + (int64_t)job.rb * pd.n2pad;
    const uint16_t* bdesc = desc + pd.b_row * 128;
    for (int seg = 0; seg < pd.nseg; ++seg) {
      const int t_begin = seg * kTilesPerSeg;
      const int t_end = min(ntiles_total, t_begin + kTilesPerSeg);
      const int tlast = t_end - 1;
      uint32_t b1r[2][16], b2r[2][16];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 16; ++i) { b1r[s][i] = 0u; b2r[s][i] = 0u; }

      const uint4* src0 = reinterpret_cast<const uint4*>(bdesc + (int64_t)st_col * 128) + st_chunk;
      // Prologue: stage tiles t_begin, t_begin + 1; chain of (t_begin, 0).
      *reinterpret_cast<uint4*>(lds + 0 * kTileBytes + st_lds) = src0[(int64_t)t_begin * 32 * 16];
      *reinterpret_cast<uint4*>(lds + 1 * kTileBytes + st_lds) =
          src0[(int64_t)min(t_begin + 1, tlast) * 32 * 16];
      __syncthreads();
      bf16x8 bfrag[8];
      load_bfrag(lds, r, h, bfrag);
      f32x16 acc0 = chain(afrag[0], bfrag, cinit);

      for (int k = 0; k < t_end - t_begin; ++k) {
        const int t = t_begin + k;
        const uint4 nxt = src0[(int64_t)min(t + 2, tlast) * 32 * 16];
        const uint32_t tbits = (uint32_t)(kTilesPerSeg - 1 - k);
#ifdef SCM_MATCH_BPREF
        // B fragments of tile t + 1 (staged since the last barrier) requested
        // a whole sub-tile ahead of their chain.
        bf16x8 bnext[8];
        load_bfrag(lds + ((k + 1) % kStages) * kTileBytes, r, h, bnext);
#endif
        // chain (t, 1) || epilogue (t, 0)
#ifdef SCM_MATCH_REFILL
        const f32x16 acc1 = chain_refill(afrag[1], bfrag, cinit,
                                         lds + ((k + 1) % kStages) * kTileBytes, r, h);
#else
        const f32x16 acc1 = chain(afrag[1], bfrag, cinit);
#endif
        const uint2 c0 = subtile_epilogue<CLAMP>(acc0, tbits, b1r[0], b2r[0], row_base0);
        // chain (t + 1, 0) || epilogue (t, 1).  The barrier keeps the next
        // B fragments from being loaded while the current ones are live.
        __builtin_amdgcn_sched_barrier(0);
#if defined(SCM_MATCH_BPREF)
#pragma unroll
        for (int q = 0; q < 8; ++q) bfrag[q] = bnext[q];
#elif !defined(SCM_MATCH_REFILL)
        load_bfrag(lds + ((k + 1) % kStages) * kTileBytes, r, h, bfrag);
#endif
        acc0 = chain(afrag[0], bfrag, cinit);
        const uint2 c1 = subtile_epilogue<CLAMP>(acc1, tbits, b1r[1], b2r[1], row_base0 + 32u);
        // Column partial of this wave: merge the two sub-tiles and the halves.
        uint32_t B1 = max(c0.x, c1.x), B2 = merge_second(c0.x, c0.y, c1.x, c1.y);
        const uint32_t o1 = __shfl_xor(B1, 32);
        const uint32_t o2 = __shfl_xor(B2, 32);
        B2 = merge_second(B1, B2, o1, o2);
        B1 = max(B1, o1);
        if (h == 0) colscratch[((k & 1) * kMatchWaves + wave) * 32 + r] = make_uint2(B1, B2);
        *reinterpret_cast<uint4*>(lds + ((k + 2) % kStages) * kTileBytes + st_lds) = nxt;
        __syncthreads();
        // One wave merges the 8 wave partials of this tile and stores them.
#ifdef SCM_DIAG_MATCH_NOCOLMERGE
        if (false) {  // diagnostics only: column results dropped
#else
        if (wave == (k & (kMatchWaves - 1)) && h == 0) {
#endif
          uint2 m = colscratch[((k & 1) * kMatchWaves + 0) * 32 + r];
#pragma unroll
          for (int w = 1; w < kMatchWaves; ++w) {
            const uint2 o = colscratch[((k & 1) * kMatchWaves + w) * 32 + r];
            m.y = merge_second(m.x, m.y, o.x, o.y);
            m.x = max(m.x, o.x);
          }
          colp[t * 32 + r] = m;
        }
      }
      __syncthreads();  // every wave done with the LDS tiles before the next segment

      // ---- Row flush for this segment: re-key with the column inside the
      // segment, reduce over the 32 lanes of each half, store.
      uint2* rr = rowres + pd.rowres_off + (int64_t)seg * pd.n1;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint32_t k1 = b1r[s][i];
          const uint32_t tl = (uint32_t)(kTilesPerSeg - 1) - (k1 & 255u);
          const uint32_t col = tl * 32u + (uint32_t)r;
          uint32_t B1 = (k1 & ~kIdxMask) | (kIdxMask - col);
          uint32_t B2 = b2r[s][i] & ~kIdxMask;
#pragma unroll
          for (int x = 1; x < 32; x <<= 1) {
            const uint32_t o1 = __shfl_xor(B1, x);
            const uint32_t o2 = __shfl_xor(B2, x);
            B2 = merge_second(B1, B2, o1, o2);
            B1 = max(B1, o1);
          }
          const int row = job.rb * kRowsPerBlock + wave * 64 + 32 * s + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (r == i + 16 * s && row < pd.n1) rr[row] = make_uint2(B1, B2);
        }
      }
    }
  }
}

// Upper bound, acosf LUT: lut[d] = acosf(min(d * 2^-18, 1.0f)), d in [0, 2^18],
// built on the host with the host libm (the reference's own acosf).
__device__ __forceinline__ float lut_at(const float* lut, uint32_t v) {
  return lut[v < kLutMax ? v : kLutMax];
}

// Ratio + distance test of FindBestMatchesOneWay on (best, second) values.
__device__ __forceinline__ bool passes(const float* lut, uint32_t best, uint32_t second,
                                       float max_ratio, float max_distance) {
  if (best == 0u) return false;  // best_i2 == -1
  const float bn = lut_at(lut, best);
  if (bn > max_distance) return false;
  const float sn = lut_at(lut, second);
  return !(bn >= max_ratio * sn);
}

// Finalize: one workgroup per pair.  Merges column partials over row blocks
// (ascending block order; strict '>' keeps the lowest row on ties), merges
// row results over column segments, applies the tests, the cross-check and an
// order-preserving compaction (matches sorted by idx1, as FindBestMatches).
__global__ __launch_bounds__(kFinThreads) void match_finalize_kernel(
    const PairDesc* __restrict__ pairs, const uint2* __restrict__ rowres,
    const uint2* __restrict__ colpart, int32_t* __restrict__ m21_scratch,
    const float* __restrict__ lut, float max_ratio, float max_distance,
    int cross_check, uint2* __restrict__ matches, int32_t* __restrict__ counts) {
  __shared__ int32_t wave_tot[kFinThreads / 64];
  __shared__ int32_t wave_off[kFinThreads / 64];
  const PairDesc pd = pairs[blockIdx.x];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  if (pd.n1 == 0 || pd.n2 == 0) {  // no descriptors on one side: no matches
    if (tid == 0) counts[blockIdx.x] = 0;
    return;
  }
  int32_t* m21 = m21_scratch + pd.m21_off;
  const uint2* cp = colpart + pd.colpart_off;
  const uint2* rr = rowres + pd.rowres_off;

  if (cross_check) {
    for (int j = tid; j < pd.n2; j += kFinThreads) {
      uint2 m = cp[j];
      int best_rb = 0;
      for (int b = 1; b < pd.nrb; ++b) {
        const uint2 o = cp[(int64_t)b * pd.n2pad + j];
        m.y = merge_second(m.x, m.y, o.x, o.y);
        if (o.x > m.x) { m.x = o.x; best_rb = b; }
      }
      const uint32_t best = m.x >> kIdxBits, second = m.y >> kIdxBits;
      const int32_t row = best_rb * kRowsPerBlock + (int32_t)(kIdxMask - (m.x & kIdxMask));
      m21[j] = passes(lut, best, second, max_ratio, max_distance) ? row : -1;
    }
    __syncthreads();
  }
  // Rows: contiguous chunk per thread for the ordered compaction.
  const int per = (pd.n1 + kFinThreads - 1) / kFinThreads;
  const int i0 = min(pd.n1, tid * per), i1 = min(pd.n1, i0 + per);
  int cnt = 0;
  for (int pass = 0; pass < 2; ++pass) {
    int out = 0;
    if (pass == 1) {
      // exclusive scan of cnt over the block
      int x = cnt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d);
        if (lane >= d) x += y;
      }
      if (lane == 63) wave_tot[wave] = x;
      __syncthreads();
      if (tid == 0) {
        int acc = 0;
        for (int w = 0; w < kFinThreads / 64; ++w) { wave_off[w] = acc; acc += wave_tot[w]; }
        counts[blockIdx.x] = acc;
      }
      __syncthreads();
      out = wave_off[wave] + x - cnt;
    }
    for (int i = i0; i < i1; ++i) {
      uint2 m = rr[i];
      int best_seg = 0;
      for (int sg = 1; sg < pd.nseg; ++sg) {
        const uint2 o = rr[(int64_t)sg * pd.n1 + i];
        m.y = merge_second(m.x, m.y, o.x, o.y);
        if (o.x > m.x) { m.x = o.x; best_seg = sg; }
      }
      const uint32_t best = m.x >> kIdxBits, second = m.y >> kIdxBits;
      const int32_t col = best_seg * (kTilesPerSeg * 32) + (int32_t)(kIdxMask - (m.x & kIdxMask));
      bool ok = passes(lut, best, second, max_ratio, max_distance);
      if (ok && cross_check) ok = (m21[col] == i);
      if (ok) {
        if (pass == 0) ++cnt;
        else matches[pd.match_off + out++] = make_uint2((uint32_t)i, (uint32_t)col);
      }
    }
  }
}

// u8 -> bf16 descriptor conversion at table load (exact: integers < 256).
__global__ void u8_to_bf16_kernel(const uint8_t* __restrict__ in,
                                  uint16_t* __restrict__ out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t base = i * 8;
  if (base >= n) return;
  if (base + 8 <= n) {
    const uint2 v = *reinterpret_cast<const uint2*>(in + base);
    uint32_t w[2] = {v.x, v.y};
    uint16_t o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float f = (float)((w[k >> 2] >> (8 * (k & 3))) & 255u);
      o[k] = (uint16_t)(__float_as_uint(f) >> 16);
    }
    *reinterpret_cast<uint4*>(out + base) = *reinterpret_cast<uint4*>(o);
  } else {
    for (int64_t k = base; k < n; ++k) out[k] = (uint16_t)(__float_as_uint((float)in[k]) >> 16);
  }
}

// ---------------------------------------------------------------------------
// Host launchers.
// ---------------------------------------------------------------------------
hipError_t launch_match_tiles(const uint16_t* desc, const MatchJob* jobs, int njobs,
                              const PairDesc* pairs, uint2* rowres, uint2* colpart,
                              bool clamp, hipStream_t stream) {
  if (njobs <= 0) return hipSuccess;
  if (clamp)
    hipLaunchKernelGGL(match_tiles_kernel<true>, dim3(njobs), dim3(kMatchThreads), 0, stream,
                       desc, jobs, pairs, rowres, colpart);
  else
    hipLaunchKernelGGL(match_tiles_kernel<false>, dim3(njobs), dim3(kMatchThreads), 0, stream,
                       desc, jobs, pairs, rowres, colpart);
  return hipGetLastError();
}

hipError_t launch_match_finalize(const PairDesc* pairs, int npairs, const uint2* rowres,
                                 const uint2* colpart, int32_t* m21, const float* lut,
                                 float max_ratio, float max_distance, int cross_check,
                                 uint2* matches, int32_t* counts, hipStream_t stream) {
  if (npairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(match_finalize_kernel, dim3(npairs), dim3(kFinThreads), 0, stream, pairs,
                     rowres, colpart, m21, lut, max_ratio, max_distance, cross_check, matches,
                     counts);
  return hipGetLastError();
}

hipError_t launch_u8_to_bf16(const uint8_t* in, uint16_t* out, int64_t n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const int64_t threads = (n + 7) / 8;
  hipLaunchKernelGGL(u8_to_bf16_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     stream, in, out, n);
  return hipGetLastError();
}

}  // namespace scm
