// Kernel 1 of the sequential-matching stage: brute-force SIFT descriptor
// similarity on MFMA with a fused, bit-exact two-way top-2 reduction, plus
// the finalize kernel (ratio / distance tests, cross-check, ordered
// compaction).
//
// Replaces colmap::MatchSiftFeaturesCPU as called from
// SequentialMatchingCPUKernel::execute (reference
// integration/op_cpp/sequential_matching.cc:154-155), i.e. the upstream
// ComputeSiftDistanceMatrix + FindBestMatchesOneWay x2 + FindBestMatches
// (SURVEY.md §8a a5-a7).  The int32 N1 x N2 matrix is never materialised.
//
// Two matchers: match_g8_kernel (default: integer MFMA on offset operands,
// see the i8 sections) with match_finalize_g8_kernel and its exact rechecks,
// and match_tiles_kernel (bf16 MFMA, SCM_MATCH_BF16=1 or max_ratio > 1) with
// match_finalize_kernel.
//
// Exactness (SURVEY.md §8a "Exactness facts"):
//  * bf16: u8 descriptors are exact in bf16; each MFMA chain starts from an
//    accumulator tuple holding 2^23, so every partial sum is an integer in
//    [2^23, 2^24) — exact in f32 — and the f32 bit pattern of the result is
//    0x4B000000 | dot (dot <= 128*255^2 < 2^23).  Verified on gfx950
//    (probes/probe_mfma.hip, including all-255 operands).  i8: integer
//    accumulation, exact by construction (see the i8 section).
//  * Ordering keys are 32-bit: key = (dot << 13) | 13 index bits, where the
//    index bits are [row code i (4 bits) | spare | tile index t (8 bits, in
//    32-column units)].  Fast variant: the host guarantees dot < 2^19 for
//    every pair of rows from exact squared norms (|a||b| < 2^19; RootSIFT u8
//    descriptors have |a|^2 ~ 2^18) and the key is ONE v_lshl_or_b32.  (bf16:
//    the pivot's operand is pre-scaled by 16 (exact) and the accumulator of
//    register i starts at 2^23 + (15 - i), so the result bits are
//    0x4B000000 | dot << 4 | (15 - i) and the key is acc << 9 | t-bits.)
//  * Otherwise the CLAMP variant uses min(dot, 2^18), which changes no
//    output: acosf(min(d * 2^-18, 1)) is 0 for every d >= 2^18, so any (best,
//    second) >= 2^18 fails the ratio test and a unique best above 2^18 keeps
//    its index.
//  * max(key) = largest dot, lowest index among ties (FindBestMatchesOneWay
//    keeps the first maximum; equal values fall to "second"); the running
//    second is med3(key, best, second).  Both merges are associative, so the
//    tile-parallel reduction equals the sequential scan bit for bit.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <climits>

#include "match_kernels.h"

namespace scm {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(16))) int i32x16;

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

// Column top-2 of one lane's 16 keys of a sub-tile (unique: the row code
// differs) as a 3-input tree, 21 ops instead of 32 for the streaming update;
// the best is re-keyed with its row inside the workgroup's 512-row block.
__device__ __forceinline__ uint2 column_top2(const uint32_t (&key)[16], uint32_t row_base) {
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

// Column partial of one 32-column sub-tile of a wave: merge the two row
// sub-tiles and the two lane halves; lanes of half 0 store it for the
// workgroup merge.
__device__ __forceinline__ void wave_col_partial(uint2 c0, uint2 c1, uint2* dst, int h, int r) {
  uint32_t B1 = max(c0.x, c1.x), B2 = merge_second(c0.x, c0.y, c1.x, c1.y);
  const uint32_t o1 = __shfl_xor(B1, 32);
  const uint32_t o2 = __shfl_xor(B2, 32);
  B2 = merge_second(B1, B2, o1, o2);
  B1 = max(B1, o1);
  if (h == 0) dst[r] = make_uint2(B1, B2);
}

// Row flush at the end of a column segment: re-key each row's best with its
// column inside the segment, reduce over the 32 lanes of each half, store.
__device__ __forceinline__ void row_flush(const uint32_t (&b1r)[2][16], const uint32_t (&b2r)[2][16],
                                          uint2* rr, int row0, int n1, int r, int h) {
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
      const int row = row0 + 32 * s + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (r == i + 16 * s && row < n1) rr[row] = make_uint2(B1, B2);
    }
  }
}

// Row flush of match_g8_kernel: each lane holds, per row, the best VALUE
// (dot + 2^22) over ITS columns only (j = lane + 32 t); reduced over the 32
// lanes of a half this gives the row's exact best with the lane of the best
// (the column's residue mod 32; ties between lanes need no tie-break: the
// second then equals the best and the row fails the ratio test) and, as
// second, the best of the OTHER lanes: a lower bound of the row's second that
// misses only the second within the winning lane.  The best column itself and
// the exact second come from match_rowcheck_g8_kernel for the rows that can
// still pass.  Stored as (dot << 13) | (kIdxMask - lane), (second << 13);
// CLAMP: min(dot, 2^18) (acosf(min(d 2^-18, 1)) is 0 for every d >= 2^18).
template <bool CLAMP>
__device__ __forceinline__ void row_flush_values(const uint32_t (&b1r)[2][16], uint2* rr, int row0,
                                                 int n1, int r, int h) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t k1 = b1r[s][i];
      uint32_t v = k1 >= (1u << 22) ? k1 - (1u << 22) : 0u;
      if (CLAMP) v = min(v, kLutMax);
      uint32_t B1 = (v << kIdxBits) | (kIdxMask - (uint32_t)r);
      uint32_t B2 = 0u;
#pragma unroll
      for (int x = 1; x < 32; x <<= 1) {
        const uint32_t o1 = __shfl_xor(B1, x);
        const uint32_t o2 = __shfl_xor(B2, x);
        B2 = merge_second(B1, B2, o1, o2);
        B1 = max(B1, o1);
      }
      const int row = row0 + 32 * s + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (r == i + 16 * s && row < n1) rr[row] = make_uint2(B1, B2);
    }
  }
}

// ===========================================================================
// bf16 matcher (SCM_MATCH_BF16=1).
// ===========================================================================
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

// Keys of one finished sub-tile: row top-2 state update; returns the
// sub-tile's column partial.
template <bool CLAMP>
__device__ __forceinline__ uint2 subtile_epilogue(const f32x16& acc, uint32_t tbits,
                                                  uint32_t (&b1r)[16], uint32_t (&b2r)[16],
                                                  uint32_t row_base) {
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
  return column_top2(key, row_base);
}

// One workgroup = one MatchJob = 512 rows of the pivot image (8 waves x 64
// rows, two 32-row MFMA sub-tiles per wave, A fragments register-resident)
// swept against every column of every neighbour image of the job, 32 columns
// per LDS tile.  Per element (fast variant): 1 v_lshl_or (key) + 2 row-state
// ops + ~1.3 column-state ops (3-input tree).
//
// Software pipeline (per wave, sub-tile granularity): the MFMA chain of
// sub-tile (t, 1) runs while the epilogue of (t, 0) executes, and the chain of
// (t + 1, 0) while the epilogue of (t, 1) executes.  B tiles rotate through
// three LDS buffers (tile t+2 is staged while t+1 is read); one barrier per
// tile.  Past the last tile of a segment the chain runs on a clamped tile and
// is discarded.
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
        // chain (t, 1) || epilogue (t, 0)
        const f32x16 acc1 = chain(afrag[1], bfrag, cinit);
        const uint2 c0 = subtile_epilogue<CLAMP>(acc0, tbits, b1r[0], b2r[0], row_base0);
        // chain (t + 1, 0) || epilogue (t, 1).  The barrier keeps the next
        // B fragments from being loaded while the current ones are live.
        __builtin_amdgcn_sched_barrier(0);
        load_bfrag(lds + ((k + 1) % kStages) * kTileBytes, r, h, bfrag);
        acc0 = chain(afrag[0], bfrag, cinit);
        const uint2 c1 = subtile_epilogue<CLAMP>(acc1, tbits, b1r[1], b2r[1], row_base0 + 32u);
        wave_col_partial(c0, c1, colscratch + ((k & 1) * kMatchWaves + wave) * 32, h, r);
        *reinterpret_cast<uint4*>(lds + ((k + 2) % kStages) * kTileBytes + st_lds) = nxt;
        __syncthreads();
        // One wave merges the 8 wave partials of this tile and stores them.
        if (wave == (k & (kMatchWaves - 1)) && h == 0) {
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
      row_flush(b1r, b2r, rowres + pd.rowres_off + (int64_t)seg * pd.n1,
                job.rb * kRowsPerBlock + wave * 64, pd.n1, r, h);
    }
  }
}

// ===========================================================================
// i8 matcher (default).
//
// v_mfma_i32_32x32x32_i8 covers K = 32 in the cycles the bf16 form needs for
// K = 16 (MI355X_MICROARCH.md, matrix cores), so a 128-long dot is 4 MFMAs
// instead of 8, and a descriptor is 128 B in HBM, L2 and LDS instead of 256.
// u8 is not an i8 range, so the table holds a' = a - 128 (the byte a ^ 0x80)
// and, per descriptor, cs = 128 * sum_d a_d (u8_to_i8_kernel); then exactly
//   a.b = a'.b' + 128 (Sa + Sb) - 2^21,        |a'.b'| <= 2^21,
// so a chain that starts from the accumulator ra_i + cb_j, with
// ra_i = cs(a_i) - 2^21 (registers, per job) and cb_j = cs(b_j) (per tile),
// ends at the exact int32 dot.  A pivot row past the image's count is a zero
// descriptor (bytes 0x80, cs 0) and yields dots of 0, like the zero padding
// of the table.  An LDS tile holds 64 columns (two 32-column sub-tiles) and
// the tile bits of a key still count 32-column units.
//
// Column side by VALUE (no index bits).  The chain starts from the per-row
// registers ra_i = cs(a_i) + 2^21 as the MFMA's C operand (no VALU), so it
// ends at x = dot - cb_j + 2^22, which lies in (0, 2^24) because cb_j <=
// 128 * 128 * 255 < 2^22.  Within a column cb_j is a constant, so the top-2
// values of the column are the top-2 of x plus (cb_j - 2^22), added once when
// the workgroup's column partial is stored: the column tree runs on the raw
// accumulators.  The column's best ROW is not tracked: with max_ratio <= 1 a
// column whose best value is tied fails the ratio test (second == best), so
// a passing column has a unique best row, and the cross-check "column j's
// best row is i" reduces to "column j passes and its best value equals row
// i's best value" (match_finalize_kernel, value mode).  The runtime selects
// the bf16 kernel (column keys with the lowest-row tie rule) when max_ratio
// > 1.  Row keys: one v_lshl_add_u32 per element, (x << 13) + ((cb_j << 13) |
// t-bits), which is (dot << 13) | t-bits mod 2^32 (the 2^22 offset shifts out).
// Per element: 1 (key) + 2 (row state) + ~1.3 (column tree) VALU ops.
// ===========================================================================
static_assert((kTile8Cols << kSeg8Log2) == kColsPerSeg, "i8 row segments of the bf16 kernel's width");

// Byte offset of 16-B chunk c (of 8) of column col in an i8 LDS tile.  The
// XOR with (col >> 1) & 7 makes each 16-lane group of a ds_read_b128 (one
// chunk, the 32 columns of one lane half) cover all 64 banks once
// (MI355X_MICROARCH.md, LDS table).
__device__ __forceinline__ int sw8(int col, int c) {
  return col * 128 + ((c ^ ((col >> 1) & 7)) << 4);
}

// B fragments of column col: chunk 4h + q feeds MFMA q, as in the A fragment.
__device__ __forceinline__ void load_bfrag8(const uint8_t* bt, int col, int h, i32x4 (&b)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) b[q] = *reinterpret_cast<const i32x4*>(bt + sw8(col, 4 * h + q));
}

// One 32 x 32 sub-tile over K = 128: 4 MFMAs, the first reading the per-row
// offsets ra as its C operand.
__device__ __forceinline__ i32x16 chain8(const i32x4 (&a)[4], const i32x4 (&b)[4],
                                         const i32x16& ra) {
  i32x16 acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[0], b[0], ra, 0, 0, 0);
#pragma unroll
  for (int q = 1; q < 4; ++q) acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[q], b[q], acc, 0, 0, 0);
  return acc;
}

// Top-2 VALUES (multiset: a tie puts the value in both) of one lane's 16
// accumulators, as a 3-input tree (21 ops).
__device__ __forceinline__ uint2 column_top2_values(const i32x16& acc) {
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = (uint32_t)acc[i];
  const uint2 p0 = top2_of3(v[0], v[1], v[2]);
  const uint2 p1 = top2_of3(v[3], v[4], v[5]);
  const uint2 p2 = top2_of3(v[6], v[7], v[8]);
  const uint2 p3 = top2_of3(v[9], v[10], v[11]);
  const uint2 p4 = top2_of3(v[12], v[13], v[14]);
  const uint2 l0 = merge3(p0, p1, p2);
  const uint2 l1 = make_uint2(max(max(p3.x, p4.x), v[15]),
                              max(med3_u32(p3.x, p4.x, v[15]), max(p3.y, p4.y)));
  return make_uint2(max(l0.x, l1.x), max(max(min(l0.x, l1.x), l0.y), l1.y));
}

__device__ __forceinline__ uint32_t merge_second_values(uint32_t b1a, uint32_t b2a,
                                                        uint32_t b1b, uint32_t b2b) {
  return max(max(b2a, b2b), min(b1a, b1b));
}

// ===========================================================================
// match_g8_kernel (default i8 matcher): LDS-DMA staging, packed row keys,
// best-only columns.
//  * B tiles and their column sums reach LDS by global_load_lds_dwordx4
//    (LDS-DMA: no staging VGPRs, no ds_write, no wave waiting for a load in
//    the tile it is issued): each wave moves 1 KiB of the 8 KiB tile, the
//    XOR-swizzled LDS image is produced by permuting the per-lane SOURCE
//    addresses (the destination of one instruction is lane-linear), tiles are
//    issued three groups ahead into a 16-stage ring, and one raw s_barrier per
//    group of 4 tiles is preceded by a counted vmcnt that retires exactly the
//    next group.
//  * Rows by VALUE: the chain ends at x = dot - cb_j + 2^22 (< 2^24), and
//    x + cb_j = dot + 2^22 for two accumulators of the lane's column (two
//    adjacent rows) is ONE v_lshl_add_u64 on the register pair; the row state
//    takes the values of the tile's two column sub-tiles with one v_max3 per
//    row: 1 VALU op per element (a keyed row state with the column index in
//    the low bits costs 1.5: v_lshl_add_u32 per element + half a max3).  Each
//    lane keeps, per row, the best value over ITS columns (j = lane mod 32);
//    row_flush_values reduces them over the lanes with the lane of the best.
//    Which column of that lane's residue class holds the best, and the exact
//    second, come from match_rowcheck_g8_kernel (an exact MFMA pass over the
//    class) for the rows that can still pass.  CLAMP variant: the same values,
//    min(dot, 2^18) applied at the flush (max commutes with the clamp).
//  * Column side by BEST VALUE ONLY: per lane a max3 tree over its 16 raw
//    accumulators (x; cb_j is constant within a column), then the two row
//    sub-tiles and the two lane halves (best of the wave's 64 rows); the
//    workgroup merge keeps, per column, the best value B1, the largest best of
//    the OTHER waves B2', and the wave of B1.  The column's true second is
//    max(B2', second within that wave's 64 rows), recomputed exactly by
//    match_recheck_g8_kernel for the columns whose cross-check outcome depends
//    on it.  With max_ratio <= 1 a column whose best value is tied fails the
//    ratio test, so the column's best row need not be tracked (the runtime
//    selects the bf16 kernel, which keeps the lowest-row rule, otherwise).
// Per element: 1 (rows) + ~0.55 (columns) VALU ops.
// colpart entry (per row block, column): x = B1 (raw accumulator units), y =
// (B2' << 3) | wave of B1.
// ===========================================================================
constexpr int kG8T = 4;                                        // tiles per barrier group
// groups in the LDS ring (DMA kG8Q - 1 ahead; 3 measured equal, profiles/r03_q3_vbench.log)
constexpr int kG8Q = 4;
constexpr int kG8Stages = kG8T * kG8Q;                         // 16 x 8 KiB of B tiles
static_assert(kG8Q >= 3, "the ring holds the group in use, the next, and one in flight");
constexpr int kG8CscGroups = 3;                                // column partials of 3 groups
constexpr int kG8CbOff = kG8Stages * kTile8Bytes;              // column sums, 64 int32 per stage
constexpr int kG8MetaOff = kG8CbOff + kG8Stages * kTile8Cols * 4;  // colpart index per tile
constexpr int kG8CscOff = kG8MetaOff + kG8Stages * 8;
constexpr int kG8LdsBytes = kG8CscOff + kG8CscGroups * kG8T * kMatch8Waves * kTile8Cols * 4;
static_assert(kMatch8Waves * 1024 == kTile8Bytes, "one 1 KiB LDS-DMA per wave per tile");
static_assert(kG8LdsBytes <= 160 * 1024, "LDS");

typedef __attribute__((address_space(3))) void lds_void;

typedef __attribute__((address_space(3))) const i32x4 lds_i32x4;
// The first sub-tile's B fragments and the two column sums of tile g (ring
// stage g mod kG8Stages), read one step ahead of their use, from per-lane LDS
// byte addresses boff (the swizzled chunk 4h + q of column r, sw8, LDS base
// included): one add per fragment, where the address arithmetic of
// load_bfrag8 took three (-0.5 to -1 % matcher time, profiles/r06_d).  adr
// keeps the four addresses for the second sub-tile's fragments (column 32 + r:
// the same swizzle, 4 KiB further, in the ds_read offset field).
__device__ __forceinline__ void g8_next(const uint8_t* lds, int g, int r, const uint32_t (&boff)[4],
                                            uint32_t (&adr)[4], i32x4 (&bf)[4], uint32_t& cb0,
                                            uint32_t& cb1) {
  const int stage = g % kG8Stages;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    adr[q] = boff[q] + (uint32_t)(stage * kTile8Bytes);
    bf[q] = *reinterpret_cast<lds_i32x4*>((size_t)adr[q]);
  }
  const int32_t* cbs = reinterpret_cast<const int32_t*>(lds + kG8CbOff + stage * kTile8Cols * 4);
  cb0 = (uint32_t)cbs[r];
  cb1 = (uint32_t)cbs[32 + r];
}
__device__ __forceinline__ void g8_c1_adr(const uint32_t (&adr)[4], i32x4 (&bf)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) bf[q] = reinterpret_cast<lds_i32x4*>((size_t)adr[q])[32 * 128 / 16];
}
#define G8_NEXT(gg) g8_next(lds, gg, r, boff, nadr, bf0, cbn0, cbn1)
#define G8_C1() g8_c1_adr(nadr, bf1)

// Row values, two accumulators per VALU op: v_lshl_add_u64 (shift 0) on a
// register pair, x + (cb_j : cb_j) = (dot + 2^22) for two adjacent rows of
// the lane's column (x + cb_j < 2^24: no carry crosses into the high half).
// The compiler does not apply the MFMA-result read hazard (wait states) to
// inline asm, so every use takes `dep`, a value computed by ordinary VALU code
// from the same MFMA result (the column max): that code has waited for the
// result, and the asm cannot issue before it.
typedef unsigned long long u64;
__device__ __forceinline__ u64 add_pair_u64(u64 x, u64 k, uint32_t dep) {
  u64 d;
  asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(d) : "v"(x), "v"(k), "v"(dep));
  return d;
}

// Row values of one finished sub-tile (this lane's column, its 16 rows);
// `cm` = g8_colmax(acc) (the hazard dependency above).
__device__ __forceinline__ void g8_keys(const i32x16& acc, u64 kq, uint32_t cm, u64 (&k)[8]) {
#pragma unroll
  for (int m = 0; m < 8; ++m)
    k[m] = add_pair_u64(((u64)(uint32_t)acc[2 * m + 1] << 32) | (uint32_t)acc[2 * m], kq, cm);
}

// Row state update with the values of the tile's two column sub-tiles.
__device__ __forceinline__ void g8_rows(const u64 (&ka)[8], const u64 (&kb)[8], uint32_t (&b1r)[16]) {
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    b1r[2 * m] = max(max(b1r[2 * m], (uint32_t)ka[m]), (uint32_t)kb[m]);
    b1r[2 * m + 1] = max(max(b1r[2 * m + 1], (uint32_t)(ka[m] >> 32)), (uint32_t)(kb[m] >> 32));
  }
}

// Largest raw accumulator of the lane's 16 rows (column side).
__device__ __forceinline__ uint32_t g8_colmax(const i32x16& acc) {
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = (uint32_t)acc[i];
  const uint32_t m0 = max(max(v[0], v[1]), v[2]), m1 = max(max(v[3], v[4]), v[5]);
  const uint32_t m2 = max(max(v[6], v[7]), v[8]), m3 = max(max(v[9], v[10]), v[11]);
  const uint32_t m4 = max(max(v[12], v[13]), v[14]);
  return max(max(max(m0, m1), m2), max(max(m3, m4), v[15]));
}

// Best raw value of a column over the wave's 64 rows (both row sub-tiles,
// both lane halves); lanes of half 0 write it for the workgroup merge.
__device__ __forceinline__ void g8_col_partial(uint32_t e0, uint32_t e1, uint32_t* dst, int h,
                                               int r) {
  const uint32_t m = max(e0, e1);
  // v_permlane32_swap(m, m) gives each lane m and its partner (lane ^ 32) in
  // the two results: a VALU exchange instead of an LDS ds_bpermute round trip.
  const auto sw = __builtin_amdgcn_permlane32_swap(m, m, false, false);
  if (h == 0) dst[r] = max((uint32_t)sw[0], (uint32_t)sw[1]);
}

// Workgroup merge of one column of a tile (lane = column): the best of the 8
// wave bests B1, the largest of the other seven B2' (a tie puts B1 there), the
// lowest wave holding B1.  Raw accumulator units (dot - cb + 2^22; the
// finalize kernel converts with the column's sum).
__device__ __forceinline__ void g8_merge(const uint32_t* src, uint2* dst) {
  uint32_t v[kMatch8Waves];
#pragma unroll
  for (int w = 0; w < kMatch8Waves; ++w) v[w] = src[w * kTile8Cols];
  uint32_t b1 = v[0], b2 = 0u, gw = 0u;
#pragma unroll
  for (int w = 1; w < kMatch8Waves; ++w) {
    b2 = max(b2, min(b1, v[w]));
    gw = v[w] > b1 ? (uint32_t)w : gw;
    b1 = max(b1, v[w]);
  }
  *dst = make_uint2(b1, (b2 << 3) | gw);
}

// One workgroup = one MatchJob (512 pivot rows, 8 waves x 64) swept against
// every column of its neighbour images, or one column part of one (the
// small-batch column split: tiles [t0, t1), row segments of 2^seg8_log2
// tiles).  The tiles of the job's pairs form one stream (tile g -> pair p,
// tile t of p).  Groups of kG8T = 4 tiles share one
// barrier: at the barrier ending group m every wave has (a) waited for its
// LDS-DMA of group m + 1, (b) finished reading group m - 1's stages, which
// then receive group m + 3, and (c) written its column partials of group
// m - 1 (the last tile's second half is written just after barrier m - 1), so
// four waves merge group m - 1's tiles.  Waves 0-3 meet barrier m after
// section 3 of tile 4m + 3, waves 4-7 after its section 1 (half a tile
// apart; every condition above holds at either point).  Between barriers
// waves drift freely, so the two waves of a SIMD overlap one's MFMA chains
// with the other's epilogue.  Per wave and tile four 4-MFMA chains in four
// sections, software pipelined (each chain under the previous epilogue), the
// chain of the next tile's first sub-tile issued before the current tile's
// last epilogue.
template <bool CLAMP>
__global__ __launch_bounds__(kMatch8Threads, 512 / kMatch8Threads) void match_g8_kernel(
    const uint8_t* __restrict__ desc8,  // a ^ 0x80, [rows][128]
    const int32_t* __restrict__ csum,   // 128 * sum_d a_d per row
    const MatchJob* __restrict__ jobs, const PairDesc* __restrict__ pairs,
    uint2* __restrict__ rowres,         // per pair [nseg][n1]
    uint2* __restrict__ colpart) {      // per pair [nrb][n2pad]
  // One array for every LDS use (a second __shared__ object can make the
  // compiler drain the LDS-DMA queue before each ds_read).
  __shared__ __attribute__((aligned(16))) uint8_t lds[kG8LdsBytes];
  uint32_t* csc = reinterpret_cast<uint32_t*>(lds + kG8CscOff);
  int64_t* meta = reinterpret_cast<int64_t*>(lds + kG8MetaOff);

  const MatchJob job = jobs[blockIdx.x];
  if (job.npairs == 0 || job.n1 <= 0) return;  // padding job of the XCD order (whole block)
  const PairDesc* __restrict__ P = pairs + job.pair0;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar
  const int r = lane & 31;
  const int h = lane >> 5;
  const int row0 = job.rb * kRowsPerBlock8 + wave * 64;

  i32x4 afrag[2][4];
  i32x16 ra[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int row = row0 + 32 * s + r;
    const bool ok = row < job.n1;
    const i32x4* src =
        reinterpret_cast<const i32x4*>(desc8 + (job.a_row + (ok ? row : 0)) * 128) + h * 4;
    const int z = (int)0x80808080u;  // a = 0
#pragma unroll
    for (int q = 0; q < 4; ++q) afrag[s][q] = ok ? src[q] : i32x4{z, z, z, z};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int rw = row0 + 32 * s + 4 * h + (i & 3) + 8 * (i >> 2);
      // unconditional load (clamped row), then select: no branch / wait per element
      const uint32_t cs = (uint32_t)csum[job.a_row + min(rw, job.n1 - 1)];
      ra[s][i] = (int)((rw < job.n1 ? cs : 0u) + (1u << 21));
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // operands in registers before any LDS-DMA

  // Tiles of pair p in this job: [p == 0 ? t0 : 0, tile_end(p)) (a column
  // part of a split pair: its first and last pair are the same).
  auto tile_end = [&](int pp) {
    const int ntp = (P[pp].n2 + kTile8Cols - 1) / kTile8Cols;
    return pp == job.npairs - 1 && job.t1 > 0 ? min(job.t1, ntp) : ntp;
  };
  int G = -job.t0;
  for (int p = 0; p < job.npairs; ++p) G += tile_end(p);
  // LDS-DMA cursor (groups ahead of the compute cursor; past the last tile it
  // re-stages the last one, so every wave issues the same number of
  // operations per group and the vmcnt counts stay fixed).
  int fp = 0, ft = job.t0;
  int64_t fb = P[0].b_row + (int64_t)job.t0 * kTile8Cols;
  int fn = tile_end(0);
  const int gpt = wave == kMatch8Waves - 1 ? 2 : 1;  // LDS-DMA operations per tile
  // LDS-DMA of a tile into ring stage `stage`: wave w moves columns 8w ..
  // 8w + 7; lane L writes LDS byte 16 L of the wave's block, i.e. (column 8w +
  // L / 8, position L % 8), which holds logical chunk (L % 8) ^ ((column >> 1)
  // & 7) (sw8); the last wave also moves the tile's 64 column sums (4 B per
  // lane).  The tile's address is a scalar cursor (fptr, fsum) advanced per
  // tile, the lane's byte offset loff a constant: a few scalar ops per tile,
  // where a 64-bit vector address and a stage modulo per tile cost 4.3 % of
  // the matcher's time (profiles/r06_a).
  const int dcol = wave * 8 + (lane >> 3);
  const uint32_t loff = (uint32_t)(dcol * 128 + (((lane & 7) ^ ((dcol >> 1) & 7)) * 16));
  const uint8_t* fptr = desc8 + fb * 128;  // tile ft of pair fp
  const int32_t* fsum = csum + fb;
  auto dma_group = [&](int grp) {
#pragma unroll
    for (int i = 0; i < kG8T; ++i) {
      const int stage = (grp * kG8T + i) & (kG8Stages - 1);
      __builtin_amdgcn_global_load_lds(fptr + loff, (lds_void*)(lds + stage * kTile8Bytes + wave * 1024),
                                       16, 0, 0);
      if (wave == kMatch8Waves - 1)
        __builtin_amdgcn_global_load_lds(fsum + lane, (lds_void*)(lds + kG8CbOff + stage * kTile8Cols * 4),
                                         4, 0, 0);
      if (++ft == fn) {
        if (fp + 1 < job.npairs) {
          ++fp;
          ft = 0;
          fb = P[fp].b_row;
          fn = tile_end(fp);
          fptr = desc8 + fb * 128;
          fsum = csum + fb;
        } else {
          ft = fn - 1;  // past the last tile: re-stage it
        }
      } else {
        fptr += kTile8Bytes;
        fsum += kTile8Cols;
      }
    }
  };
#pragma unroll
  for (int j = 0; j < kG8Q - 1; ++j) dma_group(j);
  // group 0 landed (groups 1 and 2 may be in flight)
  if (gpt == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  static_assert(kG8Q == 4 && kG8T == 4, "vmcnt constants");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  // Compute cursor.
  int p = 0, t = job.t0;
  PairDesc pd = P[0];
  int nt = tile_end(0);
  int segm = (1 << pd.seg8_log2) - 1;  // a row segment ends at tile t with (t & segm) == segm
  int64_t cpi = pd.colpart_off + (int64_t)job.rb * pd.n2pad;  // colpart index of tile 0 of pair p
  int flushed = -8;  // iteration of the last row flush (its stores)
  // Waves 4-7 (the second wave of each SIMD) meet group barrier m half a tile
  // earlier in their own stream (after section 1 of tile 4m + 3 instead of
  // section 3): they run two sections behind their SIMD partners, so one
  // wave's row-heavy half tile (sections 3-4) runs beside the other's
  // MFMA-dense half (sections 1-2): -1 % matcher time (profiles/r06_d).  A
  // stagger of two whole tiles (the same phase within a tile) measured +2.5 %,
  // static priority for waves 4-7 no change (profiles/r06_a); with the half-tile
  // stagger, priority for either half +1 to +2 %, and the loop unrolled by a
  // group (4 tiles, compile-time barrier position: 32 B of spills) +7 %
  // (profiles/r06_g).
  const bool late = wave >= kMatch8Waves / 2;
  const int nbar_loop = G / kG8T;  // barriers in the loop (full groups)

  uint32_t b1r[2][16];  // per lane and row: best key over this lane's columns
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < 16; ++i) b1r[s][i] = 0u;

  i32x4 bf0[4], bf1[4];
  uint32_t cbn0, cbn1;
  uint32_t boff[4], nadr[4];
  {
    const uint32_t lb = (uint32_t)(size_t)(lds_void*)lds;
#pragma unroll
    for (int q = 0; q < 4; ++q) boff[q] = lb + (uint32_t)sw8(r, 4 * h + q);
  }
  G8_NEXT(0);
  i32x16 acc = chain8(afrag[0], bf0, ra[0]);

  for (int g = 0; g < G; ++g) {
    const int stage = g % kG8Stages;
    const uint32_t cb0 = cbn0, cb1 = cbn1;  // read with the tile's c0 fragments
    if (tid == 0) meta[stage] = cpi + (int64_t)t * kTile8Cols;
    const u64 kq0 = ((u64)cb0 << 32) | cb0, kq1 = ((u64)cb1 << 32) | cb1;  // row value addends
    u64 k00[8], k10[8], k01[8], k11[8];
    const int m = g / kG8T;
    uint32_t* cscw =
        csc + (((m % kG8CscGroups) * kG8T + (g & (kG8T - 1))) * kMatch8Waves + wave) * kTile8Cols;
    const bool group_end = (g & (kG8T - 1)) == kG8T - 1 && g / kG8T < nbar_loop;
    // Barrier m.  This wave's DMA of group m + 1 (issued at barrier m - 2)
    // must be done: younger are group m + 2's DMA (kG8T * gpt operations) and
    // the merge stores of barriers m - 2 and m - 1 (wave w merges at barrier j
    // when ((j - 1) & 1) == w / 4).  vmcnt(kG8T * gpt) may also wait for the
    // oldest DMA of group m + 2 (issued a whole group earlier): a superset
    // wait with an immediate count, where the exact count's switch cost ~40
    // scalar ops per group (-1 %, profiles/r06_b).  After a row flush (many
    // stores) drain.
    auto barrier_block = [&](bool next) {
      if (g - flushed <= 2 * kG8T) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (gpt == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      dma_group(m + kG8Q - 1);
      if (m >= 1 && (((m - 1) & 1) == (wave >> 2))) {  // merge tile (wave & 3) of group m - 1
        const int tg = (m - 1) * kG8T + (wave & (kG8T - 1));
        const uint32_t* src =
            csc + (((m - 1) % kG8CscGroups) * kG8T + (wave & (kG8T - 1))) * kMatch8Waves * kTile8Cols;
        g8_merge(src + lane, colpart + meta[tg % kG8Stages] + lane);
      }
      if (next) G8_NEXT(g + 1);
    };
    // (s1, c0) || epilogue (s0, c0); the c1 fragments load under the epilogue
    i32x16 acc2 = chain8(afrag[1], bf0, ra[1]);
    G8_C1();
    const uint32_t e00 = g8_colmax(acc);
    g8_keys(acc, kq0, e00, k00);
    __builtin_amdgcn_sched_barrier(0);
    if (group_end && late) barrier_block(false);  // (waves 4-7: above)
    __builtin_amdgcn_sched_barrier(0);
    // (s0, c1) || epilogue (s1, c0)
    acc = chain8(afrag[0], bf1, ra[0]);
    const uint32_t e10 = g8_colmax(acc2);
    g8_keys(acc2, kq0, e10, k10);
    g8_col_partial(e00, e10, cscw, h, r);
    __builtin_amdgcn_sched_barrier(0);
    // (s1, c1) || epilogue (s0, c1); inside a group the next tile's c0
    // fragments load under the epilogue (at a group end only after the barrier)
    acc2 = chain8(afrag[1], bf1, ra[1]);
    if (!group_end || late) G8_NEXT(g + 1);
    const uint32_t e01 = g8_colmax(acc);
    g8_keys(acc, kq1, e01, k01);
    g8_rows(k00, k01, b1r[0]);
    __builtin_amdgcn_sched_barrier(0);
    if (group_end && !late) barrier_block(true);
    // (g + 1: s0, c0) || epilogue (s1, c1)
    acc = chain8(afrag[0], bf0, ra[0]);
    const uint32_t e11 = g8_colmax(acc2);
    g8_keys(acc2, kq1, e11, k11);
    g8_rows(k10, k11, b1r[1]);
    g8_col_partial(e01, e11, cscw + 32, h, r);
    // Row flush at the end of a segment (or of the pair).
    if ((t & segm) == segm || t + 1 == nt) {
      row_flush_values<CLAMP>(b1r, rowres + pd.rowres_off + (int64_t)(t >> pd.seg8_log2) * pd.n1, row0,
                pd.n1, r, h);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 16; ++i) b1r[s][i] = 0u;
      flushed = g;
    }
    if (++t == nt && p + 1 < job.npairs) {
      ++p;
      t = 0;
      pd = P[p];
      nt = tile_end(p);
      segm = (1 << pd.seg8_log2) - 1;
      cpi = pd.colpart_off + (int64_t)job.rb * pd.n2pad;
    }
  }
  // Merge of the tiles no barrier merged: groups merged so far are those
  // before the last barrier's group (barrier m merges group m - 1).
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  const int nbar = G / kG8T;                         // barriers 0 .. nbar - 1 ran
  const int first = nbar >= 1 ? (nbar - 1) * kG8T : 0;  // first unmerged tile
  const int tg = first + wave;
  if (tg < G) {
    const uint32_t* src = csc + (((tg / kG8T) % kG8CscGroups) * kG8T + (tg & (kG8T - 1))) *
                                    kMatch8Waves * kTile8Cols;
    g8_merge(src + lane, colpart + meta[tg % kG8Stages] + lane);
  }
}

// ===========================================================================
// Finalize.
// ===========================================================================
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
    int cross_check, int colvals, uint2* __restrict__ matches, int32_t* __restrict__ counts) {
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

  if (cross_check && colvals) {
    // Column partials hold top-2 dot values (i8 kernel): m21[j] = the best
    // value of a passing column (unique best row, max_ratio <= 1), else -1.
    for (int j = tid; j < pd.n2; j += kFinThreads) {
      uint2 m = cp[j];
      int b = 1;
      for (; b + 4 <= pd.nrb; b += 4) {  // four row blocks' loads in flight
        uint2 o[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) o[u] = cp[(int64_t)(b + u) * pd.n2pad + j];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          m.y = max(max(m.y, o[u].y), min(m.x, o[u].x));
          m.x = max(m.x, o[u].x);
        }
      }
      for (; b < pd.nrb; ++b) {
        const uint2 o = cp[(int64_t)b * pd.n2pad + j];
        m.y = max(max(m.y, o.y), min(m.x, o.x));
        m.x = max(m.x, o.x);
      }
      m21[j] = passes(lut, m.x, m.y, max_ratio, max_distance) ? (int32_t)m.x : -1;
    }
    __syncthreads();
  } else if (cross_check) {
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
      if (ok && cross_check) ok = m21[col] == (colvals ? (int32_t)best : i);
      if (ok) {
        if (pass == 0) ++cnt;
        else matches[pd.match_off + out++] = make_uint2((uint32_t)i, (uint32_t)col);
      }
    }
  }
}

// Finalize of the version-2 i8 matcher (best-only column partials, value
// mode: max_ratio <= 1 with the cross-check, or no cross-check):
//  1. columns (match_colmerge_g8_kernel, one thread per column): merge the
//     row blocks' (B1, B2', wave) (raw accumulator units, converted here with
//     the column's sum) into colpart row 0 as x = B1 | rb << 19, y = B2' << 3
//     | wave (B1, B2' < 2^19: fast variant dots are < 2^19, clamp-variant
//     values <= 2^18);
//  2. rows (match_finalize_g8_kernel phase 0, a workgroup per pair): merge
//     the segments' row values, ratio / distance tests with the second's
//     lower bound, the passing rows queued by residue for
//     match_rowcheck_g8_kernel, which decides them; with the cross-check a
//     row i with best column j stays a CANDIDATE only if B1(j) equals its
//     best value, the 64-row group holding B1 is the one of row i (otherwise
//     another row ties B1: the column's second equals its best and fails),
//     and column j passes with second >= B2';
//  3. candidates (match_recheck_g8_kernel), per 64-row group: the exact
//     top-2 of the group's dots of column j on MFMA, and the final column
//     test with second = max(B2', second within the group);
//  4. ordered compaction of the accepted rows (idx1 ascending; phase 1).
// The per-row decisions live in rowres segment 0 between the phases.  The
// loops keep several rows' (row blocks') loads in flight: the chain runs on
// the small-batch critical path, where a pair's workgroup is latency-bound.
constexpr int kFinU = 8;  // rows per thread and pass (loads in flight)
// match_colmerge_g8_kernel: small batches spread a pair's columns over
// workgroups of kCmThreads (one column per thread); large batches take one
// workgroup of kFinThreads per pair (the table path: a grid of many small
// workgroups took CUs from the next batch's matcher beside it, matcher 4.5 %
// slower in the overlapped step, profiles/r06_s).
constexpr int kCmThreads = 256;
constexpr int kCmWidePairs = 256;  // up to this many pairs: the wide grid

__global__ __launch_bounds__(kFinThreads) void match_colmerge_g8_kernel(
    const PairDesc* __restrict__ pairs, uint2* __restrict__ colpart,
    const int32_t* __restrict__ csum, int prio) {
  if (prio) __builtin_amdgcn_s_setprio(2);
  const PairDesc pd = pairs[blockIdx.y];
  if (pd.n1 == 0) return;
  uint2* cp = colpart + pd.colpart_off;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < pd.n2; j += gridDim.x * blockDim.x) {
    const uint2 m = cp[j];
    uint32_t b1 = m.x, b2 = m.y >> 3, w = m.y & 7u, rbest = 0u;
    // ascending row blocks, eight loads in flight; a block past nrb reads as
    // (0, 0), which changes nothing (0 > b1 never holds, max(b2, 0) = b2)
    for (int b = 1; b < pd.nrb; b += 8) {
      uint2 o[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        o[u] = b + u < pd.nrb ? cp[(int64_t)(b + u) * pd.n2pad + j] : make_uint2(0u, 0u);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool gt = o[u].x > b1;
        b2 = gt ? max(o[u].y >> 3, b1) : max(b2, o[u].x);
        w = gt ? (o[u].y & 7u) : w;
        rbest = gt ? (uint32_t)(b + u) : rbest;
        b1 = gt ? o[u].x : b1;
      }
    }
    // raw accumulator units (dot - cb_j + 2^22) -> dot values of the column
    const uint32_t cbm = (uint32_t)csum[pd.b_row + j] - (1u << 22);
    b1 += cbm;
    b2 += cbm;
    if (pd.clamp) {
      b1 = min(b1, kLutMax);
      b2 = min(b2, kLutMax);
    }
    cp[j] = make_uint2(b1 | (rbest << 19), (b2 << 3) | w);
  }
}

__global__ __launch_bounds__(kFinThreads) void match_finalize_g8_kernel(
    const PairDesc* __restrict__ pairs, uint2* __restrict__ rowres, uint2* __restrict__ rowaux,
    int32_t* __restrict__ rlist, const float* __restrict__ lut, float max_ratio,
    float max_distance, uint2* __restrict__ matches, int32_t* __restrict__ counts, int phase) {
  // bit 4 of phase: raised wave priority (the batch's verification waits for
  // this chain; launch_match_finalize_g8)
  if (phase & 4) __builtin_amdgcn_s_setprio(2);
  phase &= 3;
  __shared__ int32_t wave_tot[kFinThreads / 64];
  __shared__ int32_t bcnt[32], bcur[32];
  const PairDesc pd = pairs[blockIdx.x];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  if (pd.n1 == 0 || pd.n2 == 0) {
    if (tid == 0) counts[blockIdx.x] = 0;
    return;
  }
  uint2* rr = rowres + pd.rowres_off;
  if (phase == 0) {
  // Phase 2: per-row decisions (rows strided over the threads, coalesced;
  // kFinU rows per thread and pass).  The matcher's rows carry their best
  // VALUE, the residue (mod 32) of the best column, and as second a lower
  // bound (best of the other lanes, see row_flush_values): a row that fails
  // with it fails; a row that passes is queued in the bucket of its residue
  // (state 3) for match_rowcheck_g8_kernel, which finds the best column, the
  // exact second and (with the cross-check) whether the row can still be its
  // column's match.
  int32_t* rl = rlist + pd.rlist_off;
  uint2* ax = rowaux + pd.aux_off;
  if (tid < 32) bcnt[tid] = 0;
  __syncthreads();
  for (int i0 = tid; i0 < pd.n1; i0 += kFinU * kFinThreads) {
    uint2 m[kFinU];
#pragma unroll
    for (int u = 0; u < kFinU; ++u) {
      const int i = i0 + u * kFinThreads;
      m[u] = i < pd.n1 ? rr[i] : make_uint2(0u, 0u);
    }
    for (int sg = 1; sg < pd.nseg; ++sg) {
      uint2 o[kFinU];
#pragma unroll
      for (int u = 0; u < kFinU; ++u) {
        const int i = i0 + u * kFinThreads;
        o[u] = i < pd.n1 ? rr[(int64_t)sg * pd.n1 + i] : make_uint2(0u, 0u);
      }
#pragma unroll
      for (int u = 0; u < kFinU; ++u) {
        m[u].y = merge_second(m[u].x, m[u].y, o[u].x, o[u].y);
        m[u].x = max(m[u].x, o[u].x);
      }
    }
#pragma unroll
    for (int u = 0; u < kFinU; ++u) {
      const int i = i0 + u * kFinThreads;
      if (i >= pd.n1) break;
      const uint32_t best = m[u].x >> kIdxBits, second = m[u].y >> kIdxBits;
      const int32_t col = (int32_t)((kIdxMask - (m[u].x & kIdxMask)) & 31u);  // residue of the best
      const uint32_t state = passes(lut, best, second, max_ratio, max_distance) ? 3u : 0u;
      rr[i] = make_uint2((uint32_t)col, state);
      if (state == 3u) {
        ax[i] = make_uint2(best, second);
        atomicAdd(&bcnt[col & 31], 1);
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int b = 0; b < 32; ++b) {
      rl[b] = acc;
      bcur[b] = acc;
      acc += bcnt[b];
    }
    rl[32] = acc;
  }
  __syncthreads();
  // (the order within a bucket is immaterial: every queued row is decided
  // alone; each thread re-reads the states it wrote above)
  for (int i0 = tid; i0 < pd.n1; i0 += kFinU * kFinThreads) {
    uint2 st[kFinU];
#pragma unroll
    for (int u = 0; u < kFinU; ++u) {
      const int i = i0 + u * kFinThreads;
      st[u] = i < pd.n1 ? rr[i] : make_uint2(0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < kFinU; ++u)
      if (st[u].y == 3u) rl[33 + atomicAdd(&bcur[st[u].x & 31u], 1)] = i0 + u * kFinThreads;
  }
  return;
  }
  // Phase 4: ordered compaction (idx1 ascending), one tile of kFinThreads
  // consecutive rows at a time (the states of kFinU tiles loaded together):
  // ballot prefixes within the waves, wave offsets through LDS, a running
  // offset over the tiles.
  int run = 0;
  for (int r0 = 0; r0 < pd.n1; r0 += kFinU * kFinThreads) {
    uint2 sts[kFinU];
#pragma unroll
    for (int u = 0; u < kFinU; ++u) {
      const int i = r0 + u * kFinThreads + tid;
      sts[u] = i < pd.n1 ? rr[i] : make_uint2(0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < kFinU; ++u) {
      const int t0 = r0 + u * kFinThreads;
      if (t0 >= pd.n1) break;
      const int i = t0 + tid;
      const uint2 st = sts[u];
      const bool f = st.y == 1u;
      const uint64_t bm = __ballot(f);
      if (lane == 0) wave_tot[wave] = __popcll(bm);
      __syncthreads();
      int off = run, tot = 0;
      for (int w = 0; w < kFinThreads / 64; ++w) {
        const int c = wave_tot[w];
        off += w < wave ? c : 0;
        tot += c;
      }
      if (f) {
        const int pre = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
        matches[pd.match_off + off + pre] = make_uint2((uint32_t)i, st.x);
      }
      run += tot;
      __syncthreads();  // wave_tot is rewritten by the next tile
    }
  }
  if (tid == 0) counts[blockIdx.x] = run;
}

// Best column and exact second of the queued rows (finalize phase 2b).  The
// matcher keeps per lane only the best VALUE of each row over that lane's
// columns (j = lane + 32 t), so a row is known by its best value, the residue
// b of its best column and a lower bound of its second (the best of the other
// lanes).  One workgroup per (pair, residue b): the queued rows of bucket b
// against every column = b (mod 32) of the neighbour (staged in LDS, 256 at a
// time), on the matcher's own MFMA with the same offset operands: A = those
// columns (C operand = their sums), B = the rows; per row the exact top-2
// (multiset) over the residue class and the LOWEST column holding the class
// best (FindBestMatchesOneWay keeps the first maximum).  The row's second is
// then exact (max of the lower bound and the in-class second) and the ratio /
// distance test final; with the cross-check the row stays a candidate (state
// 2, match_recheck_g8_kernel) only if its column's best value equals the
// row's best, sits in the row's 64-row group and passes the column's test with
// the column's second lower bound; otherwise it is a match (1) or rejected (0).
constexpr int kRcThreads = 256;
constexpr int kRcChunk = 256;  // columns of one residue class staged per pass (32 KiB)

__global__ __launch_bounds__(kRcThreads) void match_rowcheck_g8_kernel(
    const PairDesc* __restrict__ pairs, uint2* __restrict__ rowres,
    const uint2* __restrict__ colpart,
    const uint2* __restrict__ rowaux, const int32_t* __restrict__ rlist,
    const uint8_t* __restrict__ desc8, const int32_t* __restrict__ csum,
    const float* __restrict__ lut, float max_ratio, float max_distance, int cross_check,
    int prio) {
  if (prio) __builtin_amdgcn_s_setprio(2);
  __shared__ __attribute__((aligned(16))) uint8_t lcol[kRcChunk * 128];
  __shared__ int32_t lcs[kRcChunk + 32];
  const PairDesc pd = pairs[blockIdx.y];
  const int b = blockIdx.x;
  if (pd.n1 == 0 || pd.n2 <= b) return;
  const int32_t* rl = rlist + pd.rlist_off;
  const int q0 = rl[b], R = rl[b + 1] - q0;
  if (R <= 0) return;
  const int32_t* rows = rl + 33 + q0;
  const int Cb = (pd.n2 - b + 31) / 32;  // columns b, b + 32, ... < n2
  const int nchunks = (Cb + kRcChunk - 1) / kRcChunk;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  uint2* rr = rowres + pd.rowres_off;
  const uint2* ax = rowaux + pd.aux_off;
  for (int g0 = 0; g0 < R; g0 += 4 * 32) {  // row groups: 4 waves x 32 rows
    const int k = g0 + wave * 32 + r;
    const bool rv = k < R;
    const int row = rows[rv ? k : 0];
    i32x4 bfr[4];
    {
      const i32x4* src = reinterpret_cast<const i32x4*>(desc8 + (pd.a_row + row) * 128) + 4 * h;
#pragma unroll
      for (int q = 0; q < 4; ++q) bfr[q] = src[q];
    }
    int t1 = INT_MIN, t2 = INT_MIN;  // this lane's top-2 (multiset) over its columns
    int j1 = 0;                      // column of t1 (first maximum in column order)
    for (int c = 0; c < nchunks; ++c) {
      const int cbeg = c * kRcChunk, cn = min(kRcChunk, Cb - cbeg);
      if (nchunks > 1 || g0 == 0) {
        __syncthreads();
        for (int e = tid; e < cn * 8; e += kRcThreads) {
          const int x = e >> 3, ch = e & 7;
          const int64_t j = b + 32 * (int64_t)(cbeg + x);
          *reinterpret_cast<i32x4*>(lcol + sw8(x, ch)) =
              *reinterpret_cast<const i32x4*>(desc8 + (pd.b_row + j) * 128 + ch * 16);
        }
        for (int x = tid; x < cn; x += kRcThreads) lcs[x] = csum[pd.b_row + b + 32 * (int64_t)(cbeg + x)];
        __syncthreads();
      }
      for (int ct = 0; ct * 32 < cn; ++ct) {
        i32x4 afr[4];
        load_bfrag8(lcol, ct * 32 + r, h, afr);  // column ct*32 + r, chunk 4h + q
        i32x16 cinit;
#pragma unroll
        for (int i = 0; i < 16; ++i) cinit[i] = lcs[ct * 32 + 4 * h + (i & 3) + 8 * (i >> 2)];
        const i32x16 acc = chain8(afr, bfr, cinit);  // a'.b' + cs(column): dot - cs(row) + 2^21
        // this lane's columns in ascending order: x = ct*32 + 4h + (i & 3) + 8 (i >> 2)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int x = ct * 32 + 4 * h + (i & 3) + 8 * (i >> 2);
          const int v = x < cn ? acc[i] : INT_MIN;
          t2 = max(t2, min(t1, v));
          j1 = v > t1 ? cbeg + x : j1;
          t1 = max(t1, v);
        }
      }
    }
    // The two lane halves hold the class's columns 4h + (i & 3) + 8 (i >> 2) of
    // each 32-column tile: merge them (symmetric in the two halves).
    const auto e1 = __builtin_amdgcn_permlane32_swap(t1, t1, false, false);
    const auto e2 = __builtin_amdgcn_permlane32_swap(t2, t2, false, false);
    const auto ej = __builtin_amdgcn_permlane32_swap(j1, j1, false, false);
    if (h == 0 && rv) {
      const int s2 = max(max((int)e2[0], (int)e2[1]), min((int)e1[0], (int)e1[1]));
      // a tie between the halves makes the second equal the best: the row fails
      // whichever column is taken
      const int jb = (int)e1[1] > (int)e1[0] ? (int)ej[1] : (int)ej[0];
      const int32_t col = b + 32 * jb;
      const uint2 a = ax[row];
      const int32_t rowsum = csum[pd.a_row + row] - (1 << 21);
      uint32_t d2 = s2 == INT_MIN ? 0u : (uint32_t)(s2 + rowsum);  // one column only: second 0
      if (pd.clamp) d2 = min(d2, kLutMax);
      const uint32_t second = max(a.y, d2);
      uint32_t state = passes(lut, a.x, second, max_ratio, max_distance) ? (cross_check ? 2u : 1u) : 0u;
      if (state == 2u) {  // can the row still be its column's match? (colpart merged by phase 0)
        constexpr uint32_t kV = (1u << 19) - 1u;
        const uint2 c = colpart[pd.colpart_off + col];
        const uint32_t b1 = c.x & kV, rb = c.x >> 19, w = c.y & 7u, b2 = c.y >> 3;
        const uint32_t grp = rb * (uint32_t)(kRowsPerBlock8 / 64) + w;
        if (b1 != a.x || grp != (uint32_t)(row >> 6) || !passes(lut, b1, b2, max_ratio, max_distance))
          state = 0u;
      }
      rr[row] = make_uint2((uint32_t)col, state);
    }
  }
}

// Phase 3 of the version-2 finalize: one wave per 64-row group of a pair
// (grid: x = groups of 4, y = pair).  The group's 64 rows are the A operand
// of the matcher's own MFMA (i8 32x32x32, the same offset operands and
// fragment layout), up to 32 candidate columns per pass the B operand; each
// lane's 16-row top-2 tree, the row sub-tiles and the lane halves give every
// candidate column the exact top-2 of the group's 64 dots.  With it, the
// column's second is max(B2', second within the group) and the cross-check
// decision of the candidate row is final.
__global__ __launch_bounds__(256) void match_recheck_g8_kernel(
    const PairDesc* __restrict__ pairs, uint2* __restrict__ rowres, uint2* __restrict__ colpart,
    const uint8_t* __restrict__ desc8, const int32_t* __restrict__ csum,
    const float* __restrict__ lut, float max_ratio, float max_distance, int prio) {
  if (prio) __builtin_amdgcn_s_setprio(2);
  __shared__ int32_t cand_lane[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const PairDesc pd = pairs[blockIdx.y];
  const int grp = blockIdx.x * 4 + wave;
  if (pd.n1 == 0 || pd.n2 == 0 || grp * 64 >= pd.n1) return;
  uint2* cp = colpart + pd.colpart_off;
  uint2* rr = rowres + pd.rowres_off;
  constexpr uint32_t kV = (1u << 19) - 1u;
  const int row = grp * 64 + lane;
  const uint2 st = row < pd.n1 ? rr[row] : make_uint2(0u, 0u);
  const uint64_t cand = __ballot(st.y == 2u);
  if (!cand) return;
  // Candidate k of the group (ascending lane) -> its lane.
  const int k = __builtin_amdgcn_mbcnt_hi((uint32_t)(cand >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)cand, 0u));
  if (st.y == 2u) cand_lane[wave][k] = lane;
  const int ncand = __popcll(cand);
  // A fragments: rows grp*64 + 32 s + r, chunks 4h + q; accumulator offsets
  // cs(a) of the rows this lane's results belong to (zero rows past n1).
  const int row0 = grp * 64;
  i32x4 afrag[2][4];
  i32x16 ra[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int rw = row0 + 32 * s + r;
    const bool ok = rw < pd.n1;
    const i32x4* src =
        reinterpret_cast<const i32x4*>(desc8 + (pd.a_row + (ok ? rw : 0)) * 128) + h * 4;
    const int z = (int)0x80808080u;
#pragma unroll
    for (int q = 0; q < 4; ++q) afrag[s][q] = ok ? src[q] : i32x4{z, z, z, z};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ri = row0 + 32 * s + 4 * h + (i & 3) + 8 * (i >> 2);
      const uint32_t cs = (uint32_t)csum[pd.a_row + min(ri, pd.n1 - 1)];
      ra[s][i] = (int)(ri < pd.n1 ? cs : 0u);
    }
  }
  __builtin_amdgcn_wave_barrier();
  for (int base = 0; base < ncand; base += 32) {
    const int c = base + r;  // this lane's candidate column slot
    const bool valid = c < ncand;
    const int L = valid ? cand_lane[wave][c] : 0;
    const int jc = __shfl((int)st.x, L);
    const int jv = valid ? jc : 0;
    i32x4 bfr[4];
    const i32x4* bsrc = reinterpret_cast<const i32x4*>(desc8 + (pd.b_row + jv) * 128) + h * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) bfr[q] = bsrc[q];
    const uint32_t cbj = (uint32_t)csum[pd.b_row + jv];
    const uint2 cpc = cp[jv];
    const i32x16 acc0 = chain8(afrag[0], bfr, ra[0]);
    const i32x16 acc1 = chain8(afrag[1], bfr, ra[1]);
    const uint2 p0 = column_top2_values(acc0), p1 = column_top2_values(acc1);
    const uint32_t t1 = max(p0.x, p1.x);
    uint32_t t2 = merge_second_values(p0.x, p0.y, p1.x, p1.y);
    const auto s1 = __builtin_amdgcn_permlane32_swap(t1, t1, false, false);
    const auto s2 = __builtin_amdgcn_permlane32_swap(t2, t2, false, false);
    // lanes of half 0: the partner's (half 1's) values are the second results
    t2 = merge_second_values(t1, t2, (uint32_t)s1[1], (uint32_t)s2[1]);
    if (h == 0 && valid) {
      uint32_t d2 = t2 + cbj - (1u << 21);  // a'.b' + 128(Sa + Sb) - 2^21
      if (pd.clamp) d2 = min(d2, kLutMax);
      const uint32_t b1 = cpc.x & kV, b2 = max(cpc.y >> 3, d2);
      rr[row0 + L] =
          make_uint2((uint32_t)jc, passes(lut, b1, b2, max_ratio, max_distance) ? 1u : 0u);
    }
  }
}

// ===========================================================================
// Table conversion at load.
// ===========================================================================
// u8 -> bf16 (exact: integers < 256).
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

// u8 -> i8 offset operands: a ^ 0x80 (= a - 128) per byte and
// cs = 128 * sum_d a_d per 128-B descriptor (8 threads per descriptor).
__global__ void u8_to_i8_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                int32_t* __restrict__ csum, int64_t nrows) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = g >> 3;
  uint32_t s = 0;
  if (row < nrows) {
    const uint4 v = reinterpret_cast<const uint4*>(in)[g];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      s += (w[e] & 255u) + ((w[e] >> 8) & 255u) + ((w[e] >> 16) & 255u) + (w[e] >> 24);
    reinterpret_cast<uint4*>(out)[g] = make_uint4(v.x ^ 0x80808080u, v.y ^ 0x80808080u,
                                                  v.z ^ 0x80808080u, v.w ^ 0x80808080u);
  }
  s += __shfl_xor(s, 1);
  s += __shfl_xor(s, 2);
  s += __shfl_xor(s, 4);
  if (row < nrows && (g & 7) == 0) csum[row] = (int32_t)(128u * s);
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

hipError_t launch_match_g8(const uint8_t* desc8, const int32_t* csum, const MatchJob* jobs,
                           int njobs, const PairDesc* pairs, uint2* rowres, uint2* colpart,
                           bool clamp, hipStream_t stream) {
  if (njobs <= 0) return hipSuccess;
  if (clamp)
    hipLaunchKernelGGL(match_g8_kernel<true>, dim3(njobs), dim3(kMatch8Threads), 0, stream, desc8,
                       csum, jobs, pairs, rowres, colpart);
  else
    hipLaunchKernelGGL(match_g8_kernel<false>, dim3(njobs), dim3(kMatch8Threads), 0, stream, desc8,
                       csum, jobs, pairs, rowres, colpart);
  return hipGetLastError();
}

hipError_t launch_match_finalize_g8(const PairDesc* pairs, int npairs, uint2* rowres,
                                    uint2* colpart, uint2* rowaux, int32_t* rlist,
                                    const uint8_t* desc8, const int32_t* csum,
                                    const float* lut, float max_ratio, float max_distance,
                                    int cross_check, uint2* matches, int32_t* counts,
                                    int max_groups, int max_cols, hipStream_t stream) {
  if (npairs <= 0) return hipSuccess;
  // The finalize chain's waves at raised issue priority over the verification
  // kernels of earlier batches beside it: the batch's own verification waits
  // for this chain (46.90/47.00K vs 46.78/46.75K pairs/s, profiles/r05_v).
  constexpr int prio = 1;
  const int pbit = prio ? 4 : 0;
  if (cross_check && max_cols > 0) {
    const bool wide = npairs <= kCmWidePairs;
    hipLaunchKernelGGL(match_colmerge_g8_kernel,
                       dim3(wide ? (unsigned)((max_cols + kCmThreads - 1) / kCmThreads) : 1u, npairs),
                       dim3(wide ? kCmThreads : kFinThreads), 0, stream, pairs, colpart, csum, prio);
  }
  hipLaunchKernelGGL(match_finalize_g8_kernel, dim3(npairs), dim3(kFinThreads), 0, stream, pairs,
                     rowres, rowaux, rlist, lut, max_ratio, max_distance, matches, counts, 0 | pbit);
  hipLaunchKernelGGL(match_rowcheck_g8_kernel, dim3(32, npairs), dim3(kRcThreads), 0, stream,
                     pairs, rowres, colpart, rowaux, rlist, desc8, csum, lut, max_ratio, max_distance,
                     cross_check, prio);
  if (cross_check && max_groups > 0)
    hipLaunchKernelGGL(match_recheck_g8_kernel, dim3((unsigned)((max_groups + 3) / 4), npairs),
                       dim3(256), 0, stream, pairs, rowres, colpart, desc8, csum, lut, max_ratio,
                       max_distance, prio);
  hipLaunchKernelGGL(match_finalize_g8_kernel, dim3(npairs), dim3(kFinThreads), 0, stream, pairs,
                     rowres, rowaux, rlist, lut, max_ratio, max_distance, matches, counts, 1 | pbit);
  return hipGetLastError();
}

hipError_t launch_match_finalize(const PairDesc* pairs, int npairs, const uint2* rowres,
                                 const uint2* colpart, int32_t* m21, const float* lut,
                                 float max_ratio, float max_distance, int cross_check,
                                 int colvals, uint2* matches, int32_t* counts,
                                 hipStream_t stream) {
  if (npairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(match_finalize_kernel, dim3(npairs), dim3(kFinThreads), 0, stream, pairs,
                     rowres, colpart, m21, lut, max_ratio, max_distance, cross_check, colvals,
                     matches, counts);
  return hipGetLastError();
}

hipError_t launch_u8_to_bf16(const uint8_t* in, uint16_t* out, int64_t n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const int64_t threads = (n + 7) / 8;
  hipLaunchKernelGGL(u8_to_bf16_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     stream, in, out, n);
  return hipGetLastError();
}

hipError_t launch_u8_to_i8(const uint8_t* in, uint8_t* out, int32_t* csum, int64_t nrows,
                           hipStream_t stream) {
  if (nrows <= 0) return hipSuccess;
  const int64_t threads = nrows * 8;
  hipLaunchKernelGGL(u8_to_i8_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     stream, in, out, csum, nrows);
  return hipGetLastError();
}

namespace {
constexpr int kUploadThreads = 256;
constexpr int kUploadMaxBlocks = 512;
__global__ void __launch_bounds__(kUploadThreads)
    stage_upload_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t n) {
  const int64_t step = (int64_t)gridDim.x * kUploadThreads;
  for (int64_t i = (int64_t)blockIdx.x * kUploadThreads + threadIdx.x; i < n; i += step)
    dst[i] = src[i];
}
}  // namespace

hipError_t launch_stage_upload(const void* host_dev_src, void* dst, size_t bytes,
                               hipStream_t stream) {
  if (bytes == 0) return hipSuccess;
  if (bytes % sizeof(uint4) != 0) return hipErrorInvalidValue;
  const int64_t n = (int64_t)(bytes / sizeof(uint4));
  const int64_t blocks = std::min<int64_t>((n + kUploadThreads - 1) / kUploadThreads, kUploadMaxBlocks);
  hipLaunchKernelGGL(stage_upload_kernel, dim3((unsigned)blocks), dim3(kUploadThreads), 0, stream,
                     reinterpret_cast<const uint4*>(host_dev_src), reinterpret_cast<uint4*>(dst), n);
  return hipGetLastError();
}

}  // namespace scm
