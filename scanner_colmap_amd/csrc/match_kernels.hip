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
// Two matchers produce the same keys and partial results and share the
// finalize kernel: match_tiles_i8_kernel (default: integer MFMA on offset
// operands, see its section) and match_tiles_kernel (bf16 MFMA, selected by
// SCM_MATCH_BF16=1).
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
#ifndef SCM_DIAG_MERGE
#define SCM_DIAG_MERGE 1  // diagnostics: 0 drops the column merge (wrong results)
#endif
// LDS ring: tile t + 3 is staged at the end of tile t and first read in tile
// t + 2 (the B-fragment prefetch).  One barrier per kBarTiles tiles (2: 2-3 %
// faster than 1): waves may then be two tiles apart, so the ring holds 6 tiles
// and the column partials 4 buffers; every staging write still has a barrier
// before its first read.  (4 would need staging further ahead: with t + 3 a
// group of 4 leaves writes and reads of a tile without a barrier between.)
#ifndef SCM_I8_BAR_TILES
#define SCM_I8_BAR_TILES 2
#endif
constexpr int kBarTiles = SCM_I8_BAR_TILES;
static_assert(kBarTiles == 1 || kBarTiles == 2, "barrier group");
constexpr int kStages8 = kBarTiles == 1 ? 4 : 6;
constexpr int kCscBufs = 2 * kBarTiles;
constexpr int kAhead8 = 3;
constexpr int kTiles8PerSeg = kTilesPerSeg / 2;  // 64-column tiles per 8192-column segment

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

// Column value partial of one 32-column sub-tile of a wave (both row
// sub-tiles, both lane halves); lanes of half 0 store it for the workgroup merge.
__device__ __forceinline__ void wave_col_partial_values(uint2 c0, uint2 c1, uint2* dst, int h, int r) {
  uint32_t B1 = max(c0.x, c1.x), B2 = merge_second_values(c0.x, c0.y, c1.x, c1.y);
  const uint32_t o1 = __shfl_xor(B1, 32);
  const uint32_t o2 = __shfl_xor(B2, 32);
  B2 = merge_second_values(B1, B2, o1, o2);
  B1 = max(B1, o1);
  if (h == 0) dst[r] = make_uint2(B1, B2);
}

// Row keys of a finished sub-tile and the row top-2 state update; returns the
// column value partial.  kc = (cb_j << 13) | t-bits; cbm = cb_j - 2^22.
template <bool CLAMP>
__device__ __forceinline__ uint2 subtile_epilogue8(const i32x16& acc, uint32_t kc, uint32_t cbm,
                                                   uint32_t tbits, uint32_t (&b1r)[16],
                                                   uint32_t (&b2r)[16]) {
#ifdef SCM_DIAG_MATCH_SKELETON
  // diagnostics only: MFMA + LDS + staging skeleton, results discarded
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) x ^= (uint32_t)acc[i];
  b1r[0] ^= x;
  return make_uint2(x, x);
#endif
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t x = (uint32_t)acc[i];
    const uint32_t key = CLAMP ? (min(x + cbm, kLutMax) << 13) | tbits : (x << 13) + kc;
    b2r[i] = med3_u32(key, b1r[i], b2r[i]);
    b1r[i] = max(b1r[i], key);
  }
  return column_top2_values(acc);
}

// Merge of the kMatch8Waves wave partials of tile k's 64 columns (one wave;
// lane = column 32 h + r) and store of the columns' top-2 dot values.
template <bool CLAMP>
__device__ __forceinline__ void merge_cols8(const uint2* colscratch, int k, int h, int r, int lane,
                                            uint32_t cbm_col, uint2* dst) {
  const uint2* src = colscratch + (k % kCscBufs) * 2 * kMatch8Waves * 32 + h * kMatch8Waves * 32 + r;
  uint2 m = src[0];
#pragma unroll
  for (int w = 1; w < kMatch8Waves; ++w) {
    const uint2 o = src[w * 32];
    m.y = merge_second_values(m.x, m.y, o.x, o.y);
    m.x = max(m.x, o.x);
  }
  m.x += cbm_col;
  m.y += cbm_col;
  if (CLAMP) {
    m.x = min(m.x, kLutMax);
    m.y = min(m.y, kLutMax);
  }
  dst[lane] = m;
}

// One workgroup = one MatchJob (512 pivot rows, 8 waves x 64) swept against
// every column of its neighbour images, 64 columns per LDS tile.  Per wave
// and tile: four 4-MFMA chains (row sub-tile s, column sub-tile c), software
// pipelined so that each chain runs under the epilogue of the previous one:
//   (s1,c0) || epi(s0,c0);  (s0,c1) || epi(s1,c0);  (s1,c1) || epi(s0,c1);
//   (t+1: s0,c0) || epi(s1,c1).
// Tiles rotate through a 4-stage LDS ring; one barrier per tile.
template <bool CLAMP>
__global__ __launch_bounds__(kMatch8Threads, 512 / kMatch8Threads) void match_tiles_i8_kernel(
    const uint8_t* __restrict__ desc8,  // a ^ 0x80, [rows][128]
    const int32_t* __restrict__ csum,   // 128 * sum_d a_d per row
    const MatchJob* __restrict__ jobs, const PairDesc* __restrict__ pairs,
    uint2* __restrict__ rowres,         // per pair [nseg][n1]
    uint2* __restrict__ colpart) {      // per pair [nrb][n2pad]
  __shared__ __attribute__((aligned(16))) uint8_t
      lds[kStages8 * kTile8Bytes + kCscBufs * 2 * kMatch8Waves * 32 * 8];
  // column partials: [tile parity][column sub-tile][wave][32]
  uint2* colscratch = reinterpret_cast<uint2*>(lds + kStages8 * kTile8Bytes);

  const MatchJob job = jobs[blockIdx.x];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int row0 = job.rb * kRowsPerBlock8 + wave * 64;

  // ---- A fragments (rows row0 + 32 s + r, chunks 4h + q) and the
  // accumulator offsets of the rows this lane's results belong to.
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
      ra[s][i] = (int)((rw < job.n1 ? (uint32_t)csum[job.a_row + rw] : 0u) + (1u << 21));
    }
  }

  // Staging role of this thread: kSt 16-B chunks of the 8 KiB tile (chunk
  // tid + kMatch8Threads * u = 8 col + c).
  constexpr int kTileChunks = kTile8Cols * 8;  // 16-B chunks per tile
  constexpr int kSt = kTileChunks / kMatch8Threads;
  static_assert(kSt * kMatch8Threads == kTileChunks, "staging covers the tile");
  int st_lds[kSt], st_off[kSt];
#pragma unroll
  for (int u = 0; u < kSt; ++u) {
    const int ch = tid + kMatch8Threads * u;
    st_lds[u] = sw8(ch >> 3, ch & 7);
    st_off[u] = (ch >> 3) * 8 + (ch & 7);  // in 16-B chunks from the tile's first column
  }

  for (int p = 0; p < job.npairs; ++p) {
    const PairDesc pd = pairs[job.pair0 + p];
    const int ntiles_total = (pd.n2 + kTile8Cols - 1) / kTile8Cols;
    uint2* colp = colpart + pd.colpart_off + (int64_t)job.rb * pd.n2pad;
    const int32_t* bsum = csum + pd.b_row;
    const i32x4* src0 = reinterpret_cast<const i32x4*>(desc8 + pd.b_row * 128);
    for (int seg = 0; seg < pd.nseg; ++seg) {
      const int t_begin = seg * kTiles8PerSeg;
      const int t_end = min(ntiles_total, t_begin + kTiles8PerSeg);
      const int tlast = t_end - 1;
      uint32_t b1r[2][16], b2r[2][16];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 16; ++i) { b1r[s][i] = 0u; b2r[s][i] = 0u; }
      // Prologue: stage tiles t_begin .. t_begin + 2, the column offsets of
      // the first three, and the chain (t_begin: s0, c0).
#pragma unroll
      for (int j = 0; j < kAhead8; ++j)
#pragma unroll
        for (int u = 0; u < kSt; ++u)
          *reinterpret_cast<i32x4*>(lds + j * kTile8Bytes + st_lds[u]) =
              src0[(int64_t)min(t_begin + j, tlast) * kTileChunks + st_off[u]];
      const int t1 = min(t_begin + 1, tlast), t2 = min(t_begin + 2, tlast);
      uint32_t cb0 = (uint32_t)bsum[t_begin * kTile8Cols + r];
      uint32_t cb1 = (uint32_t)bsum[t_begin * kTile8Cols + 32 + r];
      uint32_t cn0 = (uint32_t)bsum[t1 * kTile8Cols + r];
      uint32_t cn1 = (uint32_t)bsum[t1 * kTile8Cols + 32 + r];
      uint32_t cm0 = (uint32_t)bsum[t2 * kTile8Cols + r];
      uint32_t cm1 = (uint32_t)bsum[t2 * kTile8Cols + 32 + r];
      __syncthreads();
      i32x4 bf0[4], bf1[4];
      load_bfrag8(lds, r, h, bf0);
      i32x16 acc = chain8(afrag[0], bf0, ra[0]);

      for (int k = 0; k < t_end - t_begin; ++k) {
        const int t = t_begin + k;
        const int t3 = min(t + 3, tlast);
        i32x4 nxt[kSt];
#pragma unroll
        for (int u = 0; u < kSt; ++u) nxt[u] = src0[(int64_t)t3 * kTileChunks + st_off[u]];
        const uint32_t cf0 = (uint32_t)bsum[t3 * kTile8Cols + r];
        const uint32_t cf1 = (uint32_t)bsum[t3 * kTile8Cols + 32 + r];
        const uint32_t tb0 = (uint32_t)(kTilesPerSeg - 1 - 2 * k), tb1 = tb0 - 1u;
        const uint8_t* cur = lds + (k % kStages8) * kTile8Bytes;
        uint2* csc = colscratch + (k % kCscBufs) * 2 * kMatch8Waves * 32;
        const uint32_t kc0 = (cb0 << 13) | tb0, kc1 = (cb1 << 13) | tb1;
        const uint32_t cbm0 = cb0 - (1u << 22), cbm1 = cb1 - (1u << 22);
        // (s1, c0) || epilogue (s0, c0)
        i32x16 acc2 = chain8(afrag[1], bf0, ra[1]);
        const uint2 e00 = subtile_epilogue8<CLAMP>(acc, kc0, cbm0, tb0, b1r[0], b2r[0]);
        __builtin_amdgcn_sched_barrier(0);
        // (s0, c1) || epilogue (s1, c0)
        load_bfrag8(cur, 32 + r, h, bf1);
        acc = chain8(afrag[0], bf1, ra[0]);
        const uint2 e10 = subtile_epilogue8<CLAMP>(acc2, kc0, cbm0, tb0, b1r[1], b2r[1]);
        wave_col_partial_values(e00, e10, csc + wave * 32, h, r);
        __builtin_amdgcn_sched_barrier(0);
        // (s1, c1) || epilogue (s0, c1)
        acc2 = chain8(afrag[1], bf1, ra[1]);
        const uint2 e01 = subtile_epilogue8<CLAMP>(acc, kc1, cbm1, tb1, b1r[0], b2r[0]);
        __builtin_amdgcn_sched_barrier(0);
        // (t + 1: s0, c0) || epilogue (s1, c1)
        load_bfrag8(lds + ((k + 1) % kStages8) * kTile8Bytes, r, h, bf0);
        acc = chain8(afrag[0], bf0, ra[0]);
        const uint2 e11 = subtile_epilogue8<CLAMP>(acc2, kc1, cbm1, tb1, b1r[1], b2r[1]);
        wave_col_partial_values(e01, e11, csc + (kMatch8Waves + wave) * 32, h, r);
#pragma unroll
        for (int u = 0; u < kSt; ++u)
          *reinterpret_cast<i32x4*>(lds + ((k + 3) % kStages8) * kTile8Bytes + st_lds[u]) = nxt[u];
        // this lane's column in the merge below: 32 h + r of tile t
        const uint32_t cbm_col = h ? cbm1 : cbm0;
        cb0 = cn0;
        cb1 = cn1;
        cn0 = cm0;
        cn1 = cm1;
        cm0 = cf0;
        cm1 = cf1;
        if ((k + 1) % kBarTiles == 0) {
#ifndef SCM_DIAG_NOBARRIER  // diagnostics only: no barrier (races; timing of the barrier)
          __syncthreads();
#endif
          // One wave merges the 8 wave partials of the last kBarTiles tiles'
          // 64 columns each and stores the columns' top-2 dot values.  (All
          // waves sharing the merge, 8 columns each, measured 6 % slower:
          // every wave then waits on LDS right after the barrier.)
          if (SCM_DIAG_MERGE && wave == ((k / kBarTiles) & (kMatch8Waves - 1))) {
#pragma unroll
            for (int g = kBarTiles - 1; g > 0; --g)
              merge_cols8<CLAMP>(colscratch, k - g, h, r, lane,
                                 (uint32_t)bsum[(t - g) * kTile8Cols + lane] - (1u << 22),
                                 colp + (t - g) * kTile8Cols);
            merge_cols8<CLAMP>(colscratch, k, h, r, lane, cbm_col, colp + t * kTile8Cols);
          }
        }
      }
      if (const int rest = (t_end - t_begin) % kBarTiles) {  // tiles after the last barrier
        __syncthreads();
        const int kl = t_end - t_begin - 1;
        if (SCM_DIAG_MERGE && wave == ((kl / kBarTiles) & (kMatch8Waves - 1)))
          for (int g = rest - 1; g >= 0; --g)
            merge_cols8<CLAMP>(colscratch, kl - g, h, r, lane,
                               (uint32_t)bsum[(t_end - 1 - g) * kTile8Cols + lane] - (1u << 22),
                               colp + (t_end - 1 - g) * kTile8Cols);
      }
      __syncthreads();  // every wave done with the LDS tiles before the next segment
      row_flush(b1r, b2r, rowres + pd.rowres_off + (int64_t)seg * pd.n1, row0, pd.n1, r, h);
    }
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

hipError_t launch_match_tiles_i8(const uint8_t* desc8, const int32_t* csum, const MatchJob* jobs,
                                 int njobs, const PairDesc* pairs, uint2* rowres, uint2* colpart,
                                 bool clamp, hipStream_t stream) {
  if (njobs <= 0) return hipSuccess;
  if (clamp)
    hipLaunchKernelGGL(match_tiles_i8_kernel<true>, dim3(njobs), dim3(kMatch8Threads), 0, stream,
                       desc8, csum, jobs, pairs, rowres, colpart);
  else
    hipLaunchKernelGGL(match_tiles_i8_kernel<false>, dim3(njobs), dim3(kMatch8Threads), 0, stream,
                       desc8, csum, jobs, pairs, rowres, colpart);
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

}  // namespace scm
