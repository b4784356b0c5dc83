// Shared constants / job descriptors of the matcher kernels (match_kernels.hip)
// and their host launchers (scm_runtime.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace scm {

constexpr int kMatchWaves = 8;                   // waves per workgroup
constexpr int kMatchThreads = kMatchWaves * 64;  // 512
constexpr int kRowsPerBlock = kMatchWaves * 64;  // pivot rows per workgroup
// i8 kernel: waves per workgroup (4 = 256-row jobs, two workgroups per CU:
// +5 % isolated, no gain beside verification)
constexpr int kMatch8Waves = 8;
constexpr int kMatch8Threads = kMatch8Waves * 64;
constexpr int kRowsPerBlock8 = kMatch8Waves * 64;
constexpr int kTileBytes = 32 * 256;             // bf16 kernel: 32 descriptors per LDS tile
constexpr int kTile8Cols = 64;                   // i8 kernel: 64 descriptors per LDS tile
constexpr int kTile8Bytes = kTile8Cols * 128;    // 8 KiB
constexpr int kDescRowAlign = 64;                // descriptor rows of an image padded to this
constexpr int kTilesPerSeg = 256;                // 8 tile-index bits per key (32-column units)
constexpr int kColsPerSeg = kTilesPerSeg * 32;   // 8192 columns per segment
constexpr int kIdxBits = 13;
constexpr uint32_t kIdxMask = (1u << kIdxBits) - 1u;
constexpr uint32_t kLutMax = 1u << 18;           // acosf LUT covers [0, 2^18]
constexpr int kFinThreads = 1024;
constexpr int kXcds = 8;                         // MI355X: 8 XCDs, round-robin dispatch
constexpr int kNumCUs = 256;                     // MI355X: 32 CUs per XCD

// Column split of the i8 matcher (small batches): a pair's columns in up to
// kMaxColSplit parts of 2^seg8_log2 64-column tiles, one job and one row
// segment each.
constexpr int kMaxColSplit = 8;
constexpr int kSeg8Log2 = 7;  // unsplit: 128 tiles (8192 columns) per row segment

// One workgroup of match_tiles_kernel: 512 rows of a pivot image against
// every column of `npairs` neighbour images (pairs[pair0 .. pair0+npairs)).
// i8 kernel: the first pair from 64-column tile t0, the last up to tile t1
// (exclusive; 0 = its last tile): a column part of a split pair (npairs 1).
struct MatchJob {
  int64_t a_row;   // table row of the pivot image's descriptor 0
  int32_t rb;      // row block
  int32_t n1;      // pivot keypoints
  int32_t pair0;   // first PairDesc of this pivot
  int32_t npairs;
  int32_t t0, t1;
};

struct PairDesc {
  int64_t b_row;        // table row of the neighbour's descriptor 0
  int64_t rowres_off;   // uint2 offset: [nseg][n1]
  int64_t colpart_off;  // uint2 offset: [nrb][n2pad]
  int64_t m21_off;      // int32 offset: [n2]
  int64_t match_off;    // uint2 offset: [n1]
  int64_t a_row;        // table row of the pivot's descriptor 0 (finalize recompute)
  int64_t aux_off;      // uint2 offset: [n1] row (best, second lower bound) (v2 finalize)
  int64_t rlist_off;    // int32 offset: [33 + n1] row-recheck buckets (v2 finalize)
  int32_t n1, n2, n2pad, nseg, nrb;
  int32_t clamp;        // 1: the pivot run took the CLAMP matcher variant
  int32_t seg8_log2;    // i8 kernel: 64-column tiles per row segment, log2 (7: 8192 columns)
  int32_t pad_;
};

hipError_t launch_match_tiles(const uint16_t* desc, const MatchJob* jobs, int njobs,
                              const PairDesc* pairs, uint2* rowres, uint2* colpart,
                              bool clamp, hipStream_t stream);
// Version-2 i8 matcher (LDS-DMA staging, best-only column partials) and its
// finalize (exact recompute of the deciding column seconds).
hipError_t launch_match_g8(const uint8_t* desc8, const int32_t* csum, const MatchJob* jobs,
                           int njobs, const PairDesc* pairs, uint2* rowres, uint2* colpart,
                           bool clamp, hipStream_t stream);
hipError_t launch_match_finalize_g8(const PairDesc* pairs, int npairs, uint2* rowres,
                                    uint2* colpart, uint2* rowaux, int32_t* rlist,
                                    const uint8_t* desc8, const int32_t* csum,
                                    const float* lut, float max_ratio, float max_distance,
                                    int cross_check, uint2* matches, int32_t* counts,
                                    int max_groups, int max_cols, hipStream_t stream);
hipError_t launch_match_finalize(const PairDesc* pairs, int npairs, const uint2* rowres,
                                 const uint2* colpart, int32_t* m21, const float* lut,
                                 float max_ratio, float max_distance, int cross_check,
                                 int colvals, uint2* matches, int32_t* counts,
                                 hipStream_t stream);
hipError_t launch_u8_to_bf16(const uint8_t* in, uint16_t* out, int64_t n, hipStream_t stream);
hipError_t launch_u8_to_i8(const uint8_t* in, uint8_t* out, int32_t* csum, int64_t nrows,
                           hipStream_t stream);
// Copies `bytes` (a multiple of 16) from pinned host memory (its device
// address, hipHostGetDevicePointer) into device memory with a kernel on
// `stream`: a batch's descriptor tables, uploaded on the stream's own queue
// instead of the copy engine, where a copy waits behind every earlier copy of
// another stream that shares the engine (profiles/r06_ah).
hipError_t launch_stage_upload(const void* host_dev_src, void* dst, size_t bytes, hipStream_t stream);

}  // namespace scm
