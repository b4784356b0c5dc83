/*
 * scm.h — C ABI of the MI355X-native sequential SIFT feature-matching stage.
 *
 * Drop-in boundary for the reference's Scanner op
 *   REGISTER_OP(SequentialMatchingCPU) / SequentialMatchingCPUKernel
 *   (reference integration/op_cpp/sequential_matching.cc:27-205)
 * loaded by integration/feature_matching.py:39-54.
 *
 * All buffers crossing this boundary are host memory laid out exactly as the
 * reference's io.cc codecs write them (integration/op_cpp/io.cc), so a Scanner
 * kernel (see scanner_colmap_amd/scanner_op/) or any FFI (ctypes, see
 * scanner_colmap_amd/_abi.py) can call it with the bytes Scanner hands over.
 * Plain C types only: no torch / HIP types in the signatures.
 *
 * Error convention: every int-returning entry point returns SCM_OK (0) on
 * success and a negative SCM_E_* code otherwise; scm_last_error() returns a
 * thread-local message.  The reference aborts the worker through glog CHECK
 * (no return codes); the Scanner-side op maps a non-zero status to the same
 * fatal abort (scanner_colmap_amd/scanner_op/sequential_matching_gpu.cc).
 *
 * Threading (reference: one kernel instance per Scanner pipeline instance,
 * execute() serial per instance, sequential_matching.cc:103): an scm_context
 * is NOT re-entrant; distinct contexts may be used from distinct threads.
 */
#ifndef SCM_H_
#define SCM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SCM_ABI_VERSION 6

enum {
  SCM_OK = 0,
  SCM_E_INVALID = -1,   /* malformed argument / element bytes            */
  SCM_E_DEVICE = -2,    /* HIP runtime error, or no gfx950 device        */
  SCM_E_NOMEM = -3,     /* host or device allocation failed              */
  SCM_E_CAPACITY = -4,  /* caller buffer too small (size written back)   */
  SCM_E_STATE = -5      /* call order (e.g. table_run before table_load) */
};

/* colmap::TwoViewGeometry::ConfigurationType [upstream
 * estimators/two_view_geometry.h], SURVEY.md §8a a18. */
enum {
  SCM_TVG_UNDEFINED = 0,
  SCM_TVG_DEGENERATE = 1,
  SCM_TVG_CALIBRATED = 2,
  SCM_TVG_UNCALIBRATED = 3,
  SCM_TVG_PLANAR = 4,
  SCM_TVG_PANORAMIC = 5,
  SCM_TVG_PLANAR_OR_PANORAMIC = 6,
  SCM_TVG_WATERMARK = 7,
  SCM_TVG_MULTIPLE = 8
};

/* Options.  Fields 1-14 mirror siftFeatureMatchingArgs (reference
 * integration/op_cpp/colmap.proto:6-49), overlap/loop fields mirror
 * SequentialMatchingArgs (colmap.proto:55-65), and the remaining fields are
 * the colmap::TwoViewGeometry::Options / RANSACOptions defaults that
 * sequential_matching.cc:64-75 leaves untouched.  scm_default_options() fills
 * the proto2 defaults — the values the reference runs with, because
 * feature_matching.py:50-54 passes no op args. */
typedef struct scm_matching_options {
  int32_t use_gpu;                   /* colmap.proto:7   default 0      */
  int32_t gpu_index;                 /* colmap.proto:11  default "-1"   */
  double max_ratio;                  /* colmap.proto:14  default 0.8    */
  double max_distance;               /* colmap.proto:17  default 0.7    */
  int32_t cross_check;               /* colmap.proto:20  default 1      */
  int32_t max_num_matches;           /* colmap.proto:23  default 32768  */
  float max_error;                   /* colmap.proto:26  default 4.0    */
  double confidence;                 /* colmap.proto:29  default 0.999  */
  int32_t min_num_trials;            /* colmap.proto:33  default 30     */
  int32_t max_num_trials;            /* colmap.proto:34  default 10000  */
  double min_inlier_ratio;           /* colmap.proto:38  default 0.25   */
  int32_t min_num_inliers;           /* colmap.proto:42  default 15     */
  int32_t multiple_models;           /* colmap.proto:45  default 0      */
  int32_t guided_matching;           /* colmap.proto:48  default 0      */
  int32_t loop_detection;            /* colmap.proto:57  default 0      */
  int32_t overlap;                   /* colmap.proto:59  default 10     */
  int32_t quadratic_overlap;         /* colmap.proto:62  default 0      */
  double min_E_F_inlier_ratio;       /* COLMAP default 0.95             */
  double max_H_inlier_ratio;         /* COLMAP default 0.8              */
  double watermark_min_inlier_ratio; /* COLMAP default 0.7              */
  double watermark_border_size;      /* COLMAP default 0.1              */
  int32_t detect_watermark;          /* COLMAP default 1                */
  double dyn_num_trials_multiplier;  /* COLMAP RANSACOptions default 3  */
  /* The reference's RANSAC PRNG is thread-local and time-seeded (COLMAP
   * SetPRNGSeed is never called), so its geometry output is not reproducible.
   * Here every pair draws from a fresh std::mt19937 seeded with
   * scm_pair_seed(ransac_seed, image_id1, image_id2). */
  uint32_t ransac_seed;              /* default 0                       */
} scm_matching_options;

/* One Scanner element: a borrowed, read-only byte range (scanner::Element,
 * reference io.cc:67-68). */
typedef struct scm_element {
  const uint8_t* buffer;
  size_t size;
} scm_element;

/* An output element produced by the library (scanner::new_buffer +
 * insert_element, io.cc:157/272/86).  Release with scm_blob_free. */
typedef struct scm_blob {
  uint8_t* data;
  size_t size;
} scm_blob;

typedef struct scm_context scm_context;

/* ---- options / utilities -------------------------------------------- */
int32_t scm_abi_version(void);
const char* scm_last_error(void);
void scm_default_options(scm_matching_options* opts);
/* Decode a serialised SequentialMatchingArgs (proto2 wire format) into opts,
 * starting from the defaults — replaces SequentialMatchingArgs::ParseFromArray
 * + parseConfigs (sequential_matching.cc:36-76). */
int scm_parse_args(const uint8_t* bytes, size_t size, scm_matching_options* opts);
uint32_t scm_pair_seed(uint32_t base_seed, uint32_t image_id1, uint32_t image_id2);
void scm_blob_free(scm_blob* blob);

/* ---- kernel instance (SequentialMatchingCPUKernel ctor, :30-33) ------- */
/* Binds one HIP device (Scanner KernelConfig.devices[0]); owns one stream
 * and its HBM workspace.  Fails with SCM_E_DEVICE if no gfx950 device. */
int scm_context_create(int32_t device_index, const scm_matching_options* opts,
                       scm_context** out);
void scm_context_destroy(scm_context* ctx);

/* ---- hot path, pair granularity -------------------------------------- */
/* colmap::MatchSiftFeaturesCPU replacement (sequential_matching.cc:154-155):
 * u8 descriptors, row-major N x 128.  Writes the cross-checked matches as
 * (idx1, idx2) uint32 pairs sorted by idx1 into matches[0 .. 2*cap).  On
 * SCM_E_CAPACITY *num_matches holds the required count. */
int scm_match_pair(scm_context* ctx, const uint8_t* desc1, int64_t n1,
                   const uint8_t* desc2, int64_t n2, uint32_t* matches,
                   int64_t cap, int64_t* num_matches);

/* verifyTwoViewGeometry + post-filter replacement (sequential_matching.cc:
 * 84-101, 164-178): keypoints are FeatureKeypoint rows {x,y,a11,a12,a21,a22}
 * (float32, 24 B).  Writes one TwoViewGeometry in the io.cc per-TVG byte
 * layout (io.cc:279-292) to *tvg_out. */
int scm_verify_pair(scm_context* ctx, const float* kp1, int64_t n1,
                    const float* kp2, int64_t n2, const uint32_t* matches,
                    int64_t num_matches, uint32_t image_id1, uint32_t image_id2,
                    scm_blob* tvg_out);

/* ---- hot path, op granularity ---------------------------------------- */
/* SequentialMatchingCPUKernel::execute replacement (:103-185) for ONE output
 * row: stencil_size elements of each input column (image_ids: size_t id,
 * io.cc:67; keypoints: io.cc:115-147 vector blob; descriptors: io.cc:180-194
 * matrix blob).  Produces the two output elements pair_image_ids
 * (io.cc:151-176) and two_view_geometries (io.cc:256-297). */
int scm_execute_stencil(scm_context* ctx, int64_t stencil_size,
                        const scm_element* image_ids,
                        const scm_element* keypoints,
                        const scm_element* descriptors,
                        scm_blob* pair_image_ids_out, scm_blob* tvgs_out);

/* The same for a Scanner batch of `batch` stencils (a `.batch()` kernel's
 * StenciledBatchedElements, sequential_matching.cc:189-191 registers the
 * kernel with .batch()): element (b, s) of each column at index
 * b * stencil_size + s; writes `batch` output elements to each of
 * pair_image_ids_out[] / tvgs_out[] (caller arrays).  Every output row is
 * byte-identical to scm_execute_stencil on that stencil alone.  The
 * reference's execute() reads only batch element 0 (:106-108) and emits one
 * row; this entry point handles every element.  Images stay resident in HBM
 * from one call to the next, so consecutive stencils upload only their new
 * images, and all pairs of the call run through the pipelined batch path.
 * Images are identified by content (id, feature counts and 64-bit hashes of
 * the keypoint and descriptor bytes), never by id alone: PrepareImage ids
 * are per-instance counters (prepare_image.cc:11-20), so one id may name two
 * images, and every element is matched with its own bytes as the reference
 * decodes them (sequential_matching.cc:115-122).  Element buffers the
 * previous call also handed over (same addresses and sizes) take that call's
 * content keys at once (when a sample of their words is unchanged) and are
 * re-hashed while the GPU runs; if a buffer was rewritten in place the run is
 * discarded and the call runs again with every key hashed first, so the
 * outputs always follow the bytes. */
int scm_execute_batch(scm_context* ctx, int64_t batch, int64_t stencil_size,
                      const scm_element* image_ids,
                      const scm_element* keypoints,
                      const scm_element* descriptors,
                      scm_blob* pair_image_ids_out, scm_blob* tvgs_out);
/* Images the execute() cache reused / uploaded so far (cumulative). */
int scm_stencil_stats(scm_context* ctx, int64_t* reused, int64_t* uploaded);
/* Content-key speculation of scm_execute_batch so far (cumulative): elements
 * whose buffers took the previous call's key while the GPU ran; elements whose
 * buffers the previous call also handed over but whose sampled words changed
 * (a recycled buffer holding another image: hashed before the run instead);
 * calls whose speculated key did not hold (buffer rewritten in place with
 * its sampled words unchanged) and ran again -- the image cache is kept, so
 * the rerun uploads only the changed images.  Diagnostics (bench, tests). */
int scm_stencil_spec_stats(scm_context* ctx, int64_t* speculated, int64_t* rejected,
                           int64_t* retried);
/* Drops the execute() image cache (Scanner Kernel::reset(), called when a
 * kernel instance starts on a new stream of rows): the next call uploads
 * every image it needs.  Never needed for correctness -- the cache is keyed
 * by image content -- it returns the cache's HBM. */
int scm_stencil_cache_clear(scm_context* ctx);

/* ---- table granularity (HBM-resident batch path) ---------------------- */
/* Decode and upload num_rows rows of the `extraction` table (columns
 * image_id / keypoints / descriptors, feature_matching.py:61-68) into HBM. */
int scm_table_load(scm_context* ctx, int64_t num_rows,
                   const scm_element* image_ids, const scm_element* keypoints,
                   const scm_element* descriptors);
/* Run the stencil range(0, overlap) (feature_matching.py:43) for output rows
 * [row_begin, row_end) of the loaded table; writes (row_end - row_begin)
 * pair_image_ids and two_view_geometries elements.  Row i is paired with rows
 * i+1 .. min(i+overlap-1, num_rows-1). */
int scm_table_run(scm_context* ctx, int64_t overlap, int64_t row_begin,
                  int64_t row_end, scm_blob* pair_image_ids_out,
                  scm_blob* tvgs_out);
/* Same run, one packed output: rows_out receives a single buffer holding, for
 * each output row r in order, the pair_image_ids element followed by the
 * two_view_geometries element; row_offsets (2 * (row_end - row_begin) + 1
 * entries, caller-allocated) receives the byte offset of each element and the
 * total size last: element 2r spans [row_offsets[2r], row_offsets[2r+1]),
 * element 2r+1 spans [row_offsets[2r+1], row_offsets[2r+2]).  Saves one
 * allocation per element on the serving path (the bytes are identical). */
int scm_table_run_packed(scm_context* ctx, int64_t overlap, int64_t row_begin,
                         int64_t row_end, scm_blob* rows_out,
                         int64_t* row_offsets);
/* Streamed form of scm_table_run_packed: `passes` runs of the row range
 * [row_begin, row_end) as ONE batch stream, so the batches of pass k + 1 enter
 * the pipeline while the last batches of pass k are still being verified and
 * the GPU does not drain between passes (the serving shape: consecutive
 * tables, or a table re-run, back to back).  As soon as pass k's rows are
 * serialised, on_pass(user, k, rows, row_offsets) is called on the calling
 * thread, passes in order: `rows` (rows_size bytes) is a packed buffer the
 * callee owns (free it with scm_blob_free on {rows, rows_size}), `row_offsets` the 2 * (row_end - row_begin) + 1 element
 * offsets of scm_table_run_packed (valid during the call only).  Every pass's
 * bytes equal scm_table_run_packed's.  With scm_set_keep_matches the raw
 * matches of the last pass are kept.  scm_table_timings then reports the
 * whole streamed run. */
typedef void (*scm_pass_fn)(void* user, int64_t pass, uint8_t* rows, size_t rows_size,
                            const int64_t* row_offsets);
int scm_table_run_passes(scm_context* ctx, int64_t overlap, int64_t row_begin,
                         int64_t row_end, int64_t passes, scm_pass_fn on_pass, void* user);
/* Chunked form of scm_table_run_packed for the multi-GPU gather (SURVEY.md
 * §8e: the row gather overlaps the tail of the compute): the rows of
 * [row_begin, row_end) are handed over batch by batch, in row order, as soon
 * as each batch is serialised -- on_chunk(user, first_row, num_rows, rows,
 * rows_size, row_offsets) on the calling thread, with `rows` a packed buffer
 * of num_rows rows the callee owns (scm_blob_free on {rows, rows_size}) and
 * `row_offsets` its 2 * num_rows + 1 element offsets (valid during the call
 * only).  The chunks' rows, concatenated, equal scm_table_run_packed's bytes.
 * No chunk is handed over for an empty range. */
typedef void (*scm_chunk_fn)(void* user, int64_t first_row, int64_t num_rows, uint8_t* rows,
                             size_t rows_size, const int64_t* row_offsets);
int scm_table_run_chunks(scm_context* ctx, int64_t overlap, int64_t row_begin,
                         int64_t row_end, scm_chunk_fn on_chunk, void* user);
/* Keep (keep != 0) the raw cross-checked matches of every pair of the
 * following table runs for scm_table_matches; off by default. */
int scm_set_keep_matches(scm_context* ctx, int32_t keep);
/* Keep the raw matches only of the pairs whose pivot row lies in
 * [row_begin, row_end) (a bounded debug output for spot checks of long runs:
 * the bench keeps a few rows of its timed run for the parity check);
 * row_end == row_begin turns keeping off. */
int scm_set_keep_matches_range(scm_context* ctx, int64_t row_begin, int64_t row_end);
/* Also keep the pairs whose pivot row lies in [row_begin, row_end), beside the
 * ranges already kept (the bench's parity sample: the first rows and rows
 * past the first batch boundary and at the table's end). */
int scm_add_keep_matches_range(scm_context* ctx, int64_t row_begin, int64_t row_end);
/* Raw cross-checked matches of the most recent scm_table_run for the pair
 * (row, row + offset), offset in [1, overlap); the debug `matches` output the
 * bit-exact checks read.  Requires scm_set_keep_matches. */
int scm_table_matches(scm_context* ctx, int64_t row, int64_t offset,
                      uint32_t* matches, int64_t cap, int64_t* num_matches);

/* Per-stage device time of the most recent scm_table_run, milliseconds,
 * measured with HIP events on the context's stream:
 * t[0] = descriptor-distance + top-2 kernel, t[1] = match finalize,
 * t[2] = RANSAC hypothesis kernels, t[3] = whole run (wall),
 * t[4] = number of descriptor-distance kernel launches of the run,
 * t[5] = inlier-scoring kernels (F + H), t[6] / t[7] = F / H (model, point)
 * residual evaluations of the sequential LO-RANSAC up to its stop;
 * t[8] / t[9] = host time of the last scm_execute_batch: content keys of its
 * elements, then the image table (reuse + upload staging); t[10] = its
 * pipeline run (GPU stages and their host steps up to the serialised rows),
 * t[11] = building its output blobs; t[12..15] = the run's watermark
 * decisions of small batches taken from the speculative pass / recomputed
 * and equal / recomputed and different (both with SCM_DIAG_SPEC_CHECK=1) /
 * speculation void (H aborted in its last window) and recomputed.  n: the
 * entries the caller holds (at most 16 are written). */
int scm_table_timings(scm_context* ctx, double* t, int32_t n);
/* Measurement only: serial != 0 runs the following table runs with matching
 * and verification one after the other instead of overlapped (no stage
 * shares the GPU), so scm_table_timings reports isolated kernel times; the
 * output bytes are identical.  Off by default (SCM_SERIAL=1 sets the initial
 * value). */
int scm_set_serial(scm_context* ctx, int32_t serial);

/* ---- SIFT extraction (the producer of the
 * `extraction` table; replaces SiftExtractionKernel::execute,
 * integration/op_cpp/extraction_op.cc:70-121, REGISTER_OP(SiftExtraction)
 * :124-130: input image_id + frame, outputs keypoints, descriptors, cameras).
 * A frame is a Scanner Frame's buffer: height x width x channels bytes,
 * row-major, channels 1, 3 or 4; as the reference's raw-bits FreeImage
 * bitmap, channel 2 takes the red weight of the grey conversion. */
typedef struct scm_frame {
  const uint8_t* data;
  int32_t width;
  int32_t height;
  int32_t channels;
} scm_frame;
/* n frames -> per frame the keypoints element (write_vector_to_element),
 * the descriptors element (write_matrix_to_element, u8 128 per row) and the
 * camera element (write_camera_to_element, io.cc:307-335); each blob
 * library-allocated (scm_blob_free).  COLMAP's default
 * SiftExtractionOptions; a frame larger than max_image_size (3200) is
 * first reduced as resizeBitmap does (extraction_op.cc:28-39: grey, FreeImage
 * bilinear rescale by 3200 / max(w, h)).  Any frame of at least 1 x 1 runs,
 * as VLFeat's filter does (octaves too small for an interior pixel detect
 * nothing); a frame that overflows the workspace's keypoint capacities grows
 * them and runs again (the reference has no capacity limit).  SCM_E_INVALID:
 * a null argument, an empty frame or a channel count other than 1, 3, 4.
 * The frames run on the context's four streams, in stream order with its
 * other calls; on any error no output blob stays allocated. */
int scm_extract_frames(scm_context* ctx, int64_t n, const uint64_t* image_ids,
                       const scm_frame* frames, scm_blob* keypoints_out,
                       scm_blob* descriptors_out, scm_blob* cameras_out);

#ifdef __cplusplus
}
#endif

#endif /* SCM_H_ */
