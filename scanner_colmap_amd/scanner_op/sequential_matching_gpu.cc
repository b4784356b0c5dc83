// Scanner op `SequentialMatchingGPU`: the MI355X drop-in for the reference's
// `SequentialMatchingCPU` (reference integration/op_cpp/sequential_matching.cc:
// 27-205).  Same stencil inputs (image_ids, keypoints, descriptors), same two
// outputs (pair_image_ids, two_view_geometries) in the same io.cc byte layout,
// host (CPU_DEVICE) output buffers, one kernel instance per Scanner pipeline
// instance bound to config.devices[0].  All computation goes through the C ABI
// of include/scm.h (libscm.so); this file only adapts Scanner's element
// containers to it.  Build it next to the reference ops with Scanner's
// build_op and link libscm.so.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "scanner/api/kernel.h"
#include "scanner/api/op.h"
#include "scanner/util/memory.h"
#include "scm.h"

namespace {

// The reference aborts the worker on failure (glog CHECK inside COLMAP);
// a non-zero status from the library does the same here.
void scm_check(int rc, const char* what) {
  if (rc != SCM_OK) {
    std::fprintf(stderr, "SequentialMatchingGPU: %s failed (%d): %s\n", what, rc,
                 scm_last_error());
    std::abort();
  }
}

}  // namespace

class SequentialMatchingGPUKernel : public scanner::StenciledBatchedKernel,
                                    public scanner::VideoKernel {
 public:
  // Reference constructor + parseConfigs (sequential_matching.cc:30-76).
  explicit SequentialMatchingGPUKernel(const scanner::KernelConfig& config)
      : scanner::StenciledBatchedKernel(config) {
    scm_matching_options opts;
    scm_check(scm_parse_args(config.args.data(), config.args.size(), &opts), "scm_parse_args");
    const int device = config.devices.empty() ? 0 : config.devices[0].id;
    scm_check(scm_context_create(device, &opts, &ctx_), "scm_context_create");
  }

  ~SequentialMatchingGPUKernel() override { scm_context_destroy(ctx_); }

  // A new run of rows: drop the HBM image cache.  The cache is keyed by image
  // content, so this only returns its memory; outputs never depend on it.
  void reset() override { scm_check(scm_stencil_cache_clear(ctx_), "scm_stencil_cache_clear"); }

  // Reference execute (sequential_matching.cc:103-185): column c, batch
  // element b, stencil offset s -> input_cols[c][b][s].  The reference reads
  // only b = 0 and emits one row (:106-108); every element of the batch is
  // matched here (one scm_execute_batch call, one output row per element),
  // so `batch=` on the op call amortises the GPU pipeline over many rows.
  void execute(const scanner::StenciledBatchedElements& input_cols,
               scanner::BatchedElements& output_cols) override {
    const size_t nb = input_cols[0].size();
    if (nb == 0) return;
    const size_t k = input_cols[0][0].size();
    std::vector<scm_element> e_ids(nb * k), e_kps(nb * k), e_descs(nb * k);
    for (size_t b = 0; b < nb; ++b) {
      const auto& ids = input_cols[0][b];
      const auto& kps = input_cols[1][b];
      const auto& descs = input_cols[2][b];
      if (ids.size() != k || kps.size() != k || descs.size() != k) {
        std::fprintf(stderr, "SequentialMatchingGPU: ragged stencils in one batch\n");
        std::abort();
      }
      for (size_t s = 0; s < k; ++s) {
        e_ids[b * k + s] = {ids[s].buffer, ids[s].size};
        e_kps[b * k + s] = {kps[s].buffer, kps[s].size};
        e_descs[b * k + s] = {descs[s].buffer, descs[s].size};
      }
    }
    std::vector<scm_blob> pair_ids(nb, scm_blob{nullptr, 0}), tvgs(nb, scm_blob{nullptr, 0});
    scm_check(scm_execute_batch(ctx_, (int64_t)nb, (int64_t)k, e_ids.data(), e_kps.data(),
                                e_descs.data(), pair_ids.data(), tvgs.data()),
              "scm_execute_batch");
    for (size_t b = 0; b < nb; ++b) {
      emit(output_cols[0], &pair_ids[b]);
      emit(output_cols[1], &tvgs[b]);
    }
  }

 private:
  // io.cc:157-176: the element is a scanner::new_buffer on the CPU device,
  // owned by Scanner after insert_element.
  static void emit(scanner::Elements& col, scm_blob* blob) {
    scanner::u8* buf = scanner::new_buffer(scanner::CPU_DEVICE, blob->size);
    std::memcpy(buf, blob->data, blob->size);
    scanner::insert_element(col, buf, blob->size);
    scm_blob_free(blob);
  }

  scm_context* ctx_ = nullptr;
};

// Same signature as REGISTER_OP(SequentialMatchingCPU) (sequential_matching.cc:
// 193-200).  The reference names a protobuf message that colmap.proto does not
// define ("featureMatchingArgs"); the kernel parses SequentialMatchingArgs,
// which is what is registered here.
REGISTER_OP(SequentialMatchingGPU)
    .stencil()
    .input("image_ids")
    .input("keypoints")
    .input("descriptors")
    .output("pair_image_ids")
    .output("two_view_geometries")
    .protobuf_name("SequentialMatchingArgs");

// Placement: the kernel holds a GPU (config.devices[0] is the GPU Scanner
// assigned to this pipeline instance), but every column stays in host
// memory -- execute() hands the element bytes to scm_execute_batch, which
// stages them into its own HBM image cache, and the outputs are
// new_buffer(CPU_DEVICE) elements.  Without these declarations Scanner's
// evaluator would move the inputs to the GPU before execute() and treat the
// outputs as device buffers.
REGISTER_KERNEL(SequentialMatchingGPU, SequentialMatchingGPUKernel)
    .device(scanner::DeviceType::GPU)
    .input_device("image_ids", scanner::DeviceType::CPU)
    .input_device("keypoints", scanner::DeviceType::CPU)
    .input_device("descriptors", scanner::DeviceType::CPU)
    .output_device("pair_image_ids", scanner::DeviceType::CPU)
    .output_device("two_view_geometries", scanner::DeviceType::CPU)
    .batch()
    .num_devices(1);
