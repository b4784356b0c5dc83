// Scanner op `SiftExtractionGPU`: the MI355X drop-in for the reference's
// `SiftExtraction` (reference integration/op_cpp/extraction_op.cc:22-130;
// SURVEY.md §8f rank 4, the producer of the `extraction` table).  Same inputs
// (image_ids, frame column frames), same three outputs (keypoints,
// descriptors, cameras) in the same io.cc byte layout, host (CPU_DEVICE)
// output buffers, one kernel instance per pipeline instance bound to
// config.devices[0].  All computation goes through scm_extract_frames
// (include/scm.h, libscm.so); this file only adapts Scanner's elements.
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "scanner/api/kernel.h"
#include "scanner/api/op.h"
#include "scanner/util/memory.h"
#include "scm.h"

namespace {

// The reference aborts the worker on failure (glog CHECK inside COLMAP).
void scm_check(int rc, const char* what) {
  if (rc != SCM_OK) {
    std::fprintf(stderr, "SiftExtractionGPU: %s failed (%d): %s\n", what, rc, scm_last_error());
    std::abort();
  }
}

}  // namespace

class SiftExtractionGPUKernel : public scanner::Kernel, public scanner::VideoKernel {
 public:
  explicit SiftExtractionGPUKernel(const scanner::KernelConfig& config) : scanner::Kernel(config) {
    scm_matching_options opts;  // the context also serves matching; extraction ignores them
    scm_default_options(&opts);
    const int device = config.devices.empty() ? 0 : config.devices[0].id;
    scm_check(scm_context_create(device, &opts, &ctx_), "scm_context_create");
  }

  ~SiftExtractionGPUKernel() override { scm_context_destroy(ctx_); }

  // Reference execute (extraction_op.cc:70-121): the image id (size_t,
  // read_single_from_element), the frame, then keypoints, descriptors and
  // the camera into the three output elements.
  void execute(const scanner::Elements& input_cols, scanner::Elements& output_cols) override {
    const scanner::Element& image_id_col = input_cols[0];
    const scanner::Element& frame_col = input_cols[1];
    uint64_t image_id = 0;
    std::memcpy(&image_id, image_id_col.buffer, sizeof(image_id));
    scanner::check_frame(scanner::CPU_DEVICE, frame_col);
    const scanner::Frame* frame = frame_col.as_const_frame();
    const scm_frame f{frame->data, frame->width(), frame->height(), frame->channels()};
    scm_blob out[3] = {{nullptr, 0}, {nullptr, 0}, {nullptr, 0}};
    scm_check(scm_extract_frames(ctx_, 1, &image_id, &f, &out[0], &out[1], &out[2]),
              "scm_extract_frames");
    for (int c = 0; c < 3; ++c) {
      scanner::u8* buf = scanner::new_buffer(scanner::CPU_DEVICE, out[c].size);
      std::memcpy(buf, out[c].data, out[c].size);
      scanner::insert_element(output_cols[c], buf, out[c].size);
      scm_blob_free(&out[c]);
    }
  }

 private:
  scm_context* ctx_ = nullptr;
};

// Same signature as REGISTER_OP(SiftExtraction) (extraction_op.cc:124-130).
REGISTER_OP(SiftExtractionGPU)
    .input("image_ids")
    .frame_input("frames")
    .output("keypoints")
    .output("descriptors")
    .output("cameras")
    .protobuf_name("siftExtractionArgs");

// Placement: a GPU kernel whose columns all stay in host memory -- the frame
// is read as host bytes (check_frame(CPU_DEVICE, ...) above) and uploaded by
// scm_extract_frames, the outputs are new_buffer(CPU_DEVICE) elements.
// Without these declarations Scanner's evaluator would hand execute() the
// frame in device memory and treat the outputs as device buffers.
REGISTER_KERNEL(SiftExtractionGPU, SiftExtractionGPUKernel)
    .device(scanner::DeviceType::GPU)
    .input_device("image_ids", scanner::DeviceType::CPU)
    .input_device("frames", scanner::DeviceType::CPU)
    .output_device("keypoints", scanner::DeviceType::CPU)
    .output_device("descriptors", scanner::DeviceType::CPU)
    .output_device("cameras", scanner::DeviceType::CPU)
    .num_devices(1);
