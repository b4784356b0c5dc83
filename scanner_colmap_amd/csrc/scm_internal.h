// Internal declarations shared by the host runtime translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/scm.h"
#include "match_kernels.h"

namespace scm {

void set_error(const std::string& msg);

#define SCM_HIP(call)                                                        \
  do {                                                                       \
    hipError_t e_ = (call);                                                  \
    if (e_ != hipSuccess) {                                                  \
      ::scm::set_error(std::string(#call) + ": " + hipGetErrorString(e_));   \
      return SCM_E_DEVICE;                                                   \
    }                                                                        \
  } while (0)

#define SCM_TRY(call)        \
  do {                       \
    int rc_ = (call);        \
    if (rc_ != SCM_OK) return rc_; \
  } while (0)

// Grow-only device buffer (allocation happens outside the launch sequence).
struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  int ensure(size_t need) {
    if (need <= bytes) return SCM_OK;
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
    size_t want = need + need / 4 + 4096;
    if (hipMalloc(&ptr, want) != hipSuccess) {
      set_error("hipMalloc of " + std::to_string(want) + " bytes failed");
      return SCM_E_NOMEM;
    }
    bytes = want;
    return SCM_OK;
  }
  template <typename T> T* as() const { return reinterpret_cast<T*>(ptr); }
  void release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
  }
};

// Pinned host staging buffer.
struct HostBuf {
  void* ptr = nullptr;
  void* dptr = nullptr;  // its device address (kernels read it: launch_stage_upload)
  size_t bytes = 0;
  int ensure(size_t need) {
    if (need <= bytes) return SCM_OK;
    if (ptr) (void)hipHostFree(ptr);
    ptr = nullptr;
    bytes = 0;
    size_t want = need + need / 4 + 4096;
    if (hipHostMalloc(&ptr, want, hipHostMallocDefault) != hipSuccess) {
      set_error("hipHostMalloc failed");
      return SCM_E_NOMEM;
    }
    if (hipHostGetDevicePointer(&dptr, ptr, 0) != hipSuccess) {
      (void)hipHostFree(ptr);
      ptr = dptr = nullptr;
      set_error("hipHostGetDevicePointer failed");
      return SCM_E_DEVICE;
    }
    bytes = want;
    return SCM_OK;
  }
  template <typename T> T* as() const { return reinterpret_cast<T*>(ptr); }
  void release() {
    if (ptr) (void)hipHostFree(ptr);
    ptr = dptr = nullptr;
    bytes = 0;
  }
};

struct Match {
  uint32_t idx1, idx2;
};

// Decoded view of one table row (borrowed pointers into Scanner elements).
struct RowView {
  uint32_t id = 0;
  const float* kp = nullptr;  // FeatureKeypoint rows, 6 floats
  int64_t nkp = 0;
  const uint8_t* desc = nullptr;
  int64_t ndesc = 0;
};

int decode_row(const scm_element& id, const scm_element& kp, const scm_element& desc,
               RowView* out);

// One TwoViewGeometry as the op emits it (F, H row-major in memory).
struct Tvg {
  int32_t config = SCM_TVG_UNDEFINED;
  double F[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  double tri_angle = 0.0;
  std::vector<Match> inlier_matches;
};

void append_tvg(std::vector<uint8_t>* out, const Tvg& t);
int make_blob(const std::vector<uint8_t>& bytes, scm_blob* out);
// Large-output buffer recycling (scm_codec.cpp): take a parked block (its
// usable size in *cap) or nullptr; give parks a block of >= 16 MiB.
void* pool_take(size_t* cap);
bool pool_give(void* p);
std::vector<uint8_t> tvg_list_bytes(const std::vector<Tvg>& list);
std::vector<uint8_t> id_list_bytes(const std::vector<uint32_t>& ids);

// GPU SIFT extraction (scm_sift.cpp): per-context state, created on first use.
// streams: kSiftSlotStreams streams the slots borrow (nullptr: their own).
constexpr int kSiftSlotStreams = 4;
struct SiftState;
void sift_state_destroy(SiftState* s);
int sift_extract_frames(SiftState** state, int device, const hipStream_t* streams, int64_t n,
                        const uint64_t* ids, const scm_frame* frames, scm_blob* kp_out,
                        scm_blob* desc_out, scm_blob* cam_out);

}  // namespace scm
