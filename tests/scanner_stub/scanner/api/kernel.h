// Test stub (see tests/scanner_stub/README.md): Scanner kernel interfaces.
#pragma once
#include <cstdlib>
#include <vector>

#include "scanner/util/common.h"
#include "scanner/util/memory.h"

namespace scanner {
struct KernelConfig {
  std::vector<DeviceHandle> devices;
  std::vector<u8> args;  // serialised protobuf op arguments
};

class StenciledBatchedKernel {
 public:
  explicit StenciledBatchedKernel(const KernelConfig& config) : config_(config) {}
  virtual ~StenciledBatchedKernel() = default;
  virtual void execute(const StenciledBatchedElements& input_cols,
                       BatchedElements& output_cols) = 0;
  // Scanner calls reset() when an instance starts on a new run of rows.
  virtual void reset() {}

 protected:
  KernelConfig config_;
};

// Non-batched, non-stenciled kernel: one element per column per call.
class Kernel {
 public:
  explicit Kernel(const KernelConfig& config) : config_(config) {}
  virtual ~Kernel() = default;
  virtual void execute(const Elements& input_cols, Elements& output_cols) = 0;

 protected:
  KernelConfig config_;
};

class VideoKernel {};

// Frames handed to a CPU kernel live in host memory.
inline void check_frame(const DeviceHandle& device, const Element& e) {
  if (device.type != DeviceType::CPU || !e.is_frame) std::abort();
}
}  // namespace scanner
