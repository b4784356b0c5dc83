// Test stub (see tests/scanner_stub/README.md): Scanner kernel interfaces.
#pragma once
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

 protected:
  KernelConfig config_;
};

class VideoKernel {};
}  // namespace scanner
