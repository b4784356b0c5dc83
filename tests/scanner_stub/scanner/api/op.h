// Test stub (see tests/scanner_stub/README.md): op / kernel registration.
// REGISTER_KERNEL records a factory so a test driver can instantiate the
// kernel by op name, as a Scanner worker would.
#pragma once
#include <functional>
#include <map>
#include <string>
#include <type_traits>
#include <vector>

#include "scanner/api/kernel.h"

namespace scanner {
struct OpInfo {
  std::string name;
  bool stencil = false;
  std::vector<std::string> inputs, outputs;
  std::vector<bool> frame_inputs;  // per input: a frame column
  std::string protobuf_name;
};

struct KernelInfo {
  DeviceType device = DeviceType::CPU;
  bool batch = false;
  int num_devices = 1;
  // Column placement (Scanner KernelBuilder::input_device / output_device):
  // a column listed here lives on that device whatever the kernel's own
  // device is; an unlisted column lives on the kernel's device.  Scanner's
  // evaluator copies an input column to that device before execute() and
  // treats an output column's buffers as allocated there.
  std::map<std::string, DeviceType> input_devices, output_devices;
  std::function<StenciledBatchedKernel*(const KernelConfig&)> make;  // stenciled / batched kernels
  std::function<Kernel*(const KernelConfig&)> make_plain;            // scanner::Kernel
};

inline std::map<std::string, OpInfo>& op_registry() {
  static std::map<std::string, OpInfo> r;
  return r;
}
inline std::map<std::string, KernelInfo>& kernel_registry() {
  static std::map<std::string, KernelInfo> r;
  return r;
}

struct OpBuilder {
  OpInfo* info;
  explicit OpBuilder(const std::string& name) : info(&op_registry()[name]) { info->name = name; }
  OpBuilder& stencil() { info->stencil = true; return *this; }
  OpBuilder& input(const std::string& c) {
    info->inputs.push_back(c);
    info->frame_inputs.push_back(false);
    return *this;
  }
  OpBuilder& frame_input(const std::string& c) {
    info->inputs.push_back(c);
    info->frame_inputs.push_back(true);
    return *this;
  }
  OpBuilder& output(const std::string& c) { info->outputs.push_back(c); return *this; }
  OpBuilder& protobuf_name(const std::string& n) { info->protobuf_name = n; return *this; }
};

struct KernelBuilder {
  KernelInfo* info;
  explicit KernelBuilder(const std::string& name) : info(&kernel_registry()[name]) {}
  template <typename K>
  static KernelBuilder of(const std::string& name) {
    KernelBuilder b(name);
    if constexpr (std::is_base_of<StenciledBatchedKernel, K>::value)
      b.info->make = [](const KernelConfig& c) -> StenciledBatchedKernel* { return new K(c); };
    else
      b.info->make_plain = [](const KernelConfig& c) -> Kernel* { return new K(c); };
    return b;
  }
  KernelBuilder& device(DeviceType d) { info->device = d; return *this; }
  KernelBuilder& batch() { info->batch = true; return *this; }
  KernelBuilder& num_devices(int n) { info->num_devices = n; return *this; }
  KernelBuilder& input_device(const std::string& col, DeviceType d) {
    info->input_devices[col] = d;
    return *this;
  }
  KernelBuilder& output_device(const std::string& col, DeviceType d) {
    info->output_devices[col] = d;
    return *this;
  }
};

// Where a Scanner worker places a kernel's column: the declared device, else
// the kernel's own device.
inline DeviceType input_placement(const KernelInfo& k, const std::string& col) {
  auto it = k.input_devices.find(col);
  return it == k.input_devices.end() ? k.device : it->second;
}
inline DeviceType output_placement(const KernelInfo& k, const std::string& col) {
  auto it = k.output_devices.find(col);
  return it == k.output_devices.end() ? k.device : it->second;
}

// The drivers hand every column over in host memory and free every output
// with delete_buffer(CPU_DEVICE, ...), so -- as under a real Scanner worker,
// which would move a GPU-placed column to device memory -- a kernel whose
// columns are not all CPU-placed cannot run here.  Returns the first such
// column ("" when every column is on the CPU).
inline std::string first_non_cpu_column(const OpInfo& op, const KernelInfo& k) {
  for (const auto& c : op.inputs)
    if (input_placement(k, c) != DeviceType::CPU) return "input " + c;
  for (const auto& c : op.outputs)
    if (output_placement(k, c) != DeviceType::CPU) return "output " + c;
  return "";
}
}  // namespace scanner

#define SCANNER_STUB_CAT2(a, b) a##b
#define SCANNER_STUB_CAT(a, b) SCANNER_STUB_CAT2(a, b)
#define REGISTER_OP(name) \
  static ::scanner::OpBuilder SCANNER_STUB_CAT(op_builder_, __LINE__) = ::scanner::OpBuilder(#name)
#define REGISTER_KERNEL(name, kernel)                                           \
  static ::scanner::KernelBuilder SCANNER_STUB_CAT(kernel_builder_, __LINE__) = \
      ::scanner::KernelBuilder::of<kernel>(#name)
