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
};
}  // namespace scanner

#define SCANNER_STUB_CAT2(a, b) a##b
#define SCANNER_STUB_CAT(a, b) SCANNER_STUB_CAT2(a, b)
#define REGISTER_OP(name) \
  static ::scanner::OpBuilder SCANNER_STUB_CAT(op_builder_, __LINE__) = ::scanner::OpBuilder(#name)
#define REGISTER_KERNEL(name, kernel)                                           \
  static ::scanner::KernelBuilder SCANNER_STUB_CAT(kernel_builder_, __LINE__) = \
      ::scanner::KernelBuilder::of<kernel>(#name)
