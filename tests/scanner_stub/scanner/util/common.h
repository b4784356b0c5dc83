// Test stub (see tests/scanner_stub/README.md): Scanner common types.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace scanner {
using u8 = uint8_t;

enum class DeviceType { CPU, GPU };

struct DeviceHandle {
  DeviceType type;
  int32_t id;
};

inline const DeviceHandle CPU_DEVICE = {DeviceType::CPU, 0};

struct Element {
  u8* buffer = nullptr;
  size_t size = 0;
};

using Elements = std::vector<Element>;
using BatchedElements = std::vector<Elements>;                      // [column][batch]
using StenciledBatchedElements = std::vector<std::vector<Elements>>;  // [column][batch][stencil]
}  // namespace scanner
