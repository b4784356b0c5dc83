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

// A decoded video frame (height x width x channels bytes, row-major).
struct Frame {
  int32_t w = 0, h = 0, c = 0;
  u8* data = nullptr;
  int32_t width() const { return w; }
  int32_t height() const { return h; }
  int32_t channels() const { return c; }
};

struct Element {
  u8* buffer = nullptr;  // for a frame column: the Frame (as_const_frame)
  size_t size = 0;
  bool is_frame = false;
  const Frame* as_const_frame() const { return reinterpret_cast<const Frame*>(buffer); }
};

using Elements = std::vector<Element>;
using BatchedElements = std::vector<Elements>;                      // [column][batch]
using StenciledBatchedElements = std::vector<std::vector<Elements>>;  // [column][batch][stencil]
}  // namespace scanner
