// Test stub (see tests/scanner_stub/README.md): Scanner buffers.
#pragma once
#include <cstdlib>

#include "scanner/util/common.h"

namespace scanner {
inline u8* new_buffer(DeviceHandle device, size_t size) {
  (void)device;  // the stub only hands out host memory
  return static_cast<u8*>(std::malloc(size ? size : 1));
}
inline void delete_buffer(DeviceHandle device, u8* buffer) {
  (void)device;
  std::free(buffer);
}
inline void insert_element(Elements& col, u8* buffer, size_t size) {
  Element e;
  e.buffer = buffer;
  e.size = size;
  col.push_back(e);
}
// Output element of a non-batched kernel (io.cc insert_element(element, ...)).
inline void insert_element(Element& element, u8* buffer, size_t size) {
  element.buffer = buffer;
  element.size = size;
}
}  // namespace scanner
