// Test driver (see tests/scanner_stub/README.md): instantiates a registered
// kernel by op name, as a Scanner worker would, and runs execute() on one
// stencil read from files:  drive_op OP DIR K [DEVICE]
//   DIR/args (optional): serialised op arguments
//   DIR/in_<c>_<s>: element s of input column c (c = 0 ids, 1 keypoints, 2 descriptors)
//   writes DIR/out_<c> for every output column.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "scanner/api/kernel.h"
#include "scanner/api/op.h"

static bool read_file(const std::string& path, std::vector<scanner::u8>* out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  out->assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  return true;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s OP DIR K [DEVICE]\n", argv[0]);
    return 2;
  }
  const std::string op = argv[1], dir = argv[2];
  const int k = std::atoi(argv[3]);
  const int device = argc > 4 ? std::atoi(argv[4]) : 0;
  auto it = scanner::kernel_registry().find(op);
  if (it == scanner::kernel_registry().end()) {
    std::fprintf(stderr, "op %s not registered\n", op.c_str());
    return 2;
  }
  const scanner::OpInfo& info = scanner::op_registry()[op];
  scanner::KernelConfig config;
  config.devices.push_back({it->second.device, device});
  read_file(dir + "/args", &config.args);

  std::vector<std::vector<std::vector<scanner::u8>>> store(info.inputs.size());
  scanner::StenciledBatchedElements in(info.inputs.size());
  for (size_t c = 0; c < info.inputs.size(); ++c) {
    store[c].resize(k);
    in[c].resize(1);
    for (int s = 0; s < k; ++s) {
      if (!read_file(dir + "/in_" + std::to_string(c) + "_" + std::to_string(s), &store[c][s])) {
        std::fprintf(stderr, "missing input %zu/%d\n", c, s);
        return 2;
      }
      scanner::Element e;
      e.buffer = store[c][s].data();
      e.size = store[c][s].size();
      in[c][0].push_back(e);
    }
  }
  scanner::BatchedElements out(info.outputs.size());
  scanner::StenciledBatchedKernel* kernel = it->second.make(config);
  kernel->execute(in, out);
  for (size_t c = 0; c < out.size(); ++c) {
    if (out[c].size() != 1) {
      std::fprintf(stderr, "column %zu: %zu elements\n", c, out[c].size());
      return 1;
    }
    std::ofstream f(dir + "/out_" + std::to_string(c), std::ios::binary);
    f.write(reinterpret_cast<const char*>(out[c][0].buffer), (std::streamsize)out[c][0].size);
    scanner::delete_buffer(scanner::CPU_DEVICE, out[c][0].buffer);
  }
  delete kernel;
  return 0;
}
