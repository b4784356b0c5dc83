// Test driver (see tests/scanner_stub/README.md): instantiates a registered
// kernel by op name, as a Scanner worker would, and runs execute() on
// stencils read from files.
//   drive_op OP DIR K [DEVICE]: one stencil;
//     DIR/in_<c>_<s>: element s of input column c (c = 0 ids, 1 keypoints, 2 descriptors)
//     writes DIR/out_<c> for every output column.
//   drive_op OP DIR K DEVICE NROWS BATCH: a table of NROWS rows (DIR/in_<c>_<r>)
//     run as Scanner runs a stencil range(0, K) op with batch BATCH: output rows
//     0..NROWS-1 in consecutive execute() calls of up to BATCH stencils, the
//     stencil of row r being rows min(r + s, NROWS - 1); writes DIR/out_<c>_<r>.
//   DIR/args (optional): serialised op arguments
#include <cstdio>
#include <algorithm>
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
  // drive_op --placements OP: print the kernel's device and every column's
  // placement ("input <col> CPU|GPU", "output <col> CPU|GPU").
  if (argc == 3 && std::string(argv[1]) == "--placements") {
    auto k = scanner::kernel_registry().find(argv[2]);
    if (k == scanner::kernel_registry().end()) return 2;
    const scanner::OpInfo& op = scanner::op_registry()[argv[2]];
    auto name = [](scanner::DeviceType d) { return d == scanner::DeviceType::CPU ? "CPU" : "GPU"; };
    std::printf("kernel %s\n", name(k->second.device));
    for (const auto& c : op.inputs)
      std::printf("input %s %s\n", c.c_str(), name(scanner::input_placement(k->second, c)));
    for (const auto& c : op.outputs)
      std::printf("output %s %s\n", c.c_str(), name(scanner::output_placement(k->second, c)));
    return 0;
  }
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
  // Column placement: the inputs below are host buffers and the outputs are
  // freed as host buffers, which is what a Scanner worker does only for
  // CPU-placed columns (KernelBuilder::input_device / output_device).
  const std::string misplaced = scanner::first_non_cpu_column(info, it->second);
  if (!misplaced.empty()) {
    std::fprintf(stderr, "op %s: %s is not placed on the CPU device\n", op.c_str(),
                 misplaced.c_str());
    return 3;
  }
  scanner::KernelConfig config;
  config.devices.push_back({it->second.device, device});
  read_file(dir + "/args", &config.args);

  const int nrows = argc > 5 ? std::atoi(argv[5]) : 0;
  const int batch = argc > 6 ? std::max(1, std::atoi(argv[6])) : 1;
  const bool table = nrows > 0;
  const int nfiles = table ? nrows : k;
  std::vector<std::vector<std::vector<scanner::u8>>> store(info.inputs.size());
  for (size_t c = 0; c < info.inputs.size(); ++c) {
    store[c].resize(nfiles);
    for (int s = 0; s < nfiles; ++s)
      if (!read_file(dir + "/in_" + std::to_string(c) + "_" + std::to_string(s), &store[c][s])) {
        std::fprintf(stderr, "missing input %zu/%d\n", c, s);
        return 2;
      }
  }
  scanner::StenciledBatchedKernel* kernel = it->second.make(config);
  const int rows_out = table ? nrows : 1;
  for (int r0 = 0; r0 < rows_out; r0 += batch) {
    const int nb = table ? std::min(batch, rows_out - r0) : 1;
    scanner::StenciledBatchedElements in(info.inputs.size());
    for (size_t c = 0; c < info.inputs.size(); ++c) {
      in[c].resize(nb);
      for (int b = 0; b < nb; ++b)
        for (int s = 0; s < k; ++s) {
          const int row = table ? std::min(r0 + b + s, nrows - 1) : s;
          scanner::Element e;
          e.buffer = store[c][row].data();
          e.size = store[c][row].size();
          in[c][b].push_back(e);
        }
    }
    scanner::BatchedElements out(info.outputs.size());
    kernel->execute(in, out);
    for (size_t c = 0; c < out.size(); ++c) {
      if (out[c].size() != (size_t)nb) {
        std::fprintf(stderr, "column %zu: %zu elements for %d stencils\n", c, out[c].size(), nb);
        return 1;
      }
      for (int b = 0; b < nb; ++b) {
        const std::string name = table ? "/out_" + std::to_string(c) + "_" + std::to_string(r0 + b)
                                       : "/out_" + std::to_string(c);
        std::ofstream f(dir + name, std::ios::binary);
        f.write(reinterpret_cast<const char*>(out[c][b].buffer), (std::streamsize)out[c][b].size);
        scanner::delete_buffer(scanner::CPU_DEVICE, out[c][b].buffer);
      }
    }
  }
  delete kernel;
  return 0;
}
