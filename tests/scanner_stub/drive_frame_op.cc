// Test driver (see tests/scanner_stub/README.md) for a non-batched frame op
// (scanner::Kernel, e.g. SiftExtractionGPU): instantiates the registered
// kernel by op name and calls execute() once per row, as a Scanner worker
// runs such an op over a table.
//   drive_frame_op OP DIR NROWS [DEVICE]
//     DIR/in_0_<r>: row r's image id element (size_t);
//     DIR/frame_<r>: row r's frame bytes, DIR/shape_<r>: "width height channels";
//     writes DIR/out_<c>_<r> for every output column.
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
    std::fprintf(stderr, "usage: %s OP DIR NROWS [DEVICE]\n", argv[0]);
    return 2;
  }
  const std::string op = argv[1], dir = argv[2];
  const int nrows = std::atoi(argv[3]);
  const int device = argc > 4 ? std::atoi(argv[4]) : 0;
  auto it = scanner::kernel_registry().find(op);
  if (it == scanner::kernel_registry().end() || !it->second.make_plain) {
    std::fprintf(stderr, "op %s not registered as a plain kernel\n", op.c_str());
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
  scanner::Kernel* kernel = it->second.make_plain(config);
  for (int r = 0; r < nrows; ++r) {
    std::vector<scanner::u8> id, frame;
    if (!read_file(dir + "/in_0_" + std::to_string(r), &id) ||
        !read_file(dir + "/frame_" + std::to_string(r), &frame)) {
      std::fprintf(stderr, "missing input of row %d\n", r);
      return 2;
    }
    scanner::Frame f;
    std::ifstream sh(dir + "/shape_" + std::to_string(r));
    sh >> f.w >> f.h >> f.c;
    f.data = frame.data();
    scanner::Elements in(info.inputs.size());
    for (size_t c = 0; c < info.inputs.size(); ++c) {
      if (info.frame_inputs[c]) {
        in[c].buffer = reinterpret_cast<scanner::u8*>(&f);
        in[c].size = frame.size();
        in[c].is_frame = true;
      } else {
        in[c].buffer = id.data();
        in[c].size = id.size();
      }
    }
    scanner::Elements out(info.outputs.size());
    kernel->execute(in, out);
    for (size_t c = 0; c < out.size(); ++c) {
      std::ofstream o(dir + "/out_" + std::to_string(c) + "_" + std::to_string(r), std::ios::binary);
      o.write(reinterpret_cast<const char*>(out[c].buffer), (std::streamsize)out[c].size);
      scanner::delete_buffer(scanner::CPU_DEVICE, out[c].buffer);
    }
  }
  delete kernel;
  return 0;
}
