// Sanitizer driver of the CPU oracle (TEST INFRASTRUCTURE ONLY; SURVEY.md §5
// "race detection / memory checking": the reference has none, the plan is an
// ASan + UBSan build of the CPU restatement).  Built by `make -C oracle asan`
// into build/oracle_asan with AddressSanitizer and UndefinedBehaviorSanitizer
// linked statically (no preloaded runtime needed), and run by
// tests/test_oracle_asan.py on a small seeded table.
//
// usage: oracle_asan IN OUT OVERLAP
//   IN : u64 num_rows, then per row three length-prefixed (u64) io.cc
//        elements: image id, keypoints, descriptors;
//   OUT: per output row two length-prefixed elements, pair_image_ids and
//        two_view_geometries (oracle_table_run over every row).
// usage: oracle_asan --sift WIDTH HEIGHT CHANNELS SEED
//   the SIFT extraction op (oracle_sift_extract) on a seeded pseudo-random
//   frame; prints the three element sizes.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../include/scm.h"

extern "C" {
void oracle_default_options(scm_matching_options* o);
int oracle_table_run(const scm_matching_options* o, int64_t num_rows, const scm_element* ids,
                     const scm_element* kps, const scm_element* descs, int64_t overlap,
                     int64_t row_begin, int64_t row_end, uint8_t** ids_out, size_t* ids_sizes,
                     uint8_t** tvg_out, size_t* tvg_sizes);
void oracle_free(uint8_t* p);
int oracle_sift_extract(const uint8_t* frame, int32_t width, int32_t height, int32_t channels,
                        uint64_t image_id, uint8_t** kp_out, size_t* kp_size, uint8_t** desc_out,
                        size_t* desc_size, uint8_t** cam_out, size_t* cam_size);
}

namespace {

bool read_u64(FILE* f, uint64_t* v) { return std::fread(v, 8, 1, f) == 1; }

bool read_blob(FILE* f, std::vector<uint8_t>* b) {
  uint64_t n = 0;
  if (!read_u64(f, &n) || n > (1ull << 32)) return false;
  b->resize(n);
  return n == 0 || std::fread(b->data(), 1, n, f) == n;
}

void write_blob(FILE* f, const uint8_t* p, uint64_t n) {
  std::fwrite(&n, 8, 1, f);
  if (n) std::fwrite(p, 1, n, f);
}

}  // namespace

int sift_main(int w, int h, int c, uint32_t seed) {
  std::vector<uint8_t> f((size_t)w * h * c);
  uint32_t x = seed * 2654435761u + 1u;
  for (size_t i = 0; i < f.size(); ++i) {  // smooth-ish texture: blobs plus noise
    x = x * 1664525u + 1013904223u;
    const size_t p = i / c;
    const int yy = (int)(p / w), xx = (int)(p % w);
    f[i] = (uint8_t)(((xx * 37 + yy * 61) % 97) * 2 + (x >> 28));
  }
  uint8_t *a = nullptr, *b = nullptr, *d = nullptr;
  size_t na = 0, nb = 0, nd = 0;
  const int rc = oracle_sift_extract(f.data(), w, h, c, 1, &a, &na, &b, &nb, &d, &nd);
  if (rc != 0) return 3;
  std::printf("%zu %zu %zu\n", na, nb, nd);
  oracle_free(a);
  oracle_free(b);
  oracle_free(d);
  return 0;
}

int main(int argc, char** argv) {
  if (argc == 6 && std::string(argv[1]) == "--sift")
    return sift_main(std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4]),
                     (uint32_t)std::atoi(argv[5]));
  if (argc != 4) {
    std::fprintf(stderr, "usage: %s IN OUT OVERLAP\n", argv[0]);
    return 2;
  }
  FILE* in = std::fopen(argv[1], "rb");
  if (!in) return 2;
  uint64_t n = 0;
  if (!read_u64(in, &n) || n == 0 || n > 100000) return 2;
  std::vector<std::vector<uint8_t>> blobs(3 * n);
  for (auto& b : blobs)
    if (!read_blob(in, &b)) return 2;
  std::fclose(in);
  std::vector<scm_element> ids(n), kps(n), descs(n);
  for (uint64_t i = 0; i < n; ++i) {
    ids[i] = {blobs[3 * i].data(), blobs[3 * i].size()};
    kps[i] = {blobs[3 * i + 1].data(), blobs[3 * i + 1].size()};
    descs[i] = {blobs[3 * i + 2].data(), blobs[3 * i + 2].size()};
  }
  scm_matching_options o;
  oracle_default_options(&o);
  std::vector<uint8_t*> a(n), b(n);
  std::vector<size_t> na(n), nb(n);
  const int rc = oracle_table_run(&o, (int64_t)n, ids.data(), kps.data(), descs.data(),
                                  std::atoll(argv[3]), 0, (int64_t)n, a.data(), na.data(),
                                  b.data(), nb.data());
  if (rc != SCM_OK) return 3;
  FILE* out = std::fopen(argv[2], "wb");
  if (!out) return 2;
  for (uint64_t i = 0; i < n; ++i) {
    write_blob(out, a[i], na[i]);
    write_blob(out, b[i], nb[i]);
    oracle_free(a[i]);
    oracle_free(b[i]);
  }
  std::fclose(out);
  return 0;
}
