// Stress driver of the runtime's host worker pool (scanner_colmap_amd/csrc/
// scm_pool.h), built and run by tests/test_worker_pool.py under
// ThreadSanitizer: run() and launch()/wait() jobs of varying sizes back to
// back (a job's last task ends it while late workers may still be waking, and
// the next job reuses the other slot), every task's effect checked, and the
// destructor with workers still asleep.  usage: pool_stress ITERATIONS
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "scm_pool.h"

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  {
    scm::WorkerPool p, q;
    p.start(7);
    q.start(3);
    std::vector<int64_t> out(64);
    for (int it = 0; it < iters; ++it) {
      const int n = 1 + (it * 7) % 37;
      for (int i = 0; i < n; ++i) out[i] = -1;
      p.run(n, [&](int64_t i) { out[i] = i * it; });
      for (int i = 0; i < n; ++i)
        if (out[i] != (int64_t)i * it) {
          std::printf("run %d: task %d not done\n", it, i);
          return 1;
        }
      std::atomic<int64_t> sum{0};
      q.launch(n, [&](int64_t i) { sum += i + 1; });
      q.wait();
      if (sum != (int64_t)n * (n + 1) / 2) {
        std::printf("launch %d: sum %lld\n", it, (long long)sum.load());
        return 1;
      }
      if (it % 5 == 0) p.run(0, [](int64_t) {});  // empty jobs
    }
  }
  scm::WorkerPool idle;  // destroyed with its workers asleep, no job ever run
  idle.start(4);
  std::printf("ok\n");
  return 0;
}
