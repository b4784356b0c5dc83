// Host worker pool of the runtime (scm_runtime.cpp): content hashing and
// upload staging of the drop-in path.  Plain C++ (no HIP), so that
// tests/test_worker_pool.py can build it alone under ThreadSanitizer.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace scm {

// Persistent host worker threads (content hashing, upload staging): run()
// executes f(0 .. n-1) on the workers and the calling thread and returns when
// all are done; launch() starts them on the workers only and wait() joins
// (the caller meanwhile drives the GPU).  One job at a time per pool.  A job
// is done when its last task is: the caller never waits for every worker to
// wake up (a sleeping thread's wake-up is tens of microseconds, on the drop-in
// path's critical host steps).  Jobs alternate between two slots; a worker
// joins the current job under the lock and leaves its slot's count when out
// of tasks, and launch() reuses a slot only when no worker is left in it.
class WorkerPool {
 public:
  void start(int workers) {
    for (int i = 0; i < workers; ++i) th_.emplace_back([this] { loop(); });
  }
  ~WorkerPool() {
    {
      std::unique_lock<std::mutex> l(m_);
      out_.wait(l, [&] { return job_[0].active == 0 && job_[1].active == 0; });
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void launch(int64_t n, std::function<void(int64_t)> f) {
    if (th_.empty()) {
      for (int64_t i = 0; i < n; ++i) f(i);
      return;
    }
    {
      std::unique_lock<std::mutex> l(m_);
      Job& j = job_[(gen_ + 1) & 1];
      out_.wait(l, [&] { return j.active == 0; });
      j.fn = std::move(f);
      j.n = n;
      j.next.store(0);
      j.finished.store(0);
      ++gen_;
    }
    cv_.notify_all();
    busy_ = true;
  }
  void wait() {
    if (!busy_) return;
    Job& j = job_[gen_ & 1];  // (gen_ is written by this thread only)
    std::unique_lock<std::mutex> l(m_);
    done_.wait(l, [&] { return j.finished.load() >= j.n; });
    busy_ = false;
  }
  void run(int64_t n, std::function<void(int64_t)> f) {
    if (n <= 1 || th_.empty()) {
      for (int64_t i = 0; i < n; ++i) f(i);
      return;
    }
    launch(n, std::move(f));
    work(job_[gen_ & 1]);
    wait();
  }

 private:
  struct Job {
    std::function<void(int64_t)> fn;
    int64_t n = 0;
    std::atomic<int64_t> next{0}, finished{0};
    int active = 0;  // workers inside (guarded by m_)
  };
  void work(Job& j) {
    for (;;) {
      const int64_t i = j.next.fetch_add(1);
      if (i >= j.n) return;
      j.fn(i);
      if (j.finished.fetch_add(1) + 1 == j.n) {
        std::lock_guard<std::mutex> l(m_);
        done_.notify_all();
      }
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      Job* j;
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        j = &job_[seen & 1];
        ++j->active;
      }
      work(*j);
      std::lock_guard<std::mutex> l(m_);
      if (--j->active == 0) out_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_, out_;
  Job job_[2];
  uint64_t gen_ = 0;
  bool stop_ = false, busy_ = false;
};

}  // namespace scm
