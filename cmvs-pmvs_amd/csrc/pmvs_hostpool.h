// pmvs_hostpool.h -- a persistent pool of host threads (host code only): included by
// pmvs_kernels.hip and by the CPU test tests/csrc/hostpool_test.cpp.
#pragma once
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace pmvsdev {

// A persistent pool of host threads for the per-batch host work of the refine (the start-point
// angles below).  run(nt, f) calls f(t, nt') for t in [0, nt') (nt' = nt capped by the pool, t = 0 on
// the caller's thread) and returns after every call returned; false (nothing run) when another
// thread is using the pool.
class HostPool {
 public:
  // never destroyed: the workers wait on the condition variable until the process ends (no join at
  // exit, and a forked child, which has none of them, never touches them: run() checks the pid)
  static HostPool& get() {
    static HostPool* pool = new HostPool();
    return *pool;
  }
  template <class F>
  bool run(int nt, F&& f) {
    if (getpid() != pid_) return false;  // a forked child has none of the workers
    std::unique_lock<std::mutex> use(use_, std::try_to_lock);
    if (!use.owns_lock()) return false;
    nt = std::max(1, std::min(nt, (int)workers_.size() + 1));
    std::function<void(int, int)> job = [&f](int t, int k) { f(t, k); };
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = &job;
      nt_ = nt;
      pending_ = nt - 1;
      ++gen_;
    }
    cv_.notify_all();
    job(0, nt);
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [&] { return pending_ == 0; });
    job_ = nullptr;
    return true;
  }

 private:
  HostPool() : pid_(getpid()) {
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    for (int t = 1; t < std::min(8, hw); ++t) workers_.emplace_back([this, t] { loop(t); });
  }
  void loop(int t) {
    unsigned long long seen = 0;
    for (;;) {
      std::function<void(int, int)>* job;
      int nt;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        job = job_;
        nt = nt_;
      }
      if (t < nt) {
        (*job)(t, nt);
        std::lock_guard<std::mutex> g(m_);
        if (--pending_ == 0) done_.notify_one();
      }
    }
  }
  const pid_t pid_;
  std::vector<std::thread> workers_;
  std::mutex use_, m_;
  std::condition_variable cv_, done_;
  std::function<void(int, int)>* job_ = nullptr;
  int nt_ = 0, pending_ = 0;
  unsigned long long gen_ = 0;
};

}  // namespace pmvsdev
