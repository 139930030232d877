// Minimal fixed-size thread pool with a parallel-for (CPU parse fan-out across cameras).
#pragma once

#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "common.h"

namespace vep {

class ThreadPool {
 public:
  explicit ThreadPool(int n, std::function<void()> init = {}) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this, init] {
      name_thread("vep-pool");
      if (init) init();
      run();
    });
  }
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return int(th_.size()); }

  // Run fn(i) for i in [0, n) on the pool; blocks until all are done.
  void parallel_for(int n, const std::function<void(int)>& fn) {
    if (n <= 0) return;
    if (th_.empty()) {
      for (int i = 0; i < n; ++i) fn(i);
      return;
    }
    std::unique_lock<std::mutex> g(mu_);
    fn_ = &fn;
    n_ = n;
    next_ = 0;
    done_ = 0;
    ++gen_;
    cv_.notify_all();
    done_cv_.wait(g, [&] { return done_ == n_; });
    fn_ = nullptr;
  }

 private:
  void run() {
    u_int64_t seen = 0;
    std::unique_lock<std::mutex> g(mu_);
    for (;;) {
      cv_.wait(g, [&] { return stop_ || (gen_ != seen && fn_ && next_ < n_); });
      if (stop_) return;
      while (fn_ && next_ < n_) {
        int i = next_++;
        const std::function<void(int)>* f = fn_;
        g.unlock();
        (*f)(i);
        g.lock();
        if (++done_ == n_) done_cv_.notify_all();
      }
      seen = gen_;
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0, next_ = 0, done_ = 0;
  u_int64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace vep
