// Shared fan-out pool for parallelism *inside* one picture's parse (independent slices of an
// H.265 picture): any number of threads (the cameras' parse strands) may call run() at once.
//
// run(n, fn) queues fn(0..n-1); the caller takes indices itself while idle pool threads help, so a
// call completes even when every pool thread is busy with other callers' work (no deadlock, no
// oversubscription beyond the pool), and a camera whose picture has one slice pays nothing.
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace vep {

class FanOut {
 public:
  // init runs first on every pool thread (host domain pinning, hostplan.h)
  explicit FanOut(int threads, std::function<void()> init = {});
  ~FanOut();
  FanOut(const FanOut&) = delete;
  FanOut& operator=(const FanOut&) = delete;
  // The calling thread's pool: the host domain's (bind_thread, set on the parse strands of a GPU
  // worker's domain), else the process-wide pool (VEP_FANOUT_THREADS, else the CPU budget - 3).
  static FanOut& shared();
  static void bind_thread(FanOut* pool);
  int size() const { return int(th_.size()); }
  // fn(i) for i in [0, n); returns when every call has returned (rethrows the first exception).
  void run(int n, const std::function<void(int)>& fn);

 private:
  struct Task {
    const std::function<void(int)>* fn = nullptr;
    int n = 0;
    std::atomic<int> next{0}, done{0};
    std::mutex mu;
    std::condition_variable cv;
    std::exception_ptr err;
  };
  static void work(Task& t);  // take indices until none are left
  void loop();
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::shared_ptr<Task>> q_;
  bool stop_ = false;
};

}  // namespace vep
