// Shared fan-out pool: see fanout.h.
#include "fanout.h"

#include <algorithm>
#include <cstdlib>

#include "ioloop.h"

namespace vep {

namespace {
thread_local FanOut* tls_pool = nullptr;
}

void FanOut::bind_thread(FanOut* pool) { tls_pool = pool; }

FanOut::FanOut(int threads, std::function<void()> init) {
  for (int i = 0; i < threads; ++i) th_.emplace_back([this, init] {
    name_thread("vep-fanout");
    if (init) init();
    loop();
  });
}

FanOut::~FanOut() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : th_) t.join();
}

FanOut& FanOut::shared() {
  if (tls_pool) return *tls_pool;
  // the same CPU share as the parse strands (VEP_INGEST_PARSE_THREADS, else the process's CPU
  // budget minus the socket loops and the GPU launcher): a picture's slices run on the cores its
  // camera's strand would otherwise leave idle, not beyond the process's share
  static FanOut pool([] {
    if (const char* e = std::getenv("VEP_FANOUT_THREADS")) return std::clamp(std::atoi(e), 0, 256);
    if (const char* e = std::getenv("VEP_INGEST_PARSE_THREADS")) return std::clamp(std::atoi(e) - 1, 0, 256);
    return std::clamp(cpu_budget() - 3, 0, 31);
  }());
  return pool;
}

void FanOut::work(Task& t) {
  for (int i = t.next.fetch_add(1); i < t.n; i = t.next.fetch_add(1)) {
    try {
      (*t.fn)(i);
    } catch (...) {
      std::lock_guard<std::mutex> g(t.mu);
      if (!t.err) t.err = std::current_exception();
    }
    if (t.done.fetch_add(1) + 1 == t.n) {
      std::lock_guard<std::mutex> g(t.mu);
      t.cv.notify_all();
    }
  }
}

void FanOut::loop() {
  std::unique_lock<std::mutex> g(mu_);
  for (;;) {
    cv_.wait(g, [&] { return stop_ || !q_.empty(); });
    if (stop_) return;
    std::shared_ptr<Task> t = q_.front();
    if (t->next.load() >= t->n) {  // every index taken: retire it from the queue
      q_.pop_front();
      continue;
    }
    g.unlock();
    work(*t);
    g.lock();
  }
}

void FanOut::run(int n, const std::function<void(int)>& fn) {
  if (n <= 0) return;
  if (n == 1 || th_.empty()) {
    for (int i = 0; i < n; ++i) fn(i);
    return;
  }
  auto t = std::make_shared<Task>();
  t->fn = &fn;
  t->n = n;
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(t);
  }
  cv_.notify_all();
  work(*t);  // the caller takes its share (all of it when the pool is busy)
  {
    std::unique_lock<std::mutex> g(t->mu);
    t->cv.wait(g, [&] { return t->done.load() == t->n; });
  }
  {
    std::lock_guard<std::mutex> g(mu_);  // (pool threads may still hold a reference: harmless)
    for (auto it = q_.begin(); it != q_.end(); ++it)
      if (*it == t) {
        q_.erase(it);
        break;
      }
  }
  if (t->err) std::rethrow_exception(t->err);
}

}  // namespace vep
