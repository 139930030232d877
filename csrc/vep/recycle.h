// Recycling of large per-picture host buffers. A parsed 1080p H.264 picture carries ~1.2 MB of
// records (MB records, coefficient and motion pools) and a reference picture ~0.4 MB of
// colocated motion. Allocated fresh per picture, those buffers come back from the allocator as
// untouched pages: every picture then pays a few hundred page faults (fault + zeroing, under
// the process-wide mm lock that all parse threads share). The pool hands out objects whose
// vectors keep their capacity and are already resident.
//
// acquire() returns a shared_ptr whose deleter puts the object back (up to `cap` kept); objects
// that outlive the pool are deleted normally. `reset(T&)` restores default state while keeping
// capacities; it runs outside the pool lock (it may drop references that recycle other objects).
#pragma once

#include <memory>
#include <mutex>
#include <vector>

namespace vep {

template <class T>
class Recycler : public std::enable_shared_from_this<Recycler<T>> {
 public:
  static std::shared_ptr<Recycler> make(size_t cap) { return std::shared_ptr<Recycler>(new Recycler(cap)); }

  template <class Reset>
  std::shared_ptr<T> acquire(Reset&& reset) {
    std::unique_ptr<T> p;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!free_.empty()) {
        p = std::move(free_.back());
        free_.pop_back();
      }
    }
    if (p) reset(*p);
    else p.reset(new T());
    std::weak_ptr<Recycler> wp = this->shared_from_this();
    return std::shared_ptr<T>(p.release(), [wp](T* q) {
      if (auto pool = wp.lock()) {
        std::lock_guard<std::mutex> g(pool->mu_);
        if (pool->free_.size() < pool->cap_) {
          pool->free_.emplace_back(q);
          return;
        }
      }
      delete q;
    });
  }

 private:
  explicit Recycler(size_t cap) : cap_(cap) {}
  std::mutex mu_;
  std::vector<std::unique_ptr<T>> free_;
  size_t cap_;
};

}  // namespace vep
