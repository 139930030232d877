// Device-accessible host memory for ingest: a size-class pool of pinned (hipHostMalloc, mapped)
// blocks that access units are finalised into, and a registry translating host addresses inside
// such blocks to device addresses.
//
// Why: the native decoder references PCM samples *in place* in the received slice bytes. When
// those bytes already sit in pinned memory the worker's critical path does no host copy at all —
// a gather kernel on the copy stream pulls each slice straight over PCIe into the device staging
// buffer. The one host copy that remains (RTP reassembly -> pinned block) runs on the camera's
// own ingest thread, in parallel across cameras. Replaces the reference's
// ndarray/tobytes/SerializeToString/Redis copy chain (python/read_image.py:94-121).
#pragma once

#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <type_traits>
#include <vector>

#include "common.h"

namespace vep::hostmem {

// Enable the pinned pool (called once a Worker owns a GPU; HIP must be initialised). Until
// then, and on CPU-only hosts, pinned_block() returns nullptr and AUs stay in pageable memory.
void enable_pool(size_t max_bytes = size_t(8) << 30);
bool pool_enabled();

// The GPU whose NUMA node the calling thread's new pinned blocks should sit on (a host domain's
// threads bind their worker's device, hostplan.h; -1: unbound). Blocks are pooled per device.
void bind_thread_device(int device);

// A block of at least n bytes from the pool (nullptr if disabled or over budget). The memory is
// returned to the pool when the last reference drops.
std::shared_ptr<u8> pinned_block(size_t n);

// Device address of [p, p + n) if the range lies inside a registered pinned region, else nullptr.
const u8* device_address(const u8* p, size_t n);

// Register / unregister externally allocated pinned memory (e.g. a staging buffer).
void register_range(const u8* host, size_t n, const u8* dev);
void unregister_range(const u8* host);

// Raw allocation for containers: from the pinned pool when it is enabled (so the GPU can read
// the memory in place, see device_address), else from the heap. free_bytes tells them apart.
void* alloc_bytes(size_t n);
void free_bytes(void* p);

// Growable array of trivially copyable per-picture reconstruction records in pool memory (the
// std::vector subset the parser uses). Pictures are recycled with their capacity, so after
// warm-up nothing is allocated; the worker gathers the records to the GPU over PCIe instead of
// copying them into its staging buffer on the host. Appends are plain memcpy (a std::vector with
// a custom allocator would construct element by element).
template <class T>
class PodVec {
  static_assert(std::is_trivially_copyable_v<T>, "PodVec holds plain records");

 public:
  PodVec() = default;
  PodVec(const PodVec& o) { append(o.p_, o.n_); }
  PodVec(PodVec&& o) noexcept : p_(o.p_), n_(o.n_), cap_(o.cap_) { o.p_ = nullptr, o.n_ = o.cap_ = 0; }
  PodVec& operator=(const PodVec& o) {
    if (this != &o) {
      n_ = 0;
      append(o.p_, o.n_);
    }
    return *this;
  }
  PodVec& operator=(PodVec&& o) noexcept {
    if (this != &o) {
      free_bytes(p_);
      p_ = o.p_, n_ = o.n_, cap_ = o.cap_;
      o.p_ = nullptr, o.n_ = o.cap_ = 0;
    }
    return *this;
  }
  ~PodVec() { free_bytes(p_); }

  size_t size() const { return n_; }
  size_t capacity() const { return cap_; }
  bool empty() const { return n_ == 0; }
  T* data() { return p_; }
  const T* data() const { return p_; }
  T& operator[](size_t i) { return p_[i]; }
  const T& operator[](size_t i) const { return p_[i]; }
  T* begin() { return p_; }
  T* end() { return p_ + n_; }
  const T* begin() const { return p_; }
  const T* end() const { return p_ + n_; }
  T& back() { return p_[n_ - 1]; }

  void clear() { n_ = 0; }
  void reserve(size_t c) {
    if (c > cap_) grow(c);
  }
  void resize(size_t n) { resize(n, T{}); }
  void resize(size_t n, const T& v) {
    if (n > cap_) grow(std::max(n, 2 * cap_));
    for (size_t i = n_; i < n; ++i) p_[i] = v;
    n_ = n;
  }
  void assign(size_t n, const T& v) {
    n_ = 0;
    resize(n, v);
  }
  void append(const T* src, size_t k) {
    if (n_ + k > cap_) grow(std::max(n_ + k, 2 * cap_));
    if (k) std::memcpy(static_cast<void*>(p_ + n_), src, k * sizeof(T));
    n_ += k;
  }
  void push_back(const T& v) { append(&v, 1); }
  // k more entries, left uninitialised (the caller writes every one); returns the first
  T* extend(size_t k) {
    if (n_ + k > cap_) grow(std::max(n_ + k, 2 * cap_));
    T* q = p_ + n_;
    n_ += k;
    return q;
  }
  // (std::vector's range insert, at the end only)
  T* insert(T* pos, const T* first, const T* last) {
    const size_t at = size_t(pos - p_);
    VEP_CHECK(at == n_, "PodVec inserts append only");
    append(first, size_t(last - first));
    return p_ + at;
  }

 private:
  void grow(size_t c) {
    T* q = static_cast<T*>(alloc_bytes(c * sizeof(T)));
    if (n_) std::memcpy(static_cast<void*>(q), p_, n_ * sizeof(T));
    free_bytes(p_);
    p_ = q;
    cap_ = c;
  }
  T* p_ = nullptr;
  size_t n_ = 0, cap_ = 0;
};
template <class T>
using pinned_vector = PodVec<T>;

struct PoolStats {
  u64 chunks = 0, bytes_reserved = 0, blocks_live = 0, blocks_reused = 0, fallbacks = 0;
};
PoolStats pool_stats();

}  // namespace vep::hostmem
