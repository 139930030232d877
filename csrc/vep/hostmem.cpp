// Pinned ingest pool + host->device address registry. See hostmem.h.
#include "hostmem.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <new>
#include <array>
#include <map>
#include <shared_mutex>

namespace vep::hostmem {

namespace {

struct Region {
  size_t len;
  const u8* dev;
};

// Size classes: 2^16 .. 2^26 bytes (64 KiB .. 64 MiB); larger requests get a dedicated chunk.
constexpr int kMinShift = 16, kMaxShift = 26;

struct Pool {
  std::shared_mutex reg_mu;
  std::map<const u8*, Region> regions;  // host base -> (len, device base)
  std::mutex mu;
  // free blocks per (device the allocating thread was bound to, size class): a domain reuses
  // blocks on its own NUMA node
  std::map<int, std::array<std::vector<u8*>, kMaxShift + 1>> free_;
  bool enabled = false;
  size_t max_bytes = 0;
  PoolStats st;
};

Pool& pool() {
  static Pool* p = new Pool();  // intentionally leaked: blocks may outlive static destruction
  return *p;
}

int class_of(size_t n) {
  int s = kMinShift;
  while (s < kMaxShift && (size_t(1) << s) < n) ++s;
  return (size_t(1) << s) >= n ? s : -1;
}

u8* new_chunk(size_t bytes) {
  void* h = nullptr;
  if (hipHostMalloc(&h, bytes, hipHostMallocDefault) != hipSuccess || !h) return nullptr;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) d = h;
  register_range(static_cast<u8*>(h), bytes, static_cast<u8*>(d));
  return static_cast<u8*>(h);
}

thread_local int tls_device = -1;

}  // namespace

void bind_thread_device(int device) { tls_device = device; }

void enable_pool(size_t max_bytes) {
  Pool& p = pool();
  std::lock_guard<std::mutex> g(p.mu);
  p.enabled = true;
  p.max_bytes = std::max(p.max_bytes, max_bytes);
}

bool pool_enabled() {
  Pool& p = pool();
  std::lock_guard<std::mutex> g(p.mu);
  return p.enabled;
}

std::shared_ptr<u8> pinned_block(size_t n) {
  Pool& p = pool();
  const int cls = class_of(n);
  const int dev = tls_device;
  u8* blk = nullptr;
  {
    std::lock_guard<std::mutex> g(p.mu);
    if (!p.enabled) return nullptr;
    auto& fl = p.free_[dev];
    if (cls >= 0 && !fl[size_t(cls)].empty()) {
      blk = fl[size_t(cls)].back();
      fl[size_t(cls)].pop_back();
      ++p.st.blocks_reused;
      ++p.st.blocks_live;
    }
  }
  if (!blk) {
    const size_t bytes = cls >= 0 ? (size_t(1) << cls) : ((n + 0xFFFFF) & ~size_t(0xFFFFF));
    {
      std::lock_guard<std::mutex> g(p.mu);
      if (p.st.bytes_reserved + bytes > p.max_bytes) {
        ++p.st.fallbacks;
        return nullptr;
      }
      p.st.bytes_reserved += bytes;  // reserve before the (slow) allocation
    }
    blk = new_chunk(bytes);
    std::lock_guard<std::mutex> g(p.mu);
    if (!blk) {
      p.st.bytes_reserved -= bytes;
      ++p.st.fallbacks;
      return nullptr;
    }
    ++p.st.chunks;
    ++p.st.blocks_live;
  }
  return std::shared_ptr<u8>(blk, [cls, dev](u8* b) {
    Pool& q = pool();
    std::lock_guard<std::mutex> g(q.mu);
    --q.st.blocks_live;
    // pooled, never returned to the driver; a dedicated (> 64 MiB) chunk is recycled as a
    // top-class block (it is at least that large)
    q.free_[dev][size_t(cls >= 0 ? cls : kMaxShift)].push_back(b);
  });
}

namespace {
struct Live {  // pool blocks handed to containers, keyed by address
  std::mutex mu;
  std::map<void*, std::shared_ptr<u8>> blocks;
};
Live& live() {
  static Live* l = new Live();  // leaked like the pool
  return *l;
}
}  // namespace

void* alloc_bytes(size_t n) {
  n = std::max<size_t>(n, 1);
  if (pool_enabled()) {
    if (std::shared_ptr<u8> b = pinned_block(n)) {
      void* p = b.get();
      Live& l = live();
      std::lock_guard<std::mutex> g(l.mu);
      l.blocks.emplace(p, std::move(b));
      return p;
    }
  }
  void* p = std::malloc(n);
  if (!p) throw std::bad_alloc();
  return p;
}

void free_bytes(void* p) {
  if (!p) return;
  std::shared_ptr<u8> keep;  // released outside the lock (its deleter takes the pool lock)
  {
    Live& l = live();
    std::lock_guard<std::mutex> g(l.mu);
    auto it = l.blocks.find(p);
    if (it != l.blocks.end()) {
      keep = std::move(it->second);
      l.blocks.erase(it);
    }
  }
  if (!keep) std::free(p);
}

const u8* device_address(const u8* p, size_t n) {
  Pool& q = pool();
  std::shared_lock<std::shared_mutex> g(q.reg_mu);
  auto it = q.regions.upper_bound(p);
  if (it == q.regions.begin()) return nullptr;
  --it;
  const u8* base = it->first;
  if (p < base || p + n > base + it->second.len) return nullptr;
  return it->second.dev + (p - base);
}

void register_range(const u8* host, size_t n, const u8* dev) {
  Pool& q = pool();
  std::unique_lock<std::shared_mutex> g(q.reg_mu);
  q.regions[host] = Region{n, dev ? dev : host};
}

void unregister_range(const u8* host) {
  Pool& q = pool();
  std::unique_lock<std::shared_mutex> g(q.reg_mu);
  q.regions.erase(host);
}

PoolStats pool_stats() {
  Pool& q = pool();
  std::lock_guard<std::mutex> g(q.mu);
  return q.st;
}

}  // namespace vep::hostmem
