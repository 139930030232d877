// vep — MI355X-native multi-camera video edge hub: shared native utilities.
#pragma once

#include <pthread.h>

#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace vep {

using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i16 = int16_t;
using i32 = int32_t;
using i64 = int64_t;

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define VEP_CHECK(cond, msg)                                                   \
  do {                                                                         \
    if (!(cond)) throw ::vep::Error(std::string("vep: ") + (msg));             \
  } while (0)

inline i64 now_ms() {
  using namespace std::chrono;
  return duration_cast<milliseconds>(system_clock::now().time_since_epoch()).count();
}

// Names the calling thread (at most 15 characters; /proc/<pid>/task/<tid>/comm): the bench's
// per-role CPU accounting and `top -H` tell the parse pool from the I/O loops and the GPU feeder.
inline void name_thread(const char* name) { ::pthread_setname_np(::pthread_self(), name); }

inline i64 mono_us() {
  using namespace std::chrono;
  return duration_cast<microseconds>(steady_clock::now().time_since_epoch()).count();
}

// Macroblock geometry of an H.264 4:2:0 8-bit picture.
constexpr int kMbSize = 16;
constexpr int kPcmLumaBytes = 256;
constexpr int kPcmChromaBytes = 64;  // per plane
constexpr int kPcmMbBytes = kPcmLumaBytes + 2 * kPcmChromaBytes;  // 384 = 24 x 16 B
constexpr int kPcmMaxSamples = 512;  // (H.264 4:2:2 I_PCM: 256 + 2 x 128 samples)

// 64-byte aligned growable byte buffer (host, pageable).
class AlignedBuf {
 public:
  AlignedBuf() = default;
  explicit AlignedBuf(size_t n) { resize(n); }
  ~AlignedBuf() { std::free(p_); }
  AlignedBuf(const AlignedBuf&) = delete;
  AlignedBuf& operator=(const AlignedBuf&) = delete;
  AlignedBuf(AlignedBuf&& o) noexcept : p_(o.p_), n_(o.n_), cap_(o.cap_) {
    o.p_ = nullptr;
    o.n_ = o.cap_ = 0;
  }
  AlignedBuf& operator=(AlignedBuf&& o) noexcept {
    if (this != &o) {
      std::free(p_);
      p_ = o.p_;
      n_ = o.n_;
      cap_ = o.cap_;
      o.p_ = nullptr;
      o.n_ = o.cap_ = 0;
    }
    return *this;
  }
  void reserve(size_t n) {
    if (n <= cap_) return;
    size_t c = ((n > 2 * cap_ ? n : 2 * cap_) + 63) & ~size_t(63);
    void* q = std::aligned_alloc(64, c);
    VEP_CHECK(q, "aligned_alloc failed");
    if (p_) {
      std::memcpy(q, p_, n_);
      std::free(p_);
    }
    p_ = static_cast<u8*>(q);
    cap_ = c;
  }
  void resize(size_t n) {
    reserve(n);
    n_ = n;
  }
  void clear() { n_ = 0; }
  u8* data() { return p_; }
  const u8* data() const { return p_; }
  size_t size() const { return n_; }

 private:
  u8* p_ = nullptr;
  size_t n_ = 0, cap_ = 0;
};

}  // namespace vep
