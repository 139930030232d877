// Bit-level readers/writers for H.264/H.265 RBSP and the NAL emulation-prevention layer.
//
// Reference parity: these replace the bitstream handling that the reference delegates to
// FFmpeg/libavcodec via PyAV (python/read_image.py:87 `p.decode()`).
#pragma once

#include "common.h"

namespace vep {

// MSB-first reader over an RBSP (emulation-prevention bytes already removed).
class BitReader {
 public:
  BitReader(const u8* p, size_t n) : p_(p), n_(n) {}

  size_t bitpos() const { return pos_; }
  size_t bits_left() const { return n_ * 8 > pos_ ? n_ * 8 - pos_ : 0; }
  bool byte_aligned() const { return (pos_ & 7) == 0; }
  size_t bytepos() const { return pos_ >> 3; }
  const u8* data() const { return p_; }
  size_t size() const { return n_; }

  u32 u1() {
    VEP_CHECK(pos_ < n_ * 8, "bitstream overrun");
    u32 b = (p_[pos_ >> 3] >> (7 - (pos_ & 7))) & 1u;
    ++pos_;
    return b;
  }
  u32 u(int n) {
    u32 v = 0;
    // fast path: byte-wise when aligned
    while (n >= 8 && byte_aligned()) {
      VEP_CHECK(pos_ + 8 <= n_ * 8, "bitstream overrun");
      v = (v << 8) | p_[pos_ >> 3];
      pos_ += 8;
      n -= 8;
    }
    for (int i = 0; i < n; ++i) v = (v << 1) | u1();
    return v;
  }
  u32 ue() {
    int lz = 0;
    while (u1() == 0) {
      ++lz;
      VEP_CHECK(lz < 32, "exp-golomb code too long");
    }
    if (lz == 0) return 0;
    return ((1u << lz) - 1u) + u(lz);
  }
  i32 se() {
    u32 k = ue();
    return (k & 1) ? i32((k + 1) >> 1) : -i32(k >> 1);
  }
  void skip(size_t nbits) {
    VEP_CHECK(pos_ + nbits <= n_ * 8, "bitstream overrun");
    pos_ += nbits;
  }
  void align() { pos_ = (pos_ + 7) & ~size_t(7); }
  void seek_byte(size_t b) { pos_ = b * 8; }

  // Position (in bits) of the rbsp_stop_one_bit: more_rbsp_data() is true while pos < this.
  size_t stop_bit_pos() const {
    size_t i = n_;
    while (i > 0 && p_[i - 1] == 0) --i;  // cabac_zero_words / trailing zeros
    if (i == 0) return 0;
    u8 last = p_[i - 1];
    int tz = __builtin_ctz(last);
    return (i - 1) * 8 + (7 - tz);
  }

 private:
  const u8* p_;
  size_t n_;
  size_t pos_ = 0;
};

// MSB-first writer producing an RBSP.
class BitWriter {
 public:
  void u1(u32 b) {
    cur_ = (cur_ << 1) | (b & 1u);
    if (++nb_ == 8) flush_byte();
  }
  void u(int n, u32 v) {
    for (int i = n - 1; i >= 0; --i) u1((v >> i) & 1u);
  }
  void ue(u32 v) {
    u64 x = u64(v) + 1;
    int len = 64 - __builtin_clzll(x);
    for (int i = 0; i < len - 1; ++i) u1(0);
    for (int i = len - 1; i >= 0; --i) u1(u32(x >> i) & 1u);
  }
  void se(i32 v) { ue(v > 0 ? u32(2 * v - 1) : u32(-2 * i64(v))); }
  bool byte_aligned() const { return nb_ == 0; }
  void align_zero() {
    while (nb_ != 0) u1(0);
  }
  void trailing() {  // rbsp_trailing_bits
    u1(1);
    align_zero();
  }
  // Append raw aligned bytes (PCM samples).
  void bytes(const u8* p, size_t n) {
    VEP_CHECK(nb_ == 0, "raw bytes must be byte aligned");
    out_.insert(out_.end(), p, p + n);
  }
  std::vector<u8>& buf() { return out_; }

 private:
  void flush_byte() {
    out_.push_back(u8(cur_));
    cur_ = 0;
    nb_ = 0;
  }
  std::vector<u8> out_;
  u32 cur_ = 0;
  int nb_ = 0;
};

// Insert emulation-prevention bytes (00 00 0x, x<=3 -> 00 00 03 0x). Appends to `out`.
inline void rbsp_to_ebsp(const u8* p, size_t n, std::vector<u8>& out) {
  out.reserve(out.size() + n + n / 64 + 4);
  int zeros = 0;
  for (size_t i = 0; i < n; ++i) {
    u8 b = p[i];
    if (zeros >= 2 && b <= 3) {
      out.push_back(3);
      zeros = 0;
    }
    out.push_back(b);
    zeros = (b == 0) ? zeros + 1 : 0;
  }
}

// Positions (indices into p) of emulation-prevention 0x03 bytes. Uses memchr to hop
// between zero bytes so PCM payloads (samples never 0) are scanned at memchr speed.
inline void find_epb(const u8* p, size_t n, std::vector<u32>& out) {
  out.clear();
  size_t i = 0;
  while (i + 2 < n) {
    const void* z = std::memchr(p + i, 0, n - i - 2);
    if (!z) break;
    size_t k = size_t(static_cast<const u8*>(z) - p);
    if (p[k + 1] == 0 && p[k + 2] == 3) {
      out.push_back(u32(k + 2));
      i = k + 3;
    } else {
      i = k + 1;
    }
  }
}

// Remove emulation-prevention bytes: EBSP -> RBSP. Returns RBSP length.
inline size_t ebsp_to_rbsp(const u8* p, size_t n, u8* out) {
  size_t o = 0;
  int zeros = 0;
  for (size_t i = 0; i < n; ++i) {
    u8 b = p[i];
    if (zeros >= 2 && b == 3) {
      zeros = 0;
      continue;
    }
    out[o++] = b;
    zeros = (b == 0) ? zeros + 1 : 0;
  }
  return o;
}

}  // namespace vep
