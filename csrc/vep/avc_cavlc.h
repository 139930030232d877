// CAVLC entropy layer of H.264 (§9.2): a branch-light bit reader, the coeff_token /
// total_zeros / run_before code tables as single-lookup decode tables (built once from the
// code lists of Tables 9-5, 9-7, 9-8, 9-9a and 9-10), and the matching encoder.
#pragma once

#include "bits.h"
#include "common.h"

namespace vep::avc {

// MSB-first reader with 32-bit lookahead over an RBSP. Reading past the end yields zero bits and
// is reported by overrun() (checked once per macroblock instead of per bit).
class Bits {
 public:
  Bits(const u8* p, size_t n, size_t bitpos = 0) : p_(p), n_(n), pos_(bitpos) {}
  u32 peek32() const {
    const size_t byte = pos_ >> 3;
    u64 v = 0;
    if (byte + 8 <= n_) {
      std::memcpy(&v, p_ + byte, 8);
      v = __builtin_bswap64(v);
    } else {
      for (size_t i = 0; i < 8; ++i) v = (v << 8) | (byte + i < n_ ? p_[byte + i] : 0u);
    }
    return u32((v << (pos_ & 7)) >> 32);
  }
  void skip(size_t n) { pos_ += n; }
  u32 u(int n) {
    if (n == 0) return 0;
    const u32 v = peek32() >> (32 - n);
    pos_ += size_t(n);
    return v;
  }
  u32 u1() { return u(1); }
  u32 ue() {
    const u32 w = peek32();
    VEP_CHECK(w != 0, "exp-golomb code too long");
    const int lz = __builtin_clz(w);
    if (lz <= 15) {
      const int len = 2 * lz + 1;
      pos_ += size_t(len);
      return (w >> (32 - len)) - 1;
    }
    pos_ += size_t(lz);
    return u(lz + 1) - 1;
  }
  i32 se() {
    const u32 k = ue();
    return (k & 1) ? i32((k + 1) >> 1) : -i32(k >> 1);
  }
  size_t pos() const { return pos_; }
  void seek(size_t bit) { pos_ = bit; }
  void align() { pos_ = (pos_ + 7) & ~size_t(7); }
  bool overrun() const { return pos_ > n_ * 8; }
  const u8* data() const { return p_; }
  size_t size() const { return n_; }

 private:
  const u8* p_;
  size_t n_;
  size_t pos_;
};

// coded_block_pattern of me(v) codeNum (Table 9-4, ChromaArrayType 1/2): Intra_4x4 / Inter.
inline constexpr u8 kCbpIntra[48] = {47, 31, 15, 0,  23, 27, 29, 30, 7,  11, 13, 14, 39, 43, 45, 46,
                                     16, 3,  5,  10, 12, 19, 21, 26, 28, 35, 37, 42, 44, 1,  2,  4,
                                     8,  17, 18, 20, 24, 6,  9,  22, 25, 32, 33, 34, 36, 40, 38, 41};
inline constexpr u8 kCbpInter[48] = {0,  16, 1,  2,  4,  8,  32, 3,  5,  10, 12, 15, 47, 7,  11, 13,
                                     14, 6,  9,  31, 35, 37, 42, 44, 33, 34, 36, 40, 39, 43, 45, 46,
                                     17, 18, 20, 24, 19, 21, 26, 28, 23, 27, 29, 30, 22, 25, 38, 41};

// coeff_token class: 0..3 for nC ranges [0,2) [2,4) [4,8) [8,inf), 4 for chroma DC 4:2:0
// (nC = -1), 5 for chroma DC 4:2:2 (nC = -2).
inline int coeff_token_class(int nc) {
  return nc == -2 ? 5 : nc < 0 ? 4 : nc < 2 ? 0 : nc < 4 ? 1 : nc < 8 ? 2 : 3;
}

struct CoeffToken {
  int total, trailing;
};

CoeffToken read_coeff_token(Bits& br, int cls);
// max_coeff 4 / 8: the chroma DC tables of 4:2:0 (Table 9-9a) / 4:2:2 (Table 9-9b)
int read_total_zeros(Bits& br, int total_coeff, int max_coeff);
int read_run_before(Bits& br, int zeros_left);

// Parse one residual_block_cavlc (§7.3.5.3.3), handing every nonzero coefficient to
// put(scan_index, level) (scan_index in [0, max_coeff)). Returns TotalCoeff.
template <class Put>
inline int read_residual_block_cb(Bits& br, int nc, int max_coeff, Put&& put) {
  const CoeffToken t = read_coeff_token(br, coeff_token_class(nc));
  if (t.total == 0) return 0;
  VEP_CHECK(t.total <= max_coeff, "TotalCoeff exceeds maxNumCoeff");
  int level[16];
  int suffix_len = (t.total > 10 && t.trailing < 3) ? 1 : 0;
  for (int i = 0; i < t.total; ++i) {
    if (i < t.trailing) {
      level[i] = br.u1() ? -1 : 1;
      continue;
    }
    const u32 w = br.peek32();
    VEP_CHECK(w != 0, "level_prefix too long");
    const int prefix = __builtin_clz(w);
    br.skip(size_t(prefix) + 1);
    int code = (prefix < 15 ? prefix : 15) << suffix_len;
    const int ssize = (prefix == 14 && suffix_len == 0) ? 4 : (prefix >= 15 ? prefix - 3 : suffix_len);
    if (ssize > 0) code += int(br.u(ssize));
    if (prefix >= 15 && suffix_len == 0) code += 15;
    if (prefix >= 16) code += (1 << (prefix - 3)) - 4096;
    if (i == t.trailing && t.trailing < 3) code += 2;
    level[i] = (code % 2 == 0) ? (code + 2) >> 1 : (-code - 1) >> 1;
    if (suffix_len == 0) suffix_len = 1;
    const int a = level[i] < 0 ? -level[i] : level[i];
    if (a > (3 << (suffix_len - 1)) && suffix_len < 6) ++suffix_len;
  }
  int left = 0;
  if (t.total < max_coeff) left = read_total_zeros(br, t.total, max_coeff);
  VEP_CHECK(t.total + left <= max_coeff, "total_zeros out of range");
  // levels arrive highest frequency first: walk scan positions downwards from the last one
  int pos = t.total + left - 1;
  for (int i = 0; i < t.total - 1; ++i) {
    put(pos, level[i]);
    int run = 0;
    if (left > 0) {
      run = read_run_before(br, left);
      left -= run;
      VEP_CHECK(left >= 0, "run_before exceeds zerosLeft");
    }
    pos -= run + 1;
  }
  put(pos, level[t.total - 1]);
  return t.total;
}

// Parse one residual_block_cavlc (§7.3.5.3.3) into coeff[0 .. max_coeff-1] (scan order; the
// caller zeroes coeff). Returns TotalCoeff.
inline int read_residual_block(Bits& br, int nc, int max_coeff, int* coeff) {
  return read_residual_block_cb(br, nc, max_coeff, [coeff](int k, int v) { coeff[k] = v; });
}

// Encoder side: coeff[0 .. max_coeff-1] in scan order; levels must satisfy |level| <= 2047.
// Returns TotalCoeff.
int write_residual_block(BitWriter& bw, int nc, int max_coeff, const int* coeff);

}  // namespace vep::avc
