// CABAC arithmetic coding engine (H.265 §9.3.4.3 / §9.3.5; identical engine to H.264 §9.3.3.2):
// 9-bit-offset decoder, 10-bit-low encoder with outstanding-bit carry resolution, the 64-state
// probability model and the slice-QP-dependent context initialisation.
//
// Used by the native HEVC subset codec (hevc.h) for the handful of context-coded syntax elements
// a PCM/skip picture needs (cu_skip_flag, pred_mode_flag, part_mode) plus the terminating bins
// (pcm_flag, end_of_slice_segment_flag). Replaces libavcodec's CABAC inside PyAV in the reference
// (python/read_image.py:87 `p.decode()`).
#pragma once

#include <atomic>
#include <cstring>

#include "common.h"

namespace vep::cabac {

#define VEP_CABAC_INLINE inline __attribute__((always_inline))

// rangeTabLPS[pStateIdx][qRangeIdx] (H.265 Table 9-52 / H.264 Table 9-44).
inline constexpr u8 kRangeLps[64][4] = {
    {128, 176, 208, 240}, {128, 167, 197, 227}, {128, 158, 187, 216}, {123, 150, 178, 205},
    {116, 142, 169, 195}, {111, 135, 160, 185}, {105, 128, 152, 175}, {100, 122, 144, 166},
    {95, 116, 137, 158},  {90, 110, 130, 150},  {85, 104, 123, 142},  {81, 99, 117, 135},
    {77, 94, 111, 128},   {73, 89, 105, 122},   {69, 85, 100, 116},   {66, 80, 95, 110},
    {62, 76, 90, 104},    {59, 72, 86, 99},     {56, 69, 81, 94},     {53, 65, 77, 89},
    {51, 62, 73, 85},     {48, 59, 69, 80},     {46, 56, 66, 76},     {43, 53, 63, 72},
    {41, 50, 59, 69},     {39, 48, 56, 65},     {37, 45, 54, 62},     {35, 43, 51, 59},
    {33, 41, 48, 56},     {32, 39, 46, 53},     {30, 37, 43, 50},     {29, 35, 41, 48},
    {27, 33, 39, 45},     {26, 31, 37, 43},     {24, 30, 35, 41},     {23, 28, 33, 39},
    {22, 27, 32, 37},     {21, 26, 30, 35},     {20, 24, 29, 33},     {19, 23, 27, 31},
    {18, 22, 26, 30},     {17, 21, 25, 28},     {16, 20, 23, 27},     {15, 19, 22, 25},
    {14, 18, 21, 24},     {14, 17, 20, 23},     {13, 16, 19, 22},     {12, 15, 18, 21},
    {12, 14, 17, 20},     {11, 14, 16, 19},     {11, 13, 15, 18},     {10, 12, 15, 17},
    {10, 12, 14, 16},     {9, 11, 13, 15},      {9, 11, 12, 14},      {8, 10, 12, 14},
    {8, 9, 11, 13},       {7, 9, 11, 12},       {7, 9, 10, 12},       {7, 8, 10, 11},
    {6, 8, 9, 11},        {6, 7, 9, 10},        {6, 7, 8, 9},         {2, 2, 2, 2},
};

// transIdxLps (Table 9-53); transIdxMps is min(s + 1, 62) (63 is the terminate state).
inline constexpr u8 kNextLps[64] = {
    0,  0,  1,  2,  2,  4,  4,  5,  6,  7,  8,  9,  9,  11, 11, 12, 13, 13, 15, 15, 16, 16,
    18, 18, 19, 19, 21, 21, 22, 22, 23, 24, 24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30,
    31, 32, 32, 33, 33, 33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63,
};
// Packed state s = pStateIdx << 1 | valMps. Both transitions in one table:
// kTrans[is_lps][s] = the next packed state (an LPS in state 0 flips valMps).
struct StateTrans {
  u16 t[2][128];
  constexpr StateTrans() : t{} {
    for (int st = 0; st < 64; ++st)
      for (int m = 0; m < 2; ++m) {
        const int s = st << 1 | m;
        t[0][s] = u16((st < 62 ? st + 1 : st) << 1 | m);
        t[1][s] = u16(kNextLps[st] << 1 | (st == 0 ? m ^ 1 : m));
      }
  }
};
inline constexpr StateTrans kTrans{};

// A context is one u64 carrying everything a bin needs from it:
//   bits  0..31  rangeTabLPS[pStateIdx][qRangeIdx 0..3], a byte each
//   bits 32..38  packed state s (bit 32 = valMps)
//   bits 40..46  packed state after an LPS, bits 48..54 after an MPS.
// The LPS range is then a shift of the context word by the range's two quantisation bits (no
// table load on the range -> range dependency chain), and both successor words are loaded from
// the context alone while that chain runs, so the outcome only selects one (a cmov): the next
// bin of the same context waits on a select and a store-forward, not on a load indexed by the
// outcome. (Not a smaller type: u8/u16 stores may alias any object, and every context update
// would force the arithmetic decoder's registers back to memory when reached through a pointer.)
struct CtxWords {
  u64 e[128];
  constexpr CtxWords() : e() {
    for (int s = 0; s < 128; ++s) {
      const int st = s >> 1;
      u64 w = 0;
      for (int q = 0; q < 4; ++q) w |= u64(kRangeLps[st][q]) << (8 * q);
      w |= u64(s) << 32 | u64(kTrans.t[1][s]) << 40 | u64(kTrans.t[0][s]) << 48;
      e[s] = w;
    }
  }
};
inline constexpr CtxWords kCtxWords{};

struct Ctx {
  u64 e = kCtxWords.e[0];

  int state() const { return int((e >> 33) & 63); }
  int mps() const { return int((e >> 32) & 1); }
  void set(int state, int mps) { e = kCtxWords.e[(state << 1 | mps) & 127]; }
  // §9.3.2.2: initValue -> (pStateIdx, valMps) for SliceQpY.
  void init(int init_value, int qp) {
    const int slope = init_value >> 4, offset = init_value & 15;
    const int m = slope * 5 - 45, n = (offset << 3) - 16;
    const int q = qp < 0 ? 0 : (qp > 51 ? 51 : qp);
    int pre = ((m * q) >> 4) + n;
    pre = pre < 1 ? 1 : (pre > 126 ? 126 : pre);
    const int mp = pre <= 63 ? 0 : 1;
    set(mp ? pre - 64 : 63 - pre, mp);
  }
  // rangeTabLPS[pStateIdx][qRangeIdx] for a range in [256, 510]
  static VEP_CABAC_INLINE u32 lps_of(u64 e, u32 range) { return u32(e >> ((range >> 3) & 24u)) & 0xFFu; }
  static VEP_CABAC_INLINE u64 after(u64 e, u32 is_lps) {
    const u64 el = kCtxWords.e[(e >> 40) & 127], em = kCtxWords.e[(e >> 48) & 127];
    return is_lps ? el : em;
  }
};

// Arithmetic decoder over an RBSP (byte positions are RBSP offsets). Bits are pulled from a
// 64-bit MSB-aligned cache (refilled a word at a time) and renormalisation is one clz + shift;
// a context-coded bin is branch-free apart from the rare refill (an MPS / LPS outcome is close to
// unpredictable on residual data). (A variant keeping the offset scaled with a 16-bit look-ahead
// window and a marker bit measured 13% slower on the parse benchmark: the extra shift sits on
// the range -> offset dependency chain.)
//
// Hot loops (residual blocks) also work on a local copy of the decoder (`Decoder d = engine;
// ...; engine = d;`): a copy whose address never escapes (every member is force-inlined) stays
// in registers for the whole block.
class Decoder {
 public:
  Decoder(const u8* p, size_t n, size_t bytepos) : p_(p), n_(n) { start(bytepos); }

  // §9.3.2.5: (re)initialise at a byte position (slice data start, or after PCM samples).
  void start(size_t bytepos) {
    byte_ = bytepos;
    cache_ = 0;
    cbits_ = 0;
    range_ = 510;
    offset_ = bits(9);
  }
  VEP_CABAC_INLINE u32 decision(Ctx& c) {
    ++nbins_;
    const u64 e = c.e;
    const u32 lps = Ctx::lps_of(e, range_);
    u64 e_lps = kCtxWords.e[(e >> 40) & 127], e_mps = kCtxWords.e[(e >> 48) & 127];
    // (both words loaded here, off the bin's chain: without this the compiler selects the
    // address by the outcome and loads after it, putting the load back on the same-context chain)
    asm("" : "+r"(e_lps), "+r"(e_mps));
    const u32 rmps = range_ - lps;
    const u32 is_lps = offset_ >= rmps ? 1u : 0u;
    offset_ -= rmps & (0u - is_lps);
    range_ = is_lps ? lps : rmps;
    c.e = is_lps ? e_lps : e_mps;
    renorm();
    return (u32(e >> 32) & 1u) ^ is_lps;
  }
  // §9.3.3.2.2.3. After a 1 (pcm_flag / end_of_slice_flag) the bit position is exactly the end
  // of the encoder's flush (the flush's final 1 bit included).
  u32 terminate() {
    ++nbins_;
    range_ -= 2;
    if (offset_ >= range_) return 1;
    renorm();
    return 0;
  }
  VEP_CABAC_INLINE u32 bypass() {
    ++nbins_;
    offset_ = (offset_ << 1) | bits(1);
    const u32 b = offset_ >= range_ ? 1u : 0u;  // (branch-free: signs are close to random)
    offset_ -= range_ & (0u - b);
    return b;
  }
  size_t bitpos() const { return byte_ * 8 - size_t(cbits_); }
  u64 bins() const { return nbins_; }  // bins decoded (decision + bypass + terminate)
  size_t aligned_bytepos() const { return (bitpos() + 7) >> 3; }
 private:
  VEP_CABAC_INLINE void renorm() {  // range_ in [2, 510]: shift it back to >= 256 (0 when it already is)
    const int sh = __builtin_clz(range_) - 23;
    range_ <<= sh;
    offset_ = (offset_ << sh) | bits0(sh);
  }
  VEP_CABAC_INLINE u32 bits(int k) {  // 1 <= k <= 9
    if (__builtin_expect(cbits_ < k, 0)) refill();
    const u32 v = u32(cache_ >> (64 - k));
    cache_ <<= k;
    cbits_ -= k;
    return v;
  }
  VEP_CABAC_INLINE u32 bits0(int k) {  // 0 <= k <= 8 (k = 0 reads nothing)
    if (__builtin_expect(cbits_ < k, 0)) refill();
    const u32 v = u32((cache_ >> 1) >> (63 - k));
    cache_ <<= k;
    cbits_ -= k;
    return v;
  }
  VEP_CABAC_INLINE void refill() {
    if (__builtin_expect(byte_ + 8 <= n_, 1)) {  // whole bytes that fit behind the cached bits, one load
      u64 w;
      std::memcpy(&w, p_ + byte_, 8);
      w = __builtin_bswap64(w);
      const int take = (64 - cbits_) >> 3;
      if (take < 8) w &= ~0ull << (64 - 8 * take);
      cache_ |= w >> cbits_;
      cbits_ += 8 * take;
      byte_ += size_t(take);
      return;
    }
    const Tail t = refill_tail(p_, n_, byte_, cache_, cbits_);
    byte_ = t.byte;
    cache_ = t.cache;
    cbits_ = t.cbits;
  }
  // The last bytes of the buffer, out of line (values in and out: the hot loops' register copies
  // of the decoder never have their address taken). Reading past the end yields zeros (the
  // trailing bits); the caller bounds the walk.
  struct Tail {
    size_t byte;
    u64 cache;
    int cbits;
  };
  __attribute__((noinline)) static Tail refill_tail(const u8* p, size_t n, size_t byte, u64 cache, int cbits) {
    while (cbits <= 56) {
      const u64 b = byte < n ? p[byte] : 0;
      ++byte;
      cache |= b << (56 - cbits);
      cbits += 8;
    }
    return Tail{byte, cache, cbits};
  }
  const u8* p_;
  size_t n_;
  size_t byte_ = 0;
  u64 cache_ = 0;
  int cbits_ = 0;
  u32 range_ = 510, offset_ = 0;
  u64 nbins_ = 0;  // (a register in the hot loops' local copies: off the range / offset chain)
};

// Process-wide count of bins decoded (slices add their decoder's count when they end): the parse
// benchmarks' bins per picture and cycles per bin.
inline std::atomic<u64>& bins_decoded() {
  static std::atomic<u64> n{0};
  return n;
}

// Arithmetic encoder appending to a byte-aligned RBSP buffer (§9.3.5).
class Encoder {
 public:
  explicit Encoder(std::vector<u8>& out) : out_(out) { start(); }

  void start() {  // InitEncoder: must be at a byte boundary
    VEP_CHECK(nbits_ == 0, "CABAC encoder must start byte aligned");
    low_ = 0;
    range_ = 510;
    first_ = true;
    outstanding_ = 0;
  }
  void decision(Ctx& c, u32 bin) {
    const u32 lps = Ctx::lps_of(c.e, range_);
    range_ -= lps;
    const u32 is_lps = bin != u32(c.mps()) ? 1u : 0u;
    if (is_lps) {
      low_ += range_;
      range_ = lps;
    }
    c.e = Ctx::after(c.e, is_lps);
    renorm();
  }
  void terminate(u32 bin) {
    range_ -= 2;
    if (bin) {
      low_ += range_;
      flush();
    } else {
      renorm();
    }
  }
  void bypass(u32 bin) {
    low_ <<= 1;
    if (bin) low_ += range_;
    if (low_ >= 1024) {
      put(1);
      low_ -= 1024;
    } else if (low_ < 512) {
      put(0);
    } else {
      low_ -= 512;
      ++outstanding_;
    }
  }
  // Raw bits after a flush (pcm_alignment_zero_bit, byte_alignment()).
  void align_zero() {
    while (nbits_ != 0) bit(0);
  }
  void raw_bytes(const u8* p, size_t n) {
    VEP_CHECK(nbits_ == 0, "raw bytes must be byte aligned");
    out_.insert(out_.end(), p, p + n);
  }
  bool byte_aligned() const { return nbits_ == 0; }

 private:
  void flush() {  // EncodeFlush: the final written bit is 1 (rbsp_stop_one_bit at slice end)
    range_ = 2;
    renorm();
    put((low_ >> 9) & 1);
    bit(((low_ >> 8) & 1));
    bit(1);
  }
  void renorm() {
    while (range_ < 256) {
      if (low_ < 256) {
        put(0);
      } else if (low_ >= 512) {
        low_ -= 512;
        put(1);
      } else {
        low_ -= 256;
        ++outstanding_;
      }
      range_ <<= 1;
      low_ <<= 1;
    }
  }
  void put(u32 b) {
    if (first_) {
      first_ = false;
    } else {
      bit(b);
    }
    while (outstanding_ > 0) {
      bit(1 - b);
      --outstanding_;
    }
  }
  void bit(u32 b) {
    cur_ = (cur_ << 1) | (b & 1u);
    if (++nbits_ == 8) {
      out_.push_back(u8(cur_));
      cur_ = 0;
      nbits_ = 0;
    }
  }
  std::vector<u8>& out_;
  u32 low_ = 0, range_ = 510;
  bool first_ = true;
  u32 outstanding_ = 0;
  u32 cur_ = 0;
  int nbits_ = 0;
};

}  // namespace vep::cabac
