// CAVLC code tables and the residual_block_cavlc reader/writer (ITU-T H.264 §9.2).
#include "avc_cavlc.h"

namespace vep::avc {

namespace {

// Table 9-5, index total_coeff * 4 + trailing_ones: code length / value per nC class.
const u8 kCtLen[4][4 * 17] = {
    {1,  0,  0,  0,  6,  2,  0,  0,  8,  6,  3,  0,  9,  8,  7,  5,  10, 9,  8,  6,  11, 10, 9,
     7,  13, 11, 10, 8,  13, 13, 11, 9,  13, 13, 13, 10, 14, 14, 13, 11, 14, 14, 14, 13, 15, 15,
     14, 14, 15, 15, 15, 14, 16, 15, 15, 15, 16, 16, 16, 15, 16, 16, 16, 16, 16, 16, 16, 16},
    {2,  0,  0,  0,  6,  2,  0,  0,  6,  5,  3,  0,  7,  6,  6,  4,  8,  6,  6,  4,  8,  7,  7,
     5,  9,  8,  8,  6,  11, 9,  9,  6,  11, 11, 11, 7,  12, 11, 11, 9,  12, 12, 12, 11, 12, 12,
     12, 11, 13, 13, 13, 12, 13, 13, 13, 13, 13, 14, 13, 13, 14, 14, 14, 13, 14, 14, 14, 14},
    {4, 0, 0, 0, 6, 4, 0, 0, 6, 5,  4,  0,  6,  5,  5,  4,  7,  5,  5,  4,  7,  5,  5,
     4, 7, 6, 6, 4, 7, 6, 6, 4, 8,  7,  7,  5,  8,  8,  7,  6,  9,  8,  8,  7,  9,  9,
     8, 8, 9, 9, 9, 8, 10, 9, 9, 9, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10},
    {6, 0, 0, 0, 6, 6, 0, 0, 6, 6, 6, 0, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6,
     6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6,
     6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6}};
const u8 kCtBits[4][4 * 17] = {
    {1,  0,  0,  0,  5,  1,  0,  0,  7,  4,  1,  0,  7,  6,  5,  3, 7,  6,  5, 3, 7,  6,  5,
     4,  15, 6,  5,  4,  11, 14, 5,  4,  8,  10, 13, 4,  15, 14, 9, 4,  11, 10, 13, 12, 15, 14,
     9,  12, 11, 10, 13, 8,  15, 1,  9,  12, 11, 14, 13, 8,  7,  10, 9,  12, 4,  6,  5,  8},
    {3,  0,  0,  0,  11, 2,  0,  0,  7,  7,  3,  0,  7,  10, 9,  5,  7,  6,  5,  4,  4,  6,  5,
     6,  7,  6,  5,  8,  15, 6,  5,  4,  11, 14, 13, 4,  15, 10, 9,  4,  11, 14, 13, 12, 8,  10,
     9,  8,  15, 14, 13, 12, 11, 10, 9,  12, 7,  11, 6,  8,  9,  8,  10, 1,  7,  6,  5,  4},
    {15, 0,  0,  0,  15, 14, 0,  0,  11, 15, 13, 0,  8,  12, 14, 12, 15, 10, 11, 11, 11, 8,  9,
     10, 9,  14, 13, 9,  8,  10, 9,  8,  15, 14, 13, 13, 11, 14, 10, 12, 15, 10, 13, 12, 11, 14,
     9,  12, 8,  10, 13, 8,  13, 7,  9,  12, 9,  12, 11, 10, 5,  8,  7,  6,  1,  4,  3,  2},
    {3,  0,  0,  0,  0,  1,  0,  0,  4,  5,  6,  0,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18,
     19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41,
     42, 43, 44, 45, 46, 47, 48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62, 63}};
// nC == -1 (chroma DC, 4:2:0), index total_coeff * 4 + trailing_ones.
const u8 kCdcLen[4 * 5] = {2, 0, 0, 0, 6, 1, 0, 0, 6, 6, 3, 0, 6, 7, 7, 6, 6, 8, 8, 7};
const u8 kCdcBits[4 * 5] = {1, 0, 0, 0, 7, 1, 0, 0, 4, 6, 1, 0, 3, 3, 2, 5, 2, 3, 2, 0};

// nC == -2 (chroma DC, 4:2:2: up to 8 coefficients), index total_coeff * 4 + trailing_ones.
const u8 kCdc422Len[4 * 9] = {1, 0, 0, 0, 7, 2, 0, 0, 7, 7, 3, 0, 9, 7, 7, 5, 9, 9, 7, 6,
                              10, 10, 9, 7, 11, 11, 10, 7, 12, 12, 11, 10, 13, 12, 12, 11};
const u8 kCdc422Bits[4 * 9] = {1, 0, 0, 0, 15, 1, 0, 0, 14, 13, 1, 0, 7, 12, 11, 1, 6, 5, 10, 1,
                               7, 6, 4, 9, 7, 6, 5, 8, 7, 6, 5, 4, 7, 5, 4, 4};

// Tables 9-7 / 9-8: total_zeros for 4x4 blocks, [total_coeff - 1][total_zeros].
const u8 kTzLen[15][16] = {{1, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 9},
                           {3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 6, 6, 6, 6},
                           {4, 3, 3, 3, 4, 4, 3, 3, 4, 5, 5, 6, 5, 6},
                           {5, 3, 4, 4, 3, 3, 3, 4, 3, 4, 5, 5, 5},
                           {4, 4, 4, 3, 3, 3, 3, 3, 4, 5, 4, 5},
                           {6, 5, 3, 3, 3, 3, 3, 3, 4, 3, 6},
                           {6, 5, 3, 3, 3, 2, 3, 4, 3, 6},
                           {6, 4, 5, 3, 2, 2, 3, 3, 6},
                           {6, 6, 4, 2, 2, 3, 2, 5},
                           {5, 5, 3, 2, 2, 2, 4},
                           {4, 4, 3, 3, 1, 3},
                           {4, 4, 2, 1, 3},
                           {3, 3, 1, 2},
                           {2, 2, 1},
                           {1, 1}};
const u8 kTzBits[15][16] = {{1, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 1},
                            {7, 6, 5, 4, 3, 5, 4, 3, 2, 3, 2, 3, 2, 1, 0},
                            {5, 7, 6, 5, 4, 3, 4, 3, 2, 3, 2, 1, 1, 0},
                            {3, 7, 5, 4, 6, 5, 4, 3, 3, 2, 2, 1, 0},
                            {5, 4, 3, 7, 6, 5, 4, 3, 2, 1, 1, 0},
                            {1, 1, 7, 6, 5, 4, 3, 2, 1, 1, 0},
                            {1, 1, 5, 4, 3, 3, 2, 1, 1, 0},
                            {1, 1, 1, 3, 3, 2, 2, 1, 0},
                            {1, 0, 1, 3, 2, 1, 1, 1},
                            {1, 0, 1, 3, 2, 1, 1},
                            {0, 1, 1, 2, 1, 3},
                            {0, 1, 1, 1, 1},
                            {0, 1, 1, 1},
                            {0, 1, 1},
                            {0, 1}};
// Table 9-9a: total_zeros for chroma DC 2x2, [total_coeff - 1][total_zeros].
const u8 kTzDcLen[3][4] = {{1, 2, 3, 3}, {1, 2, 2, 0}, {1, 1, 0, 0}};
const u8 kTzDcBits[3][4] = {{1, 1, 1, 0}, {1, 1, 0, 0}, {1, 0, 0, 0}};
// Table 9-9b: total_zeros for chroma DC 2x4 (4:2:2), [total_coeff - 1][total_zeros].
const u8 kTzDc422Len[7][8] = {{1, 3, 3, 4, 4, 4, 5, 5}, {3, 2, 3, 3, 3, 3, 3}, {3, 3, 2, 2, 3, 3},
                              {3, 2, 2, 2, 3}, {2, 2, 2, 2}, {2, 2, 1}, {1, 1}};
const u8 kTzDc422Bits[7][8] = {{1, 2, 3, 2, 3, 1, 1, 0}, {0, 1, 1, 4, 5, 6, 7}, {0, 1, 1, 2, 6, 7},
                               {6, 0, 1, 2, 7}, {0, 1, 2, 3}, {0, 1, 1}, {0, 1}};
// Table 9-10: run_before, [min(zeros_left, 7) - 1][run_before].
const u8 kRunLen[7][16] = {{1, 1},          {1, 2, 2},       {2, 2, 2, 2},
                           {2, 2, 2, 3, 3}, {2, 2, 3, 3, 3, 3}, {2, 3, 3, 3, 3, 3, 3},
                           {3, 3, 3, 3, 3, 3, 3, 4, 5, 6, 7, 8, 9, 10, 11}};
const u8 kRunBits[7][16] = {{1, 0},          {1, 1, 0},       {3, 2, 1, 0},
                            {3, 2, 1, 1, 0}, {3, 2, 3, 2, 1, 0}, {3, 0, 1, 3, 2, 5, 4},
                            {7, 6, 5, 4, 3, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1}};

// Single-lookup decode table: index = next `bits` bits; entry = len << 8 | value (0 = invalid).
struct Lut {
  int bits = 0;
  std::vector<u16> e;
  void init(int b) {
    bits = b;
    e.assign(size_t(1) << b, 0);
  }
  void add(int len, u32 code, int value) {
    if (len == 0) return;
    const int pad = bits - len;
    const u32 base = code << pad;
    for (u32 s = 0; s < (1u << pad); ++s) e[base | s] = u16(len << 8 | value);
  }
  int read(Bits& br) const {
    const u16 v = e[br.peek32() >> (32 - bits)];
    VEP_CHECK(v != 0, "invalid CAVLC code");
    br.skip(v >> 8);
    return v & 0xff;
  }
};

struct Tables {
  Lut ct[6];     // coeff_token classes 0-2, 4 and 5 (class 3 is a 6-bit FLC)
  Lut tz[15], tzdc[3], tzdc422[7], run[7];
  Tables() {
    const int maxlen[3] = {16, 14, 10};
    for (int c = 0; c < 3; ++c) {
      ct[c].init(maxlen[c]);
      for (int i = 0; i < 4 * 17; ++i) ct[c].add(kCtLen[c][i], kCtBits[c][i], i);
    }
    ct[4].init(8);
    for (int i = 0; i < 4 * 5; ++i) ct[4].add(kCdcLen[i], kCdcBits[i], i);
    ct[5].init(13);
    for (int i = 0; i < 4 * 9; ++i) ct[5].add(kCdc422Len[i], kCdc422Bits[i], i);
    for (int t = 0; t < 7; ++t) {
      tzdc422[t].init(5);
      for (int z = 0; z < 8 - t; ++z) tzdc422[t].add(kTzDc422Len[t][z], kTzDc422Bits[t][z], z);
    }
    for (int t = 0; t < 15; ++t) {
      tz[t].init(9);
      for (int z = 0; z < 16 - t; ++z) tz[t].add(kTzLen[t][z], kTzBits[t][z], z);
    }
    for (int t = 0; t < 3; ++t) {
      tzdc[t].init(3);
      for (int z = 0; z < 4 - t; ++z) tzdc[t].add(kTzDcLen[t][z], kTzDcBits[t][z], z);
    }
    for (int k = 0; k < 7; ++k) {
      run[k].init(11);
      const int n = k < 6 ? k + 2 : 15;
      for (int r = 0; r < n; ++r) run[k].add(kRunLen[k][r], kRunBits[k][r], r);
    }
  }
};

const Tables kTables;  // built at load time: no guard check on the hot path
inline const Tables& tables() { return kTables; }

}  // namespace

CoeffToken read_coeff_token(Bits& br, int cls) {
  if (cls == 3) {
    const u32 c = br.u(6);
    if (c == 3) return {0, 0};
    const CoeffToken t{int(c >> 2) + 1, int(c & 3)};
    VEP_CHECK(t.trailing <= t.total, "invalid coeff_token");
    return t;
  }
  const int v = tables().ct[cls].read(br);
  return {v >> 2, v & 3};
}

int read_total_zeros(Bits& br, int tc, int max_coeff) {
  if (max_coeff == 4) return tables().tzdc[tc - 1].read(br);
  if (max_coeff == 8) return tables().tzdc422[tc - 1].read(br);
  return tables().tz[tc - 1].read(br);
}

int read_run_before(Bits& br, int zeros_left) {
  return tables().run[(zeros_left < 7 ? zeros_left : 7) - 1].read(br);
}

// --------------------------------------------------------------------------------- writer

int write_residual_block(BitWriter& bw, int nc, int max_coeff, const int* coeff) {
  int pos[16], lv[16], total = 0;
  for (int k = max_coeff - 1; k >= 0; --k)  // reverse scan order: highest frequency first
    if (coeff[k] != 0) {
      pos[total] = k;
      lv[total] = coeff[k];
      ++total;
    }
  int t1 = 0;
  while (t1 < total && t1 < 3 && (lv[t1] == 1 || lv[t1] == -1)) ++t1;
  const int cls = coeff_token_class(nc);
  if (cls == 3) {
    bw.u(6, total == 0 ? 3u : u32(((total - 1) << 2) | t1));
  } else if (cls == 4) {
    bw.u(kCdcLen[total * 4 + t1], kCdcBits[total * 4 + t1]);
  } else if (cls == 5) {
    bw.u(kCdc422Len[total * 4 + t1], kCdc422Bits[total * 4 + t1]);
  } else {
    bw.u(kCtLen[cls][total * 4 + t1], kCtBits[cls][total * 4 + t1]);
  }
  if (total == 0) return 0;
  int sl = (total > 10 && t1 < 3) ? 1 : 0;
  for (int i = 0; i < total; ++i) {
    if (i < t1) {
      bw.u1(lv[i] < 0 ? 1u : 0u);
      continue;
    }
    int code = lv[i] > 0 ? 2 * lv[i] - 2 : -2 * lv[i] - 1;
    if (i == t1 && t1 < 3) code -= 2;
    int prefix, ssize, suffix;
    if (sl == 0) {
      if (code < 14) {
        prefix = code, ssize = 0, suffix = 0;
      } else if (code < 30) {
        prefix = 14, ssize = 4, suffix = code - 14;
      } else {
        prefix = 15, ssize = 12, suffix = code - 30;
      }
    } else if (code < (15 << sl)) {
      prefix = code >> sl, ssize = sl, suffix = code & ((1 << sl) - 1);
    } else {
      prefix = 15, ssize = 12, suffix = code - (15 << sl);
    }
    VEP_CHECK(suffix < (1 << 12), "level too large for the synthetic encoder");
    for (int z = 0; z < prefix; ++z) bw.u1(0);
    bw.u1(1);
    if (ssize) bw.u(ssize, u32(suffix));
    if (sl == 0) sl = 1;
    const int a = lv[i] < 0 ? -lv[i] : lv[i];
    if (a > (3 << (sl - 1)) && sl < 6) ++sl;
  }
  const int zeros = pos[0] + 1 - total;
  if (total < max_coeff) {
    if (max_coeff == 4) bw.u(kTzDcLen[total - 1][zeros], kTzDcBits[total - 1][zeros]);
    else if (max_coeff == 8) bw.u(kTzDc422Len[total - 1][zeros], kTzDc422Bits[total - 1][zeros]);
    else bw.u(kTzLen[total - 1][zeros], kTzBits[total - 1][zeros]);
  }
  int left = zeros;
  for (int i = 0; i < total - 1 && left > 0; ++i) {
    const int run = pos[i] - pos[i + 1] - 1;
    const int k = (left < 7 ? left : 7) - 1;
    bw.u(kRunLen[k][run], kRunBits[k][run]);
    left -= run;
  }
  return total;
}

}  // namespace vep::avc
