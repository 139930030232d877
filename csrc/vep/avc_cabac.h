// CABAC entropy layer of H.264 (§9.3): context initialisation tables (m, n) for the frame-coded
// 4:2:0 syntax elements, and every syntax element's binarization written once for both
// directions.
//
// `AvcBins<E>` is symmetric: E is either the arithmetic decoder adapter (bins are read, the
// value arguments are ignored) or the encoder adapter (the value arguments are written and the
// same bins come back), so the decoder (avc_mb.cpp) and the synthetic High-profile encoder
// (avc_enc_high.cpp) share one binarization and one context-selection code path.
// Context-index increments that depend on neighbouring macroblocks are derived by the caller
// (the MB layer owns the neighbour state) and passed in.
//
// Coverage: cabac_init_idc 0 (the P/B model x264 and most camera encoders use) and the I-slice
// model; streams with cabac_init_idc 1 or 2 are rejected as UnsupportedStream (their tables
// are not carried). Field / MBAFF contexts (277-398, 436-459) are not used: interlaced coding
// is rejected before slice data.
//
// Reference parity: replaces libavcodec's CABAC decoding behind PyAV (python/read_image.py:87
// `p.decode()`) for the Main/High-profile streams IP cameras send.
#pragma once

#include "cabac.h"
#include "common.h"

namespace vep::avc {

using i8 = int8_t;
constexpr int kCabacCtx = 460;

// ctxIdxInc of significant_coeff_flag / last_significant_coeff_flag for 8x8 blocks (frame
// coded), by scanning position (Table 9-43).
extern const u8 kSig8x8Frame[63];
extern const u8 kLast8x8[63];

// Residual block categories (ctxBlockCat, Table 9-42) and their context offsets.
enum BlockCat : int { kCatLumaDc = 0, kCatLumaAc = 1, kCatLuma4x4 = 2, kCatChromaDc = 3, kCatChromaAc = 4,
                      kCatLuma8x8 = 5 };
inline constexpr int kCbfCatOff[5] = {0, 4, 8, 12, 16};
inline constexpr int kSigCatOff[5] = {0, 15, 29, 44, 47};
inline constexpr int kAbsCatOff[5] = {0, 10, 20, 30, 39};

// §9.3.1.1 context initialisation for SliceQPY. `model` -1 = I slices, 0 = cabac_init_idc 0.
void cabac_init_contexts(cabac::Ctx* ctx, int model, int qp);

// Decoder adapter: bins are read; the value arguments are ignored.
struct BinDecoder {
  static constexpr bool kWrite = false;
  cabac::Decoder& d;
  cabac::Ctx* ctx;
  u32 bin(int i, u32) { return d.decision(ctx[i]); }
  u32 byp(u32) { return d.bypass(); }
  u32 term(u32) { return d.terminate(); }
};

// Encoder adapter: the value arguments are written and returned.
struct BinEncoder {
  static constexpr bool kWrite = true;
  cabac::Encoder& e;
  cabac::Ctx* ctx;
  u32 bin(int i, u32 v) {
    e.decision(ctx[i], v & 1u);
    return v & 1u;
  }
  u32 byp(u32 v) {
    e.bypass(v & 1u);
    return v & 1u;
  }
  u32 term(u32 v) {
    e.terminate(v & 1u);
    return v & 1u;
  }
};

// Syntax-element binarizations (§9.3.2) and their context selection (§9.3.3.1). Each returns
// the element's value (decoded, or the one written).
template <class E>
struct AvcBins {
  E& e;

  u32 bin(int i, bool v) { return e.bin(i, v ? 1u : 0u); }
  u32 byp(bool v) { return e.byp(v ? 1u : 0u); }

  // k-th order Exp-Golomb suffix in bypass bins (UEGk suffix, §9.3.2.3).
  int eg(int k, int v) {
    int out = 0;
    while (byp(v >= (1 << k))) {
      out += 1 << k;
      v -= 1 << k;
      ++k;
      VEP_CHECK(k < 24, "CABAC Exp-Golomb suffix too long");
    }
    while (k--) out += int(byp((v >> k) & 1)) << k;
    return out;
  }

  u32 mb_skip(bool b_slice, int inc, bool v) { return bin((b_slice ? 24 : 11) + inc, v); }
  u32 end_of_slice(bool v) { return e.term(v ? 1u : 0u); }
  u32 transform_8x8(int inc, bool v) { return bin(399 + inc, v); }

  // Intra mb_type body (Table 9-36) shared by I slices (prefix-free) and the intra suffix of
  // P/B slices: value = I-slice mb_type (0 I_NxN, 1..24 I_16x16, 25 I_PCM).
  int intra_type(int c0, int c1, int c2, int c3, int c4, int c5, int v) {
    if (!bin(c0, v != 0)) return 0;
    if (e.term(v == 25 ? 1u : 0u)) return 25;
    const int w = (v >= 1 && v <= 24) ? v - 1 : 0;
    const int vl = w / 12, vc = (w / 4) % 3, vp = w % 4;
    const int l = int(bin(c1, vl != 0));
    int c = int(bin(c2, vc != 0));
    if (c) c += int(bin(c3, vc == 2));
    int p = int(bin(c4, (vp >> 1) & 1)) << 1;
    p |= int(bin(c5, vp & 1));
    return 1 + p + 4 * c + 12 * l;
  }
  int mb_type_i(int inc, int v) { return intra_type(3 + inc, 3 + 3, 3 + 4, 3 + 5, 3 + 6, 3 + 7, v); }
  // P slices: 0 P_L0_16x16, 1 P_L0_L0_16x8, 2 P_L0_L0_8x16, 3 P_8x8; 5 + I type for intra.
  int mb_type_p(int v) {
    if (bin(14, v >= 5)) return 5 + intra_type(17, 18, 19, 19, 20, 20, v - 5);
    if (!bin(15, v == 1 || v == 2)) return bin(16, v == 3) ? 3 : 0;
    return bin(17, v == 1) ? 1 : 2;
  }
  // B slices: 0..22 (Table 7-14); 23 + I type for intra.
  int mb_type_b(int inc, int v) {
    if (!bin(27 + inc, v != 0)) return 0;
    if (!bin(27 + 3, v >= 3)) return 1 + int(bin(27 + 5, v == 2));
    int eb;
    if (v >= 3 && v <= 10) eb = v - 3;
    else if (v == 11) eb = 14;
    else if (v == 22) eb = 15;
    else if (v >= 23) eb = 13;
    else eb = (v + 4) >> 1;
    int b = int(bin(27 + 4, (eb >> 3) & 1)) << 3;
    b |= int(bin(27 + 5, (eb >> 2) & 1)) << 2;
    b |= int(bin(27 + 5, (eb >> 1) & 1)) << 1;
    b |= int(bin(27 + 5, eb & 1));
    if (b < 8) return b + 3;
    if (b == 13) return 23 + intra_type(32, 33, 34, 34, 35, 35, v - 23);
    if (b == 14) return 11;
    if (b == 15) return 22;
    b = (b << 1) | int(bin(27 + 5, (v + 4) & 1));
    return b - 4;
  }
  int sub_mb_type_p(int v) {
    if (bin(21, v == 0)) return 0;
    if (!bin(22, v != 1)) return 1;
    return bin(23, v == 2) ? 2 : 3;
  }
  int sub_mb_type_b(int v) {
    if (!bin(36, v != 0)) return 0;
    if (!bin(37, v >= 3)) return 1 + int(bin(39, v == 2));
    int t = 3;
    if (bin(38, v >= 7)) {
      if (bin(39, v >= 11)) return 11 + int(bin(39, v == 12));
      t = 7;
    }
    const int r = v - t;
    int x = int(bin(39, (r >> 1) & 1)) << 1;
    x |= int(bin(39, r & 1));
    return t + x;
  }
  int ref_idx(int inc, int v) {
    if (!bin(54 + inc, v > 0)) return 0;
    int k = 1, c = 54 + 4;
    while (bin(c, v > k)) {
      ++k;
      c = 54 + 5;
      VEP_CHECK(k < 32, "ref_idx out of range");
    }
    return k;
  }
  // base 40 (horizontal) / 47 (vertical); inc from the neighbours' absMvdComp sum.
  int mvd(int base, int inc, int v) {
    const int a = v < 0 ? -v : v;
    if (!bin(base + inc, a > 0)) return 0;
    int k = 1, c = base + 3;
    while (k < 9 && bin(c, a > k)) {
      ++k;
      if (c < base + 6) ++c;
    }
    if (k >= 9) k += eg(3, a - 9);
    return byp(v < 0) ? -k : k;
  }
  int qp_delta(int inc, int v) {
    const int m = v > 0 ? 2 * v - 1 : -2 * v;
    if (!bin(60 + inc, m > 0)) return 0;
    int k = 1, c = 60 + 2;
    while (bin(c, m > k)) {
      ++k;
      c = 60 + 3;
      VEP_CHECK(k <= 103, "mb_qp_delta out of range");
    }
    return (k & 1) ? (k + 1) / 2 : -(k / 2);
  }
  int chroma_mode(int inc, int v) {
    if (!bin(64 + inc, v > 0)) return 0;
    if (!bin(64 + 3, v > 1)) return 1;
    return bin(64 + 3, v > 2) ? 3 : 2;
  }
  u32 prev_intra_flag(bool v) { return bin(68, v); }
  int rem_intra_mode(int v) {
    int r = int(bin(69, v & 1));
    r |= int(bin(69, (v >> 1) & 1)) << 1;
    r |= int(bin(69, (v >> 2) & 1)) << 2;
    return r;
  }
  u32 cbp_luma_bin(int inc, bool v) { return bin(73 + inc, v); }
  u32 cbp_chroma_bin(int inc, bool v) { return bin(77 + inc, v); }

  // residual_block_cabac (§7.3.5.3.3): coef[0 .. n-1] levels in scan order. Read: only the
  // non-zero entries are written (the caller need not clear `coef`); write: the levels to code.
  // `nzpos` receives the scan positions of the non-zero levels (ascending). cbf_inc < 0:
  // coded_block_flag not coded (8x8 luma blocks of 4:2:0). Returns the number of non-zero levels.
  int residual(int cat, int cbf_inc, int n, int* coef, u8* nzpos) {
    int last_nz = -1;
    if constexpr (E::kWrite)
      for (int i = 0; i < n; ++i)
        if (coef[i]) last_nz = i;
    if (cbf_inc >= 0 && !bin(85 + kCbfCatOff[cat] + cbf_inc, last_nz >= 0)) return 0;
    const bool b8 = cat == kCatLuma8x8;
    int num = 0, i = 0;
    if (b8) {
      for (; i < 63; ++i) {
        if (bin(402 + kSig8x8Frame[i], E::kWrite && coef[i] != 0)) {
          nzpos[num++] = u8(i);
          if (bin(417 + kLast8x8[i], i == last_nz)) break;
        }
      }
    } else {
      const int sig_base = 105 + kSigCatOff[cat], last_base = 166 + kSigCatOff[cat];
      const bool cdc = cat == kCatChromaDc;
      const int dsh = n == 8 ? 1 : 0;  // chroma DC: ctxIdxInc = Min(i / NumC8x8, 2) (4:2:2: NumC8x8 2)
      for (; i < n - 1; ++i) {
        const int si = cdc ? ((i >> dsh) < 2 ? (i >> dsh) : 2) : i;
        if (bin(sig_base + si, E::kWrite && coef[i] != 0)) {
          nzpos[num++] = u8(i);
          if (bin(last_base + si, i == last_nz)) break;
        }
      }
    }
    if (i == n - 1) nzpos[num++] = u8(n - 1);
    const int abs_base = b8 ? 426 : 227 + kAbsCatOff[cat];
    const int gt1_max = cat == kCatChromaDc ? 3 : 4;
    int gt1 = 0, eq1 = 0;
    for (int k = num - 1; k >= 0; --k) {
      const int p = nzpos[k];
      const int c = E::kWrite ? coef[p] : 0;
      const int a = (c < 0 ? -c : c) - 1;
      int v = 0;
      if (bin(abs_base + (gt1 != 0 ? 0 : (eq1 + 1 < 4 ? eq1 + 1 : 4)), a > 0)) {
        v = 1;
        const int cx = abs_base + 5 + (gt1 < gt1_max ? gt1 : gt1_max);
        while (v < 14 && bin(cx, a > v)) ++v;
        if (v >= 14) v += eg(0, a - 14);
      }
      const int level = v + 1;
      if (level == 1) ++eq1;
      else ++gt1;
      coef[p] = byp(c < 0) ? -level : level;
    }
    return num;
  }
};

// Decoder direction of residual_block_cabac, the parse hot loop (most bins of a High-profile
// picture): same bins, same context selection as the generic body above, with the arithmetic
// decoder held in a local copy so range/offset/bit cache stay in registers across the context
// byte updates (see cabac.h). One instantiation per block category: the context bases, the
// scan length and the 8x8 / chroma DC special cases are constants of the loop.
template <int CAT>
inline int residual_dec(cabac::Ctx* const ctx, cabac::Decoder& engine, int cbf_inc, int n_dc, int* coef,
                        u8* nzpos) {
  constexpr bool b8 = CAT == kCatLuma8x8, cdc = CAT == kCatChromaDc;
  // (chroma DC: 4 or, in 4:2:2, 8 coefficients; the others are fixed)
  constexpr int kN = CAT == kCatLumaAc || CAT == kCatChromaAc ? 15 : (b8 ? 64 : 16);
  const int n = cdc ? n_dc : kN;
  cabac::Decoder d = engine;
  // (cbf_inc < 0: no coded_block_flag — the 8x8 blocks of 4:2:0)
  if (!b8 && cbf_inc >= 0 && !d.decision(ctx[85 + kCbfCatOff[b8 ? 0 : CAT] + cbf_inc])) {
    engine = d;
    return 0;
  }
  int num = 0, i = 0;
  if constexpr (b8) {
    cabac::Ctx* const sig = ctx + 402;
    cabac::Ctx* const last = ctx + 417;
    for (; i < 63; ++i)
      if (d.decision(sig[kSig8x8Frame[i]])) {
        nzpos[num++] = u8(i);
        if (d.decision(last[kLast8x8[i]])) break;
      }
  } else {
    cabac::Ctx* const sig = ctx + 105 + kSigCatOff[CAT];
    cabac::Ctx* const last = ctx + 166 + kSigCatOff[CAT];
    if constexpr (cdc) {
      const int dsh = n == 8 ? 1 : 0;  // Min(i / NumC8x8, 2): 4:2:2 has NumC8x8 = 2
      for (; i < n - 1; ++i) {
        const int si = (i >> dsh) < 2 ? (i >> dsh) : 2;
        if (d.decision(sig[si])) {
          nzpos[num++] = u8(i);
          if (d.decision(last[si])) break;
        }
      }
    } else {
      for (; i < kN - 1; ++i)
        if (d.decision(sig[i])) {
          nzpos[num++] = u8(i);
          if (d.decision(last[i])) break;
        }
    }
  }
  if (i == n - 1) nzpos[num++] = u8(n - 1);
  cabac::Ctx* const absc = ctx + (b8 ? 426 : 227 + kAbsCatOff[b8 ? 0 : CAT]);
  constexpr int gt1_max = cdc ? 3 : 4;
  int gt1 = 0, eq1 = 0;
  for (int k = num - 1; k >= 0; --k) {
    int level = 1;
    if (d.decision(absc[gt1 != 0 ? 0 : (eq1 < 3 ? eq1 + 1 : 4)])) {
      cabac::Ctx& cx = absc[5 + (gt1 < gt1_max ? gt1 : gt1_max)];
      int v = 1;
      while (v < 14 && d.decision(cx)) ++v;
      if (v >= 14) {  // UEG0 suffix
        int kk = 0;
        while (d.bypass()) {
          v += 1 << kk;
          ++kk;
          VEP_CHECK(kk < 24, "CABAC Exp-Golomb suffix too long");
        }
        while (kk--) v += int(d.bypass()) << kk;
      }
      level = v + 1;
      ++gt1;
    } else {
      ++eq1;
    }
    const int neg = -int(d.bypass());  // coeff_sign_flag: 0 / -1
    coef[nzpos[k]] = (level ^ neg) - neg;
  }
  engine = d;
  return num;
}

template <>
inline int AvcBins<BinDecoder>::residual(int cat, int cbf_inc, int n, int* coef, u8* nzpos) {
  switch (cat) {
    case kCatLumaDc: return residual_dec<kCatLumaDc>(e.ctx, e.d, cbf_inc, n, coef, nzpos);
    case kCatLumaAc: return residual_dec<kCatLumaAc>(e.ctx, e.d, cbf_inc, n, coef, nzpos);
    case kCatLuma4x4: return residual_dec<kCatLuma4x4>(e.ctx, e.d, cbf_inc, n, coef, nzpos);
    case kCatChromaDc: return residual_dec<kCatChromaDc>(e.ctx, e.d, cbf_inc, n, coef, nzpos);
    case kCatChromaAc: return residual_dec<kCatChromaAc>(e.ctx, e.d, cbf_inc, n, coef, nzpos);
    default: return residual_dec<kCatLuma8x8>(e.ctx, e.d, cbf_inc, n, coef, nzpos);
  }
}

// Decoder direction of mvd_lX (UEG3, signed, uCoff 9), the second-largest bin consumer of P/B
// pictures; local engine copy as above.
template <>
inline int AvcBins<BinDecoder>::mvd(int base, int inc, int) {
  cabac::Ctx* const ctx = e.ctx;
  cabac::Decoder d = e.d;
  if (!d.decision(ctx[base + inc])) {
    e.d = d;
    return 0;
  }
  int k = 1, c = base + 3;
  while (k < 9 && d.decision(ctx[c])) {
    ++k;
    if (c < base + 6) ++c;
  }
  if (k >= 9) {  // UEG3 suffix
    int kk = 3;
    while (d.bypass()) {
      k += 1 << kk;
      ++kk;
      VEP_CHECK(kk < 24, "CABAC Exp-Golomb suffix too long");
    }
    while (kk--) k += int(d.bypass()) << kk;
  }
  const int r = d.bypass() ? -k : k;
  e.d = d;
  return r;
}

}  // namespace vep::avc
