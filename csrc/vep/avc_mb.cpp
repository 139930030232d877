// Generic H.264 macroblock layer (§7.3.5, §7.4.5, §8.4.1, §8.4.2.3, §8.5, §9.2, §9.3): I, P and B
// macroblocks in CAVLC and CABAC slices, Intra 4x4 / 8x8 / 16x16 and I_PCM, every inter
// partition and sub-partition shape, spatial and temporal direct prediction (B_Skip,
// B_Direct_16x16, B_Direct_8x8), explicit and implicit weighted prediction, 4x4 and 8x8
// transforms with scaling matrices. Output: MbState (neighbour / colocated state) and the
// MbRec + dequantised coefficient blocks + motion vectors + weights the reconstruction kernels
// consume (avc.h).
//
// The fast CAVLC path for Baseline-style slices (avc.cpp MbDecoder, fused nC cache) stays the
// default for those; this layer takes every slice that needs anything beyond it.
//
// Reference parity: libavcodec's h264 macroblock decoding behind PyAV `packet.decode()`
// (python/read_image.py:87).
#include <algorithm>
#include <memory>
#include <cstddef>
#include <cstring>

#include "avc_cabac.h"
#include "avc_cavlc.h"
#include "avc_internal.h"

namespace vep::avc {

namespace {

// LevelScale4x4 / LevelScale8x8 (§8.5.9, §8.5.13.1): weightScale (scaling list, raster) times
// normAdjust, per list and qP % 6.
struct Dequant {
  int ls4[6][6][16];  // [Intra Y, Cb, Cr, Inter Y, Cb, Cr][m][raster]
  int ls8[2][6][64];  // [Intra Y, Inter Y][m][raster]
  explicit Dequant(const h264::ScalingLists& sl) {
    for (int l = 0; l < 6; ++l)
      for (int m = 0; m < 6; ++m)
        for (int k = 0; k < 16; ++k) {
          const int pos = kZigzag4x4[k];
          ls4[l][m][pos] = int(sl.l4[l][k]) * norm_adjust(m, pos >> 2, pos & 3);
        }
    for (int l = 0; l < 2; ++l)
      for (int m = 0; m < 6; ++m)
        for (int k = 0; k < 64; ++k) {
          const int pos = kZigzag8x8[k];
          ls8[l][m][pos] = int(sl.l8[l][k]) * norm_adjust8(m, pos >> 3, pos & 7);
        }
  }
};

// The LevelScale tables of the slice's scaling lists, rebuilt only when they change (per parse
// thread: nearly every stream keeps one set of lists).
const Dequant& dequant_for(const h264::ScalingLists& sl) {
  thread_local h264::ScalingLists last;
  thread_local std::unique_ptr<Dequant> dq;
  if (!dq || std::memcmp(&last, &sl, sizeof sl) != 0) {
    dq = std::make_unique<Dequant>(sl);
    last = sl;
  }
  return *dq;
}

inline int scale4(int c, int ls, int qp) {
  return qp >= 24 ? (c * ls) * (1 << (qp / 6 - 4)) : (c * ls + (1 << (3 - qp / 6))) >> (4 - qp / 6);
}
inline int scale8(int c, int ls, int qp) {
  return qp >= 36 ? (c * ls) * (1 << (qp / 6 - 6)) : (c * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
}

// B mb_type 0..22 (Table 7-14): prediction flags (bit 0 list 0, bit 1 list 1) per partition.
constexpr u8 kBPart[23][2] = {{0, 0}, {1, 0}, {2, 0}, {3, 0}, {1, 1}, {1, 1}, {2, 2}, {2, 2},
                              {1, 2}, {1, 2}, {2, 1}, {2, 1}, {1, 3}, {1, 3}, {2, 3}, {2, 3},
                              {3, 1}, {3, 1}, {3, 2}, {3, 2}, {3, 3}, {3, 3}, {0, 0}};
// B sub_mb_type 0..12 (Table 7-18): prediction flags, sub-partition shape (0 8x8, 1 8x4, 2 4x8,
// 3 4x4). P sub_mb_type 0..3 is list 0 with shape = value.
constexpr u8 kBSub[13][2] = {{0, 0}, {1, 0}, {2, 0}, {3, 0}, {1, 1}, {1, 2}, {2, 1},
                             {2, 2}, {3, 1}, {3, 2}, {1, 3}, {2, 3}, {3, 3}};
constexpr int kSubParts[4] = {1, 2, 2, 4};

inline int raster_b8(int blk) { return ((blk >> 3) << 1) | ((blk & 3) >> 1); }
inline u16 b8_blocks(int b8) { return u16(0x33u << ((b8 & 1) * 2 + (b8 >> 1) * 8)); }
inline int clip3i(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }

// kCabac: entropy mode; kWrite: encoder direction (values come from `want` and are written;
// every context derivation, predictor and record is the decoder's).
template <bool kCabac, bool kWrite>
class MbLayer {
  using Bins = std::conditional_t<kWrite, AvcBins<BinEncoder>, AvcBins<BinDecoder>>;

 public:
  MbLayer(MbNeighbours& nb, Picture& pic, const SliceEnv& env, const Dequant& dq)
      : nb_(nb), pic_(pic), env_(env), sh_(*env.sh), pps_(*env.pps), sps_(*env.sps), dq_(dq),
        scan4_(env.field ? kFieldScan4x4 : kZigzag4x4), scan8_(env.field ? kFieldScan8x8 : kZigzag8x8) {
    type_ = sh_.type();
    qp_ = sh_.qp;
    bd_ = sps_.bit_depth_luma;
    qpbd_ = 6 * (sps_.bit_depth_luma - 8);
    qpbdc_ = 6 * (sps_.bit_depth_chroma - 8);
    cf_ = sps_.chroma_format_idc;
    nbc_ = cf_ == 2 ? 8 : 4;
    weighted_ = (type_ == h264::kP && pps_.weighted_pred) || (type_ == h264::kB && pps_.weighted_bipred_idc != 0);
    implicit_ = type_ == h264::kB && pps_.weighted_bipred_idc == 2;
    // per-slice lookup tables of emit(): DPB slot by (refIdx + 1) per list (0xFF: refIdx -1 or
    // no such list entry), QP'C of both chroma components by QP'Y
    for (int l = 0; l < 2; ++l) {
      std::fill(std::begin(slot_[l]), std::end(slot_[l]), u8(0xFF));
      if (const auto* lst = env_.list[l])
        for (size_t k = 0; k < lst->size() && k + 1 < std::size(slot_[l]); ++k)
          if ((*lst)[k].slot >= 0) slot_[l][k + 1] = u8((*lst)[k].slot);
    }
    for (int q = 0; q < 52 + qpbd_ && q < int(std::size(qpc_tab_[0])); ++q) {
      qpc_tab_[0][q] = u8(chroma_qp_bd(q - qpbd_, pps_.chroma_qp_index_offset, qpbdc_) + qpbdc_);
      qpc_tab_[1][q] = u8(chroma_qp_bd(q - qpbd_, pps_.second_chroma_qp_index_offset, qpbdc_) + qpbdc_);
    }
    // B_Skip / B_Direct_16x16 take direct16_spatial() (no weights, spatial, 8x8 inference)
    fast_direct_ = !kWrite && type_ == h264::kB && sh_.direct_spatial && sps_.direct_8x8 && !weighted_;
  }

  // entropy sources / sinks (the ones of the mode are used)
  Bits* br = nullptr;            // CAVLC read
  BitWriter* bw = nullptr;       // CAVLC write
  Bins* bins = nullptr;          // CABAC
  cabac::Decoder* cabac = nullptr;  // CABAC read (I_PCM repositioning)
  cabac::Encoder* cenc = nullptr;   // CABAC write (I_PCM raw bytes)
  const MbDesc* want = nullptr;     // write mode: the macroblock being written
  int prev_qpd_nz = 0;  // mb_qp_delta of the previous MB in decoding order != 0 (CABAC context)

  int qp() const { return qp_; }

  // CAVLC primitives in both directions
  int ue(u32 v) {
    if constexpr (kWrite) {
      bw->ue(v);
      return int(v);
    } else {
      return int(br->ue());
    }
  }
  int se(int v) {
    if constexpr (kWrite) {
      bw->se(v);
      return v;
    } else {
      return br->se();
    }
  }
  int u(int n, u32 v) {
    if constexpr (kWrite) {
      bw->u(n, v);
      return int(v);
    } else {
      return int(br->u(n));
    }
  }

  // MbState{} except the motion vectors (a skipped MB writes every vector a reader can look at:
  // list 0 for P_Skip — list 1 of a P slice is never read — and both lists for B_Skip; a coded
  // MB clears them in coded_mb())
  static void clear_but_mv(MbState& s) {
    static const MbState z{};
    std::memcpy(static_cast<void*>(&s), &z, offsetof(MbState, mv));
    std::memcpy(static_cast<void*>(&s.mvd), &z.mvd, sizeof(MbState) - offsetof(MbState, mvd));
  }

  bool read_skip_flag(int mb, bool v = false) {
    MbState& s = nb_.at(mb);
    if constexpr (kWrite) s = MbState{};
    else clear_but_mv(s);
    s.slice = u16(env_.slice);
    nb_.begin(mb);
    auto cond = [&](int m) { return m >= 0 && !nb_.at(m).skip ? 1 : 0; };
    const int inc = cond(nb_.mb_at(mb, -1, 0)) + cond(nb_.mb_at(mb, 0, -1));
    return bins->mb_skip(type_ == h264::kB, inc, v) != 0;
  }

  void skip_mb(int mb, bool fresh) {
    MbState& s = nb_.at(mb);
    if (fresh) {
      s = MbState{};
      s.slice = u16(env_.slice);
      nb_.begin(mb);
    }
    s.kind = kSkip;
    s.skip = 1;
    s.qp = u8(qp_ + qpbd_);
    MbResidual res;
    res.luma = 0;
    res.chroma = 0;
    if (type_ == h264::kP) {
      s.ref[0][0] = s.ref[0][1] = s.ref[0][2] = s.ref[0][3] = 0;
      need_ref(0, 0);
      int mv[2];
      nb_.pskip_mv(mb, mv);
      for (auto& v : s.mv[0]) {
        v[0] = i16(mv[0]);
        v[1] = i16(mv[1]);
      }
    } else {
      s.direct16 = 1;
      s.direct8 = 0xF;
      if (fast_direct_) direct16_spatial(mb, s);
      else direct(mb, s, 0xF);
    }
    prev_qpd_nz = 0;
    if (!weighted_ && !kWrite) emit_skip(mb, s);
    else emit(mb, s, res, 0, 0, nullptr);
  }

  void coded_mb(int mb, bool fresh) {
    MbState& s = nb_.at(mb);
    if (fresh) {
      s = MbState{};
      s.slice = u16(env_.slice);
      nb_.begin(mb);
    } else if constexpr (!kWrite) {
      std::memset(static_cast<void*>(s.mv), 0, sizeof s.mv);  // (read_skip_flag() left them)
    }
    int mbt = read_mb_type(mb, kWrite ? want->mb_type : 0);
    int itype = -1;
    if (type_ == h264::kI) {
      itype = mbt;
    } else if (type_ == h264::kP) {
      VEP_CHECK(mbt <= 30, "bad P mb_type");
      if (mbt >= 5) itype = mbt - 5;
    } else {
      VEP_CHECK(mbt <= 48, "bad B mb_type");
      if (mbt >= 23) itype = mbt - 23;
    }
    VEP_CHECK(itype <= 25, "bad intra mb_type");
    MbResidual res;
    res.luma = 0;
    res.chroma = 0;
    if (itype == 25) {
      pcm_mb(mb, s, res);
      return;
    }
    int cbp = 0, i16_mode = 0;
    const bool intra = itype >= 0;
    bool no_small = true;  // noSubMbPartSizeLessThan8x8Flag
    if (itype == 0) {
      if (pps_.transform_8x8_mode) s.t8x8 = u8(read_t8x8(mb, kWrite && want->t8x8));
      s.kind = s.t8x8 ? kI8x8 : kI4x4;
      intra_modes(mb, s);
      s.chroma_mode = u8(read_chroma_mode(mb, kWrite ? want->chroma_mode : 0));
    } else if (itype > 0) {
      s.kind = kI16x16;
      i16_mode = (itype - 1) % 4;
      cbp = (((itype - 1) / 4) % 3) << 4 | (itype >= 13 ? 15 : 0);
      std::fill(std::begin(s.i4), std::end(s.i4), u8(2));
      s.chroma_mode = u8(read_chroma_mode(mb, kWrite ? want->chroma_mode : 0));
      VEP_CHECK(!mono() || (cbp >> 4) == 0, "4:0:0: Intra_16x16 type with chroma coefficients");
    } else {
      s.kind = kInter;
      no_small = inter_pred(mb, s, mbt);
    }
    VEP_CHECK(s.chroma_mode <= 3, "bad intra_chroma_pred_mode");
    if (s.kind != kI16x16) cbp = read_cbp(mb, s, intra, kWrite ? want->cbp : 0);
    s.cbp = u8(cbp);
    if (s.kind == kInter && (cbp & 15) && pps_.transform_8x8_mode && no_small &&
        !(type_ == h264::kB && mbt == 0 && !sps_.direct_8x8))
      s.t8x8 = u8(read_t8x8(mb, kWrite && want->t8x8));
    int qp = qp_;
    if ((cbp & 15) || (cbp >> 4) || s.kind == kI16x16) {
      const int dqp = read_qp_delta(kWrite ? want->qp_delta : 0);
      VEP_CHECK(dqp >= -(26 + qpbd_ / 2) && dqp <= 25 + qpbd_ / 2, "mb_qp_delta out of range");
      qp = (qp + dqp + 52 + 2 * qpbd_) % (52 + qpbd_) - qpbd_;  // (7-37: QPY in -QpBdOffsetY..51)
      prev_qpd_nz = dqp != 0;
    } else {
      prev_qpd_nz = 0;
    }
    qp_ = qp;
    s.qp = u8(qp + qpbd_);
    residual(mb, s, res, cbp & 15, cbp >> 4, qp + qpbd_, intra);
    emit(mb, s, res, i16_mode, s.chroma_mode, nullptr);
  }

  // Motion a skipped MB at `mb` would get (encoder decisions): P_Skip or B_Skip / direct.
  void skip_motion(int mb, MbState& out) {
    MbState& s = nb_.at(mb);
    s = MbState{};
    s.slice = u16(env_.slice);
    nb_.begin(mb);
    out = MbState{};
    out.slice = s.slice;
    if (type_ == h264::kP) {
      for (int k = 0; k < 4; ++k) out.ref[0][k] = 0;
      int mv[2];
      nb_.pskip_mv(mb, mv);
      for (auto& v : out.mv[0]) {
        v[0] = i16(mv[0]);
        v[1] = i16(mv[1]);
      }
    } else {
      direct(mb, out, 0xF);
    }
    s = MbState{};  // (the MB is written later)
  }

  // Pictures the slice's MBs reference (list entries that must exist).
  void need_ref(int list, int idx) {  // (slot_: the list's entries with a picture)
    VEP_CHECK(idx >= 0 && idx < 32 && slot_[list][idx + 1] != 0xFF, "ref_idx names a missing reference picture");
  }

 private:
  // ------------------------------------------------------------------ syntax elements
  int read_mb_type(int mb, int v) {
    if constexpr (kCabac) {
      if (type_ == h264::kI) {
        auto cond = [&](int m) {
          if (m < 0) return 0;
          const u8 k = nb_.at(m).kind;
          return (k == kI4x4 || k == kI8x8) ? 0 : 1;
        };
        return bins->mb_type_i(cond(nb_.mb_at(mb, -1, 0)) + cond(nb_.mb_at(mb, 0, -1)), v);
      }
      if (type_ == h264::kP) return bins->mb_type_p(v);
      auto cond = [&](int m) { return m >= 0 && !nb_.at(m).direct16 ? 1 : 0; };
      return bins->mb_type_b(cond(nb_.mb_at(mb, -1, 0)) + cond(nb_.mb_at(mb, 0, -1)), v);
    } else {
      return ue(u32(v));
    }
  }
  int read_t8x8(int mb, bool v) {
    if constexpr (kCabac) {
      auto cond = [&](int m) { return m >= 0 && nb_.at(m).t8x8 ? 1 : 0; };
      return int(bins->transform_8x8(cond(nb_.mb_at(mb, -1, 0)) + cond(nb_.mb_at(mb, 0, -1)), v));
    } else {
      return u(1, v ? 1u : 0u);
    }
  }
  int read_chroma_mode(int mb, int v) {
    if (mono()) return 0;  // 4:0:0: no intra_chroma_pred_mode (the grey planes stay 128)
    if constexpr (kCabac) {
      auto cond = [&](int m) {
        if (m < 0) return 0;
        const MbState& n = nb_.at(m);
        return is_intra(n.kind) && n.kind != kIPcm && n.chroma_mode != 0 ? 1 : 0;
      };
      return bins->chroma_mode(cond(nb_.mb_at(mb, -1, 0)) + cond(nb_.mb_at(mb, 0, -1)), v);
    } else {
      return ue(u32(v));
    }
  }
  int read_mode(int pred, int v) {  // prev_intra{4x4,8x8}_pred_mode_flag + rem
    const bool same = v == pred;
    const int rem_v = v < pred ? v : v - 1;
    if constexpr (kCabac) {
      if (bins->prev_intra_flag(same)) return pred;
      const int rem = bins->rem_intra_mode(rem_v);
      return rem < pred ? rem : rem + 1;
    } else {
      if (u(1, same ? 1u : 0u)) return pred;
      const int rem = u(3, u32(rem_v));
      return rem < pred ? rem : rem + 1;
    }
  }
  int read_sub_type(int v) {
    if constexpr (kCabac) return type_ == h264::kB ? bins->sub_mb_type_b(v) : bins->sub_mb_type_p(v);
    else return ue(u32(v));
  }
  int read_ref(int mb, int list, int x4, int y4, int v) {
    const int n = sh_.num_ref_idx[list];
    if (n <= 1) return 0;
    int r;
    if constexpr (kCabac) {
      auto cond = [&](int x, int y) {
        const int m = nb_.mb_at(mb, x, y);
        if (m < 0) return 0;
        const MbState& nbs = nb_.at(m);
        if (m != mb && (nbs.skip || is_intra(nbs.kind))) return 0;
        const int b8 = (((y & 15) >> 3) << 1) | ((x & 15) >> 3);
        if ((nbs.direct8 >> b8) & 1) return 0;
        return nbs.ref[list][b8] > 0 ? 1 : 0;
      };
      r = bins->ref_idx(cond(x4 * 4 - 1, y4 * 4) + 2 * cond(x4 * 4, y4 * 4 - 1), v);
    } else {
      if (n == 2) r = u(1, v ? 0u : 1u) ^ 1;
      else r = ue(u32(v));
    }
    VEP_CHECK(r < n, "ref_idx out of range");
    need_ref(list, r);
    return r;
  }
  int read_mvd(int mb, int list, int x4, int y4, int comp, int v) {
    if constexpr (kCabac) {
      auto am = [&](int x, int y) -> int {
        const int m = nb_.mb_at(mb, x, y);
        if (m < 0) return 0;
        const MbState& n = nb_.at(m);
        return n.mvd[list][((y & 15) >> 2) * 4 + ((x & 15) >> 2)][comp];
      };
      const int sum = am(x4 * 4 - 1, y4 * 4) + am(x4 * 4, y4 * 4 - 1);
      return bins->mvd(comp ? 47 : 40, sum < 3 ? 0 : (sum > 32 ? 2 : 1), v);
    } else {
      return se(v);
    }
  }
  int read_cbp(int mb, const MbState& s, bool intra, int v) {
    if constexpr (kCabac) {
      const int am = nb_.mb_at(mb, -1, 0), bm = nb_.mb_at(mb, 0, -1);
      int luma = 0;
      for (int b8 = 0; b8 < 4; ++b8) {
        auto cond = [&](int m, int nb8, bool cur) {
          if (cur) return ((luma >> nb8) & 1) ? 0 : 1;
          if (m < 0) return 0;
          return ((nb_.at(m).cbp >> nb8) & 1) ? 0 : 1;
        };
        const int ca = (b8 & 1) ? cond(mb, b8 - 1, true) : cond(am, b8 + 1, false);
        const int cb = (b8 & 2) ? cond(mb, b8 - 2, true) : cond(bm, b8 + 2, false);
        luma |= int(bins->cbp_luma_bin(ca + 2 * cb, (v >> b8) & 1)) << b8;
      }
      auto cc = [&](int m, int thr) { return m >= 0 && (nb_.at(m).cbp >> 4) >= thr ? 1 : 0; };
      const int vc = v >> 4;
      int chroma = 0;
      if (!mono() && bins->cbp_chroma_bin(cc(am, 1) + 2 * cc(bm, 1), vc != 0))
        chroma = 1 + int(bins->cbp_chroma_bin(4 + cc(am, 2) + 2 * cc(bm, 2), vc == 2));
      (void)s;
      (void)intra;
      return luma | chroma << 4;
    } else {
      (void)mb;
      (void)s;
      // (4:0:0: the 16-entry luma-only mapping of Table 9-4)
      static constexpr u8 kIntraMono[16] = {15, 0, 7, 11, 13, 14, 3, 5, 10, 12, 1, 2, 4, 8, 6, 9};
      static constexpr u8 kInterMono[16] = {0, 1, 2, 4, 8, 3, 5, 10, 12, 15, 7, 11, 13, 14, 6, 9};
      const u32 n = mono() ? 16 : 48;
      const u8* tab = mono() ? (intra ? kIntraMono : kInterMono) : (intra ? kCbpIntra : kCbpInter);
      u32 code = 0;
      if constexpr (kWrite)
        while (code < n && tab[code] != v) ++code;
      const u32 me = u32(ue(code));
      VEP_CHECK(me < n, "bad coded_block_pattern");
      return tab[me];
    }
  }
  int read_qp_delta(int v) {
    if constexpr (kCabac) return bins->qp_delta(prev_qpd_nz ? 1 : 0, v);
    else return se(v);
  }

  // ------------------------------------------------------------------ I_PCM
  void pcm_mb(int mb, MbState& s, MbResidual& res) {
    s.kind = kIPcm;
    s.cbp = 0x2F;
    s.cbf = 0xFFFF;
    s.cbf_dc = 7;
    s.cbf_cac[0] = s.cbf_cac[1] = u8((1u << nbc_) - 1);
    std::fill(std::begin(s.tc), std::end(s.tc), u8(16));
    for (auto& c : s.tcc) std::fill(std::begin(c), std::end(c), u8(16));
    s.qp = u8(qp_ + qpbd_);
    const u8* pcm;
    const size_t nb = mono() ? 256 : pcm_samples();  // (4:0:0: luma samples only)
    if (bd_ > 8 || cf_ == 2) {  // High 10 / 4:2:2: bd-bit samples (u(v)), kept as u16 / u8 in the record
      pcm_wide(mb, s, res, nb);
      return;
    }
    if constexpr (kWrite) {
      pcm = want->pcm;
      VEP_CHECK(pcm, "I_PCM macroblock without samples");
      if constexpr (kCabac) {
        cenc->align_zero();  // pcm_alignment_zero_bit (the terminate bin flushed the engine)
        cenc->raw_bytes(pcm, nb);
        cenc->start();
      } else {
        bw->align_zero();
        bw->bytes(pcm, nb);
      }
    } else if constexpr (kCabac) {
      const size_t off = cabac->aligned_bytepos();
      VEP_CHECK(off + nb <= data_n, "truncated I_PCM macroblock");
      pcm = data + off;
      cabac->start(off + nb);
    } else {
      br->align();
      const size_t off = br->pos() >> 3;
      VEP_CHECK(off + nb <= br->size(), "truncated I_PCM macroblock");
      pcm = br->data() + off;
      br->skip(nb * 8);
    }
    if (mono()) {  // the record's chroma samples: grey
      std::memcpy(pcm_mono_, pcm, 256);
      std::memset(pcm_mono_ + 256, 128, kPcmMbBytes - 256);
      pcm = pcm_mono_;
    }
    prev_qpd_nz = 0;
    emit(mb, s, res, 0, 0, pcm);
  }

  // Samples of an I_PCM MB in the record: 384 (4:2:0 / 4:0:0), 512 (4:2:2).
  size_t pcm_samples() const { return cf_ == 2 ? size_t(kPcmMaxSamples) : size_t(kPcmMbBytes); }
  // I_PCM above 8 bits or in 4:2:2: ns samples of bd_ bits (luma, then Cb, then Cr), byte-aligned
  // at both ends (ns * bd_ is a multiple of 8). want->pcm: u16 samples above 8 bits, else bytes.
  // The record holds u16 samples above 8 bits, bytes at 8 bits.
  void pcm_wide(int mb, MbState& s, MbResidual& res, size_t ns) {
    const size_t nbytes = ns * size_t(bd_) / 8, total = pcm_samples();
    if constexpr (kWrite) {
      VEP_CHECK(want->pcm, "I_PCM macroblock without samples");
      const u16* src16 = reinterpret_cast<const u16*>(want->pcm);
      for (size_t i = 0; i < total; ++i)
        pcm16_[i] = i < ns ? (bd_ > 8 ? src16[i] : u16(want->pcm[i])) : u16(1 << (bd_ - 1));
      BitWriter w;
      for (size_t i = 0; i < ns; ++i) w.u(bd_, pcm16_[i]);
      VEP_CHECK(w.buf().size() == nbytes, "I_PCM sample block size");
      if constexpr (kCabac) {
        cenc->align_zero();
        cenc->raw_bytes(w.buf().data(), nbytes);
        cenc->start();
      } else {
        bw->align_zero();
        bw->bytes(w.buf().data(), nbytes);
      }
    } else {
      const u8* p;
      if constexpr (kCabac) {
        const size_t off = cabac->aligned_bytepos();
        VEP_CHECK(off + nbytes <= data_n, "truncated I_PCM macroblock");
        p = data + off;
        cabac->start(off + nbytes);
      } else {
        br->align();
        const size_t off = br->pos() >> 3;
        VEP_CHECK(off + nbytes <= br->size(), "truncated I_PCM macroblock");
        p = br->data() + off;
        br->skip(nbytes * 8);
      }
      BitReader r(p, nbytes);
      for (size_t i = 0; i < total; ++i) pcm16_[i] = i < ns ? u16(r.u(bd_)) : u16(1 << (bd_ - 1));
    }
    prev_qpd_nz = 0;
    if (bd_ > 8) {
      emit(mb, s, res, 0, 0, reinterpret_cast<const u8*>(pcm16_));
    } else {
      for (size_t i = 0; i < total; ++i) pcm8_[i] = u8(pcm16_[i]);
      emit(mb, s, res, 0, 0, pcm8_);
    }
  }

  bool mono() const { return sps_.chroma_format_idc == 0; }
  u8 pcm_mono_[kPcmMbBytes];
  u16 pcm16_[kPcmMaxSamples];
  u8 pcm8_[kPcmMaxSamples];
  int bd_ = 8, qpbd_ = 0, qpbdc_ = 0;  // bit depth, QpBdOffsetY / C (High 10)
  int cf_ = 1, nbc_ = 4;               // chroma_format_idc, chroma 4x4 blocks per component

 public:
  const u8* data = nullptr;  // CABAC: slice RBSP (I_PCM samples are read in place)
  size_t data_n = 0;

 private:
  // ------------------------------------------------------------------ intra modes
  void intra_modes(int mb, MbState& s) {
    const bool ci = pps_.constrained_intra_pred;
    if (s.t8x8) {
      for (int b8 = 0; b8 < 4; ++b8) {
        const int m = read_mode(nb_.pred_intra8x8(mb, b8, ci), kWrite ? want->ipred[b8] : 0);
        VEP_CHECK(m <= 8, "Intra_8x8 mode out of range");
        for (u16 w = b8_blocks(b8); w; w &= w - 1) s.i4[__builtin_ctz(w)] = u8(m);
      }
    } else {
      for (int idx = 0; idx < 16; ++idx) {
        const int r = blk_to_raster(idx);
        s.i4[r] = u8(read_mode(nb_.pred_intra4x4(mb, r, ci), kWrite ? want->ipred[r] : 0));
        VEP_CHECK(s.i4[r] <= 8, "Intra_4x4 mode out of range");
      }
    }
  }

  // ------------------------------------------------------------------ inter prediction
  struct Part {
    int x4, y4, w4, h4, shape;
  };
  static u16 part_mask(const Part& p) {
    static constexpr u16 kRows[5] = {0, 0x1, 0x11, 0x111, 0x1111};  // bit 0 of h4 rows
    return u16((((1u << p.w4) - 1u) << p.x4) * kRows[p.h4] << (4 * p.y4));
  }
  static void set_mvd(MbState& s, int list, const Part& p, int dx, int dy) {
    const u8 ax = u8(std::min(dx < 0 ? -dx : dx, 127)), ay = u8(std::min(dy < 0 ? -dy : dy, 127));
    for (int y = p.y4; y < p.y4 + p.h4; ++y)
      for (int x = p.x4; x < p.x4 + p.w4; ++x) {
        s.mvd[list][y * 4 + x][0] = ax;
        s.mvd[list][y * 4 + x][1] = ay;
      }
  }
  static void set_mv(MbState& s, int list, const Part& p, int mx, int my) {
    VEP_CHECK(mx >= -32768 && mx <= 32767 && my >= -32768 && my <= 32767, "motion vector out of range");
    for (int y = p.y4; y < p.y4 + p.h4; ++y)
      for (int x = p.x4; x < p.x4 + p.w4; ++x) {
        s.mv[list][y * 4 + x][0] = i16(mx);
        s.mv[list][y * 4 + x][1] = i16(my);
      }
  }

  // Returns noSubMbPartSizeLessThan8x8Flag.
  bool inter_pred(int mb, MbState& s, int mbt) {
    const bool b = type_ == h264::kB;
    if (b && mbt == 0) {  // B_Direct_16x16
      s.direct16 = 1;
      s.direct8 = 0xF;
      if (fast_direct_) direct16_spatial(mb, s);
      else direct(mb, s, 0xF);
      return true;
    }
    if ((!b && mbt <= 2) || (b && mbt <= 21)) {
      Part parts[2];
      int np;
      u8 pred[2];
      int shape;
      if (!b) {
        shape = mbt;  // 0 16x16, 1 16x8, 2 8x16
        pred[0] = pred[1] = 1;
      } else {
        shape = mbt <= 3 ? 0 : ((mbt & 1) ? 2 : 1);
        pred[0] = kBPart[mbt][0];
        pred[1] = kBPart[mbt][1];
      }
      np = shape == 0 ? 1 : 2;
      for (int i = 0; i < np; ++i) {
        if (shape == 0) parts[i] = {0, 0, 4, 4, 0};
        else if (shape == 1) parts[i] = {0, 2 * i, 4, 2, 1};
        else parts[i] = {2 * i, 0, 2, 4, 2};
      }
      int refs[2][2] = {{-1, -1}, {-1, -1}};
      for (int l = 0; l < 2; ++l)
        for (int i = 0; i < np; ++i) {
          if (!((pred[i] >> l) & 1)) continue;
          refs[l][i] = read_ref(mb, l, parts[i].x4, parts[i].y4, kWrite ? want->ref[l][i] : 0);
          const Part& p = parts[i];
          for (int y = p.y4 / 2; y < (p.y4 + p.h4) / 2; ++y)
            for (int x = p.x4 / 2; x < (p.x4 + p.w4) / 2; ++x) s.ref[l][y * 2 + x] = i8(refs[l][i]);
        }
      int mvd[2][2][2] = {};
      if constexpr (kWrite) {  // the decoder's predictors in decoding order give the mvds to code
        for (int l = 0; l < 2; ++l) {
          u16 done = 0;
          for (int i = 0; i < np; ++i) {
            if (!((pred[i] >> l) & 1)) continue;
            const Part& p = parts[i];
            int mvp[2];
            nb_.pred_mv(mb, p.x4, p.y4, p.w4, p.h4, l, refs[l][i], done, p.shape, mvp);
            const i16* w = want->mv[l][p.y4 * 4 + p.x4];
            mvd[l][i][0] = w[0] - mvp[0];
            mvd[l][i][1] = w[1] - mvp[1];
            set_mv(s, l, p, w[0], w[1]);
            done |= part_mask(p);
          }
        }
      }
      for (int l = 0; l < 2; ++l)
        for (int i = 0; i < np; ++i) {
          if (!((pred[i] >> l) & 1)) continue;
          mvd[l][i][0] = read_mvd(mb, l, parts[i].x4, parts[i].y4, 0, mvd[l][i][0]);
          mvd[l][i][1] = read_mvd(mb, l, parts[i].x4, parts[i].y4, 1, mvd[l][i][1]);
          set_mvd(s, l, parts[i], mvd[l][i][0], mvd[l][i][1]);
        }
      if constexpr (!kWrite) {
        for (int l = 0; l < 2; ++l) {
          u16 done = 0;
          for (int i = 0; i < np; ++i) {
            if (!((pred[i] >> l) & 1)) continue;
            const Part& p = parts[i];
            int mvp[2];
            nb_.pred_mv(mb, p.x4, p.y4, p.w4, p.h4, l, refs[l][i], done, p.shape, mvp);
            set_mv(s, l, p, mvp[0] + mvd[l][i][0], mvp[1] + mvd[l][i][1]);
            done |= part_mask(p);
          }
        }
      }
      return true;
    }
    // P_8x8 / P_8x8ref0 / B_8x8
    int sub[4];
    bool no_small = true;
    for (int i = 0; i < 4; ++i) {
      sub[i] = read_sub_type(kWrite ? want->sub[i] : 0);
      VEP_CHECK(sub[i] <= (b ? 12 : 3), "bad sub_mb_type");
    }
    u8 spred[4], sshape[4];
    for (int i = 0; i < 4; ++i) {
      if (b) {
        spred[i] = kBSub[sub[i]][0];
        sshape[i] = kBSub[sub[i]][1];
        if (sub[i] == 0) {
          s.direct8 |= u8(1u << i);
          if (!sps_.direct_8x8) no_small = false;
        }
      } else {
        spred[i] = 1;
        sshape[i] = u8(sub[i]);
      }
      if (sshape[i] != 0) no_small = false;
    }
    for (int l = 0; l < 2; ++l)
      for (int i = 0; i < 4; ++i) {
        if (!((spred[i] >> l) & 1)) continue;
        const int r = (!b && mbt == 4) ? 0 : read_ref(mb, l, (i & 1) * 2, (i >> 1) * 2, kWrite ? want->ref[l][i] : 0);
        if (!b && mbt == 4) need_ref(0, 0);
        s.ref[l][i] = i8(r);
      }
    int mvd[2][4][4][2] = {};
    auto sub_part = [&](int i, int j) -> Part {
      const int x8 = (i & 1) * 2, y8 = (i >> 1) * 2;
      switch (sshape[i]) {
        case 0: return {x8, y8, 2, 2, 0};
        case 1: return {x8, y8 + j, 2, 1, 0};
        case 2: return {x8 + j, y8, 1, 2, 0};
        default: return {x8 + (j & 1), y8 + (j >> 1), 1, 1, 0};
      }
    };
    // motion in 8x8 order (direct 8x8s included, so later sub-partitions predict from them);
    // write mode derives the mvds to code here, before the mvd syntax
    auto derive = [&](bool write) {
      if (s.direct8) direct(mb, s, s.direct8);
      u16 done[2] = {0, 0};
      for (int i = 0; i < 4; ++i) {
        if ((s.direct8 >> i) & 1) {
          done[0] |= b8_blocks(i);
          done[1] |= b8_blocks(i);
          continue;
        }
        for (int l = 0; l < 2; ++l) {
          if (!((spred[i] >> l) & 1)) continue;
          for (int j = 0; j < kSubParts[sshape[i]]; ++j) {
            const Part p = sub_part(i, j);
            int mvp[2];
            nb_.pred_mv(mb, p.x4, p.y4, p.w4, p.h4, l, s.ref[l][i], done[l], 0, mvp);
            if (write) {
              const i16* w = want->mv[l][p.y4 * 4 + p.x4];
              mvd[l][i][j][0] = w[0] - mvp[0];
              mvd[l][i][j][1] = w[1] - mvp[1];
            }
            set_mv(s, l, p, mvp[0] + mvd[l][i][j][0], mvp[1] + mvd[l][i][j][1]);
            done[l] |= part_mask(p);
          }
        }
        done[0] |= b8_blocks(i);
        done[1] |= b8_blocks(i);
      }
    };
    if constexpr (kWrite) derive(true);
    for (int l = 0; l < 2; ++l)
      for (int i = 0; i < 4; ++i) {
        if (!((spred[i] >> l) & 1)) continue;
        for (int j = 0; j < kSubParts[sshape[i]]; ++j) {
          const Part p = sub_part(i, j);
          mvd[l][i][j][0] = read_mvd(mb, l, p.x4, p.y4, 0, mvd[l][i][j][0]);
          mvd[l][i][j][1] = read_mvd(mb, l, p.x4, p.y4, 1, mvd[l][i][j][1]);
          set_mvd(s, l, p, mvd[l][i][j][0], mvd[l][i][j][1]);
        }
      }
    if constexpr (!kWrite) derive(false);
    return no_small;
  }

  // ------------------------------------------------------------------ direct prediction
  // Motion of the 8x8 blocks in `mask` by the slice's direct mode (§8.4.1.2). Spatial mode uses
  // the whole MB's neighbours (identical for every 8x8), temporal mode the colocated picture.
  void direct(int mb, MbState& s, int mask) {
    VEP_CHECK(env_.list[1] && !env_.list[1]->empty() && (*env_.list[1])[0].slot >= 0,
              "direct prediction without a list-1 reference");
    const ListEntry& c1 = (*env_.list[1])[0];
    const ColMotion* col = c1.col;
    VEP_CHECK(col && col->wmbs == nb_.wmbs() && col->hmbs == nb_.hmbs() && col->corners == sps_.direct_8x8,
              "colocated picture motion missing");
    // direct_8x8_inference: every 4x4 block of an 8x8 takes the motion derived from the 8x8's
    // outer corner block of the colocated MB, i.e. one derivation per 8x8
    const bool infer = sps_.direct_8x8;
    auto fill = [&](int l, int b8, int blk, int mx, int my) {
      if (!infer) {
        s.mv[l][blk][0] = i16(mx);
        s.mv[l][blk][1] = i16(my);
        return;
      }
      for (u16 w = b8_blocks(b8); w; w &= w - 1) {
        const int k = __builtin_ctz(w);
        s.mv[l][k][0] = i16(mx);
        s.mv[l][k][1] = i16(my);
      }
    };
    if (sh_.direct_spatial) {
      int ref[2], mvp[2][2];
      for (int l = 0; l < 2; ++l) nb_.direct_spatial_pred(mb, l, ref[l], mvp[l]);
      const bool zero = ref[0] < 0 && ref[1] < 0;
      if (zero) ref[0] = ref[1] = 0;
      for (int l = 0; l < 2; ++l)
        if (ref[l] >= 0) need_ref(l, ref[l]);
      for (int b8 = 0; b8 < 4; ++b8) {
        if (!((mask >> b8) & 1)) continue;
        for (int l = 0; l < 2; ++l) s.ref[l][b8] = i8(ref[l]);
        for (u16 w = infer ? u16(1u << ((b8 & 1) * 2 + (b8 >> 1) * 8)) : b8_blocks(b8); w; w &= w - 1) {
          const int blk = __builtin_ctz(w);
          const ColMotion::Blk& cb = col->b[col->index(mb, blk)];
          const bool col_zero = !c1.long_term && cb.ref == 0 && cb.mv[0] >= -1 && cb.mv[0] <= 1 && cb.mv[1] >= -1 &&
                                cb.mv[1] <= 1;
          for (int l = 0; l < 2; ++l) {
            const bool use = ref[l] >= 0 && !zero && !(ref[l] == 0 && col_zero);
            fill(l, b8, blk, use ? mvp[l][0] : 0, use ? mvp[l][1] : 0);
          }
        }
      }
      return;
    }
    // temporal (§8.4.1.2.3)
    const auto& l0 = *env_.list[0];
    for (int b8 = 0; b8 < 4; ++b8) {
      if (!((mask >> b8) & 1)) continue;
      int r0 = 0;
      for (u16 w = infer ? u16(1u << ((b8 & 1) * 2 + (b8 >> 1) * 8)) : b8_blocks(b8); w; w &= w - 1) {
        const int blk = __builtin_ctz(w);
        const ColMotion::Blk& cb = col->b[col->index(mb, blk)];
        int mvc[2] = {0, 0};
        r0 = 0;
        if (cb.ref >= 0) {
          mvc[0] = cb.mv[0];
          mvc[1] = cb.mv[1];
          r0 = -1;
          for (size_t k = 0; k < l0.size() && r0 < 0; ++k)
            if (l0[k].slot >= 0 && l0[k].uid == cb.pid) r0 = int(k);
          if (r0 < 0) r0 = 0;  // the colocated reference is gone (non-conforming): conceal
        }
        need_ref(0, r0);
        const ListEntry& p0 = l0[size_t(r0)];
        int m0[2], m1[2];
        const int td = clip3i(-128, 127, c1.poc - p0.poc);
        if (td == 0 || p0.long_term) {
          m0[0] = mvc[0];
          m0[1] = mvc[1];
          m1[0] = m1[1] = 0;
        } else {
          const int tb = clip3i(-128, 127, env_.cur_poc - p0.poc);
          const int tx = (16384 + std::abs(td / 2)) / td;
          const int dsf = clip3i(-1024, 1023, (tb * tx + 32) >> 6);
          for (int k = 0; k < 2; ++k) {
            m0[k] = (dsf * mvc[k] + 128) >> 8;
            m1[k] = m0[k] - mvc[k];
          }
        }
        fill(0, b8, blk, clip3i(-32768, 32767, m0[0]), clip3i(-32768, 32767, m0[1]));
        fill(1, b8, blk, clip3i(-32768, 32767, m1[0]), clip3i(-32768, 32767, m1[1]));
      }
      s.ref[0][b8] = i8(r0);
      s.ref[1][b8] = 0;
    }
  }

  // direct() for the whole MB (mask 0xF) in the slices fast_direct_ names: spatial mode with
  // direct_8x8_inference, so each 8x8 takes its outer corner's colocated block and the four 4x4
  // blocks of an 8x8 share one vector. Same derivation as direct(); both lists' neighbour motion
  // in one fetch, the colocated picture checked once per slice, vectors written as words.
  void direct16_spatial(int mb, MbState& s) {
    if (!dcol_) {  // (the checks of direct(), on the slice's first direct MB)
      VEP_CHECK(env_.list[1] && !env_.list[1]->empty() && (*env_.list[1])[0].slot >= 0,
                "direct prediction without a list-1 reference");
      const ListEntry& c1 = (*env_.list[1])[0];
      VEP_CHECK(c1.col && c1.col->wmbs == nb_.wmbs() && c1.col->hmbs == nb_.hmbs() && c1.col->corners,
                "colocated picture motion missing");
      dcol_ = c1.col;
      dcol_long_ = c1.long_term;
    }
    int ref[2], mvp[2][2];
    nb_.direct_spatial_both(ref, mvp);
    const bool zero = ref[0] < 0 && ref[1] < 0;
    if (zero) ref[0] = ref[1] = 0;
    u32 pv[2];
    for (int l = 0; l < 2; ++l) {
      if (ref[l] >= 0) need_ref(l, ref[l]);
      const bool use = ref[l] >= 0 && !zero;
      pv[l] = use ? (u32(u16(mvp[l][0])) | u32(u16(mvp[l][1])) << 16) : 0u;
      std::memset(s.ref[l], ref[l], 4);
    }
    const ColMotion::Blk* cb = &dcol_->b[size_t(mb) * 4];
    u32 v8[2][4];
    for (int b8 = 0; b8 < 4; ++b8) {
      const bool col_zero = !dcol_long_ && cb[b8].ref == 0 && cb[b8].mv[0] >= -1 && cb[b8].mv[0] <= 1 &&
                            cb[b8].mv[1] >= -1 && cb[b8].mv[1] <= 1;
      for (int l = 0; l < 2; ++l) v8[l][b8] = (ref[l] == 0 && col_zero) ? 0u : pv[l];
    }
    for (int l = 0; l < 2; ++l) {
      u32 row[2][4];  // the two rows of 4x4 blocks an 8x8 row spans: (b8 0, 0, 1, 1)
      for (int h = 0; h < 2; ++h) {
        row[h][0] = row[h][1] = v8[l][2 * h];
        row[h][2] = row[h][3] = v8[l][2 * h + 1];
      }
      u8* mv = reinterpret_cast<u8*>(&s.mv[l][0][0]);
      for (int y = 0; y < 4; ++y) std::memcpy(mv + 16 * y, row[y >> 1], 16);
    }
  }

  // ------------------------------------------------------------------ weighted prediction
  WpEntry weights(int r0, int r1) { return wp_entry(env_, r0, r1); }

  // ------------------------------------------------------------------ residual
  // coded_block_flag context increments (§9.3.3.1.1.9).
  int cbf_luma_inc(int mb, int blk, bool intra) {
    auto cond = [&](int m, int nblk) -> int {
      if (m < 0) return intra ? 1 : 0;
      const MbState& n = nb_.at(m);
      if (n.kind == kIPcm) return 1;
      if (n.skip) return 0;
      if (!((n.cbp >> raster_b8(nblk)) & 1)) return 0;
      if (n.t8x8) return 1;
      return (n.cbf >> nblk) & 1;
    };
    const int bx = blk & 3, by = blk >> 2;
    const int a = bx > 0 ? cond(mb, blk - 1) : cond(nb_.mb_at(mb, -1, 0), blk + 3);
    const int b = by > 0 ? cond(mb, blk - 4) : cond(nb_.mb_at(mb, 0, -1), blk + 12);
    return a + 2 * b;
  }
  int cbf_dc_inc(int mb, int bit, bool intra) {  // bit 0 luma DC, 1 Cb DC, 2 Cr DC
    auto cond = [&](int m) -> int {
      if (m < 0) return intra ? 1 : 0;
      const MbState& n = nb_.at(m);
      if (n.kind == kIPcm) return 1;
      if (bit == 0) return n.kind == kI16x16 ? (n.cbf_dc & 1) : 0;
      if (n.skip || (n.cbp >> 4) == 0) return 0;
      return (n.cbf_dc >> bit) & 1;
    };
    return cond(nb_.mb_at(mb, -1, 0)) + 2 * cond(nb_.mb_at(mb, 0, -1));
  }
  int cbf_cac_inc(int mb, int c, int b, bool intra) {
    auto cond = [&](int m, int nb2, bool cur) -> int {
      if (cur) return (nb_.at(mb).cbf_cac[c] >> nb2) & 1;
      if (m < 0) return intra ? 1 : 0;
      const MbState& n = nb_.at(m);
      if (n.kind == kIPcm) return 1;
      if (n.skip || (n.cbp >> 4) != 2) return 0;
      return (n.cbf_cac[c] >> nb2) & 1;
    };
    const int bx = b & 1, by = b >> 1;
    const int a = bx ? cond(mb, b - 1, true) : cond(nb_.mb_at(mb, -1, 0), b + 1, false);
    const int bb = by ? cond(mb, b - 2, true) : cond(nb_.mb_at(mb, 0, -1), b + nbc_ - 2, false);
    return a + 2 * bb;
  }

  // One residual block: its non-zero levels lv[nzpos[j]] (scan order positions, j < the
  // returned TotalCoeff; other entries of lv are unspecified when reading). Write mode: the
  // levels of `src` are coded.
  int read_block(int cat, int cbf_inc, int nc, int n, int* lv, u8* nzpos, const int* src) {
    if constexpr (kWrite) std::memcpy(lv, src, size_t(n) * sizeof(int));
    (void)src;
    if constexpr (kCabac) {
      (void)nc;
      return bins->residual(cat, cbf_inc, n, lv, nzpos);
    } else {
      (void)cat;
      (void)cbf_inc;
      int t = 0;
      if constexpr (kWrite) {
        for (int k = 0; k < n; ++k)
          if (lv[k]) nzpos[t++] = u8(k);
        write_residual_block(*bw, nc, n, lv);
        return t;
      } else {
        read_residual_block_cb(*br, nc, n, [&](int k, int l) {
          lv[k] = l;
          nzpos[t++] = u8(k);
        });
        return t;
      }
    }
  }

  void residual(int mb, MbState& s, MbResidual& res, int cbp_luma, int cbp_chroma, int qp, bool intra) {
    const int ly = intra ? 0 : 3;
    const int q6 = qp / 6, qm = qp % 6;
    int lv[64];
    u8 nzp[64];
    if (s.kind == kI16x16) {
      const int inc = kCabac ? cbf_dc_inc(mb, 0, true) : 0;
      const int nc = kCabac ? 0 : nb_.nc_luma(mb, 0);
      int dcy[16] = {};
      const int tdc = read_block(kCatLumaDc, inc, nc, 16, lv, nzp, kWrite ? want->dc : nullptr);
      if (tdc > 0) {
        s.cbf_dc |= 1;
        int c[16] = {};
        for (int j = 0; j < tdc; ++j) c[scan4_[nzp[j]]] = lv[nzp[j]];
        hadamard4x4(c);
        const int ls = dq_.ls4[ly][qm][0];
        for (int k = 0; k < 16; ++k)
          dcy[k] = qp >= 36 ? c[k] * ls * (1 << (q6 - 6)) : (c[k] * ls + (1 << (5 - q6))) >> (6 - q6);
      }
      for (int idx = 0; idx < 16; ++idx) {
        const int r = blk_to_raster(idx);
        i16* d = res.blk[r];
        bool nz = dcy[r] != 0;
        std::memset(d, 0, 16 * sizeof(i16));
        d[0] = sat16(dcy[r]);
        if (cbp_luma) {
          const int binc = kCabac ? cbf_luma_inc(mb, r, true) : 0;
          const int bnc = kCabac ? 0 : nb_.nc_luma(mb, r);
          const int tc = read_block(kCatLumaAc, binc, bnc, 15, lv, nzp, kWrite ? want->ac[r] : nullptr);
          for (int j = 0; j < tc; ++j) {
            const int k = nzp[j];
            const int pos = scan4_[k + 1];
            const int v = scale4(lv[k], dq_.ls4[ly][qm][pos], qp);
            d[pos] = sat16(v);
            nz |= v != 0;
          }
          s.tc[r] = u8(tc);
          if (tc) s.cbf |= u16(1u << r);
        }
        if (nz) res.luma |= u16(1u << r);
      }
    } else if (s.t8x8) {
      res.t8 = true;
      const int l8 = intra ? 0 : 1;
      for (int b8 = 0; b8 < 4; ++b8) {
        if (!((cbp_luma >> b8) & 1)) continue;
        i16* d = res.b8[b8];
        std::memset(d, 0, 64 * sizeof(i16));
        bool nz = false;
        int total = 0;
        auto put = [&](int k, int level) {  // k: 8x8 scan position
          const int pos = scan8_[k];
          const int v = scale8(level, dq_.ls8[l8][qm][pos], qp);
          d[pos] = sat16(v);
          nz |= v != 0;
        };
        if constexpr (kCabac) {
          total = read_block(kCatLuma8x8, -1, 0, 64, lv, nzp, kWrite ? want->l8[b8] : nullptr);
          for (int j = 0; j < total; ++j) put(nzp[j], lv[nzp[j]]);
          for (u16 w = b8_blocks(b8); w; w &= w - 1) s.tc[__builtin_ctz(w)] = u8(std::min(total, 16));
        } else {
          for (int i4 = 0; i4 < 4; ++i4) {  // CAVLC: four interleaved 4x4 scans
            const int r = blk_to_raster(b8 * 4 + i4);
            int part[16] = {};
            if constexpr (kWrite)
              for (int k = 0; k < 16; ++k) part[k] = want->l8[b8][4 * k + i4];
            const int tc = read_block(kCatLuma4x4, 0, nb_.nc_luma(mb, r), 16, lv, nzp, part);
            s.tc[r] = u8(tc);
            total += tc;
            for (int j = 0; j < tc; ++j) put(4 * nzp[j] + i4, lv[nzp[j]]);
          }
        }
        if (total) {
          s.cbf |= b8_blocks(b8);
          nz8_ |= b8_blocks(b8);
        }
        if (nz) res.luma |= b8_blocks(b8);
      }
    } else {
      for (int idx = 0; idx < 16; ++idx) {
        const int r = blk_to_raster(idx);
        if (!((cbp_luma >> (idx >> 2)) & 1)) continue;
        const int binc = kCabac ? cbf_luma_inc(mb, r, intra) : 0;
        const int bnc = kCabac ? 0 : nb_.nc_luma(mb, r);
        const int tc = read_block(kCatLuma4x4, binc, bnc, 16, lv, nzp, kWrite ? want->ac[r] : nullptr);
        s.tc[r] = u8(tc);
        if (!tc) continue;
        s.cbf |= u16(1u << r);
        i16* d = res.blk[r];
        std::memset(d, 0, 16 * sizeof(i16));
        bool nz = false;
        for (int j = 0; j < tc; ++j) {
          const int k = nzp[j];
          const int pos = scan4_[k];
          const int v = scale4(lv[k], dq_.ls4[ly][qm][pos], qp);
          d[pos] = sat16(v);
          nz |= v != 0;
        }
        if (nz) res.luma |= u16(1u << r);
      }
    }
    if (cbp_chroma) {
      // (qp = QP'Y; QP'C = QPC + QpBdOffsetC, QPC from QPY, Table 8-15)
      const int qpc[2] = {chroma_qp_bd(qp - qpbd_, pps_.chroma_qp_index_offset, qpbdc_) + qpbdc_,
                          chroma_qp_bd(qp - qpbd_, pps_.second_chroma_qp_index_offset, qpbdc_) + qpbdc_};
      const int nbc = nbc_;  // chroma 4x4 blocks per component (4:2:2: 8, 2 wide x 4 tall)
      int dcv[2][8] = {};
      for (int c = 0; c < 2; ++c) {
        const int inc = kCabac ? cbf_dc_inc(mb, 1 + c, intra) : 0;
        int v8[8];
        // (CAVLC nC -1 / -2: the 4:2:0 / 4:2:2 chroma DC coeff_token tables)
        const int t = read_block(kCatChromaDc, inc, cf_ == 2 ? -2 : -1, nbc, v8, nzp, kWrite ? want->cdc[c] : nullptr);
        if (t > 0) {
          s.cbf_dc |= u8(2 << c);
          int u[8] = {0, 0, 0, 0, 0, 0, 0, 0};
          for (int j = 0; j < t; ++j) u[nzp[j]] = v8[nzp[j]];
          if (cf_ == 2) {  // 2x4 DC at qP,DC = QP'C + 3 (§8.5.11.2)
            const int qpdc = qpc[c] + 3;
            chroma422_dc(u, qpdc, dq_.ls4[ly + 1 + c][qpdc % 6][0], dcv[c]);
          } else {
            const int f[4] = {u[0] + u[1] + u[2] + u[3], u[0] - u[1] + u[2] - u[3], u[0] + u[1] - u[2] - u[3],
                              u[0] - u[1] - u[2] + u[3]};
            const int ls = dq_.ls4[ly + 1 + c][qpc[c] % 6][0];
            for (int b = 0; b < 4; ++b) dcv[c][b] = ((f[b] * ls) * (1 << (qpc[c] / 6))) >> 5;
          }
        }
      }
      for (int c = 0; c < 2; ++c) {
        const int lc = ly + 1 + c;
        for (int b = 0; b < nbc; ++b) {  // (4:2:2: the two 8x8s top to bottom, raster 2x2 in each)
          i16* d = res.blk[16 + c * nbc + b];
          bool nz = dcv[c][b] != 0;
          std::memset(d, 0, 16 * sizeof(i16));
          d[0] = sat16(dcv[c][b]);
          if (cbp_chroma & 2) {
            const int binc = kCabac ? cbf_cac_inc(mb, c, b, intra) : 0;
            const int bnc = kCabac ? 0 : nb_.nc_chroma(mb, c, b, nbc);
            const int tc = read_block(kCatChromaAc, binc, bnc, 15, lv, nzp, kWrite ? want->cac[c][b] : nullptr);
            s.tcc[c][b] = u8(tc);
            if (tc) s.cbf_cac[c] |= u8(1u << b);
            for (int j = 0; j < tc; ++j) {
              const int k = nzp[j];
              const int pos = scan4_[k + 1];
              const int v = scale4(lv[k], dq_.ls4[lc][qpc[c] % 6][pos], qpc[c]);
              d[pos] = sat16(v);
              nz |= v != 0;
            }
          }
          if (nz) res.chroma |= u16(1u << (c * nbc + b));
        }
      }
    }
    if constexpr (!kCabac && !kWrite) VEP_CHECK(!br->overrun(), "slice data overrun");
  }

  // ------------------------------------------------------------------ MbRec
  void emit(int mb, const MbState& s, const MbResidual& res, int i16_mode, int chroma_mode, const u8* pcm) {
    MbRec m{};
    m.kind = s.kind;
    // (biased by QpBdOffset: Picture::qp_bias / qpc_bias; I_PCM: QPY 0)
    m.qp = u8(s.kind == kIPcm ? qpbd_ : s.qp);
    VEP_CHECK(m.qp < std::size(qpc_tab_[0]), "macroblock QP out of range");
    m.qpc = qpc_tab_[0][m.qp];
    m.qpc2 = qpc_tab_[1][m.qp];
    m.i16_mode = u8(i16_mode);
    m.chroma_mode = u8(chroma_mode);
    m.dbk = u8((sh_.disable_deblocking == 1 ? 1 : 0) | (sh_.disable_deblocking == 2 ? 2 : 0));
    m.alpha_off = i8(sh_.alpha_off);
    m.beta_off = i8(sh_.beta_off);
    m.slice = s.slice;
    m.flags = s.t8x8 && s.kind != kI8x8 ? kMbT8x8 : 0;
    if (s.kind == kI8x8) m.flags = kMbT8x8;
    bool l1 = false;
    const bool intra = is_intra(s.kind);
    for (int k = 0; k < 4; ++k) {
      // (refIdx -1..31 by construction: read_ref() / direct() checked the entry exists)
      m.ref[k] = intra ? u8(0xFF) : slot_[0][s.ref[0][k] + 1];
      m.ref1[k] = intra ? u8(0xFF) : slot_[1][s.ref[1][k] + 1];
      l1 |= !intra && s.ref[1][k] >= 0;
    }
    if (l1) m.flags |= kMbL1;
    // deblocking bS 2: 4x4 blocks with coefficients (8x8 transform: all blocks of the 8x8)
    u16 nz = 0;
    if (s.t8x8) {
      nz = nz8_;
      if (!kCabac)
        for (int b8 = 0; b8 < 4; ++b8) {
          bool any = false;
          for (u16 w = b8_blocks(b8); w; w &= w - 1) any |= s.tc[__builtin_ctz(w)] != 0;
          if (any) nz |= b8_blocks(b8);
        }
    } else {
      nz = s.cbf;  // (4x4 transforms: the coded_block_flag bits are exactly the blocks with levels;
                   // I_PCM: all set, as its total_coeff 16)
    }
    nz8_ = 0;
    m.nz = nz;
    if (s.kind == kI4x4)
      for (int r = 0; r < 16; ++r) m.i4[r >> 1] |= u8(s.i4[r] << ((r & 1) * 4));
    if (s.kind == kI8x8)
      for (int b8 = 0; b8 < 4; ++b8) m.i4[b8 >> 1] |= u8(s.i4[(b8 & 1) * 2 + (b8 >> 1) * 8] << ((b8 & 1) * 4));
    WpEntry wp[4];
    bool use_wp = false;
    if (weighted_ && !is_intra(s.kind)) {
      for (int k = 0; k < 4; ++k) {
        wp[k] = weights(s.ref[0][k], s.ref[1][k]);
        const WpEntry& e = wp[k];
        for (int c = 0; c < 3; ++c)
          use_wp |= !(e.lwd[c] == 0 && e.w0[c] == 1 && e.w1[c] == 1 && e.o[c] == 0) &&
                    !(e.w0[c] == (1 << e.lwd[c]) && e.w1[c] == (1 << e.lwd[c]) && e.o[c] == 0);
      }
      if (use_wp) m.flags |= kMbWp;
    }
    store_mb(pic_, mb, m, s, &res, pcm, use_wp ? wp : nullptr);
  }

  // emit() of a skipped MB without weights: the record's header straight from the slice tables
  void emit_skip(int mb, const MbState& s) {
    MbRec m{};
    m.kind = kSkip;
    m.qp = s.qp;
    VEP_CHECK(m.qp < std::size(qpc_tab_[0]), "macroblock QP out of range");
    m.qpc = qpc_tab_[0][m.qp];
    m.qpc2 = qpc_tab_[1][m.qp];
    m.dbk = u8((sh_.disable_deblocking == 1 ? 1 : 0) | (sh_.disable_deblocking == 2 ? 2 : 0));
    m.alpha_off = i8(sh_.alpha_off);
    m.beta_off = i8(sh_.beta_off);
    m.slice = s.slice;
    bool l1 = false;
    for (int k = 0; k < 4; ++k) {
      m.ref[k] = slot_[0][s.ref[0][k] + 1];
      m.ref1[k] = slot_[1][s.ref[1][k] + 1];
      l1 |= s.ref[1][k] >= 0;
    }
    m.flags = l1 ? kMbL1 : 0;
    nz8_ = 0;
    store_skip_mb(pic_, mb, m, s);
  }

  MbNeighbours& nb_;
  Picture& pic_;
  const SliceEnv& env_;
  const SliceHdr& sh_;
  const h264::Pps& pps_;
  const h264::Sps& sps_;
  const Dequant& dq_;
  const u8* scan4_;  // 4x4 scan: zig-zag (frame) or field
  const u8* scan8_;  // 8x8 scan
  int type_ = 0;
  int qp_ = 26;
  bool weighted_ = false, implicit_ = false;
  u16 nz8_ = 0;  // CABAC 8x8 blocks with coefficients (current MB)
  u8 slot_[2][33];     // DPB slot by refIdx + 1 per list (0xFF: none)
  u8 qpc_tab_[2][96];  // QP'C (Cb, Cr) by QP'Y
  bool fast_direct_ = false;
  const ColMotion* dcol_ = nullptr;  // direct16_spatial(): the checked colocated motion
  bool dcol_long_ = false;
};

}  // namespace

// WpEntry of an 8x8 partition with reference indices (r0, r1) (-1 = list unused): explicit
// weights from the slice header, implicit weights from POC distances (§8.4.2.3).
WpEntry wp_entry(const SliceEnv& env, int r0, int r1) {
  const SliceHdr& sh = *env.sh;
  const bool implicit = sh.type() == h264::kB && env.pps->weighted_bipred_idc == 2;
  WpEntry e{};
  for (int c = 0; c < 3; ++c) {
    e.w0[c] = e.w1[c] = 1;
    e.o[c] = 0;
    e.lwd[c] = 0;
  }
  if (implicit) {
    if (r0 < 0 || r1 < 0) return e;
    const ListEntry& p0 = (*env.list[0])[size_t(r0)];
    const ListEntry& p1 = (*env.list[1])[size_t(r1)];
    int w0 = 32, w1 = 32;
    const int td = clip3i(-128, 127, p1.poc - p0.poc);
    if (td != 0 && !p0.long_term && !p1.long_term) {
      const int tb = clip3i(-128, 127, env.cur_poc - p0.poc);
      const int tx = (16384 + std::abs(td / 2)) / td;
      const int dsf = clip3i(-1024, 1023, (tb * tx + 32) >> 6);
      if ((dsf >> 2) >= -64 && (dsf >> 2) <= 128) {
        w1 = dsf >> 2;
        w0 = 64 - w1;
      }
    }
    for (int c = 0; c < 3; ++c) {
      e.w0[c] = i16(w0);
      e.w1[c] = i16(w1);
      e.lwd[c] = 5;
    }
    return e;
  }
  for (int c = 0; c < 3; ++c) e.lwd[c] = u8(c == 0 ? sh.luma_lwd : sh.chroma_lwd);
  int o0[3] = {0, 0, 0}, o1[3] = {0, 0, 0};
  if (r0 >= 0) {
    const auto& w = sh.wt[0][size_t(r0)];
    for (int c = 0; c < 3; ++c) {
      e.w0[c] = w.w[c];
      o0[c] = w.o[c];
    }
  }
  if (r1 >= 0) {
    const auto& w = sh.wt[1][size_t(r1)];
    for (int c = 0; c < 3; ++c) {
      e.w1[c] = w.w[c];
      o1[c] = w.o[c];
    }
  }
  // (offsets scaled to the sample depth, 8-301 / 8-304, before the bi-prediction average)
  for (int c = 0; c < 3; ++c) {
    const int sc = 1 << ((c == 0 ? env.sps->bit_depth_luma : env.sps->bit_depth_chroma) - 8);
    o0[c] *= sc;
    o1[c] *= sc;
    e.o[c] = i16(r0 >= 0 && r1 >= 0 ? (o0[c] + o1[c] + 1) >> 1 : (r0 >= 0 ? o0[c] : o1[c]));
  }
  return e;
}

void decode_slice_generic(MbNeighbours& nb, Picture& pic, const SliceEnv& env, const u8* data, size_t n,
                          size_t bitpos) {
  const SliceHdr& sh = *env.sh;
  const Dequant& dq = dequant_for(env.scaling);
  const int total = pic.nmbs();
  int mb = sh.first_mb;
  VEP_CHECK(mb < total, "first_mb_in_slice past end of picture");
  if (env.pps->cabac) {
    if (sh.type() != h264::kI && sh.cabac_init_idc != 0)
      throw UnsupportedStream("CABAC cabac_init_idc " + std::to_string(sh.cabac_init_idc) + " is not supported");
    const size_t start = (bitpos + 7) >> 3;  // cabac_alignment_one_bit
    VEP_CHECK(start <= n, "slice data overrun");
    cabac::Ctx ctx[kCabacCtx];
    cabac_init_contexts(ctx, sh.type() == h264::kI ? -1 : 0, std::max(0, sh.qp));  // (9-5: Clip3(0, 51, SliceQPY))
    cabac::Decoder dec(data, n, start);
    BinDecoder bd{dec, ctx};
    AvcBins<BinDecoder> bins{bd};
    MbLayer<true, false> L(nb, pic, env, dq);
    L.bins = &bins;
    L.cabac = &dec;
    L.data = data;
    L.data_n = n;
    for (;;) {
      VEP_CHECK(mb < total, "macroblock address past end of picture");
      if (sh.type() != h264::kI && L.read_skip_flag(mb)) L.skip_mb(mb, false);
      else L.coded_mb(mb, sh.type() == h264::kI);
      ++mb;
      if (bins.end_of_slice(false)) {
        cabac::bins_decoded().fetch_add(dec.bins(), std::memory_order_relaxed);
        break;
      }
      VEP_CHECK(dec.bitpos() <= n * 8 + 16, "slice data overrun");
    }
    return;
  }
  Bits br(data, n, bitpos);
  const size_t stop = BitReader(data, n).stop_bit_pos();
  MbLayer<false, false> L(nb, pic, env, dq);
  L.br = &br;
  bool more = true;
  while (more) {
    if (sh.type() != h264::kI) {
      const u32 run = br.ue();
      VEP_CHECK(u32(total - mb) >= run, "mb_skip_run past end of picture");
      for (u32 k = 0; k < run; ++k) L.skip_mb(mb++, true);
      if (run > 0) {
        more = br.pos() < stop;
        if (!more) break;
      }
    }
    VEP_CHECK(mb < total, "macroblock address past end of picture");
    L.coded_mb(mb, true);
    VEP_CHECK(!br.overrun(), "slice data overrun");
    more = br.pos() < stop;
    ++mb;
  }
}

// ---------------------------------------------------------------------------- SliceWriter

struct SliceWriter::Impl {
  const SliceEnv& env;
  BitWriter& bw;
  Dequant dq;
  bool cabac;
  bool is_i;
  int run = 0;      // CAVLC mb_skip_run
  bool first = true;
  cabac::Ctx ctx[kCabacCtx];
  std::unique_ptr<cabac::Encoder> enc;
  std::unique_ptr<BinEncoder> be;
  std::unique_ptr<AvcBins<BinEncoder>> bins;
  std::unique_ptr<MbLayer<true, true>> lc;
  std::unique_ptr<MbLayer<false, true>> lv;
  Impl(MbNeighbours& nb, Picture& pic, const SliceEnv& e, BitWriter& w)
      : env(e), bw(w), dq(e.scaling), cabac(e.pps->cabac), is_i(e.sh->type() == h264::kI) {
    if (cabac) {
      while (!bw.byte_aligned()) bw.u1(1);  // cabac_alignment_one_bit
      cabac_init_contexts(ctx, is_i ? -1 : 0, std::max(0, e.sh->qp));
      enc = std::make_unique<cabac::Encoder>(bw.buf());
      be = std::make_unique<BinEncoder>(BinEncoder{*enc, ctx});
      bins = std::make_unique<AvcBins<BinEncoder>>(AvcBins<BinEncoder>{*be});
      lc = std::make_unique<MbLayer<true, true>>(nb, pic, env, dq);
      lc->bins = bins.get();
      lc->cenc = enc.get();
    } else {
      lv = std::make_unique<MbLayer<false, true>>(nb, pic, env, dq);
      lv->bw = &bw;
    }
  }
};

SliceWriter::SliceWriter(MbNeighbours& nb, Picture& pic, const SliceEnv& env, BitWriter& bw)
    : p_(std::make_unique<Impl>(nb, pic, env, bw)) {}
SliceWriter::~SliceWriter() = default;

void SliceWriter::write_mb(int mb, const MbDesc& d) {
  Impl& p = *p_;
  VEP_CHECK(!(d.skip && p.is_i), "skipped macroblock in an I slice");
  if (p.cabac) {
    if (!p.first) p.bins->end_of_slice(false);
    p.first = false;
    p.lc->want = &d;
    if (!p.is_i && p.lc->read_skip_flag(mb, d.skip)) p.lc->skip_mb(mb, false);
    else p.lc->coded_mb(mb, p.is_i);
    return;
  }
  p.lv->want = &d;
  if (d.skip) {
    p.lv->skip_mb(mb, true);
    ++p.run;
    return;
  }
  if (!p.is_i) {
    p.bw.ue(u32(p.run));
    p.run = 0;
  }
  p.lv->coded_mb(mb, true);
}

void SliceWriter::finish() {
  Impl& p = *p_;
  if (p.cabac) {
    p.bins->end_of_slice(true);  // terminate + flush: the flush ends with the rbsp_stop_one_bit
    p.enc->align_zero();
    return;
  }
  if (p.run > 0) p.bw.ue(u32(p.run));
  p.bw.trailing();
}

void SliceWriter::skip_motion(int mb, MbState& out) {
  if (p_->cabac) p_->lc->skip_motion(mb, out);
  else p_->lv->skip_motion(mb, out);
}

int SliceWriter::qp() const { return p_->cabac ? p_->lc->qp() : p_->lv->qp(); }

}  // namespace vep::avc
