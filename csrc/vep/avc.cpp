// General H.264 decoding path: slice headers, CAVLC macroblock layer, neighbour derivations,
// DPB / reference lists and the CPU reference reconstruction. See avc.h for the CPU/GPU split.
#include "avc.h"

#include <immintrin.h>

#include <algorithm>
#include <array>

#include "avc_cavlc.h"
#include "avc_internal.h"
#include "fanout.h"

namespace vep::avc {

using h264::Pps;
using h264::Sps;

// ------------------------------------------------------------------------- MbNeighbours

void MbNeighbours::reset(int wmbs, int hmbs, bool ring) {
  w_ = wmbs;
  h_ = hmbs;
  cur_ = -1;
  run_slice_ = ~0u;
  run_start_ = 0;
  announced_ = 0;
  const size_t n = size_t(wmbs) * hmbs;
  if (++epoch_ == 0) {  // (after 2^32 pictures) no stale stamp may equal the new epoch
    epoch_ = 1;
    stamp_.clear();
  }
  // every field of an MB's state is rewritten when the MB is decoded (MbState{} first), and
  // begin() stamps the MB with the epoch and tags its state entry: nothing to clear here
  size_t ns = n;
  mask_ = ~size_t(0);
  if (ring) {  // a power of two >= 2 * (row + 2): the A / B / C / D neighbours are <= row + 1 back
    size_t r = 1;
    while (r < 2 * (size_t(wmbs) + 2)) r <<= 1;
    if (r < n) {
      ns = r;
      mask_ = r - 1;
    }
  }
  if (st_.size() != ns) st_.assign(ns, MbState{});
  if (tag_.size() != ns) tag_.assign(ns, ~0u);
  if (stamp_.size() != n) stamp_.assign(n, 0u);
}

static int coded_count(const MbState& s, int blk) {
  if (s.kind == kSkip) return 0;
  if (s.kind == kIPcm) return 16;
  return s.tc[blk];
}

int MbNeighbours::nc_luma(int mb, int blk) const {
  const int bx = blk & 3, by = blk >> 2;
  int na = -1, nb = -1;
  const int am = mb_at(mb, bx * 4 - 1, by * 4);
  if (am >= 0) na = coded_count(st_[size_t(am) & mask_], bx > 0 ? blk - 1 : blk + 3);
  const int bm = mb_at(mb, bx * 4, by * 4 - 1);
  if (bm >= 0) nb = coded_count(st_[size_t(bm) & mask_], by > 0 ? blk - 4 : blk + 12);
  if (na >= 0 && nb >= 0) return (na + nb + 1) >> 1;
  if (na >= 0) return na;
  if (nb >= 0) return nb;
  return 0;
}

int MbNeighbours::nc_chroma(int mb, int c, int blk, int nbc) const {
  const int bx = blk & 1, by = blk >> 1;
  auto count = [&](int m, int b) {
    const MbState& s = st_[size_t(m) & mask_];
    if (s.kind == kSkip) return 0;
    if (s.kind == kIPcm) return 16;
    return int(s.tcc[c][b]);
  };
  int na = -1, nb = -1;
  const int am = bx > 0 ? mb : mb_at(mb, -1, 0);
  if (am >= 0) na = count(am, bx > 0 ? blk - 1 : blk + 1);
  const int bm = by > 0 ? mb : mb_at(mb, 0, -1);
  if (bm >= 0) nb = count(bm, by > 0 ? blk - 2 : blk + nbc - 2);  // (above MB: its bottom row of blocks)
  if (na >= 0 && nb >= 0) return (na + nb + 1) >> 1;
  if (na >= 0) return na;
  if (nb >= 0) return nb;
  return 0;
}

int MbNeighbours::pred_intra4x4(int mb, int blk, bool constrained) const {
  const int bx = blk & 3, by = blk >> 2;
  const int am = mb_at(mb, bx * 4 - 1, by * 4), bm = mb_at(mb, bx * 4, by * 4 - 1);
  if (am < 0 || bm < 0) return 2;
  const MbState& a = st_[size_t(am) & mask_];
  const MbState& b = st_[size_t(bm) & mask_];
  if (constrained && (!is_intra(a.kind) || !is_intra(b.kind))) return 2;
  const int ma = a.kind == kI4x4 ? a.i4[bx > 0 ? blk - 1 : blk + 3] : 2;
  const int mbm = b.kind == kI4x4 ? b.i4[by > 0 ? blk - 4 : blk + 12] : 2;
  return ma < mbm ? ma : mbm;
}

int MbNeighbours::pred_intra8x8(int mb, int b8, bool constrained) const {
  // §8.3.2.1: neighbour 8x8 blocks A / B; an Intra_4x4 neighbour contributes the 4x4 block
  // n = 1 (A) / 2 (B) of its 8x8 — exactly the 4x4 block left of / above the 8x8's top-left
  // block, which is what MbState::i4 holds (8x8 modes are replicated over their four blocks)
  const int blk = (b8 & 1) * 2 + (b8 >> 1) * 8;
  const int bx = blk & 3, by = blk >> 2;
  const int am = mb_at(mb, bx * 4 - 1, by * 4), bm = mb_at(mb, bx * 4, by * 4 - 1);
  if (am < 0 || bm < 0) return 2;
  const MbState& a = st_[size_t(am) & mask_];
  const MbState& b = st_[size_t(bm) & mask_];
  if (constrained && (!is_intra(a.kind) || !is_intra(b.kind))) return 2;
  auto mode = [](const MbState& n, int r, int b8n) -> int {
    if (n.kind == kI8x8) return n.i4[(b8n & 1) * 2 + (b8n >> 1) * 8];
    if (n.kind == kI4x4) return n.i4[r];
    return 2;
  };
  // A: the 4x4 block left of the top-left block (right column of the left 8x8), B: above
  const int ra = bx > 0 ? blk - 1 : blk + 3, rb = by > 0 ? blk - 4 : blk + 12;
  const int b8a = ((ra >> 3) << 1) | ((ra & 3) >> 1), b8b = ((rb >> 3) << 1) | ((rb & 3) >> 1);
  const int ma = mode(a, ra, b8a), mbm = mode(b, rb, b8b);
  return ma < mbm ? ma : mbm;
}

static int median3(int a, int b, int c) { return a + b + c - std::min({a, b, c}) - std::max({a, b, c}); }

void MbNeighbours::pred_mv(int mb, int x4, int y4, int w4, int h4, int list, int ref, u16 done, int shape,
                           int out[2]) const {
  (void)h4;
  if (mb == cur_ && w4 == 4 && h4 == 4 && shape == 0) return pred_mv16(list, ref, out);  // (x4 = y4 = 0)
  const int x = x4 * 4, y = y4 * 4, w = w4 * 4;
  Nb A = motion_at(mb, x - 1, y, done, list);
  Nb B = motion_at(mb, x, y - 1, done, list);
  Nb C = motion_at(mb, x + w, y - 1, done, list);
  if (!C.avail) C = motion_at(mb, x - 1, y - 1, done, list);  // D replaces an unavailable C
  auto take = [&](const Nb& n) {
    out[0] = n.mv[0];
    out[1] = n.mv[1];
  };
  if (shape == 1) {  // 16x8
    if (y4 == 0 && B.ref == ref) return take(B);
    if (y4 != 0 && A.ref == ref) return take(A);
  } else if (shape == 2) {  // 8x16
    if (x4 == 0 && A.ref == ref) return take(A);
    if (x4 != 0 && C.ref == ref) return take(C);
  }
  if (!B.avail && !C.avail && A.avail) B = C = A;
  const int match = (A.ref == ref) + (B.ref == ref) + (C.ref == ref);
  if (match == 1) return take(A.ref == ref ? A : B.ref == ref ? B : C);
  out[0] = median3(A.mv[0], B.mv[0], C.mv[0]);
  out[1] = median3(A.mv[1], B.mv[1], C.mv[1]);
}

void MbNeighbours::pskip_mv(int mb, int out[2]) const {
  out[0] = out[1] = 0;
  if (mb == cur_) {  // the announced MB: one neighbour fetch for the checks and the predictor
    if (a_ < 0 || b_ < 0) return;
    Nb n[3];
    nb16(0, n);
    if ((n[0].ref == 0 && n[0].mv[0] == 0 && n[0].mv[1] == 0) || (n[1].ref == 0 && n[1].mv[0] == 0 && n[1].mv[1] == 0))
      return;
    pred_mv16(0, 0, out);
    return;
  }
  if (mb_at(mb, -1, 0) < 0 || mb_at(mb, 0, -1) < 0) return;
  const Nb A = motion_at(mb, -1, 0, 0, 0), B = motion_at(mb, 0, -1, 0, 0);
  if ((A.ref == 0 && A.mv[0] == 0 && A.mv[1] == 0) || (B.ref == 0 && B.mv[0] == 0 && B.mv[1] == 0))
    return;
  pred_mv(mb, 0, 0, 4, 4, 0, 0, 0, 0, out);
}

void MbNeighbours::mb_neighbour_refs(int mb, int list, int ref[3]) const {
  const Nb A = motion_at(mb, -1, 0, 0, list), B = motion_at(mb, 0, -1, 0, list);
  Nb C = motion_at(mb, 16, -1, 0, list);
  if (!C.avail) C = motion_at(mb, -1, -1, 0, list);
  ref[0] = A.ref;
  ref[1] = B.ref;
  ref[2] = C.ref;
}

void MbNeighbours::direct_spatial_pred(int mb, int list, int& ref, int mv[2]) const {
  Nb A = motion_at(mb, -1, 0, 0, list), B = motion_at(mb, 0, -1, 0, list);
  Nb C = motion_at(mb, 16, -1, 0, list);
  if (!C.avail) C = motion_at(mb, -1, -1, 0, list);
  auto minpos = [](int a, int b) { return (a >= 0 && b >= 0) ? std::min(a, b) : std::max(a, b); };
  ref = minpos(A.ref, minpos(B.ref, C.ref));
  mv[0] = mv[1] = 0;
  if (ref < 0) return;
  // the 16x16 predictor of pred_mv() for `ref` from the same A, B, C
  if (!B.avail && !C.avail && A.avail) B = C = A;
  const int match = (A.ref == ref) + (B.ref == ref) + (C.ref == ref);
  if (match == 1) {
    const Nb& n = A.ref == ref ? A : B.ref == ref ? B : C;
    mv[0] = n.mv[0];
    mv[1] = n.mv[1];
    return;
  }
  mv[0] = median3(A.mv[0], B.mv[0], C.mv[0]);
  mv[1] = median3(A.mv[1], B.mv[1], C.mv[1]);
}

// ------------------------------------------------------------------------- parameter sets

namespace {

// Stream features outside the supported subset (progressive 8-bit 4:2:0, no lossless).
void check_sps_supported(const Sps& s) {
  // (High 10: 9 / 10-bit samples, one depth for luma and chroma: the surfaces hold one)
  // (4:2:2: High 4:2:2, 8..10 bits, progressive)
  if (s.chroma_format_idc > 2 || s.bit_depth_luma > 10 || s.bit_depth_chroma != s.bit_depth_luma)
    throw UnsupportedStream("only 8-bit 4:2:0 / 4:0:0 H.264 is supported");
  // Interlaced SPS (frame_mbs_only_flag 0): frame pictures decode as progressive ones (frame
  // macroblocks, frame POC = min(top, bottom)); field pictures as half-height pictures in field
  // slots (CAVLC I / P, see Decoder::parse); MBAFF frames are rejected.
  if (!s.frame_mbs_only && s.mbaff) throw UnsupportedStream("interlaced H.264: MBAFF frames are not supported");
  if (s.transform_bypass) throw UnsupportedStream("lossless (transform bypass) H.264 is not supported");
}

const u8* unescape(const u8* p, size_t n, std::vector<u32>& epb, std::vector<u8>& scratch,
                   size_t& out_n, const u32* kb = nullptr, const u32* ke = nullptr) {
  if (kb) epb.assign(kb, ke);
  else find_epb(p, n, epb);
  if (epb.empty()) {
    out_n = n;
    return p;
  }
  scratch.resize(n);
  size_t o = 0, from = 0;
  for (u32 e : epb) {
    std::memcpy(scratch.data() + o, p + from, e - from);
    o += e - from;
    from = size_t(e) + 1;
  }
  std::memcpy(scratch.data() + o, p + from, n - from);
  out_n = o + (n - from);
  return scratch.data();
}

// Slice-level context of the macroblock walk.
struct SliceCtx {
  const SliceHdr& sh;
  const Pps& pps;
  int slice;
  bool is_p;
  int qp;
  const std::vector<ListEntry>& list0;
};

// LevelScale4x4 with flat weight matrices (16 * normAdjust4x4), per qP % 6 and raster position.
struct LevelScaleTable {
  int v[6][16];
  LevelScaleTable() {
    for (int m = 0; m < 6; ++m)
      for (int p = 0; p < 16; ++p) v[m][p] = 16 * norm_adjust(m, p >> 2, p & 3);
  }
};
const LevelScaleTable kLevelScaleTable;
const int (&kLevelScale)[6][16] = kLevelScaleTable.v;

}  // namespace

// ------------------------------------------------------------------------- slice header

static void read_ref_mods(Bits& br, std::vector<SliceHdr::RefMod>& mods) {
  if (!br.u1()) return;  // ref_pic_list_modification_flag_lX
  for (;;) {
    const int idc = int(br.ue());
    if (idc == 3) break;
    VEP_CHECK(idc <= 2, "bad modification_of_pic_nums_idc");
    mods.push_back({idc, int(br.ue())});
    VEP_CHECK(mods.size() <= 33, "too many reference list modifications");
  }
}

static SliceHdr read_slice_header(Bits& br, u8 nal_hdr, const Sps& sps, const Pps& pps) {
  SliceHdr sh;
  sh.nal_type = h264::nal_type(nal_hdr);
  sh.nal_ref_idc = h264::nal_ref_idc(nal_hdr);
  sh.first_mb = int(br.ue());
  sh.slice_type = int(br.ue());
  VEP_CHECK(sh.slice_type <= 9, "bad slice_type");
  sh.pps_id = int(br.ue());
  sh.frame_num = int(br.u(sps.log2_max_frame_num));
  if (!sps.frame_mbs_only && (sh.field_pic = br.u1())) sh.bottom_field = br.u1();
  if (sh.idr()) sh.idr_pic_id = int(br.ue());
  if (sps.poc_type == 0) {
    sh.poc_lsb = int(br.u(sps.log2_max_poc_lsb));
    if (pps.bottom_field_pic_order && !sh.field_pic) sh.delta_poc_bottom = br.se();
  } else if (sps.poc_type == 1 && !sps.delta_pic_order_always_zero) {
    sh.delta_poc[0] = br.se();
    if (pps.bottom_field_pic_order && !sh.field_pic) sh.delta_poc[1] = br.se();
  }
  if (pps.redundant_pic_cnt_present && (sh.redundant_pic_cnt = int(br.ue())) != 0)
    return sh;  // a redundant coded picture's slice: ignored (the primary picture is decoded)
  const int st = sh.type();
  if (st == h264::kSP || st == h264::kSI) throw UnsupportedStream("H.264 SP / SI slices are not supported");
  if (st == h264::kB) sh.direct_spatial = br.u1();
  sh.num_ref_idx[0] = pps.num_ref_idx_l0_default;
  sh.num_ref_idx[1] = pps.num_ref_idx_l1_default;
  if (st == h264::kP || st == h264::kB) {
    if (br.u1()) {  // num_ref_idx_active_override_flag
      sh.num_ref_idx[0] = int(br.ue()) + 1;
      if (st == h264::kB) sh.num_ref_idx[1] = int(br.ue()) + 1;
    }
    VEP_CHECK(sh.num_ref_idx[0] <= 32 && sh.num_ref_idx[1] <= 32, "num_ref_idx out of range");
    read_ref_mods(br, sh.ref_mods[0]);
    if (st == h264::kB) read_ref_mods(br, sh.ref_mods[1]);
  }
  if (st == h264::kP) sh.num_ref_idx[1] = 0;
  if (st == h264::kI) sh.num_ref_idx[0] = sh.num_ref_idx[1] = 0;
  if ((pps.weighted_pred && st == h264::kP) || (pps.weighted_bipred_idc == 1 && st == h264::kB)) {
    sh.explicit_wp = true;  // pred_weight_table()
    sh.luma_lwd = int(br.ue());
    sh.chroma_lwd = int(br.ue());
    VEP_CHECK(sh.luma_lwd <= 7 && sh.chroma_lwd <= 7, "weight denominator out of range");
    for (int l = 0; l < (st == h264::kB ? 2 : 1); ++l) {
      sh.wt[l].resize(size_t(sh.num_ref_idx[l]));
      for (auto& w : sh.wt[l]) {
        w.w[0] = i16(1 << sh.luma_lwd);
        w.w[1] = w.w[2] = i16(1 << sh.chroma_lwd);
        w.o[0] = w.o[1] = w.o[2] = 0;
        if (br.u1()) {
          w.w[0] = i16(br.se());
          w.o[0] = i16(br.se());
          VEP_CHECK(w.w[0] >= -128 && w.w[0] <= 127 && w.o[0] >= -128 && w.o[0] <= 127, "luma weight out of range");
        }
        if (br.u1())
          for (int c = 1; c < 3; ++c) {
            w.w[c] = i16(br.se());
            w.o[c] = i16(br.se());
            VEP_CHECK(w.w[c] >= -128 && w.w[c] <= 127 && w.o[c] >= -128 && w.o[c] <= 127,
                      "chroma weight out of range");
          }
      }
    }
  }
  if (sh.nal_ref_idc != 0) {
    if (sh.idr()) {
      sh.no_output_of_prior_pics = br.u1();
      sh.long_term_reference = br.u1();
    } else if ((sh.adaptive_marking = br.u1())) {
      for (;;) {
        const int op = int(br.ue());
        if (op == 0) break;
        VEP_CHECK(op <= 6, "bad memory_management_control_operation");
        SliceHdr::Mmco m{op, 0, 0};
        if (op == 1 || op == 3) m.a = int(br.ue());
        if (op == 2) m.a = int(br.ue());
        if (op == 3 || op == 6) (op == 3 ? m.b : m.a) = int(br.ue());
        if (op == 4) m.a = int(br.ue());
        sh.mmcos.push_back(m);
        VEP_CHECK(sh.mmcos.size() <= 66, "too many MMCO operations");
      }
    }
  }
  if (pps.cabac && st != h264::kI) {
    sh.cabac_init_idc = int(br.ue());
    VEP_CHECK(sh.cabac_init_idc <= 2, "bad cabac_init_idc");
  }
  sh.qp = pps.pic_init_qp + br.se();
  VEP_CHECK(sh.qp >= -6 * (sps.bit_depth_luma - 8) && sh.qp <= 51, "slice QP out of range");
  if (pps.deblocking_filter_control) {
    sh.disable_deblocking = int(br.ue());
    VEP_CHECK(sh.disable_deblocking <= 2, "bad disable_deblocking_filter_idc");
    if (sh.disable_deblocking != 1) {
      sh.alpha_off = 2 * br.se();
      sh.beta_off = 2 * br.se();
      VEP_CHECK(sh.alpha_off >= -12 && sh.alpha_off <= 12 && sh.beta_off >= -12 && sh.beta_off <= 12,
                "deblocking offsets out of range");
    }
  }
  if (sh.field_pic) {
    // Field pictures: CAVLC I / P / B. CABAC needs the field-coded context initialisation values
    // (not in any source this build can pin): it stays with the VCN backend, as does MMCO 5 in a
    // field.
    if (pps.cabac) throw UnsupportedStream("interlaced H.264: CABAC field pictures are not supported");
    // MMCO 5 in the first field of a pair (the second field then carries frame_num 0); in a
    // second field it would also drop the pair's first field: not supported
    if (sh.has_mmco5() && sh.adaptive_marking && sh.mmcos.size() != 1)
      throw UnsupportedStream("interlaced H.264: MMCO 5 with other MMCOs in a field is not supported");
  }
  return sh;
}

// ------------------------------------------------------------------------- DPB

void Decoder::reset_references() {
  pair_ = OpenPair{};
  dpb_.clear();
  pending_.clear();
  have_idr_ = false;
  max_lt_idx_ = -1;
  pinned_slot_ = -1;
}

int Decoder::pick_slot() const {
  for (int s = 0; s < dpb_slots_; ++s) {
    bool used = s == pinned_slot_ || (pair_.open && s == pair_.slot);
    for (const auto& r : dpb_) used |= r.slot == s;
    for (const auto& p : pending_) used |= p.f.slot == s;
    if (!used) return s;
  }
  throw Error("vep: decoded picture buffer overflow");
}

// §8.2.1: picture order count of the current picture (frame: min(top, bottom)).
int Decoder::compute_poc(const SliceHdr& sh, const Sps& sps) {
  const int max_fn = 1 << sps.log2_max_frame_num;
  if (sps.poc_type == 0) {
    if (sh.idr()) prev_poc_msb_ = prev_poc_lsb_ = 0;
    const int max_lsb = 1 << sps.log2_max_poc_lsb;
    int msb = prev_poc_msb_;
    if (sh.poc_lsb < prev_poc_lsb_ && prev_poc_lsb_ - sh.poc_lsb >= max_lsb / 2) msb = prev_poc_msb_ + max_lsb;
    else if (sh.poc_lsb > prev_poc_lsb_ && sh.poc_lsb - prev_poc_lsb_ > max_lsb / 2) msb = prev_poc_msb_ - max_lsb;
    const int top = msb + sh.poc_lsb, bot = sh.field_pic ? top : top + sh.delta_poc_bottom;
    if (sh.nal_ref_idc != 0) {
      if (sh.has_mmco5()) {
        prev_poc_msb_ = 0;
        prev_poc_lsb_ = top - std::min(top, bot);
      } else {
        prev_poc_msb_ = msb;
        prev_poc_lsb_ = sh.poc_lsb;
      }
    }
    return std::min(top, bot);
  }
  // types 1 and 2: FrameNumOffset
  int fno;
  if (sh.idr()) fno = 0;
  else if (prev_frame_num_ > sh.frame_num) fno = prev_frame_num_offset_ + max_fn;
  else fno = prev_frame_num_offset_;
  int poc;
  if (sps.poc_type == 1) {
    const int n = int(sps.offset_for_ref_frame.size());
    int abs_fn = n != 0 ? fno + sh.frame_num : 0;
    if (sh.nal_ref_idc == 0 && abs_fn > 0) --abs_fn;
    int expected = 0;
    if (abs_fn > 0) {
      int per_cycle = 0;
      for (int v : sps.offset_for_ref_frame) per_cycle += v;
      const int cnt = (abs_fn - 1) / n, in_cycle = (abs_fn - 1) % n;
      expected = cnt * per_cycle;
      for (int i = 0; i <= in_cycle; ++i) expected += sps.offset_for_ref_frame[size_t(i)];
    }
    if (sh.nal_ref_idc == 0) expected += sps.offset_for_non_ref_pic;
    const int top = expected + sh.delta_poc[0];
    const int bot = top + sps.offset_for_top_to_bottom_field + sh.delta_poc[1];
    // a field picture: its own field's count (bottom: expected + offset + delta_pic_order_cnt[0])
    poc = !sh.field_pic ? std::min(top, bot) : sh.bottom_field ? top + sps.offset_for_top_to_bottom_field : top;
  } else {
    poc = sh.idr() ? 0 : (sh.nal_ref_idc == 0 ? 2 * (fno + sh.frame_num) - 1 : 2 * (fno + sh.frame_num));
  }
  const bool mmco5 = sh.has_mmco5();
  prev_frame_num_offset_ = mmco5 ? 0 : fno;
  prev_frame_num_ = mmco5 ? 0 : sh.frame_num;
  return poc;
}

// §8.2.4.2 / §8.2.4.3: reference picture lists of the current slice.
void Decoder::build_lists(const SliceHdr& sh, const Sps& sps, int cur_poc) {
  const int max_fn = 1 << sps.log2_max_frame_num;
  list_[0].clear();
  list_[1].clear();
  if (sh.type() == h264::kI) return;
  std::vector<RefPic*> st, lt;
  for (auto& r : dpb_) {
    if (r.long_term) {
      lt.push_back(&r);
    } else {
      r.frame_num_wrap = r.frame_num > sh.frame_num ? r.frame_num - max_fn : r.frame_num;
      st.push_back(&r);
    }
  }
  std::sort(lt.begin(), lt.end(), [](RefPic* a, RefPic* b) { return a->lt_idx < b->lt_idx; });
  std::vector<RefPic*> init[2];
  if (sh.type() == h264::kP) {
    std::sort(st.begin(), st.end(), [](RefPic* a, RefPic* b) { return a->frame_num_wrap > b->frame_num_wrap; });
    init[0] = st;
    init[0].insert(init[0].end(), lt.begin(), lt.end());
  } else {
    std::vector<RefPic*> before, after;
    for (RefPic* r : st) (r->poc < cur_poc ? before : after).push_back(r);
    std::sort(before.begin(), before.end(), [](RefPic* a, RefPic* b) { return a->poc > b->poc; });
    std::sort(after.begin(), after.end(), [](RefPic* a, RefPic* b) { return a->poc < b->poc; });
    init[0] = before;
    init[0].insert(init[0].end(), after.begin(), after.end());
    init[0].insert(init[0].end(), lt.begin(), lt.end());
    init[1] = after;
    init[1].insert(init[1].end(), before.begin(), before.end());
    init[1].insert(init[1].end(), lt.begin(), lt.end());
    if (init[1].size() > 1 && init[1] == init[0]) std::swap(init[1][0], init[1][1]);
  }
  for (int l = 0; l < (sh.type() == h264::kB ? 2 : 1); ++l) {
    std::vector<RefPic*> list = init[l];
    int pred = sh.frame_num;
    size_t idx = 0;
    for (const auto& m : sh.ref_mods[l]) {
      RefPic* pick = nullptr;
      if (m.idc < 2) {
        const int d = m.val + 1;
        int nw = m.idc == 0 ? pred - d : pred + d;
        if (nw < 0) nw += max_fn;
        if (nw >= max_fn) nw -= max_fn;
        pred = nw;
        const int pic_num = nw > sh.frame_num ? nw - max_fn : nw;
        for (RefPic* r : st)
          if (r->frame_num_wrap == pic_num) pick = r;
      } else {
        for (RefPic* r : lt)
          if (r->lt_idx == m.val) pick = r;
      }
      if (!pick) throw Error("vep: reference list modification names a missing picture");
      ++list_mods;
      list.insert(list.begin() + long(std::min(idx, list.size())), pick);
      for (size_t k = idx + 1; k < list.size(); ++k)
        if (list[k] == pick) {
          list.erase(list.begin() + long(k));
          break;
        }
      ++idx;
    }
    list_[l].assign(size_t(sh.num_ref_idx[l]), ListEntry{});
    for (size_t i = 0; i < list_[l].size() && i < list.size(); ++i) {
      const RefPic& r = *list[i];
      list_[l][i] = ListEntry{r.slot, r.poc, r.long_term, r.uid, r.col.get()};
    }
  }
}

void Decoder::mark_references(const SliceHdr& sh, const Sps& sps, int slot, int poc, u32 uid,
                              std::shared_ptr<const ColMotion> col) {
  const int max_fn = 1 << sps.log2_max_frame_num;
  const int max_refs = std::max(1, sps.max_num_ref_frames);
  RefPic cur;
  cur.slot = slot;
  cur.frame_num = sh.frame_num;
  cur.poc = poc;
  cur.uid = uid;
  cur.col = std::move(col);
  if (sh.idr()) {
    dpb_.clear();
    if (sh.long_term_reference) {
      cur.long_term = true;
      cur.lt_idx = 0;
      max_lt_idx_ = 0;
      ++long_term_marked;
    } else {
      max_lt_idx_ = -1;
    }
    dpb_.push_back(cur);
    return;
  }
  auto wrap = [&](const RefPic& r) { return r.frame_num > sh.frame_num ? r.frame_num - max_fn : r.frame_num; };
  auto erase_if = [&](auto pred) { dpb_.erase(std::remove_if(dpb_.begin(), dpb_.end(), pred), dpb_.end()); };
  bool cur_long = false, mmco5 = false;
  int cur_lt = 0;
  if (sh.adaptive_marking) {
    for (const auto& m : sh.mmcos) {
      ++mmco_ops[m.op];
      switch (m.op) {
        case 1: {
          const int pn = sh.frame_num - (m.a + 1);
          erase_if([&](const RefPic& r) { return !r.long_term && wrap(r) == pn; });
          break;
        }
        case 2:
          erase_if([&](const RefPic& r) { return r.long_term && r.lt_idx == m.a; });
          break;
        case 3: {
          const int pn = sh.frame_num - (m.a + 1);
          erase_if([&](const RefPic& r) { return r.long_term && r.lt_idx == m.b; });
          for (auto& r : dpb_)
            if (!r.long_term && wrap(r) == pn) {
              r.long_term = true;
              r.lt_idx = m.b;
            }
          break;
        }
        case 4:
          max_lt_idx_ = m.a - 1;
          erase_if([&](const RefPic& r) { return r.long_term && r.lt_idx > max_lt_idx_; });
          break;
        case 5:
          dpb_.clear();
          max_lt_idx_ = -1;
          mmco5 = true;
          break;
        case 6:
          erase_if([&](const RefPic& r) { return r.long_term && r.lt_idx == m.a; });
          cur_long = true;
          cur_lt = m.a;
          break;
        default: break;
      }
    }
  } else {
    int n_short = 0;
    for (const auto& r : dpb_) n_short += !r.long_term;
    if (int(dpb_.size()) >= max_refs && n_short > 0) {  // sliding window
      auto it = std::min_element(dpb_.begin(), dpb_.end(), [&](const RefPic& a, const RefPic& b) {
        if (a.long_term != b.long_term) return !a.long_term;
        return wrap(a) < wrap(b);
      });
      dpb_.erase(it);
    }
  }
  cur.frame_num = mmco5 ? 0 : sh.frame_num;
  if (mmco5) cur.poc = 0;
  cur.long_term = cur_long;
  long_term_marked += cur_long ? 1 : 0;
  cur.lt_idx = cur_lt;
  dpb_.push_back(cur);
  while (int(dpb_.size()) > max_refs) {  // non-conforming stream: drop the oldest short-term
    auto it = std::min_element(dpb_.begin(), dpb_.end(), [&](const RefPic& a, const RefPic& b) {
      if (a.long_term != b.long_term) return !a.long_term;
      return wrap(a) < wrap(b);
    });
    dpb_.erase(it);
  }
}

// Field picture numbers (§8.2.4.1): a field of the current parity counts 2 * FrameNumWrap + 1
// (long-term: 2 * LongTermFrameIdx + 1), one of the other parity the even number below.
static int field_pic_num(const RefPic& r, int par, int cur_par, int frame_num, int max_fn) {
  const int wrap = r.frame_num > frame_num ? r.frame_num - max_fn : r.frame_num;
  return 2 * wrap + (par == cur_par ? 1 : 0);
}
static int field_lt_pic_num(const RefPic& r, int par, int cur_par) { return 2 * r.lt_idx + (par == cur_par ? 1 : 0); }
static ListEntry field_entry(const RefPic& r, int par, bool lt) {
  return ListEntry{2 * r.slot + par, r.poc_f[par], lt, r.uid_f[par], r.col_f[par].get()};
}

// §8.2.4.2.2 / §8.2.4.2.4 / §8.2.4.2.5: the lists of a P or B field. The reference frames
// (P: short-term by FrameNumWrap descending; B: by POC around the current field's, list 0 the
// earlier ones first, list 1 the later ones; then long-term by index) are taken apart into their
// fields, alternating parities starting with the current field's; when one parity runs out the
// other's remaining fields follow in order. A frame's POC here is the lowest of its short-term
// fields'; the first field of the current frame is a reference frame entry too. Then the slice's
// modifications (§8.2.4.3 with field picture numbers).
void Decoder::build_field_lists(const SliceHdr& sh, const Sps& sps, int cur_poc) {
  const int max_fn = 1 << sps.log2_max_frame_num;
  list_[0].clear();
  list_[1].clear();
  if (sh.type() == h264::kI) return;
  std::vector<RefPic*> st, lt;
  for (auto& r : dpb_) {
    if (r.fields & 3) {
      r.frame_num_wrap = r.frame_num > sh.frame_num ? r.frame_num - max_fn : r.frame_num;
      st.push_back(&r);
    }
    if (r.lt_fields & 3) lt.push_back(&r);
  }
  std::sort(lt.begin(), lt.end(), [](RefPic* a, RefPic* b) { return a->lt_idx < b->lt_idx; });
  const int same = sh.bottom_field ? 1 : 0;
  auto alternate = [&](const std::vector<RefPic*>& frames, bool long_term, std::vector<ListEntry>& all) {
    std::vector<ListEntry> f[2];  // [0] same parity, [1] opposite
    for (RefPic* r : frames)
      for (int k = 0; k < 2; ++k) {
        const int par = k == 0 ? same : 1 - same;
        if (((long_term ? r->lt_fields : r->fields) >> par) & 1) f[k].push_back(field_entry(*r, par, long_term));
      }
    size_t i[2] = {0, 0};
    for (int k = 0; i[0] < f[0].size() || i[1] < f[1].size(); k ^= 1) {
      const int from = i[k] < f[k].size() ? k : k ^ 1;
      all.push_back(f[from][i[from]++]);
    }
  };
  auto st_poc = [](const RefPic* r) {
    return (r->fields & 1) ? ((r->fields & 2) ? std::min(r->poc_f[0], r->poc_f[1]) : r->poc_f[0]) : r->poc_f[1];
  };
  std::vector<RefPic*> init[2];
  if (sh.type() == h264::kP) {
    std::sort(st.begin(), st.end(), [](RefPic* a, RefPic* b) { return a->frame_num_wrap > b->frame_num_wrap; });
    init[0] = st;
  } else {
    std::vector<RefPic*> before, after;
    for (RefPic* r : st) (st_poc(r) <= cur_poc ? before : after).push_back(r);
    std::sort(before.begin(), before.end(), [&](RefPic* a, RefPic* b) { return st_poc(a) > st_poc(b); });
    std::sort(after.begin(), after.end(), [&](RefPic* a, RefPic* b) { return st_poc(a) < st_poc(b); });
    init[0] = before;
    init[0].insert(init[0].end(), after.begin(), after.end());
    init[1] = after;
    init[1].insert(init[1].end(), before.begin(), before.end());
  }
  std::vector<ListEntry> all[2];
  const int nl = sh.type() == h264::kB ? 2 : 1;
  for (int l = 0; l < nl; ++l) {
    alternate(init[l], false, all[l]);
    alternate(lt, true, all[l]);
  }
  auto same_entries = [](const std::vector<ListEntry>& a, const std::vector<ListEntry>& b) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); ++i)
      if (a[i].slot != b[i].slot || a[i].long_term != b[i].long_term) return false;
    return true;
  };
  if (nl == 2 && all[1].size() > 1 && same_entries(all[0], all[1])) std::swap(all[1][0], all[1][1]);
  const int cur_pic_num = 2 * sh.frame_num + 1, max_pic = 2 * max_fn;
  for (int l = 0; l < nl; ++l) {
    std::vector<ListEntry>& list = all[l];
    int pred = cur_pic_num;
    size_t idx = 0;
    for (const auto& m : sh.ref_mods[l]) {
      bool found = false;
      ListEntry pick{};
      if (m.idc < 2) {
        int nw = m.idc == 0 ? pred - (m.val + 1) : pred + (m.val + 1);
        if (nw < 0) nw += max_pic;
        if (nw >= max_pic) nw -= max_pic;
        pred = nw;
        const int pic_num = nw > cur_pic_num ? nw - max_pic : nw;
        for (const auto& r : dpb_)
          for (int par = 0; par < 2; ++par)
            if (((r.fields >> par) & 1) && field_pic_num(r, par, same, sh.frame_num, max_fn) == pic_num) {
              pick = field_entry(r, par, false);
              found = true;
            }
      } else {
        for (const auto& r : dpb_)
          for (int par = 0; par < 2; ++par)
            if (((r.lt_fields >> par) & 1) && field_lt_pic_num(r, par, same) == m.val) {
              pick = field_entry(r, par, true);
              found = true;
            }
      }
      if (!found) throw Error("vep: reference list modification names a missing field");
      ++list_mods;
      list.insert(list.begin() + long(std::min(idx, list.size())), pick);
      for (size_t k = idx + 1; k < list.size(); ++k)
        if (list[k].slot == pick.slot && list[k].long_term == pick.long_term) {
          list.erase(list.begin() + long(k));
          break;
        }
      ++idx;
    }
    list_[l].assign(size_t(sh.num_ref_idx[l]), ListEntry{});
    for (size_t i = 0; i < list_[l].size() && i < list.size(); ++i) list_[l][i] = list[i];
  }
}

// Reference marking of a field (§8.2.5 with field picture numbers). The first field of a frame
// enters the DPB as a frame entry holding one field (after the sliding window, which works on
// frames, makes room), the second field joins its frame's entry; MMCOs mark single fields
// (1 / 2), move a field to long-term (3; a long-term frame index held by another frame frees
// it), cap the long-term indices (4) or make the current field long-term (6). The second field
// of a pair whose first field is long-term is long-term with the same index.
void Decoder::mark_field(const SliceHdr& sh, const Sps& sps, int slot, int poc, u32 uid, bool second,
                         std::shared_ptr<const ColMotion> col) {
  const int par = sh.bottom_field ? 1 : 0;
  const int max_fn = 1 << sps.log2_max_frame_num;
  const int max_refs = std::max(1, sps.max_num_ref_frames);
  const int cur_pic_num = 2 * sh.frame_num + 1;
  auto cur_entry = [&]() -> RefPic* {
    if (!second) return nullptr;
    for (auto& r : dpb_)
      if (r.slot == slot && r.frame_num == sh.frame_num && ((r.fields | r.lt_fields) & 3)) return &r;
    return nullptr;
  };
  bool cur_long = false, mmco5 = false;
  int cur_lt = 0;
  if (sh.idr() && !second) {
    dpb_.clear();
    max_lt_idx_ = sh.long_term_reference ? 0 : -1;
    cur_long = sh.long_term_reference;
    long_term_marked += cur_long ? 1 : 0;
  } else if (sh.adaptive_marking) {
    const RefPic* self = cur_entry();
    for (const auto& m : sh.mmcos) {
      ++mmco_ops[m.op];
      switch (m.op) {
        case 1:
          for (auto& r : dpb_)
            for (int p = 0; p < 2; ++p)
              if (((r.fields >> p) & 1) && field_pic_num(r, p, par, sh.frame_num, max_fn) == cur_pic_num - (m.a + 1))
                r.fields &= u8(~(1 << p));
          break;
        case 2:
          for (auto& r : dpb_)
            for (int p = 0; p < 2; ++p)
              if (((r.lt_fields >> p) & 1) && field_lt_pic_num(r, p, par) == m.a) r.lt_fields &= u8(~(1 << p));
          break;
        case 3: {
          RefPic* f = nullptr;
          int fp = 0;
          for (auto& r : dpb_)
            for (int p = 0; p < 2; ++p)
              if (((r.fields >> p) & 1) && field_pic_num(r, p, par, sh.frame_num, max_fn) == cur_pic_num - (m.a + 1)) {
                f = &r;
                fp = p;
              }
          if (!f) break;
          for (auto& r : dpb_)
            if (&r != f && (r.lt_fields & 3) && r.lt_idx == m.b) r.lt_fields = 0;
          f->fields &= u8(~(1 << fp));
          f->lt_fields |= u8(1 << fp);
          f->lt_idx = m.b;
          ++long_term_marked;
          break;
        }
        case 4:
          max_lt_idx_ = m.a - 1;
          for (auto& r : dpb_)
            if ((r.lt_fields & 3) && r.lt_idx > max_lt_idx_) r.lt_fields = 0;
          break;
        case 6:
          for (auto& r : dpb_)
            if (&r != self && (r.lt_fields & 3) && r.lt_idx == m.a) r.lt_fields = 0;
          cur_long = true;
          cur_lt = m.a;
          ++long_term_marked;
          break;
        case 5:  // every reference unused; this field counts as frame_num 0, POC 0 (first field only)
          if (second) throw UnsupportedStream("interlaced H.264: MMCO 5 in a second field is not supported");
          for (auto& r : dpb_) r.fields = r.lt_fields = 0;
          max_lt_idx_ = -1;
          mmco5 = true;
          break;
        default:
          break;
      }
    }
  } else if (!second) {  // sliding window (§8.2.5.3) on frames, for the first field of a frame
    int frames = 0, n_short = 0;
    for (const auto& r : dpb_) {
      frames += ((r.fields | r.lt_fields) & 3) ? 1 : 0;
      n_short += (r.fields & 3) ? 1 : 0;
    }
    if (frames >= max_refs && n_short > 0) {
      RefPic* oldest = nullptr;
      int ow = 0;
      for (auto& r : dpb_) {
        if (!(r.fields & 3)) continue;
        const int w = r.frame_num > sh.frame_num ? r.frame_num - max_fn : r.frame_num;
        if (!oldest || w < ow) {
          oldest = &r;
          ow = w;
        }
      }
      oldest->fields = 0;
    }
  }
  if (!cur_long && second)  // the pair's first field is long-term: so is this one
    if (const RefPic* f = cur_entry(); f && (f->lt_fields & 3)) {
      cur_long = true;
      cur_lt = f->lt_idx;
    }
  dpb_.erase(std::remove_if(dpb_.begin(), dpb_.end(), [](const RefPic& r) { return !((r.fields | r.lt_fields) & 3); }),
             dpb_.end());
  if (mmco5) poc = 0;
  RefPic* e = cur_entry();
  if (!e) {
    dpb_.push_back(RefPic{});
    e = &dpb_.back();
    e->slot = slot;
    e->frame_num = mmco5 ? 0 : sh.frame_num;
    e->poc = poc;
    e->uid = uid;
    e->fields = 0;
  }
  e->poc_f[par] = poc;
  e->uid_f[par] = uid;
  e->col_f[par] = std::move(col);
  e->poc = std::min(e->poc, poc);
  if (cur_long) {
    e->lt_fields |= u8(1 << par);
    e->lt_idx = cur_lt;
  } else {
    e->fields |= u8(1 << par);
  }
  e->long_term = (e->lt_fields & 3) && !(e->fields & 3);
}

int Decoder::reorder_depth(const Sps& sps) const {
  if (sps.max_num_reorder_frames >= 0) return sps.max_num_reorder_frames;
  if (sps.poc_type == 2 || sps.profile_idc == 66) return 0;  // output order = decoding order
  return adaptive_reorder_;
}

// C.4.5.3-style bumping in POC order: an IDR / MMCO5 picture first outputs everything still
// waiting (and itself: nothing after it can precede it); otherwise the smallest POC leaves once
// more than reorder_depth() pictures wait. A picture whose POC is below the last output one
// arrived too late for its turn: it is not output, and (without a VUI reorder depth) the
// depth learnt from the stream grows.
// Output ("bumping", C.4.5.3): pictures leave in (epoch, POC) order once more than the reorder
// depth are waiting. An IDR / MMCO5 picture starts a new epoch: the previous pictures still leave
// first (as no_output_of_prior_pics_flag = 0 requires) but one per decoded picture, like the
// steady state, so a stream with B pictures outputs one frame per access unit across GOPs
// instead of a burst at every IDR. `hard` (new picture geometry, or no reordering) outputs every
// waiting picture at once.
OutFrame Decoder::out_of(const Picture& pic) const {
  OutFrame f;
  f.slot = pic.target;
  f.info = pic.info;
  f.au = pic.au;
  f.poc = pic.poc;
  return f;
}

// The open field pair's frame leaves for the reorder buffer (its second field was decoded, or
// never came: then the missing field's rows are whatever the slot held).
void Decoder::close_pair(Picture& pic) {
  if (!pair_.open) return;
  pair_.open = false;
  OutFrame f = pair_.f;
  f.poc = pair_.have == 3 ? std::min(pair_.poc[0], pair_.poc[1]) : pair_.poc[(pair_.have >> 1) & 1];
  bump(pic, f, pair_.boundary, pair_.hard);
}

void Decoder::bump(Picture& pic, const OutFrame& f, bool new_epoch, bool hard) {
  auto before = [](const Pending& a, const Pending& b) {
    return a.epoch != b.epoch ? a.epoch < b.epoch : a.f.poc < b.f.poc;
  };
  auto take_min = [&] {
    auto it = std::min_element(pending_.begin(), pending_.end(), before);
    pic.outputs.push_back(it->f);
    last_out_poc_ = it->f.poc;
    last_out_epoch_ = i64(it->epoch);
    pending_.erase(it);
  };
  if (new_epoch) ++epoch_;
  if (hard)
    while (!pending_.empty()) take_min();
  if (last_out_epoch_ == i64(epoch_) && f.poc < last_out_poc_) {
    if (adaptive_reorder_ < 16) ++adaptive_reorder_;  // late: dropped from output
  } else {
    pending_.push_back({f, epoch_});
    while (int(pending_.size()) > reorder_cur_) take_min();
  }
  if (!pic.outputs.empty()) pinned_slot_ = pic.outputs.back().slot;
}

std::vector<OutFrame> Decoder::flush_output() {
  Picture tmp;
  close_pair(tmp);  // (a lone first field: output as it is)
  while (!pending_.empty()) {
    auto it = std::min_element(pending_.begin(), pending_.end(), [](const Pending& a, const Pending& b) {
      return a.epoch != b.epoch ? a.epoch < b.epoch : a.f.poc < b.f.poc;
    });
    tmp.outputs.push_back(it->f);
    pending_.erase(it);
  }
  if (!tmp.outputs.empty()) pinned_slot_ = tmp.outputs.back().slot;
  return tmp.outputs;
}

void Decoder::absorb_parameter_sets(const AccessUnit& au) {
  std::vector<u8> scratch;
  for (size_t i = 0; i < au.nals.size(); ++i) {
    const u8* p = au.nal(i);
    const size_t n = au.nal_size(i);
    if (n < 2) continue;
    const int t = h264::nal_type(p[0]);
    if (t != h264::kNalSps && t != h264::kNalPps) continue;
    size_t rn;
    const u8* r = unescape(p, n, epb_, scratch, rn);
    if (t == h264::kNalSps) {
      Sps s = h264::parse_sps(r, rn);
      sps_[s.sps_id] = s;
    } else {
      Pps q = h264::parse_pps(r, rn);
      pps_[q.pps_id] = q;
    }
  }
}

namespace {

class MbDecoder {
 public:
  MbDecoder(MbNeighbours& nb, Picture& pic, const SliceCtx& sc) : nb_(nb), pic_(pic), sc_(sc) {}

  void skip(int mb) {
    MbState& s = nb_.at(mb);
    s = MbState{};
    s.kind = kSkip;
    s.slice = u16(sc_.slice);
    nb_.begin(mb);
    s.qp = u8(sc_.qp);
    for (int k = 0; k < 4; ++k) s.ref[0][k] = 0;
    int mv[2];
    nb_.pskip_mv(mb, mv);
    for (auto& v : s.mv[0]) {
      v[0] = i16(mv[0]);
      v[1] = i16(mv[1]);
    }
    MbResidual res;
    emit(mb, s, res, 0, 0);
  }

  void macroblock(Bits& br, int mb) {
    const u32 mbt = br.ue();
    int it = -1;  // I-slice mb_type of an intra MB
    if (sc_.is_p) {
      VEP_CHECK(mbt <= 30, "bad P mb_type");
      if (mbt >= 5) it = int(mbt) - 5;
    } else {
      VEP_CHECK(mbt <= 25, "bad I mb_type");
      it = int(mbt);
    }
    MbState& s = nb_.at(mb);
    s = MbState{};
    s.slice = u16(sc_.slice);
    nb_.begin(mb);
    MbResidual res;
    if (it == 25) {  // I_PCM
      s.kind = kIPcm;
      std::fill(std::begin(s.tc), std::end(s.tc), u8(16));
      for (auto& c : s.tcc) std::fill(std::begin(c), std::end(c), u8(16));
      s.qp = u8(sc_.qp);
      br.align();
      const size_t off = br.pos() >> 3;
      VEP_CHECK(off + kPcmMbBytes <= br.size(), "truncated I_PCM macroblock");
      pcm_ = br.data() + off;
      br.skip(kPcmMbBytes * 8);
      emit(mb, s, res, 0, 0);
      pcm_ = nullptr;
      return;
    }
    int cbp_luma = 0, cbp_chroma = 0, i16_mode = 0, chroma_mode = 0;
    if (it == 0) {
      s.kind = kI4x4;
      for (int idx = 0; idx < 16; ++idx) {
        const int r = blk_to_raster(idx);
        const bool prev = br.u1();
        const int rem = prev ? 0 : int(br.u(3));
        const int pred = nb_.pred_intra4x4(mb, r, sc_.pps.constrained_intra_pred);
        s.i4[r] = u8(prev ? pred : (rem < pred ? rem : rem + 1));
      }
      chroma_mode = int(br.ue());
    } else if (it > 0) {
      s.kind = kI16x16;
      i16_mode = (it - 1) % 4;
      cbp_chroma = ((it - 1) / 4) % 3;
      cbp_luma = it >= 13 ? 15 : 0;
      std::fill(std::begin(s.i4), std::end(s.i4), u8(2));
      chroma_mode = int(br.ue());
    } else {
      s.kind = kInter;
      inter_pred(br, mb, s, int(mbt));
    }
    VEP_CHECK(chroma_mode <= 3, "bad intra_chroma_pred_mode");
    if (s.kind != kI16x16) {
      const u32 me = br.ue();
      VEP_CHECK(me < 48, "bad coded_block_pattern");
      const int cbp = s.kind == kI4x4 ? kCbpIntra[me] : kCbpInter[me];
      cbp_luma = cbp & 15;
      cbp_chroma = cbp >> 4;
    }
    int qp = sc_.qp;
    if (cbp_luma || cbp_chroma || s.kind == kI16x16) {
      const int dqp = br.se();
      VEP_CHECK(dqp >= -26 && dqp <= 25, "mb_qp_delta out of range");
      qp = (qp + dqp + 52) % 52;
      qp_out_ = qp;
    }
    s.qp = u8(qp);
    residual(br, mb, s, res, cbp_luma, cbp_chroma, qp);
    emit(mb, s, res, i16_mode, chroma_mode);
  }

  int qp_out_ = -1;  // updated QP_Y (the next MB's QP_Y,PRED), -1 = unchanged

 private:
  int read_ref(Bits& br) {
    const int n = sc_.sh.num_ref_idx[0];
    int r = 0;
    if (n == 2) r = int(br.u1() ^ 1u);
    else if (n > 2) r = int(br.ue());
    VEP_CHECK(r < n && sc_.list0[size_t(r)].slot >= 0, "ref_idx_l0 names a missing reference picture");
    return r;
  }

  void set_part(MbState& s, int x4, int y4, int w4, int h4, const int mv[2]) {
    for (int y = y4; y < y4 + h4; ++y)
      for (int x = x4; x < x4 + w4; ++x) {
        s.mv[0][y * 4 + x][0] = i16(mv[0]);
        s.mv[0][y * 4 + x][1] = i16(mv[1]);
      }
  }
  static u16 part_mask(int x4, int y4, int w4, int h4) {
    u16 m = 0;
    for (int y = y4; y < y4 + h4; ++y)
      for (int x = x4; x < x4 + w4; ++x) m |= u16(1u << (y * 4 + x));
    return m;
  }

  void inter_pred(Bits& br, int mb, MbState& s, int mbt) {
    struct Part {
      int x4, y4, w4, h4, ref, shape;
      int mvd[2];
    };
    Part parts[16];
    int np = 0;
    if (mbt <= 2) {
      const int n = mbt == 0 ? 1 : 2;
      int refs[2] = {0, 0};
      for (int i = 0; i < n; ++i) refs[i] = read_ref(br);
      for (int i = 0; i < n; ++i) {
        Part& p = parts[np++];
        p.ref = refs[i];
        p.mvd[0] = br.se();
        p.mvd[1] = br.se();
        if (mbt == 0) p.x4 = 0, p.y4 = 0, p.w4 = 4, p.h4 = 4, p.shape = 0;
        else if (mbt == 1) p.x4 = 0, p.y4 = 2 * i, p.w4 = 4, p.h4 = 2, p.shape = 1;
        else p.x4 = 2 * i, p.y4 = 0, p.w4 = 2, p.h4 = 4, p.shape = 2;
      }
      for (int i = 0; i < n; ++i) {
        const Part& p = parts[i];
        for (int y = p.y4 / 2; y < (p.y4 + p.h4) / 2; ++y)
          for (int x = p.x4 / 2; x < (p.x4 + p.w4) / 2; ++x) s.ref[0][y * 2 + x] = i8(p.ref);
      }
    } else {
      int sub[4], refs[4];
      for (int& t : sub) {
        t = int(br.ue());
        VEP_CHECK(t <= 3, "bad P sub_mb_type");
      }
      for (int i = 0; i < 4; ++i) refs[i] = mbt == 4 ? 0 : read_ref(br);
      for (int i = 0; i < 4; ++i) {
        s.ref[0][i] = i8(refs[i]);
        const int x8 = (i & 1) * 2, y8 = (i >> 1) * 2;
        const int cnt = sub[i] == 0 ? 1 : sub[i] == 3 ? 4 : 2;
        for (int j = 0; j < cnt; ++j) {
          Part& p = parts[np++];
          p.ref = refs[i];
          p.shape = 0;
          p.mvd[0] = br.se();
          p.mvd[1] = br.se();
          switch (sub[i]) {
            case 0: p.x4 = x8, p.y4 = y8, p.w4 = 2, p.h4 = 2; break;
            case 1: p.x4 = x8, p.y4 = y8 + j, p.w4 = 2, p.h4 = 1; break;
            case 2: p.x4 = x8 + j, p.y4 = y8, p.w4 = 1, p.h4 = 2; break;
            default: p.x4 = x8 + (j & 1), p.y4 = y8 + (j >> 1), p.w4 = 1, p.h4 = 1; break;
          }
        }
      }
    }
    u16 done = 0;
    for (int i = 0; i < np; ++i) {
      const Part& p = parts[i];
      int mvp[2];
      nb_.pred_mv(mb, p.x4, p.y4, p.w4, p.h4, 0, p.ref, done, p.shape, mvp);
      int mv[2] = {mvp[0] + p.mvd[0], mvp[1] + p.mvd[1]};
      VEP_CHECK(mv[0] >= -32768 && mv[0] <= 32767 && mv[1] >= -32768 && mv[1] <= 32767,
                "motion vector out of range");
      set_part(s, p.x4, p.y4, p.w4, p.h4, mv);
      done |= part_mask(p.x4, p.y4, p.w4, p.h4);
    }
  }

  // nC contexts (§9.2.1) of the current MB: total_coeff of the 4x4 blocks left of and above
  // every block (luma [(by + 1) * 5 + bx + 1], chroma [c][(by + 1) * 3 + bx + 1]), filled from
  // the A/B neighbours once and updated as blocks are parsed; kNa = not available.
  static constexpr u8 kNa = 0xFF;
  u8 ncl_[25];
  u8 ncc_[2][9];

  void nc_setup(int mb) {
    std::memset(ncl_, 0, sizeof ncl_);
    std::memset(ncc_, 0, sizeof ncc_);
    const int am = nb_.mb_at(mb, -1, 0), bm = nb_.mb_at(mb, 0, -1);
    const MbState* a = am >= 0 ? &nb_.at(am) : nullptr;
    const MbState* b = bm >= 0 ? &nb_.at(bm) : nullptr;
    for (int k = 0; k < 4; ++k) {
      ncl_[1 + k] = b ? b->tc[12 + k] : kNa;
      ncl_[(k + 1) * 5] = a ? a->tc[k * 4 + 3] : kNa;
    }
    ncl_[0] = kNa;
    for (int c = 0; c < 2; ++c) {
      for (int k = 0; k < 2; ++k) {
        ncc_[c][1 + k] = b ? b->tcc[c][2 + k] : kNa;
        ncc_[c][(k + 1) * 3] = a ? a->tcc[c][k * 2 + 1] : kNa;
      }
      ncc_[c][0] = kNa;
    }
  }
  static int nc_of(u8 na, u8 nb) {
    if (na != kNa && nb != kNa) return (na + nb + 1) >> 1;
    if (na != kNa) return na;
    if (nb != kNa) return nb;
    return 0;
  }
  int ncl(int r) const {
    const int i = ((r >> 2) + 1) * 5 + (r & 3) + 1;
    return nc_of(ncl_[i - 1], ncl_[i - 5]);
  }
  int ncc(int c, int b) const {
    const int i = ((b >> 1) + 1) * 3 + (b & 1) + 1;
    return nc_of(ncc_[c][i - 1], ncc_[c][i - 3]);
  }

  struct Scale {  // v = (level * ls[pos] * mul + add) >> sh  (§8.5.12.1)
    const int* ls;
    int mul, add, sh;
  };

  // Residual syntax with the scaling (§8.5.12.1, flat LevelScale) fused in: each level is
  // dequantised as it is placed into its raster position, so no level arrays or second pass.
  // Same output as dequantize_mb over MbLevels (the encoder's path).
  void residual(Bits& br, int mb, MbState& s, MbResidual& res, int cbp_luma, int cbp_chroma, int qp) {
    res.luma = 0;
    res.chroma = 0;
    nc_setup(mb);
    const bool intra16 = s.kind == kI16x16;
    auto scaler = [](int q) {
      return Scale{kLevelScale[q % 6], q >= 24 ? 1 << (q / 6 - 4) : 1, q >= 24 ? 0 : 1 << (3 - q / 6),
                   q >= 24 ? 0 : 4 - q / 6};
    };
    const auto dl = scaler(qp);
    auto luma_block = [&](int r, int start, int max_coeff, int dcv) {
      i16* d = res.blk[r];
      std::memset(d, 0, 16 * sizeof(i16));
      bool nz = dcv != 0;
      d[0] = sat16(dcv);
      const int tc = read_residual_block_cb(br, ncl(r), max_coeff, [&](int k, int l) {
        const int pos = kZigzag4x4[k + start];
        const int v = (l * dl.ls[pos] * dl.mul + dl.add) >> dl.sh;
        d[pos] = sat16(v);
        nz |= v != 0;
      });
      s.tc[r] = u8(tc);
      ncl_[((r >> 2) + 1) * 5 + (r & 3) + 1] = u8(tc);
      if (nz) res.luma |= u16(1u << r);
    };
    if (intra16) {
      int c[16] = {};
      const bool have_dc =
          read_residual_block_cb(br, ncl(0), 16, [&](int k, int l) { c[kZigzag4x4[k]] = l; }) > 0;
      int dcy[16] = {};
      if (have_dc) {
        hadamard4x4(c);
        const int ls = 16 * kNormAdjust[qp % 6][0];
        for (int k = 0; k < 16; ++k)
          dcy[k] = qp >= 36 ? c[k] * ls * (1 << (qp / 6 - 6)) : (c[k] * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
      }
      for (int idx = 0; idx < 16; ++idx) {
        const int r = blk_to_raster(idx);
        if (cbp_luma) {
          luma_block(r, 1, 15, dcy[r]);
        } else if (dcy[r] != 0) {
          i16* d = res.blk[r];
          std::memset(d, 0, 16 * sizeof(i16));
          d[0] = sat16(dcy[r]);
          res.luma |= u16(1u << r);
        }
      }
    } else {
      for (int idx = 0; idx < 16; ++idx)
        if ((cbp_luma >> (idx >> 2)) & 1) luma_block(blk_to_raster(idx), 0, 16, 0);
    }
    if (cbp_chroma) {
      const int qpc = chroma_qp(qp, sc_.pps.chroma_qp_index_offset);
      const auto dc = scaler(qpc);
      const int ls = 16 * kNormAdjust[qpc % 6][0];
      int dcv[2][4];
      for (int c = 0; c < 2; ++c) {
        int v[4] = {0, 0, 0, 0};
        read_residual_block_cb(br, -1, 4, [&](int k, int l) { v[k] = l; });
        const int f[4] = {v[0] + v[1] + v[2] + v[3], v[0] - v[1] + v[2] - v[3],
                          v[0] + v[1] - v[2] - v[3], v[0] - v[1] - v[2] + v[3]};
        for (int b = 0; b < 4; ++b) dcv[c][b] = ((f[b] * ls) * (1 << (qpc / 6))) >> 5;
      }
      for (int c = 0; c < 2; ++c)
        for (int b = 0; b < 4; ++b) {
          i16* d = res.blk[16 + c * 4 + b];
          bool nz = dcv[c][b] != 0;
          if (cbp_chroma & 2) {
            std::memset(d, 0, 16 * sizeof(i16));
            d[0] = sat16(dcv[c][b]);
            const int tc = read_residual_block_cb(br, ncc(c, b), 15, [&](int k, int l) {
              const int pos = kZigzag4x4[k + 1];
              const int v = (l * dc.ls[pos] * dc.mul + dc.add) >> dc.sh;
              d[pos] = sat16(v);
              nz |= v != 0;
            });
            s.tcc[c][b] = u8(tc);
            ncc_[c][((b >> 1) + 1) * 3 + (b & 1) + 1] = u8(tc);
          } else if (nz) {
            std::memset(d, 0, 16 * sizeof(i16));
            d[0] = sat16(dcv[c][b]);
          }
          if (nz) res.chroma |= u8(1u << (c * 4 + b));
        }
    }
    VEP_CHECK(!br.overrun(), "slice data overrun");
  }

  void emit(int mb, const MbState& s, const MbResidual& res, int i16_mode, int chroma_mode) {
    MbRec m{};
    m.kind = s.kind;
    m.qp = s.kind == kIPcm ? 0 : s.qp;
    m.qpc = u8(chroma_qp(m.qp, sc_.pps.chroma_qp_index_offset));
    m.qpc2 = m.qpc;  // (the fast path runs only when both chroma offsets are equal)
    m.i16_mode = u8(i16_mode);
    m.chroma_mode = u8(chroma_mode);
    m.dbk = u8((sc_.sh.disable_deblocking == 1 ? 1 : 0) | (sc_.sh.disable_deblocking == 2 ? 2 : 0));
    m.alpha_off = i8(sc_.sh.alpha_off);
    m.beta_off = i8(sc_.sh.beta_off);
    m.slice = s.slice;
    for (int k = 0; k < 4; ++k) {
      m.ref[k] = s.ref[0][k] >= 0 ? u8(sc_.list0[size_t(s.ref[0][k])].slot) : u8(0xFF);
      m.ref1[k] = u8(0xFF);
    }
    for (int r = 0; r < 16; ++r) m.i4[r >> 1] |= u8((s.kind == kI4x4 ? s.i4[r] : 0) << ((r & 1) * 4));
    for (int r = 0; r < 16; ++r) m.nz |= u16(s.tc[r] ? 1u << r : 0u);
    store_mb(pic_, mb, m, s, &res, pcm_, nullptr);
  }

  MbNeighbours& nb_;
  Picture& pic_;
  const SliceCtx& sc_;
  const u8* pcm_ = nullptr;
};

}  // namespace

namespace {

// The fast CAVLC MbDecoder above covers a slice when nothing beyond Baseline-style syntax is in
// use (the default synthetic camera streams); everything else goes to decode_slice_generic.
bool legacy_slice(const SliceHdr& sh, const Sps& sps, const Pps& pps) {
  return !pps.cabac && !sh.field_pic && sps.chroma_format_idc == 1 && sps.bit_depth_luma == 8 && (sh.type() == h264::kP || sh.type() == h264::kI) && !pps.transform_8x8_mode &&
         !sps.scaling_matrix_present && !pps.scaling_matrix_present && !sh.explicit_wp &&
         pps.chroma_qp_index_offset == pps.second_chroma_qp_index_offset;
}

// Surfaces a stream needs: references + pictures waiting for output + the picture being decoded
// + the newest output (kept until a newer one replaces it).
int dpb_slots_for(const Sps& sps) {
  int bound;
  if (sps.max_num_reorder_frames >= 0) bound = sps.max_num_reorder_frames;
  else if (sps.poc_type == 2 || sps.profile_idc == 66) bound = 0;
  else bound = sps.max_dpb_frames();
  return std::min(kMaxDpbSlots, std::max(1, sps.max_num_ref_frames) + bound + 2);
}

}  // namespace

static void validate_picture(const Picture& p);

// One slice kept for the parallel parse of its access unit (Decoder::parse).
struct Decoder::SliceUnit {
  MbNeighbours nb;        // this slice's neighbour state (own epoch: other slices' MBs unavailable)
  Picture shard;          // this slice's records (full-size MB array, own pools)
  ColBuild colb;          // colocated motion into the picture's table, with this slice's list uids
  std::vector<u8> rbsp;   // slice RBSP after the NAL header byte
  SliceHdr sh;
  const Sps* sps = nullptr;
  const Pps* pps = nullptr;
  size_t bitpos = 0;      // first bit of slice_data()
  int slice_idx = 0;
  std::vector<ListEntry> list[2];
  std::array<std::vector<u32>, 2> uids;
};

PicturePtr Decoder::parse(const AccessUnit& au, i64 tag, size_t* next_nal) {
  struct FenceOnExit {  // the records' non-temporal stores (store_rec) are ordered before the return
    ~FenceOnExit() {
#if defined(__x86_64__)
      _mm_sfence();
#endif
    }
  } fence;
  auto pic = pic_pool_->acquire([](Picture& p) {  // default state, pool capacities kept
    auto mbs = std::move(p.mbs);
    auto coefs = std::move(p.coefs), mvs = std::move(p.mvs);
    auto wps = std::move(p.wps);
    std::vector<OutFrame> outputs = std::move(p.outputs);
    p = Picture{};
    coefs.clear();
    mvs.clear();
    wps.clear();
    outputs.clear();
    p.mbs = std::move(mbs);
    p.coefs = std::move(coefs);
    p.mvs = std::move(mvs);
    p.wps = std::move(wps);
    p.outputs = std::move(outputs);
  });
  bool got = false;
  bool hard_flush = false;  // IDR with a new picture geometry: waiting pictures leave at once
  bool second_field = false;  // this picture completes the open field pair
  int slice_idx = 0;
  SliceHdr first;
  const Sps* act_sps = nullptr;
  const Pps* act_pps = nullptr;
  std::vector<u8> scratch;
  std::vector<std::array<std::vector<u32>, 2>> slice_uids;  // list uids per slice (colocated motion)
  ColBuild colb;
  std::shared_ptr<ColMotion> col_built;
  struct ColbGuard {  // the picture never keeps a pointer to this frame's ColBuild
    Picture* p;
    ~ColbGuard() { p->colb = nullptr; }
  } colb_guard{pic.get()};
  int nslices = 0;  // slice NALs of the access unit: several -> parsed in parallel
  for (size_t i = 0; i < au.nals.size(); ++i)
    if (au.nal_size(i) >= 2) {
      const int t = h264::nal_type(au.nal(i)[0]);
      nslices += (t == h264::kNalSlice || t == h264::kNalIdr) ? 1 : 0;
    }
  const bool par = parallel_slices_ && nslices >= 2 && FanOut::shared().size() > 0;
  int nunits = 0;
  const size_t start = next_nal ? *next_nal : 0;
  if (next_nal) *next_nal = au.nals.size();
  for (size_t i = start; i < au.nals.size(); ++i) {
    const u8* p = au.nal(i);
    const size_t n = au.nal_size(i);
    if (n < 2) continue;
    const int t = h264::nal_type(p[0]);
    if (t == h264::kNalSps || t == h264::kNalPps) {
      size_t rn;
      const u8* r = unescape(p, n, epb_, scratch, rn);
      if (t == h264::kNalSps) {
        Sps s = h264::parse_sps(r, rn);
        check_sps_supported(s);
        sps_[s.sps_id] = s;
      } else {
        Pps q = h264::parse_pps(r, rn);
        pps_[q.pps_id] = q;
      }
      continue;
    }
    if (t >= 2 && t <= 4) throw UnsupportedStream("H.264 data partitioning is not supported");
    if (t != h264::kNalSlice && t != h264::kNalIdr) continue;
    size_t rn;
    const u32 *kb = nullptr, *ke = nullptr;
    au.epb_of(i, &kb, &ke);
    const u8* r = unescape(p, n, epb_, rbsp_, rn, kb, ke);
    Bits peek(r + 1, rn - 1);
    peek.ue();
    peek.ue();
    const int pps_id = int(peek.ue());
    auto pit = pps_.find(pps_id);
    if (pit == pps_.end()) throw UnsupportedStream("slice references unknown PPS");
    auto sit = sps_.find(pit->second.sps_id);
    if (sit == sps_.end()) throw UnsupportedStream("slice references unknown SPS");
    const Sps& sps = sit->second;
    const Pps& pps = pit->second;
    check_sps_supported(sps);
    Bits br(r + 1, rn - 1);
    const SliceHdr sh = read_slice_header(br, p[0], sps, pps);
    if (sh.redundant_pic_cnt > 0) {  // §7.4.3: a decoder may ignore redundant coded pictures
      ++redundant_slices_skipped;
      continue;
    }
    if (sh.field_pic && (sps.bit_depth_luma > 8 || sps.chroma_format_idc == 2))
      throw UnsupportedStream("H.264 High 10 / 4:2:2 field pictures are not supported (progressive only)");
    if (!got) {
      first = sh;
      act_sps = &sps;
      act_pps = &pps;
      const int slots = dpb_slots_for(sps);
      VEP_CHECK(slots <= kMaxDpbSlots, "max_num_ref_frames out of range");
      const int W = sps.width_mbs, H = sps.height_mbs();
      second_field = sh.field_pic && pair_.open && pair_.bottom != int(sh.bottom_field) &&
                     pair_.frame_num == sh.frame_num;
      if (!second_field) close_pair(*pic);  // an unpaired field leaves before this picture
      if (sh.idr() && !second_field) {
        hard_flush = slots != dpb_slots_ || W != wmbs_ || H != hmbs_ || sh.field_pic != field_mode_ ||
                     sps.bit_depth_luma != bd_ || (sps.chroma_format_idc == 2) != (cf_ == 2);
        bd_ = sps.bit_depth_luma;
        cf_ = sps.chroma_format_idc == 2 ? 2 : 1;
        field_mode_ = sh.field_pic;
        have_idr_ = true;
        dpb_slots_ = slots;
        wmbs_ = W;
        hmbs_ = H;
        reorder_cur_ = reorder_depth(sps);
      } else {
        if (!have_idr_) throw Error("vep: H.264 stream does not start with an IDR picture");
        // a non-IDR picture may not change the picture size or the DPB (a mid-GOP SPS that
        // does would make earlier pictures of a batch write outside the surfaces)
        VEP_CHECK(slots == dpb_slots_ && W == wmbs_ && H == hmbs_ && sps.bit_depth_luma == bd_ &&
                      (sps.chroma_format_idc == 2) == (cf_ == 2),
                  "SPS changed without an IDR picture");
        if (sh.field_pic != field_mode_)
          throw UnsupportedStream("interlaced H.264: frame and field pictures mixed in one IDR period are not supported");
      }
      if (sh.idr() && !second_field) {
        // IDR: the DPB is emptied; pictures waiting for output stay (they leave before the
        // IDR's, bump(); no_output_of_prior_pics is not honoured: a viewer wants every frame)
        dpb_.clear();
        max_lt_idx_ = -1;
      }
      pic->poc = compute_poc(sh, sps);
      const int Hp = sh.field_pic ? H / 2 : H;  // (a field: half the frame's MB rows)
      pic->wmbs = W;
      pic->hmbs = Hp;
      // every record is written by store_mb or by the concealment pass below: a recycled
      // picture of the same size needs no clearing
      if (pic->mbs.size() != size_t(W) * Hp) pic->mbs.assign(size_t(W) * Hp, MbRec{});
      pic->coefs.reserve(size_t(W) * Hp * 32);
      pic->mvs.reserve(size_t(W) * Hp * 16);
      pic->dpb_slots = field_mode_ ? 2 * dpb_slots_ : dpb_slots_;
      pic->structure = sh.field_pic ? 1 + int(sh.bottom_field) : 0;
      pic->bd = sps.bit_depth_luma;
      pic->cf = sps.chroma_format_idc == 2 ? 2 : 1;
      pic->qp_bias = 6 * (sps.bit_depth_luma - 8);
      pic->qpc_bias = 6 * (sps.bit_depth_chroma - 8);
      pic->second_field = second_field;
      pic->constrained_intra = pps.constrained_intra_pred;
      pic->idr = sh.idr();
      PictureInfo& pi = pic->info;
      pi.coded_width = sps.coded_width();
      pi.coded_height = sps.coded_height();
      pi.width = sps.width();
      pi.height = sps.height();
      pi.crop_left = sps.crop_left;
      pi.crop_top = sps.crop_top;
      pi.pict_type = "PBISi"[sh.type()];
      pi.idr = sh.idr();
      pi.frame_num = sh.frame_num;
      pi.fps = sps.fps();
      pic->au.pts = au.pts;
      pic->au.dts = au.dts;
      pic->au.arrival_ms = au.arrival_ms;
      pic->au.keyframe = au.keyframe;
      pic->au.corrupt = au.corrupt;
      pic->au.tag = tag;
      nb_.reset(W, Hp, true);
      if (sh.field_pic) {  // field slot 2 * frame slot + parity
        const int fs = second_field ? pair_.slot : pick_slot();
        pic->target = 2 * fs + int(sh.bottom_field);
        if (!second_field) {
          pair_ = OpenPair{};
          pair_.open = true;
          pair_.slot = fs;
          pair_.frame_num = sh.frame_num;
          pair_.bottom = int(sh.bottom_field);
          pair_.ref = sh.nal_ref_idc != 0;
          pair_.boundary = sh.idr();
          pair_.hard = sh.idr() && (hard_flush || reorder_cur_ == 0);
          pair_.f.slot = fs;
          pair_.f.info = pic->info;
          pair_.f.au = pic->au;
          pair_.f.fields = true;
        }
        pair_.have |= u8(1 << int(sh.bottom_field));
        pair_.poc[int(sh.bottom_field)] = pic->poc;
      } else {
        pic->target = pick_slot();  // (pictures waiting for output keep their slots until bump)
      }
      if (sh.nal_ref_idc != 0 && sps.profile_idc != 66) {  // B slices may use this motion
        col_built = col_pool_->acquire([](ColMotion&) {});  // (every entry is written below)
        col_built->wmbs = W;
        col_built->hmbs = Hp;
        col_built->corners = sps.direct_8x8;
        col_built->b.resize(size_t(W) * Hp * size_t(sps.direct_8x8 ? 4 : 16));
        colb.col = col_built.get();
        pic->colb = &colb;
      }
      got = true;
    } else {
      VEP_CHECK(&sps == act_sps, "slices of one picture reference different SPSs");
      if (sh.field_pic != first.field_pic || sh.bottom_field != first.bottom_field) {
        // the next picture of the access unit (the pair's other field): the caller parses it next
        VEP_CHECK(next_nal != nullptr, "H.264: one access unit holds several pictures");
        *next_nal = i;
        break;
      }
      if (sh.type() == h264::kB || pic->info.pict_type == 'I') pic->info.pict_type = "PBISi"[sh.type()];
    }
    if (sh.field_pic) build_field_lists(sh, sps, pic->poc);
    else build_lists(sh, sps, pic->poc);
    std::array<std::vector<u32>, 2> uids;
    for (int l = 0; l < 2; ++l)
      for (const auto& e : list_[l]) uids[size_t(l)].push_back(e.uid);
    slice_uids.push_back(std::move(uids));
    colb.set_uids(&slice_uids.back());
    if (par) {  // kept until the access unit's last slice (parsed in parallel below)
      if (units_.size() <= size_t(nunits)) units_.push_back(std::make_unique<SliceUnit>());
      SliceUnit& u = *units_[size_t(nunits++)];
      u.rbsp.assign(r + 1, r + rn);
      u.sh = sh;
      u.sps = &sps;
      u.pps = &pps;
      u.bitpos = br.pos();
      u.slice_idx = slice_idx;
      u.list[0] = list_[0];
      u.list[1] = list_[1];
      u.uids = slice_uids.back();
    } else {
      parse_slice_data(nb_, *pic, sh, sps, pps, r + 1, rn - 1, br.pos(), slice_idx, list_);
    }
    ++slice_idx;
    VEP_CHECK(slice_idx < 65535, "too many slices");
  }
  VEP_CHECK(got, "access unit has no slice");
  (void)act_pps;
  std::vector<u8> covered;  // parallel slices: MBs some slice decoded
  if (par) {
    const int W = pic->wmbs, H = pic->hmbs;
    ColMotion* col_target = colb.col;
    FanOut::shared().run(nunits, [&](int k) {
      SliceUnit& u = *units_[size_t(k)];
      u.nb.reset(W, H, true);
      Picture& sh = u.shard;
      sh.wmbs = W;
      sh.hmbs = H;
      if (sh.mbs.size() != size_t(W) * H) sh.mbs.assign(size_t(W) * H, MbRec{});
      sh.coefs.clear();
      sh.mvs.clear();
      sh.wps.clear();
      sh.intra_mbs = sh.intra_res = sh.inter_mbs = 0;
      sh.deblock = false;
      sh.target = pic->target;
      sh.dpb_slots = pic->dpb_slots;
      sh.constrained_intra = pic->constrained_intra;
      sh.poc = pic->poc;
      sh.bd = pic->bd;
      sh.cf = pic->cf;
      sh.qp_bias = pic->qp_bias;
      sh.qpc_bias = pic->qpc_bias;
      u.colb.col = col_target;
      u.colb.set_uids(&u.uids);
      sh.colb = col_target ? &u.colb : nullptr;
      parse_slice_data(u.nb, sh, u.sh, *u.sps, *u.pps, u.rbsp.data(), u.rbsp.size(), u.bitpos, u.slice_idx, u.list);
#if defined(__x86_64__)
      _mm_sfence();  // (the shard's non-temporal record stores, before the join)
#endif
    });
    parallel_slices_run_ += u64(nunits);
    // merge in slice order: the MBs each slice decoded, pool offsets rebased
    covered.assign(size_t(pic->nmbs()), 0);
    for (int k = 0; k < nunits; ++k) {
      SliceUnit& u = *units_[size_t(k)];
      const Picture& sh = u.shard;
      const u32 coef0 = u32(pic->coefs.size()), mv0 = u32(pic->mvs.size()), wp0 = u32(pic->wps.size());
      const u32 res0 = u32(pic->intra_res);
      pic->coefs.insert(pic->coefs.end(), sh.coefs.begin(), sh.coefs.end());
      pic->mvs.insert(pic->mvs.end(), sh.mvs.begin(), sh.mvs.end());
      pic->wps.insert(pic->wps.end(), sh.wps.begin(), sh.wps.end());
      pic->intra_mbs += sh.intra_mbs;
      pic->intra_res += sh.intra_res;
      pic->inter_mbs += sh.inter_mbs;
      pic->deblock |= sh.deblock;
      for (int mb = u.sh.first_mb; mb < pic->nmbs(); ++mb) {
        if (!u.nb.announced(mb)) continue;
        VEP_CHECK(!covered[size_t(mb)], "H.264: slices overlap");
        covered[size_t(mb)] = 1;
        MbRec m = sh.mbs[size_t(mb)];
        m.coef += coef0;
        if (m.kind == kSkip || m.kind == kInter) m.mv += mv0;
        if (m.flags & kMbWp) m.wp += wp0;
        if (m.res != kNoRes) m.res += res0;
        pic->mbs[size_t(mb)] = m;
      }
    }
  }
  int ncovered = 0;
  if (par)
    for (u8 c : covered) ncovered += c;
  auto announced = [&](int mb) { return par ? covered[size_t(mb)] != 0 : nb_.announced(mb); };
  // conceal macroblocks no slice covered (lost slices): copy from the first reference, or grey
  // (an MB announced but not finished would have thrown: announced = decoded here)
  int missing = 0;
  for (int mb = 0; (par ? ncovered : nb_.announced_count()) < pic->nmbs() && mb < pic->nmbs(); ++mb) {
    MbRec& m = pic->mbs[size_t(mb)];
    if (announced(mb)) continue;
    ++missing;
    if (pic->colb) colb.none(mb);
    m = MbRec{};
    m.res = kNoRes;
    m.dbk = 1;
    m.slice = u16(0xFFFF);
    std::fill(std::begin(m.ref1), std::end(m.ref1), u8(0xFF));
    if (!dpb_.empty()) {
      m.kind = kSkip;
      int cs = dpb_.front().slot;
      if (pic->structure) {  // a field of that frame, the current parity if it holds one
        const int par = pic->structure - 1;
        cs = 2 * cs + ((((dpb_.front().fields | dpb_.front().lt_fields) >> par) & 1) ? par : 1 - par);
      }
      for (auto& rf : m.ref) rf = u8(cs);
      m.mv = u32(pic->mvs.size());
      m.flags |= kMbMv16;
      pic->mvs.resize(pic->mvs.size() + 2, 0);
      ++pic->inter_mbs;
    } else {
      m.kind = kI16x16;
      m.i16_mode = 2;
      std::fill(std::begin(m.ref), std::end(m.ref), u8(0xFF));
      ++pic->intra_mbs;
    }
  }
  pic->info.coded_mbs = pic->nmbs() - missing;
  const u32 uid = next_uid_++;
  if (first.field_pic) {
    if (first.nal_ref_idc != 0)
      mark_field(first, *act_sps, pic->target >> 1, pic->poc, uid, second_field && pair_.ref, std::move(col_built));
    if (first.has_mmco5() && !second_field) {  // POC / frame_num restart (§8.2.1): the pair
      pic->poc = 0;                            // continues with frame_num 0 and a new period
      pair_.frame_num = 0;
      pair_.poc[int(first.bottom_field)] = 0;
      pair_.boundary = true;
      pair_.hard = reorder_cur_ == 0;
    }
    if (second_field) close_pair(*pic);  // the frame is complete
  } else {
    if (first.nal_ref_idc != 0) {
      // (B slices possible: the motion for direct prediction, built as the MBs were stored)
      mark_references(first, *act_sps, pic->target, pic->poc, uid, std::move(col_built));
    }
    const bool boundary = first.idr() || first.has_mmco5();
    // MMCO 5: the picture's POC becomes 0 (tempPicOrderCnt subtracted, §8.2.1), for output order
    // too: it starts the new period the later pictures' POCs count from
    if (first.has_mmco5()) pic->poc = 0;
    bump(*pic, out_of(*pic), boundary, boundary && (hard_flush || reorder_cur_ == 0));
  }
  // (store_mb validated every record as it was written; concealed ones are built in range)
  if (missing || par) validate(*pic);
  else validate_picture(*pic);
  return pic;
}

Decoder::Decoder() {
  if (const char* e = std::getenv("VEP_AVC_SLICE_THREADS")) parallel_slices_ = e[0] != '0';
}
Decoder::~Decoder() = default;

// The slice data of one slice (either entropy layer) into `pic` through neighbour state `nb`.
void Decoder::parse_slice_data(MbNeighbours& nb, Picture& pic, const SliceHdr& sh, const Sps& sps, const Pps& pps,
                               const u8* data, size_t n, size_t bitpos, int slice_idx,
                               const std::vector<ListEntry> (&lists)[2]) {
  if (legacy_slice(sh, sps, pps)) {
    Bits br(data, n, bitpos);
    const size_t stop = BitReader(data, n).stop_bit_pos();
    SliceCtx sc{sh, pps, slice_idx, sh.type() == h264::kP, sh.qp, lists[0]};
    const int total = pic.nmbs();
    int mb = sh.first_mb;
    VEP_CHECK(mb < total, "first_mb_in_slice past end of picture");
    bool more = true;
    while (more) {
      if (sc.is_p) {
        const u32 run = br.ue();
        VEP_CHECK(u32(total - mb) >= run, "mb_skip_run past end of picture");
        MbDecoder d(nb, pic, sc);
        for (u32 k = 0; k < run; ++k) d.skip(mb++);
        if (run > 0) {
          more = br.pos() < stop;
          if (!more) break;
        }
      }
      VEP_CHECK(mb < total, "macroblock address past end of picture");
      MbDecoder d(nb, pic, sc);
      d.macroblock(br, mb);
      if (d.qp_out_ >= 0) sc.qp = d.qp_out_;
      VEP_CHECK(!br.overrun(), "slice data overrun");
      more = br.pos() < stop;
      ++mb;
    }
    return;
  }
  SliceEnv env;
  env.sh = &sh;
  env.sps = &sps;
  env.pps = &pps;
  env.slice = slice_idx;
  env.list[0] = &lists[0];
  env.list[1] = &lists[1];
  env.cur_poc = pic.poc;
  env.scaling = h264::resolve_scaling(sps, pps);
  env.field = sh.field_pic;
  decode_slice_generic(nb, pic, env, data, n, bitpos);
}

// One record against the picture's pools (store_mb checks every record as it is written, so
// the GPU never sees an out-of-range index from a malformed stream).
// (`written`: store_mb has just appended this MB's groups, so they are inside the pool by
// construction and their mask words need not be walked again.)
static inline void validate_mb(const Picture& p, const MbRec& m, bool written = false) {
  const size_t ncoef = p.coefs.size(), nmv = p.mvs.size();
  VEP_CHECK(m.kind <= kI8x8, "macroblock kind out of range");
  VEP_CHECK(p.cf == 2 || m.chroma_coded < 0x100, "chroma block mask out of range");
  VEP_CHECK(m.qp <= 51 + p.qp_bias && m.qpc <= 51 + p.qpc_bias && m.qpc2 <= 51 + p.qpc_bias,
            "macroblock QP out of range");
  if (m.kind == kIPcm) {
    const size_t ns = p.cf == 2 ? size_t(kPcmMaxSamples) : size_t(kPcmMbBytes);
    VEP_CHECK(size_t(m.coef) + (p.bd > 8 ? ns : ns / 2) <= ncoef, "I_PCM samples outside the pool");
    return;
  }
  // sparse groups: the mask words, then as many values as they announce, inside the pool
  const size_t nw = size_t(coef_words(m));
  VEP_CHECK(size_t(m.coef) + nw <= ncoef, "coefficient masks outside the pool");
  VEP_CHECK(written || size_t(m.coef) + nw + coef_values(p.coefs.data(), m) <= ncoef, "coefficients outside the pool");
  VEP_CHECK(m.chroma_mode <= 3 && m.i16_mode <= 3, "intra prediction mode out of range");
  if (m.flags & kMbT8x8)
    for (int q = 0; q < 4; ++q) {
      const u32 g = (u32(m.luma_coded) >> ((q & 1) * 2 + (q >> 1) * 8)) & 0x33u;
      VEP_CHECK(g == 0 || g == 0x33u, "8x8 residual block partially coded");
    }
  if (m.kind == kSkip || m.kind == kInter) {
    VEP_CHECK(size_t(m.mv) + size_t(mv_per_list(m.flags)) * ((m.flags & kMbL1) ? 2 : 1) <= nmv,
              "motion vectors outside the pool");
    for (int k = 0; k < 4; ++k) {
      const int r0 = m.ref[k], r1 = m.ref1[k];
      VEP_CHECK(r0 != 0xFF || r1 != 0xFF, "inter partition without a reference");
      VEP_CHECK((r0 == 0xFF || r0 < p.dpb_slots) && (r1 == 0xFF || r1 < p.dpb_slots),
                "reference slot outside the DPB");
      VEP_CHECK(r1 == 0xFF || (m.flags & kMbL1), "list-1 reference without list-1 motion");
    }
    if (m.flags & kMbWp) VEP_CHECK(size_t(m.wp) + 4 <= p.wps.size(), "weights outside the pool");
  } else if (m.kind == kI4x4) {
    for (u8 b : m.i4) VEP_CHECK((b & 15) <= 8 && (b >> 4) <= 8, "Intra_4x4 mode out of range");
  } else if (m.kind == kI8x8) {
    VEP_CHECK((m.flags & kMbT8x8) && (m.i4[0] & 15) <= 8 && (m.i4[0] >> 4) <= 8 && (m.i4[1] & 15) <= 8 &&
                  (m.i4[1] >> 4) <= 8,
              "Intra_8x8 mode out of range");
  }
  VEP_CHECK(m.res == kNoRes || (is_intra(m.kind) && m.res < u32(p.intra_res)), "residual slot out of range");
}

// validate_mb(p, m, true) as one branch-free verdict (store_mb's per-MB check): every condition
// folded into one flag, the detailed check (and its message) only when something fails.
static inline void validate_written_mb(const Picture& p, const MbRec& m) {
  const size_t ncoef = p.coefs.size(), nmv = p.mvs.size();
  bool ok = (m.kind <= kI8x8) & (p.cf == 2 || m.chroma_coded < 0x100) & (m.qp <= 51 + p.qp_bias) &
            (m.qpc <= 51 + p.qpc_bias) & (m.qpc2 <= 51 + p.qpc_bias);
  if (m.kind != kIPcm) {
    ok &= size_t(m.coef) + size_t(coef_words(m)) <= ncoef;
    ok &= (m.chroma_mode <= 3) & (m.i16_mode <= 3);
    if (m.flags & kMbT8x8)
      for (int q = 0; q < 4; ++q) {
        const u32 g = (u32(m.luma_coded) >> ((q & 1) * 2 + (q >> 1) * 8)) & 0x33u;
        ok &= (g == 0) | (g == 0x33u);
      }
    if (m.kind == kSkip || m.kind == kInter) {
      ok &= size_t(m.mv) + size_t(mv_per_list(m.flags)) * ((m.flags & kMbL1) ? 2 : 1) <= nmv;
      u32 r0w, r1w;
      std::memcpy(&r0w, m.ref, 4);
      std::memcpy(&r1w, m.ref1, 4);
      for (int k = 0; k < 4; ++k) {
        const u32 r0 = (r0w >> (8 * k)) & 0xFFu, r1 = (r1w >> (8 * k)) & 0xFFu;
        ok &= (r0 != 0xFF) | (r1 != 0xFF);
        ok &= (r0 == 0xFF) | (r0 < u32(p.dpb_slots));
        ok &= (r1 == 0xFF) | (r1 < u32(p.dpb_slots));
        ok &= (r1 == 0xFF) | ((m.flags & kMbL1) != 0);
      }
      if (m.flags & kMbWp) ok &= size_t(m.wp) + 4 <= p.wps.size();
    } else if (m.kind == kI4x4 || m.kind == kI8x8) {
      for (u8 b : m.i4) ok &= ((b & 15) <= 8) & ((b >> 4) <= 8);
      if (m.kind == kI8x8) ok &= (m.flags & kMbT8x8) != 0;
    }
    ok &= m.res == kNoRes || (is_intra(m.kind) && m.res < u32(p.intra_res));
  }
  if (!ok) validate_mb(p, m, true);  // (throws, naming the failed check)
}

static void validate_picture(const Picture& p) {
  VEP_CHECK(p.dpb_slots >= 1 && p.dpb_slots <= kMaxDpbSlots && p.target >= 0 && p.target < p.dpb_slots,
            "picture DPB slots out of range");
  VEP_CHECK(p.wmbs > 0 && p.hmbs > 0 && p.mbs.size() == size_t(p.nmbs()), "picture size mismatch");
}

void validate(const Picture& p) {
  validate_picture(p);
  for (const MbRec& m : p.mbs) validate_mb(p, m);
}

// ------------------------------------------------------------------------- shared internals

// Non-temporal stores of `bytes` (a multiple of 8) from `src` to the 8-byte aligned `dst`: for
// the parser's write-once outputs (records, colocated motion) that are read next by the GPU or
// by another picture's parse on another thread — write-allocating them only pulled their lines
// in for ownership and evicted the parser's working set. Decoder::parse ends with an sfence.
static inline void stream_words(void* dst, const void* src, size_t bytes) {
#if defined(__x86_64__)
  long long w[16];
  for (size_t o = 0; o < bytes; o += sizeof w) {
    const size_t n = bytes - o < sizeof w ? bytes - o : sizeof w;
    std::memcpy(w, static_cast<const char*>(src) + o, n);
    long long* d = reinterpret_cast<long long*>(static_cast<char*>(dst) + o);
    for (size_t k = 0; k < n / 8; ++k) _mm_stream_si64(d + k, w[k]);
  }
#else
  std::memcpy(dst, src, bytes);
#endif
}

void ColBuild::none(int mb) {
  const int per = col->corners ? 4 : 16;
  ColMotion::Blk* out = &col->b[size_t(mb) * size_t(per)];
  for (int k = 0; k < per; ++k) out[k] = ColMotion::Blk{{0, 0}, 0u, i8(-1)};
}

void ColBuild::store(int mb, const MbState& st) {
  if (is_intra(st.kind) || !uids) {
    none(mb);
    return;
  }
  static constexpr u8 kCorner[4] = {0, 3, 12, 15};  // outer corner 4x4 block of each 8x8
  const auto& lu = *uids;
  if (col->corners) {  // 48 bytes per MB, streamed (read next by a later B picture's parse)
    ColMotion::Blk out[4];
    for (int k = 0; k < 4; ++k) {
      const int l = st.ref[0][k] >= 0 ? 0 : 1;
      const int ri = st.ref[l][k];
      out[k] = ri < 0 ? ColMotion::Blk{{0, 0}, 0u, i8(-1)}
                      : ColMotion::Blk{{st.mv[l][kCorner[k]][0], st.mv[l][kCorner[k]][1]}, uid_tab[l][ri & 31], i8(ri)};
    }
    stream_words(&col->b[size_t(mb) * 4], out, sizeof out);
    return;
  }
  ColMotion::Blk* out = &col->b[size_t(mb) * 16];
  for (int blk = 0; blk < 16; ++blk) {
    const int b8 = ((blk >> 3) << 1) | ((blk & 3) >> 1);
    const int l = st.ref[0][b8] >= 0 ? 0 : 1;
    const int ri = st.ref[l][b8];
    if (ri < 0) {
      out[blk] = ColMotion::Blk{{0, 0}, 0u, i8(-1)};
      continue;
    }
    out[blk] = ColMotion::Blk{{st.mv[l][blk][0], st.mv[l][blk][1]},
                              size_t(ri) < lu[size_t(l)].size() ? lu[size_t(l)][size_t(ri)] : 0u, i8(ri)};
  }
}

std::shared_ptr<ColMotion> build_col_motion(const MbNeighbours& nb, int wmbs, int hmbs,
                                            const std::vector<std::array<std::vector<u32>, 2>>& slice_uids,
                                            bool corners, Recycler<ColMotion>* pool) {
  // (a recycled buffer keeps its entries: the loop below writes every one of them)
  auto col = pool ? pool->acquire([](ColMotion&) {}) : std::make_shared<ColMotion>();
  col->wmbs = wmbs;
  col->hmbs = hmbs;
  col->corners = corners;
  const int per = corners ? 4 : 16;
  col->b.resize(size_t(wmbs) * hmbs * size_t(per));
  static constexpr u8 kCorner[4] = {0, 3, 12, 15};  // outer corner 4x4 block of each 8x8
  for (int mb = 0; mb < wmbs * hmbs; ++mb) {
    const MbState& st = nb.at(mb);
    ColMotion::Blk* out = &col->b[size_t(mb) * size_t(per)];
    if (!nb.decoded(mb) || is_intra(st.kind) || slice_uids.empty()) {
      for (int k = 0; k < per; ++k) out[k] = ColMotion::Blk{{0, 0}, 0u, i8(-1)};
      continue;
    }
    const auto& lu = slice_uids[std::min<size_t>(st.slice, slice_uids.size() - 1)];
    for (int k = 0; k < per; ++k) {
      const int blk = corners ? kCorner[k] : k;
      const int b8 = ((blk >> 3) << 1) | ((blk & 3) >> 1);
      const int l = st.ref[0][b8] >= 0 ? 0 : 1;
      const int ri = st.ref[l][b8];
      if (ri < 0) {
        out[k] = ColMotion::Blk{{0, 0}, 0u, i8(-1)};
        continue;
      }
      out[k] = ColMotion::Blk{{st.mv[l][blk][0], st.mv[l][blk][1]},
                              size_t(ri) < lu[size_t(l)].size() ? lu[size_t(l)][size_t(ri)] : 0u, i8(ri)};
    }
  }
  return col;
}

namespace {
template <class P>
const P* yplane(const HostSurface& s) {
  if constexpr (sizeof(P) == 1) return s.y.data();
  else return s.y16.data();
}
template <class P>
const P* uvplane(const HostSurface& s) {
  if constexpr (sizeof(P) == 1) return s.uv.data();
  else return s.uv16.data();
}
template <class P>
P* yplane(HostSurface& s) {
  if constexpr (sizeof(P) == 1) return s.y.data();
  else return s.y16.data();
}
template <class P>
P* uvplane(HostSurface& s) {
  if constexpr (sizeof(P) == 1) return s.uv.data();
  else return s.uv16.data();
}

// (P: u8 surfaces, or u16 at bit depth bd, High 10)
template <class P>
void predict_inter_t(const std::vector<HostSurface>& slots, const MbRec& m, const i16* mv0, const i16* mv1,
                     const WpEntry* wp, int mx, int my, int* py, int (*pc)[128], int structure, int bd) {
  // field pictures: slot parity = field parity; a vector into the opposite-parity field is offset
  // by a quarter chroma sample vertically (Table 8-10: 2 * (bottom_cur - bottom_ref) eighths)
  auto cy_off = [&](int slot) { return structure ? 2 * ((structure == 2) - (slot & 1)) : 0; };
  const int pitch = slots[0].coded_w, wpx = pitch, hpx = slots[0].coded_h;
  for (int y = 0; y < 16; ++y)
    for (int x = 0; x < 16; ++x) {
      const int r = (y >> 2) * 4 + (x >> 2), b8 = ((y >> 3) << 1) | (x >> 3);
      const int s0 = m.ref[b8], s1 = mv1 ? m.ref1[b8] : 0xFF;
      int p0 = 0, p1 = 0;
      if (s0 != 0xFF)
        p0 = luma_qpel(yplane<P>(slots[size_t(s0)]), pitch, wpx, hpx, mx * 16 + x + (mv0[2 * r] >> 2),
                       my * 16 + y + (mv0[2 * r + 1] >> 2), mv0[2 * r] & 3, mv0[2 * r + 1] & 3, bd);
      if (s1 != 0xFF)
        p1 = luma_qpel(yplane<P>(slots[size_t(s1)]), pitch, wpx, hpx, mx * 16 + x + (mv1[2 * r] >> 2),
                       my * 16 + y + (mv1[2 * r + 1] >> 2), mv1[2 * r] & 3, mv1[2 * r + 1] & 3, bd);
      py[y * 16 + x] = wp_sample(p0, p1, s0 != 0xFF, s1 != 0xFF, wp ? wp + b8 : nullptr, 0, bd);
    }
  // chroma: 8x8 (4:2:0) or 8x16 (4:2:2, full-height chroma: chroma row y is luma row y)
  const int cf = slots[0].cf, ch = cf == 2 ? 16 : 8, chp = cf == 2 ? hpx : hpx / 2;
  for (int c = 0; c < 2; ++c)
    for (int y = 0; y < ch; ++y)
      for (int x = 0; x < 8; ++x) {
        const int ly = cf == 2 ? y : 2 * y;  // luma row of the sample
        const int r = (ly >> 2) * 4 + (x >> 1), b8 = ((ly >> 3) << 1) | (x >> 2);
        const int s0 = m.ref[b8], s1 = mv1 ? m.ref1[b8] : 0xFF;
        int p0 = 0, p1 = 0, ix, fx, iy, fy;
        if (s0 != 0xFF) {
          chroma_mv(mv0[2 * r], mv0[2 * r + 1] + cy_off(s0), cf, ix, fx, iy, fy);
          p0 = chroma_epel(uvplane<P>(slots[size_t(s0)]), pitch, wpx / 2, chp, c, mx * 8 + x + ix, my * ch + y + iy, fx, fy);
        }
        if (s1 != 0xFF) {
          chroma_mv(mv1[2 * r], mv1[2 * r + 1] + cy_off(s1), cf, ix, fx, iy, fy);
          p1 = chroma_epel(uvplane<P>(slots[size_t(s1)]), pitch, wpx / 2, chp, c, mx * 8 + x + ix, my * ch + y + iy, fx, fy);
        }
        pc[c][y * 8 + x] = wp_sample(p0, p1, s0 != 0xFF, s1 != 0xFF, wp ? wp + b8 : nullptr, 1 + c, bd);
      }
}
}  // namespace

void predict_inter(const std::vector<HostSurface>& slots, const MbRec& m, const i16* mv0, const i16* mv1,
                   const WpEntry* wp, int mx, int my, int* py, int (*pc)[128], int structure) {
  if (slots[0].wide()) predict_inter_t<u16>(slots, m, mv0, mv1, wp, mx, my, py, pc, structure, slots[0].bd);
  else predict_inter_t<u8>(slots, m, mv0, mv1, wp, mx, my, py, pc, structure, 8);
}

void dequantize_mb(const MbLevels& lv, bool i16x16, int qp, int qpc, MbResidual& res) {
  // (§8.5.6 - §8.5.12.1) scan-order levels -> dequantised raster 4x4 blocks; blocks without
  // levels are skipped (their res.blk entries are left unwritten and masked out)
  res.luma = 0;
  res.chroma = 0;
  int dcy[16];
  const bool have_dc = i16x16 && (lv.dcmask & 1);
  if (have_dc) {
    int c[16] = {};
    for (int k = 0; k < 16; ++k) c[kZigzag4x4[k]] = lv.dc[k];
    hadamard4x4(c);
    const int ls = 16 * kNormAdjust[qp % 6][0];
    for (int k = 0; k < 16; ++k)
      dcy[k] = qp >= 36 ? c[k] * ls * (1 << (qp / 6 - 6)) : (c[k] * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
  }
  const int q6 = qp / 6, qm = qp % 6;
  for (int r = 0; r < 16; ++r) {
    const bool ac = (lv.lmask >> r) & 1;
    const int dcv = have_dc ? dcy[r] : 0;
    if (!ac && dcv == 0) continue;
    i16* d = res.blk[r];
    std::memset(d, 0, 16 * sizeof(i16));
    bool nz = dcv != 0;
    d[0] = sat16(dcv);
    if (ac) {
      for (int k = i16x16 ? 1 : 0; k < 16; ++k) {
        const int l = lv.luma[r][k];
        if (!l) continue;
        const int pos = kZigzag4x4[k];
        const int v = dequant4x4(l, qp, pos >> 2, pos & 3);
        d[pos] = sat16(v);
        nz |= v != 0;
      }
    }
    if (nz) res.luma |= u16(1u << r);
  }
  (void)q6;
  (void)qm;
  const int ls = 16 * kNormAdjust[qpc % 6][0];
  for (int c = 0; c < 2; ++c) {
    const bool has_dc = (lv.dcmask >> (1 + c)) & 1;
    const int acm = (lv.cmask >> (c * 4)) & 15;
    if (!has_dc && !acm) continue;
    int f[4] = {0, 0, 0, 0};
    if (has_dc) {
      const int c0 = lv.cdc[c][0], c1 = lv.cdc[c][1], c2 = lv.cdc[c][2], c3 = lv.cdc[c][3];
      f[0] = c0 + c1 + c2 + c3;
      f[1] = c0 - c1 + c2 - c3;
      f[2] = c0 + c1 - c2 - c3;
      f[3] = c0 - c1 - c2 + c3;
    }
    for (int b = 0; b < 4; ++b) {
      const int dcv = ((f[b] * ls) * (1 << (qpc / 6))) >> 5;
      const bool ac = (acm >> b) & 1;
      if (!ac && dcv == 0) continue;
      i16* d = res.blk[16 + c * 4 + b];
      std::memset(d, 0, 16 * sizeof(i16));
      d[0] = sat16(dcv);
      bool nz = dcv != 0;
      if (ac) {
        for (int k = 1; k < 16; ++k) {
          const int l = lv.cac[c][b][k];
          if (!l) continue;
          const int pos = kZigzag4x4[k];
          const int v = dequant4x4(l, qpc, pos >> 2, pos & 3);
          d[pos] = sat16(v);
          nz |= v != 0;
        }
      }
      if (nz) res.chroma |= u8(1u << (c * 4 + b));
    }
  }
}

// Bit i set = p[i] != 0 (16 coefficients): one 256-bit compare, movemask, and a bit extract of
// every second mask bit (the host build targets x86-64-v3: AVX2 + BMI2).
static inline u16 nonzero_mask16(const i16* p) {
#if defined(__AVX2__) && defined(__BMI2__)
  const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p));
  const u32 zero = u32(_mm256_movemask_epi8(_mm256_cmpeq_epi16(v, _mm256_setzero_si256())));
  return u16(_pext_u32(~zero, 0x55555555u));
#else
  u32 m = 0;
  for (int i = 0; i < 16; ++i) m |= u32(p[i] != 0) << i;
  return u16(m);
#endif
}

// pshufb control that moves the i16 lanes selected by an 8-bit mask to the front (branch-free
// compaction of a group's non-zero values: the inner "for each set bit" loop mispredicted its
// exit on most groups).
struct Compact8 {
  alignas(16) u8 c[256][16];
  constexpr Compact8() : c() {
    for (int m = 0; m < 256; ++m) {
      int k = 0;
      for (int i = 0; i < 8; ++i)
        if ((m >> i) & 1) {
          c[m][2 * k] = u8(2 * i);
          c[m][2 * k + 1] = u8(2 * i + 1);
          ++k;
        }
      for (int j = 2 * k; j < 16; ++j) c[m][j] = 0x80;  // (zeros; overwritten by the next group)
    }
  }
};
static constexpr Compact8 kCompact8{};

// The non-zero values of 16 coefficients (mask = nonzero_mask16(p)) to out; writes up to 8
// entries past the last value (the caller leaves that slack).
static inline i16* compact16(const i16* p, u32 mask, i16* out) {
#if defined(__SSSE3__)
  const __m128i lo = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
  const __m128i hi = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 8));
  const u32 m0 = mask & 0xFFu, m1 = mask >> 8;
  _mm_storeu_si128(reinterpret_cast<__m128i*>(out),
                   _mm_shuffle_epi8(lo, _mm_load_si128(reinterpret_cast<const __m128i*>(kCompact8.c[m0]))));
  out += __builtin_popcount(m0);
  _mm_storeu_si128(reinterpret_cast<__m128i*>(out),
                   _mm_shuffle_epi8(hi, _mm_load_si128(reinterpret_cast<const __m128i*>(kCompact8.c[m1]))));
  return out + __builtin_popcount(m1);
#else
  for (int i = 0; i < 16; ++i) {  // (branch-free: store every value, advance on non-zero)
    *out = p[i];
    out += (mask >> i) & 1;
  }
  return out;
#endif
}

// Granularity of one list's motion (16 raster 4x4 vectors as words): bit 0 every vector equals
// block 0's (kMbMv16), bit 1 every vector equals its 8x8's top-left block's (kMbMv8x8).
static inline u32 motion_uniformity(const i16* mv) {
#if defined(__AVX2__)
  const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(mv));       // blocks 0..7
  const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(mv + 16));  // blocks 8..15
  const __m256i v0 = _mm256_broadcastd_epi32(_mm256_castsi256_si128(a));
  const __m256i tl = _mm256_setr_epi32(0, 0, 2, 2, 0, 0, 2, 2);  // top-left block of each 8x8
  const u32 all = u32(_mm256_movemask_epi8(_mm256_and_si256(_mm256_cmpeq_epi32(a, v0), _mm256_cmpeq_epi32(b, v0))));
  const u32 q8 = u32(_mm256_movemask_epi8(_mm256_and_si256(_mm256_cmpeq_epi32(a, _mm256_permutevar8x32_epi32(a, tl)),
                                                           _mm256_cmpeq_epi32(b, _mm256_permutevar8x32_epi32(b, tl)))));
  return (all == 0xFFFFFFFFu ? 1u : 0u) | (q8 == 0xFFFFFFFFu ? 2u : 0u);
#else
  u32 v[16];
  std::memcpy(v, mv, sizeof v);
  bool u16 = true, u8x8 = true;
  for (int b = 1; b < 16; ++b) u16 &= v[b] == v[0];
  for (int b = 0; b < 16; ++b) u8x8 &= v[b] == v[((b >> 3) << 3) | (b & 2)];
  return (u16 ? 1u : 0u) | (u8x8 ? 2u : 0u);
#endif
}

// The MB's motion into the picture's vector pool at the coarsest granularity that represents
// every list used exactly (sets m.mv and the kMbMv16 / kMbMv8x8 flag).
static inline void store_motion(Picture& pic, MbRec& m, const MbState& s) {
  const int nl = (m.flags & kMbL1) ? 2 : 1;
  u32 u = 3;
  for (int l = 0; l < nl; ++l) u &= motion_uniformity(&s.mv[l][0][0]);
  m.flags |= (u & 1) ? kMbMv16 : ((u & 2) ? kMbMv8x8 : 0);
  m.mv = u32(pic.mvs.size());
  const int per = (u & 1) ? 2 : ((u & 2) ? 8 : 32);
  i16* out = pic.mvs.extend(size_t(per * nl));
  for (int l = 0; l < nl; ++l, out += per) {
    const i16* v = &s.mv[l][0][0];
    if (per == 2) {
      std::memcpy(out, v, 4);
    } else if (per == 8) {  // blocks 0, 2, 8, 10
      std::memcpy(out, v, 4);
      std::memcpy(out + 2, v + 4, 4);
      std::memcpy(out + 4, v + 16, 4);
      std::memcpy(out + 6, v + 20, 4);
    } else {
      std::memcpy(out, v, 64);
    }
  }
}

// Records leave the parser with non-temporal stores (stream_words): pic.mbs (56 bytes per MB,
// 457 KB per 1080p picture) is written once and read next by the GPU's record gather over PCIe
// (or, on the CPU backend, by the reconstruction much later).
static inline void store_rec(MbRec* dst, const MbRec& m) {
  static_assert(sizeof(MbRec) % 8 == 0 && sizeof(ColMotion::Blk) * 4 % 8 == 0, "8-byte words");
  stream_words(dst, &m, sizeof(MbRec));
}

void store_skip_mb(Picture& pic, int mb, MbRec& m, const MbState& s) {
  m.coef = u32(pic.coefs.size());
  m.luma_coded = 0;
  m.chroma_coded = 0;
  m.wp = 0;
  m.res = kNoRes;
  store_motion(pic, m, s);
  ++pic.inter_mbs;
  if (!(m.dbk & 1)) pic.deblock = true;
  // (validate_mb's checks that can fail for a skipped MB: the reference slots)
  for (int k = 0; k < 4; ++k) {
    const int r0 = m.ref[k], r1 = m.ref1[k];
    VEP_CHECK((r0 != 0xFF || r1 != 0xFF) && (r0 == 0xFF || r0 < pic.dpb_slots) && (r1 == 0xFF || r1 < pic.dpb_slots) &&
                  (r1 == 0xFF || (m.flags & kMbL1)),
              "skipped macroblock reference slot outside the DPB");
  }
  VEP_CHECK(m.qp <= 51 + pic.qp_bias && m.qpc <= 51 + pic.qpc_bias && m.qpc2 <= 51 + pic.qpc_bias,
            "macroblock QP out of range");
  store_rec(&pic.mbs[size_t(mb)], m);
  if (pic.colb) pic.colb->store(mb, s);
}

void store_mb(Picture& pic, int mb, MbRec m, const MbState& s, const MbResidual* res, const u8* pcm,
              const WpEntry* wp) {
  m.coef = u32(pic.coefs.size());
  m.luma_coded = 0;
  m.chroma_coded = 0;
  if (m.kind == kIPcm) {
    VEP_CHECK(pcm, "I_PCM macroblock without samples");
    // (8-bit: sample bytes; High 10: u16 samples; 384 samples, 4:2:2 512)
    const size_t ns = pic.cf == 2 ? size_t(kPcmMaxSamples) : size_t(kPcmMbBytes);
    const size_t o = pic.coefs.size(), nb = pic.bd > 8 ? 2 * ns : ns;
    pic.coefs.resize(o + nb / 2);
    std::memcpy(pic.coefs.data() + o, pcm, nb);
  } else if (res && (res->luma | res->chroma)) {
    m.luma_coded = res->luma;
    m.chroma_coded = res->chroma;
    if (res->t8) m.flags |= kMbT8x8;
    // sparse groups (avc_recon.h): the mask words, then the non-zero values
    const i16* grp[32];  // (16 luma + 16 chroma groups in 4:2:2)
    int ng = 0;
    if (res->t8) {
      for (int q = 0; q < 4; ++q)
        if ((res->luma >> ((q & 1) * 2 + (q >> 1) * 8)) & 1)
          for (int w = 0; w < 4; ++w) grp[ng++] = res->b8[q] + 16 * w;
    } else {
      for (u32 w = res->luma; w; w &= w - 1) grp[ng++] = res->blk[__builtin_ctz(w)];
    }
    for (u32 w = res->chroma; w; w &= w - 1) grp[ng++] = res->blk[16 + __builtin_ctz(w)];
    u16 mask[32];
    int nv = 0;
    for (int g = 0; g < ng; ++g) {
      mask[g] = nonzero_mask16(grp[g]);
      nv += __builtin_popcount(mask[g]);
    }
    // appended without zero-filling (the pool is reserved per picture), with 8 entries of slack
    // for the last group's 16-byte stores, trimmed after
    const size_t o = pic.coefs.size();
    i16* out = pic.coefs.extend(size_t(ng + nv) + 8);
    std::memcpy(out, mask, size_t(ng) * sizeof(u16));
    i16* v = out + ng;
    for (int g = 0; g < ng; ++g) v = compact16(grp[g], mask[g], v);
    pic.coefs.resize(o + size_t(ng + nv));
  }
  m.mv = 0;
  m.wp = 0;
  m.flags &= u8(~(kMbMv8x8 | kMbMv16));
  if (m.kind == kSkip || m.kind == kInter) {
    store_motion(pic, m, s);
    if (wp && (m.flags & kMbWp)) {
      m.wp = u32(pic.wps.size());
      pic.wps.insert(pic.wps.end(), wp, wp + 4);
    } else {
      m.flags &= u8(~kMbWp);
    }
    ++pic.inter_mbs;
  } else if (m.kind == kIPcm) {
    ++pic.inter_mbs;  // no neighbour dependency: reconstructed in the parallel pass
  } else {
    ++pic.intra_mbs;
  }
  m.res = is_intra(m.kind) && m.kind != kIPcm && (m.luma_coded | m.chroma_coded) ? u32(pic.intra_res++) : kNoRes;
  if (!(m.dbk & 1)) pic.deblock = true;
  validate_written_mb(pic, m);
  store_rec(&pic.mbs[size_t(mb)], m);
  if (pic.colb) pic.colb->store(mb, s);
}

// ------------------------------------------------------------------------- CPU reconstruction

namespace {

// Intra availability of MB (nx, ny) for the current MB m (§6.4.11 + constrained_intra_pred).
bool intra_avail(const Picture& pic, const MbRec& m, int nx, int ny) {
  if (nx < 0 || ny < 0 || nx >= pic.wmbs) return false;
  const MbRec& n = pic.mbs[size_t(ny) * pic.wmbs + nx];
  if (n.slice != m.slice) return false;
  return !(pic.constrained_intra && !is_intra(n.kind));
}

// `dense`: the MB's coefficients expanded (expand_coefs, avc_recon.h)
const i16* luma_res(const i16* dense, const MbRec& m, int r) {
  if (!((m.luma_coded >> r) & 1)) return nullptr;
  return dense + 16 * r;
}

const i16* chroma_res(const i16* dense, const MbRec& m, int c, int b, int nbc) {
  const int k = c * nbc + b;
  if (!((m.chroma_coded >> k) & 1)) return nullptr;
  return dense + 256 + 16 * k;
}

// Luma residual samples of the whole MB (raster 16x16), from 4x4 or 8x8 transform blocks.
void luma_residual(const i16* dense, const MbRec& m, int* out) {
  std::memset(out, 0, 256 * sizeof(int));
  if (m.flags & kMbT8x8) {
    for (int q = 0; q < 4; ++q) {
      if (!((m.luma_coded >> ((q & 1) * 2 + (q >> 1) * 8)) & 1)) continue;
      int r[64];
      idct8x8(dense + 64 * q, r);
      for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) out[((q >> 1) * 8 + i) * 16 + (q & 1) * 8 + j] = r[i * 8 + j];
    }
    return;
  }
  for (int blk = 0; blk < 16; ++blk) {
    const i16* d = luma_res(dense, m, blk);
    if (!d) continue;
    int r[16];
    idct4x4(d, r);
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) out[((blk >> 2) * 4 + i) * 16 + (blk & 3) * 4 + j] = r[i * 4 + j];
  }
}

template <class P>
struct Recon {
  const Picture& pic;
  std::vector<HostSurface>& slots;
  HostSurface& T;
  int pitch, wpx, hpx, bd;
  int cf, ch, nbc;  // chroma format, chroma MB height (8 / 16), chroma 4x4 blocks per component
  i16 dense[kDenseCoefs];  // the current MB's coefficients (load())

  void load(const MbRec& m) {
    if (m.kind != kIPcm) expand_coefs(pic.coefs.data(), m, dense);
  }

  P& Y(int x, int y) { return yplane<P>(T)[size_t(y) * pitch + x]; }
  P& C(int x, int y, int c) { return uvplane<P>(T)[size_t(y) * pitch + 2 * x + c]; }
  P px(int v) const { return P(clip1(v, bd)); }

  void chroma_store(const MbRec& m, int mx, int my, int c, const int* pred /*8 x ch*/) {
    for (int b = 0; b < nbc; ++b) {
      const i16* d = chroma_res(dense, m, c, b, nbc);
      int res[16] = {};
      if (d) idct4x4(d, res);
      const int bx = (b & 1) * 4, by = (b >> 1) * 4;
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
          C(mx * 8 + bx + j, my * ch + by + i, c) = px(pred[(by + i) * 8 + bx + j] + res[i * 4 + j]);
    }
  }

  void inter(const MbRec& m, int mx, int my) {
    i16 e[2][32];  // expanded to one vector per 4x4 block
    const i16* base = &pic.mvs[size_t(m.mv)];
    for (int l = 0; l < ((m.flags & kMbL1) ? 2 : 1); ++l)
      for (int b = 0; b < 16; ++b) {
        const i16* v = base + mv_sub(m.flags, l, b);
        e[l][2 * b] = v[0];
        e[l][2 * b + 1] = v[1];
      }
    const i16* mv0 = e[0];
    const i16* mv1 = (m.flags & kMbL1) ? e[1] : nullptr;
    const WpEntry* wp = (m.flags & kMbWp) ? &pic.wps[m.wp] : nullptr;
    int py[256], pc[2][128], res[256];
    predict_inter_t<P>(slots, m, mv0, mv1, wp, mx, my, py, pc, pic.structure, bd);
    luma_residual(dense, m, res);
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) Y(mx * 16 + x, my * 16 + y) = px(py[y * 16 + x] + res[y * 16 + x]);
    for (int c = 0; c < 2; ++c) chroma_store(m, mx, my, c, pc[c]);
  }

  void pcm(const MbRec& m, int mx, int my) {  // (u8 surfaces: sample bytes; u16: samples; 384 / 4:2:2 512)
    const P* s = reinterpret_cast<const P*>(pic.coefs.data() + m.coef);
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) Y(mx * 16 + x, my * 16 + y) = s[y * 16 + x];
    for (int c = 0; c < 2; ++c)
      for (int y = 0; y < ch; ++y)
        for (int x = 0; x < 8; ++x) C(mx * 8 + x, my * ch + y, c) = s[256 + c * 8 * ch + y * 8 + x];
  }

  void intra_chroma(const MbRec& m, int mb, int mx, int my) {
    for (int c = 0; c < 2; ++c) {
      IntraChromaNb n;
      chroma_neighbours(pic, mb, c, T, n);
      const PredConst k = m.chroma_mode == 3 ? chroma_plane_const(n, cf) : PredConst{0, 0, 0, 0};
      int cp[128];
      for (int y = 0; y < ch; ++y)
        for (int x = 0; x < 8; ++x) cp[y * 8 + x] = chroma_pred(n, k, m.chroma_mode, x, y, bd, cf);
      chroma_store(m, mx, my, c, cp);
    }
  }

  void intra16(const MbRec& m, int mb, int mx, int my) {
    Intra16Nb n;
    intra16_neighbours(pic, mb, T, n);
    const PredConst k = intra16x16_const(n, m.i16_mode, bd);
    int res[256];
    luma_residual(dense, m, res);
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x)
        Y(mx * 16 + x, my * 16 + y) = px(intra16x16_pred(n, k, m.i16_mode, x, y, bd) + res[y * 16 + x]);
  }

  void intra4(const MbRec& m, int mb, int mx, int my) {
    for (int idx = 0; idx < 16; ++idx) {
      const int r = blk_to_raster(idx), bx = r & 3, by = r >> 2;
      Intra4Nb n;
      intra4x4_neighbours(pic, mb, idx, T, n);
      const int mode = i4_mode(m, r);
      const i16* d = luma_res(dense, m, r);
      int res[16] = {};
      if (d) idct4x4(d, res);
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
          Y(mx * 16 + bx * 4 + j, my * 16 + by * 4 + i) = px(intra4x4_pred(n, mode, j, i, bd) + res[i * 4 + j]);
    }
  }

  void intra8(const MbRec& m, int mb, int mx, int my) {
    for (int q = 0; q < 4; ++q) {
      int f[25];
      bool top, left;
      intra8x8_neighbours(pic, mb, q, T, f, top, left);
      const int mode = i4_mode(m, q);
      int res[64] = {};
      if ((m.luma_coded >> ((q & 1) * 2 + (q >> 1) * 8)) & 1) idct8x8(dense + 64 * q, res);
      const int x0 = mx * 16 + (q & 1) * 8, y0 = my * 16 + (q >> 1) * 8;
      for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) Y(x0 + j, y0 + i) = px(intra8x8_pred(f, top, left, mode, j, i, bd) + res[i * 8 + j]);
    }
  }
};

}  // namespace

// Filtered Intra_8x8 reference samples of 8x8 block q (§8.3.2.2, §8.3.2.2.1) from the surface
// being reconstructed.
void intra8x8_neighbours(const Picture& pic, int mb, int q, const HostSurface& T, int* f, bool& has_top,
                         bool& has_left) {
  const MbRec& m = pic.mbs[size_t(mb)];
  const int mx = mb % pic.wmbs, my = mb / pic.wmbs, pitch = T.coded_w;
  const bool A = intra_avail(pic, m, mx - 1, my), B = intra_avail(pic, m, mx, my - 1),
             Cm = intra_avail(pic, m, mx + 1, my - 1), D = intra_avail(pic, m, mx - 1, my - 1);
  const int bx = q & 1, by = q >> 1;
  const int x0 = mx * 16 + bx * 8, y0 = my * 16 + by * 8;
  has_top = by > 0 || B;
  has_left = bx > 0 || A;
  const bool has_tl = (bx > 0 && by > 0) || (bx == 0 && by == 0 ? D : bx == 0 ? A : B);
  const bool has_tr = by == 0 ? (bx == 0 ? B : Cm) : (bx == 0);  // block 2's top-right is block 1
  auto P = [&](int x, int y) { return T.wide() ? int(T.y16[size_t(y) * pitch + x]) : int(T.y[size_t(y) * pitch + x]); };
  int t[17], l[8];  // t[0] = p[-1,-1], t[1 + x] = p[x,-1]
  t[0] = has_tl ? P(x0 - 1, y0 - 1) : 128;
  for (int k = 0; k < 8; ++k) {
    t[1 + k] = has_top ? P(x0 + k, y0 - 1) : 128;
    l[k] = has_left ? P(x0 - 1, y0 + k) : 128;
  }
  for (int k = 8; k < 16; ++k) t[1 + k] = has_tr ? P(x0 + k, y0 - 1) : t[8];
  for (int k = 0; k < 25; ++k) f[k] = 128;
  intra8x8_filter([&](int x) { return t[1 + x]; }, [&](int y) { return l[y]; }, has_top, has_left, has_tl, f);
}

void intra4x4_neighbours(const Picture& pic, int mb, int idx, const HostSurface& T, Intra4Nb& n) {
  const MbRec& m = pic.mbs[size_t(mb)];
  const int mx = mb % pic.wmbs, my = mb / pic.wmbs, pitch = T.coded_w;
  const bool A = intra_avail(pic, m, mx - 1, my), B = intra_avail(pic, m, mx, my - 1),
             Cm = intra_avail(pic, m, mx + 1, my - 1), D = intra_avail(pic, m, mx - 1, my - 1);
  const int r = blk_to_raster(idx), bx = r & 3, by = r >> 2;
  const int x0 = mx * 16 + bx * 4, y0 = my * 16 + by * 4;
  auto P = [&](int x, int y) { return T.wide() ? int(T.y16[size_t(y) * pitch + x]) : int(T.y[size_t(y) * pitch + x]); };
  n.has_top = by > 0 || B;
  n.has_left = bx > 0 || A;
  n.has_tl = (bx > 0 && by > 0) || (bx == 0 && by == 0 ? D : bx == 0 ? A : B);
  const bool tr = by == 0 ? (bx < 3 ? B : Cm) : (bx < 3 && raster_to_blk((by - 1) * 4 + bx + 1) < idx);
  n.t[0] = n.has_tl ? P(x0 - 1, y0 - 1) : 128;
  for (int k = 0; k < 4; ++k) {
    n.t[1 + k] = n.has_top ? P(x0 + k, y0 - 1) : 128;
    n.l[k] = n.has_left ? P(x0 - 1, y0 + k) : 128;
  }
  for (int k = 0; k < 4; ++k) n.t[5 + k] = tr ? P(x0 + 4 + k, y0 - 1) : n.t[4];
}

void intra16_neighbours(const Picture& pic, int mb, const HostSurface& T, Intra16Nb& n) {
  const MbRec& m = pic.mbs[size_t(mb)];
  const int mx = mb % pic.wmbs, my = mb / pic.wmbs, pitch = T.coded_w;
  auto P = [&](int x, int y) { return T.wide() ? int(T.y16[size_t(y) * pitch + x]) : int(T.y[size_t(y) * pitch + x]); };
  n.has_left = intra_avail(pic, m, mx - 1, my);
  n.has_top = intra_avail(pic, m, mx, my - 1);
  n.has_tl = intra_avail(pic, m, mx - 1, my - 1);
  n.top[0] = n.has_tl ? P(mx * 16 - 1, my * 16 - 1) : 128;
  for (int k = 0; k < 16; ++k) {
    n.top[k + 1] = n.has_top ? P(mx * 16 + k, my * 16 - 1) : 128;
    n.left[k] = n.has_left ? P(mx * 16 - 1, my * 16 + k) : 128;
  }
}

void chroma_neighbours(const Picture& pic, int mb, int c, const HostSurface& T, IntraChromaNb& n) {
  const MbRec& m = pic.mbs[size_t(mb)];
  const int mx = mb % pic.wmbs, my = mb / pic.wmbs, pitch = T.coded_w;
  auto P = [&](int x, int y) {
    return T.wide() ? int(T.uv16[size_t(y) * pitch + 2 * x + c]) : int(T.uv[size_t(y) * pitch + 2 * x + c]);
  };
  n.has_left = intra_avail(pic, m, mx - 1, my);
  n.has_top = intra_avail(pic, m, mx, my - 1);
  n.has_tl = intra_avail(pic, m, mx - 1, my - 1);
  const int ch = T.cf == 2 ? 16 : 8;  // chroma MB height (4:2:2: 16 rows)
  n.top[0] = n.has_tl ? P(mx * 8 - 1, my * ch - 1) : 128;
  for (int k = 0; k < 8; ++k) n.top[k + 1] = n.has_top ? P(mx * 8 + k, my * ch - 1) : 128;
  for (int k = 0; k < ch; ++k) n.left[k] = n.has_left ? P(mx * 8 - 1, my * ch + k) : 128;
}

namespace {
template <class P>
void reconstruct_mb_t(const Picture& pic, int mb, std::vector<HostSurface>& slots) {
  HostSurface& T = slots[size_t(pic.target)];
  const int wpx = pic.wmbs * 16, hpx = pic.hmbs * 16;
  Recon<P> r{pic, slots, T, wpx, wpx, hpx, T.wide() ? T.bd : 8, T.cf, T.cf == 2 ? 16 : 8, T.cf == 2 ? 8 : 4, {}};
  const MbRec& m = pic.mbs[size_t(mb)];
  r.load(m);
  const int mx = mb % pic.wmbs, my = mb / pic.wmbs;
  switch (m.kind) {
    case kSkip:
    case kInter:
      for (int k = 0; k < 8; ++k) {
        const u8 s = k < 4 ? m.ref[k] : ((m.flags & kMbL1) ? m.ref1[k - 4] : u8(0xFF));
        VEP_CHECK(s == 0xFF || (s < slots.size() && slots[s].coded_w == wpx && slots[s].coded_h == hpx),
                  "missing reference surface");
      }
      r.inter(m, mx, my);
      break;
    case kIPcm: r.pcm(m, mx, my); break;
    case kI16x16:
      r.intra16(m, mb, mx, my);
      r.intra_chroma(m, mb, mx, my);
      break;
    case kI8x8:
      r.intra8(m, mb, mx, my);
      r.intra_chroma(m, mb, mx, my);
      break;
    default:
      r.intra4(m, mb, mx, my);
      r.intra_chroma(m, mb, mx, my);
      break;
  }
}

template <class P>
void deblock_t(const Picture& pic, HostSurface& T) {
  static const i16 kZeroMv[64] = {};
  const int W = pic.wmbs, pitch = T.coded_w, bd = T.wide() ? T.bd : 8;
  const int qb = pic.qp_bias, qcb = pic.qpc_bias;
  const bool cf2 = T.cf == 2;
  P* Yp = yplane<P>(T);
  P* UV = uvplane<P>(T);
  auto mvs = [&](const MbRec& r) { return is_intra(r.kind) ? kZeroMv : &pic.mvs[size_t(r.mv)]; };
  for (int mb = 0; mb < pic.nmbs(); ++mb) {
    const MbRec& q = pic.mbs[size_t(mb)];
    if (q.dbk & 1) continue;
    const int mx = mb % W, my = mb / W;
    const bool left = mx > 0 && !((q.dbk & 2) && pic.mbs[size_t(mb - 1)].slice != q.slice);
    const bool top = my > 0 && !((q.dbk & 2) && pic.mbs[size_t(mb - W)].slice != q.slice);
    const i16* mq = mvs(q);
    for (int dir = 0; dir < 2; ++dir) {  // 0: vertical edges, 1: horizontal edges
      for (int e = 0; e < 4; ++e) {
        if (e == 0 && !(dir == 0 ? left : top)) continue;
        const MbRec& p = e > 0 ? q : pic.mbs[size_t(dir == 0 ? mb - 1 : mb - W)];
        const i16* mp = mvs(p);
        // luma: no 4x4 edges inside 8x8 transform blocks; chroma (4x4 transforms): the edges at
        // chroma samples 0 and 4 (luma edges 0 and 2), and in 4:2:2 every horizontal edge (chroma
        // rows 0, 4, 8, 12 = luma rows: the odd ones also inside luma 8x8 transform blocks)
        const bool luma_edge = !((e & 1) && (q.flags & kMbT8x8));
        const bool chroma_edge = cf2 ? (dir == 1 || !(e & 1)) : !(e & 1);
        if (!luma_edge && !chroma_edge) continue;
        const EdgeParams ep = edge_params(p.qp - qb, q.qp - qb, q.alpha_off, q.beta_off, bd);
        const EdgeParams epcs[2] = {edge_params(p.qpc - qcb, q.qpc - qcb, q.alpha_off, q.beta_off, bd),
                                    edge_params(p.qpc2 - qcb, q.qpc2 - qcb, q.alpha_off, q.beta_off, bd)};
        int bs[16];
        for (int k = 0; k < 16; ++k) {
          const int bq = dir == 0 ? (k >> 2) * 4 + e : e * 4 + (k >> 2);
          const int bp = e > 0 ? (dir == 0 ? bq - 1 : bq - 4) : (dir == 0 ? bq + 3 : bq + 12);
          bs[k] = boundary_strength(p, bp, mp, q, bq, mq, e == 0, pic.structure != 0, dir == 0);
        }
        for (int k = 0; k < 16 && luma_edge; ++k) {
          if (!bs[k]) continue;
          if (dir == 0) filter_line(Yp + size_t(my * 16 + k) * pitch + mx * 16 + 4 * e, 1, bs[k], ep, false, bd);
          else filter_line(Yp + size_t(my * 16 + 4 * e) * pitch + mx * 16 + k, long(pitch), bs[k], ep, false, bd);
        }
        if (!chroma_edge) continue;
        const int ch = cf2 ? 16 : 8;  // chroma MB height
        for (int c = 0; c < 2; ++c)
          for (int k = 0; k < (dir == 0 ? ch : 8); ++k) {
            const EdgeParams& epc = epcs[c];
            // bS of the luma line through the chroma line: vertical edges row k (4:2:0: 2k),
            // horizontal edges column 2k
            const int b = bs[dir == 0 && cf2 ? k : 2 * k];
            if (!b) continue;
            if (dir == 0)
              filter_line(UV + size_t(my * ch + k) * pitch + (mx * 8 + 2 * e) * 2 + c, 2, b, epc, true, bd);
            else  // (chroma row of edge e: 4:2:0 2e, 4:2:2 4e)
              filter_line(UV + size_t(my * ch + (cf2 ? 4 : 2) * e) * pitch + (mx * 8 + k) * 2 + c, long(pitch), b,
                          epc, true, bd);
          }
      }
    }
  }
}
}  // namespace

void cpu_reconstruct_mb(const Picture& pic, int mb, std::vector<HostSurface>& slots) {
  if (slots[size_t(pic.target)].wide()) reconstruct_mb_t<u16>(pic, mb, slots);
  else reconstruct_mb_t<u8>(pic, mb, slots);
}

void cpu_deblock(const Picture& pic, HostSurface& T) {
  if (T.wide()) deblock_t<u16>(pic, T);
  else deblock_t<u8>(pic, T);
}

void weave_fields(const HostSurface& top, const HostSurface& bottom, HostSurface& frame) {
  VEP_CHECK(top.coded_w == bottom.coded_w && top.coded_h == bottom.coded_h && !top.wide(), "weave: field sizes");
  const int w = top.coded_w, fh = top.coded_h;
  if (frame.coded_w != w || frame.coded_h != 2 * fh) frame.alloc(w, 2 * fh);
  for (int r = 0; r < 2 * fh; ++r)
    std::memcpy(&frame.y[size_t(r) * w], &(r & 1 ? bottom : top).y[size_t(r >> 1) * w], size_t(w));
  for (int r = 0; r < fh; ++r)
    std::memcpy(&frame.uv[size_t(r) * w], &(r & 1 ? bottom : top).uv[size_t(r >> 1) * w], size_t(w));
}

void cpu_reconstruct(const Picture& pic, std::vector<HostSurface>& slots) {
  VEP_CHECK(pic.target >= 0 && pic.target < int(slots.size()), "target slot out of range");
  HostSurface& T = slots[size_t(pic.target)];
  VEP_CHECK(T.coded_w == pic.wmbs * 16 && T.coded_h == pic.hmbs * 16 && T.bd == pic.bd && T.cf == pic.cf,
            "surface size mismatch");
  for (int mb = 0; mb < pic.nmbs(); ++mb) cpu_reconstruct_mb(pic, mb, slots);
  if (pic.deblock) cpu_deblock(pic, T);
}

}  // namespace vep::avc
