// The HEVC CTU layer (§7.3.8 syntax, §9.3 CABAC binarization / context selection) and the
// reconstruction it drives, written once for both directions: `CtuLayer<RD>` decodes, and
// `CtuLayer<WR>` encodes the decisions of a CtuDecider through the same code (see hevc_ctu.h).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <thread>

#include "hevc_ctu.h"
#include "hevc_recon.h"

namespace vep::hevc {

void PicCtx::init_tiles() {
  pps->tile_bounds(wctb, hctb, col_bd, row_bd);
  const size_t nctb = size_t(wctb) * size_t(hctb);
  rs2ts.resize(nctb);
  ts2rs.resize(nctb);
  tile.resize(nctb);
  const int tc = int(col_bd.size()) - 1, tr = int(row_bd.size()) - 1;
  int ts = 0;
  for (int ty = 0; ty < tr; ++ty)  // tiles in raster order, CTBs in raster order inside a tile
    for (int tx = 0; tx < tc; ++tx)
      for (int y = row_bd[size_t(ty)]; y < row_bd[size_t(ty) + 1]; ++y)
        for (int x = col_bd[size_t(tx)]; x < col_bd[size_t(tx) + 1]; ++x) {
          const int rs = y * wctb + x;
          rs2ts[size_t(rs)] = ts;
          ts2rs[size_t(ts)] = rs;
          tile[size_t(rs)] = u16(ty * tc + tx);
          ++ts;
        }
}

void PicCtx::init_scaling() {
  scaling = sps->scaling_list;
  if (!scaling) return;
  // PPS lists replace the SPS ones; an SPS without explicit data uses the default lists
  const ScalingList& sl = pps->scaling_list ? pps->sl : sps->sl;
  for (int size_id = 0; size_id < 4; ++size_id)
    for (int m = 0; m < 6; ++m) {
      const int n = 4 << size_id;
      sf[size_id][m].resize(size_t(n) * n);
      sl.factors(size_id, m, sf[size_id][m].data());
    }
}

namespace {

struct RD {
  static constexpr bool kW = false;
  cabac::Decoder& d;
  cabac::Ctx* c;
  u32 bin(int i, u32) { return d.decision(c[i]); }
  u32 byp(u32) { return d.bypass(); }
  u32 term(u32) { return d.terminate(); }
};

struct WR {
  static constexpr bool kW = true;
  cabac::Encoder& e;
  cabac::Ctx* c;
  u32 bin(int i, u32 v) {
    e.decision(c[i], v & 1u);
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

// partition rectangles (x, y, w, h) of a CU of size n per PartMode
int pu_rects(int part, int n, int r[4][4]) {
  const int h = n / 2, q = n / 4;
  switch (part) {
    case 0: r[0][0] = 0, r[0][1] = 0, r[0][2] = n, r[0][3] = n; return 1;
    case 1: r[0][0] = 0, r[0][1] = 0, r[0][2] = n, r[0][3] = h; r[1][0] = 0, r[1][1] = h, r[1][2] = n, r[1][3] = h; return 2;
    case 2: r[0][0] = 0, r[0][1] = 0, r[0][2] = h, r[0][3] = n; r[1][0] = h, r[1][1] = 0, r[1][2] = h, r[1][3] = n; return 2;
    case 3:
      for (int k = 0; k < 4; ++k) r[k][0] = (k & 1) * h, r[k][1] = (k >> 1) * h, r[k][2] = h, r[k][3] = h;
      return 4;
    case 4: r[0][0] = 0, r[0][1] = 0, r[0][2] = n, r[0][3] = q; r[1][0] = 0, r[1][1] = q, r[1][2] = n, r[1][3] = n - q; return 2;
    case 5: r[0][0] = 0, r[0][1] = 0, r[0][2] = n, r[0][3] = n - q; r[1][0] = 0, r[1][1] = n - q, r[1][2] = n, r[1][3] = q; return 2;
    case 6: r[0][0] = 0, r[0][1] = 0, r[0][2] = q, r[0][3] = n; r[1][0] = q, r[1][1] = 0, r[1][2] = n - q, r[1][3] = n; return 2;
    default: r[0][0] = 0, r[0][1] = 0, r[0][2] = n - q, r[0][3] = n; r[1][0] = n - q, r[1][1] = 0, r[1][2] = q, r[1][3] = n; return 2;
  }
}

template <class E>
class CtuLayer {
 public:
  static constexpr bool kWrite = E::kW;

  CtuLayer(PicCtx& pc, int si, E& e, CtuDecider* dec)
      : pc_(pc), si_(si), sl_(pc.slices[size_t(si)]), sh_(sl_.sh), sps_(*pc.sps), pps_(*pc.pps), e_(e), dec_(dec),
        g_(pc.gpu), st_(&pc.stats), bypass_(&pc.any_bypass) {
    slice_qp_ = sl_.qp;
    qp_last_ = slice_qp_;
    log2_min_qg_ = sps_.log2_ctb - (pps_.cu_qp_delta ? pps_.diff_cu_qp_delta_depth : 0);
  }

  // Outputs into a slice's own shard instead of the picture (parallel slices).
  void use_shard(SliceShard& sh) {
    g_ = pc_.gpu ? &sh.g : nullptr;
    st_ = &sh.stats;
    bypass_ = &sh.any_bypass;
  }

  cabac::Decoder* rd = nullptr;  // (read mode: PCM samples, re-initialisation)
  cabac::Encoder* wr = nullptr;
  const u8* data = nullptr;
  size_t data_n = 0;

  // -------------------------------------------------------------------- CTU
  void ctu(int addr, bool last) {
    const int rx = addr % pc_.wctb, ry = addr / pc_.wctb;
    const int x0 = rx << sps_.log2_ctb, y0 = ry << sps_.log2_ctb;
    if (!pc_.prefilled) {
      pc_.slice[size_t(addr)] = u16(si_);
      pc_.sord[size_t(addr)] = u16(sl_.ord);
    }
    if (sh_.sao_luma || sh_.sao_chroma) sao(rx, ry);
    quadtree(x0, y0, sps_.log2_ctb, 0);
    const u32 end = e_.term(last ? 1u : 0u);
    if constexpr (!kWrite) last_read_ = end != 0;
  }
  bool end_of_slice() const { return last_read_; }
  // qPY_PREV: SliceQpY again for the next quantization group (first QG of a tile, or of a CTB
  // row with WPP), or the QP of the previous segment's last CU (dependent slice segment)
  void reset_qp_prediction() { first_qg_ = true; }
  void continue_qp_prediction(int qp_last) {
    first_qg_ = false;
    qp_last_ = qp_last;
  }
  int qp_last() const { return qp_last_; }

 private:
  u32 bin(int ctx, u32 v) { return e_.bin(ctx, v); }
  u32 byp(u32 v) { return e_.byp(v); }
  u32 fl(int n, u32 v) {  // fixed length, bypass, MSB first
    u32 r = 0;
    for (int i = n - 1; i >= 0; --i) r |= byp((v >> i) & 1u) << i;
    return r;
  }
  int egk(int k, int v) {  // k-th order Exp-Golomb, bypass (§9.3.3.3)
    int out = 0;
    while (byp(v >= (1 << k))) {
      out += 1 << k;
      v -= 1 << k;
      ++k;
      VEP_CHECK(k < 31, "Exp-Golomb prefix too long");
    }
    while (k--) out += int(byp((v >> k) & 1)) << k;
    return out;
  }

  // -------------------------------------------------------------------- SAO (§7.3.8.3)
  void sao(int rx, int ry) {
    SaoParams want{};
    bool ml = false, mu = false;
    if constexpr (kWrite) dec_->sao(rx, ry, want, ml, mu);
    const int addr = ry * pc_.wctb + rx;
    bool merge_left = false, merge_up = false;
    // §7.3.8.3: the left / up CTB must be in the slice (address >= SliceAddrRs) and the tile
    const auto same_tile = [&](int a) { return pc_.tile[size_t(a)] == pc_.tile[size_t(addr)]; };
    if (rx > 0 && addr - 1 >= sl_.addr_rs && same_tile(addr - 1)) merge_left = bin(kCtxSaoMerge, ml);
    if (ry > 0 && !merge_left && addr - pc_.wctb >= sl_.addr_rs && same_tile(addr - pc_.wctb))
      merge_up = bin(kCtxSaoMerge, mu);
    SaoParams& p = pc_.sao[size_t(addr)];
    if (merge_left) {
      p = pc_.sao[size_t(addr - 1)];
      return;
    }
    if (merge_up) {
      p = pc_.sao[size_t(addr - pc_.wctb)];
      return;
    }
    p = SaoParams{};
    for (int c = 0; c < 3; ++c) {
      if (!((sh_.sao_luma && c == 0) || (sh_.sao_chroma && c > 0))) continue;
      if (c < 2) {  // sao_type_idx: TR cMax 2, bin 0 context, bin 1 bypass
        const int t = want.type[c];
        int v = 0;
        if (bin(kCtxSaoType, t != 0)) v = 1 + int(byp(t == 2));
        p.type[c] = u8(v);
      } else {
        p.type[2] = p.type[1];
      }
      if (!p.type[c]) continue;
      int abs[4];
      const int cmax = (1 << (std::min(c ? pc_.bd_c : pc_.bd_y, 10) - 5)) - 1;  // 7 at 8 bits, 31 at 10
      for (int i = 0; i < 4; ++i) {  // TR cMax, bypass
        const int a = std::abs(int(want.off[c][i]));
        int v = 0;
        while (v < cmax && byp(a > v)) ++v;
        abs[i] = v;
      }
      if (p.type[c] == 1) {
        for (int i = 0; i < 4; ++i) {
          int sgn = 0;
          if (abs[i]) sgn = int(byp(want.off[c][i] < 0));
          p.off[c][i] = i8(sgn ? -abs[i] : abs[i]);
        }
        p.band[c] = u8(fl(5, want.band[c]));
      } else {
        for (int i = 0; i < 4; ++i) p.off[c][i] = i8(i < 2 ? abs[i] : -abs[i]);
        if (c == 0) p.eo[0] = u8(fl(2, want.eo[0]));
        if (c == 1) p.eo[1] = u8(fl(2, want.eo[1]));
        if (c == 2) p.eo[2] = p.eo[1];
      }
    }
  }

  // -------------------------------------------------------------------- coding quadtree
  void quadtree(int x0, int y0, int log2, int depth) {
    const int n = 1 << log2;
    bool split;
    if (x0 + n <= pc_.W && y0 + n <= pc_.H && log2 > sps_.log2_min_cb) {
      int inc = 0;
      if (pc_.avail(x0, y0, x0 - 1, y0, pc_.done) && pc_.depth[pc_.i4(x0 - 1, y0)] > depth) ++inc;
      if (pc_.avail(x0, y0, x0, y0 - 1, pc_.done) && pc_.depth[pc_.i4(x0, y0 - 1)] > depth) ++inc;
      bool want = false;
      if constexpr (kWrite) want = dec_->split(x0, y0, log2);
      split = bin(kCtxSplitCu + inc, want);
    } else {
      split = log2 > sps_.log2_min_cb;
    }
    if (log2 >= log2_min_qg_) {  // start of a quantization group
      qg_x_ = x0;
      qg_y_ = y0;
      qg_coded_ = false;
      cu_qp_delta_ = 0;
      // qPY_PREV (§8.6.1): SliceQpY for the first quantization group of a slice, a tile or (WPP) a
      // CTB row, else the QP of the previous QG's last CU. (The quadtree passes a QG start at
      // every level down to Log2MinCuQpDeltaSize, several at the same position: the first-QG
      // state ends with the first coded CU, not with the first of those passes.)
      qp_prev_ = first_qg_ ? slice_qp_ : qp_last_;
      qp_pred_ = predict_qp();
    }
    if (split) {
      const int h = n >> 1;
      for (int k = 0; k < 4; ++k) {
        const int x = x0 + (k & 1) * h, y = y0 + (k >> 1) * h;
        if (x < pc_.W && y < pc_.H) quadtree(x, y, log2 - 1, depth + 1);
      }
      return;
    }
    coding_unit(x0, y0, log2, depth);
  }

  int predict_qp() const {
    auto qp_at = [&](int xn, int yn) {
      if (!pc_.avail(qg_x_, qg_y_, xn, yn, pc_.done)) return qp_prev_;
      if (pc_.ctb_of(xn, yn) != pc_.ctb_of(qg_x_, qg_y_)) return qp_prev_;
      return int(pc_.qp[pc_.i4(xn, yn)]);
    };
    return (qp_at(qg_x_ - 1, qg_y_) + qp_at(qg_x_, qg_y_ - 1) + 1) >> 1;
  }
  // QpY (§8.6.1), in -QpBdOffsetY .. 51
  int qp_y() const {
    const int off = pc_.qp_off_y;
    return ((qp_pred_ + cu_qp_delta_ + 52 + 2 * off) % (52 + off)) - off;
  }

  // f(k) for every 4x4 block index of the rectangle clipped to the picture: row by row over
  // consecutive indices (the per-block bookkeeping of skip-heavy pictures is a large share of
  // the parse, so no per-block index arithmetic or bound checks).
  template <class F>
  void for4(int x0, int y0, int w, int h, F f) {
    const int xe = std::min(x0 + w, pc_.W), ye = std::min(y0 + h, pc_.H);
    if (xe <= x0) return;
    const size_t cnt = size_t((xe - x0 + 3) >> 2);
    for (int y = y0; y < ye; y += 4) {
      const size_t k0 = pc_.i4(x0, y);
      for (size_t k = k0; k < k0 + cnt; ++k) f(k);
    }
  }

  // for4() storing one constant byte into a per-4x4 map: a memset per row of 4x4 blocks
  void fill4(void* map, int x0, int y0, int w, int h, u8 v) {
    u8* const m = static_cast<u8*>(map);
    const int xe = std::min(x0 + w, pc_.W), ye = std::min(y0 + h, pc_.H);
    if (xe <= x0) return;
    const size_t cnt = size_t((xe - x0 + 3) >> 2);
    for (int y = y0; y < ye; y += 4) std::memset(m + pc_.i4(x0, y), v, cnt);
  }

  // -------------------------------------------------------------------- coding unit
  void coding_unit(int x0, int y0, int log2, int depth) {
    const int n = 1 << log2;
    CuDesc want;
    if constexpr (kWrite) dec_->cu(x0, y0, log2, want);
    cu_ = CuState{};
    cu_.x0 = x0;
    cu_.y0 = y0;
    cu_.log2 = log2;
    // (raw pointers held in locals: a u8 store through pc_.X[k] may alias the vectors' own data
    // pointers, which would otherwise be reloaded after every store of these per-4x4 loops)
    u8* const m_depth = pc_.depth.data();
    u8* const m_edge = pc_.edge.data();
    u8* const m_cbf = pc_.cbf.data();
    u8* const m_pcm = pc_.pcm.data();
    fill4(m_depth, x0, y0, n, n, u8(depth));
    fill4(m_edge, x0, y0, n, n, 0);
    fill4(m_cbf, x0, y0, n, n, 0);
    fill4(m_pcm, x0, y0, n, n, 0);
    // CU boundaries are transform and prediction block edges
    for4(x0, y0, 4, n, [=](size_t k) { m_edge[k] |= kEdgeTuV | kEdgePuV; });
    for4(x0, y0, n, 4, [=](size_t k) { m_edge[k] |= kEdgeTuH | kEdgePuH; });
    cu_.bypass = false;
    if (pps_.transquant_bypass) {
      cu_.bypass = bin(kCtxTransquantBypass, want.bypass) != 0;
      u8* const m_byp = pc_.bypass.data();
      const u8 bv = u8(cu_.bypass);
      fill4(m_byp, x0, y0, n, n, bv);
      if (cu_.bypass) *bypass_ = true;
    }
    bool skip = false;
    if (sh_.slice_type != kI) {
      int inc = 0;
      if (pc_.avail(x0, y0, x0 - 1, y0, pc_.done) && pc_.skip[pc_.i4(x0 - 1, y0)]) ++inc;
      if (pc_.avail(x0, y0, x0, y0 - 1, pc_.done) && pc_.skip[pc_.i4(x0, y0 - 1)]) ++inc;
      skip = bin(kCtxSkip + inc, want.skip);
    }
    u8* const m_skip = pc_.skip.data();
    fill4(m_skip, x0, y0, n, n, u8(skip));
    bool intra = false, pcm = false;
    int part = 0;
    if (skip) {
      cu_.intra = false;
      u8* const m_intra = pc_.intra.data();
      fill4(m_intra, x0, y0, n, n, 0);
      prediction_unit(x0, y0, n, n, 0, 0, want.pu[0], true);
      ++st_->skip;
    } else {
      intra = sh_.slice_type == kI ? true : bin(kCtxPredMode, want.intra) != 0;
      cu_.intra = intra;
      if (!intra || log2 == sps_.log2_min_cb) part = part_mode(intra, log2, want.part);
      cu_.part = part;
      if (intra) {
        for4(x0, y0, n, n, [&](size_t k) {
          pc_.intra[k] = 1;
          pc_.mf[k] = MvField{};
        });
        if (part == 0 && sps_.pcm && log2 >= sps_.log2_min_pcm && log2 <= sps_.log2_max_pcm)
          pcm = e_.term(want.pcm ? 1u : 0u) != 0;
        if (pcm) {
          pcm_sample(x0, y0, log2, want.pcm_samples);
          ++st_->pcm;
        } else {
          intra_modes(x0, y0, log2, part, want);
          ++st_->intra;
        }
      } else {
        u8* const m_intra = pc_.intra.data();
        fill4(m_intra, x0, y0, n, n, 0);
        int r[4][4];
        const int np = pu_rects(part, n, r);
        for (int k = 0; k < np; ++k) prediction_unit(x0 + r[k][0], y0 + r[k][1], r[k][2], r[k][3], k, part, want.pu[k], false);
        ++st_->inter;
        if (part >= 4) ++st_->amp;
      }
    }
    if (!cu_.intra) predict_inter_cu();
    if (!pcm && !skip) {
      bool root = true;
      if (!intra && !(part == 0 && cu_.merge0)) {
        bool want_root = false;
        if constexpr (kWrite) want_root = plan_residual(want);
        root = bin(kCtxRqtRootCbf, want_root) != 0;
      } else if constexpr (kWrite) {
        // rqt_root_cbf is inferred 1 here: a merge 2Nx2N CU without residual would be a skip CU,
        // so give it the smallest residual (inter prediction does not depend on it)
        if (!plan_residual(want) && !intra) levels_[TuKey{0, x0, y0}].lv[0] = 1, levels_[TuKey{0, x0, y0}].any = true;
      }
      if (root) {
        const int max_depth = intra ? sps_.max_th_depth_intra + (part == 3 ? 1 : 0) : sps_.max_th_depth_inter;
        cu_.max_trafo_depth = max_depth;
        cu_.tu_target = want.tu_log2;
        transform_tree(x0, y0, x0, y0, log2, 0, 0, true, true);
      } else if (intra) {
        VEP_CHECK(false, "intra CU without a transform tree");
      }
    }
    const int q = qp_y();
    i8* const m_qp = pc_.qp.data();
    u8* const m_done = pc_.done.data();
    u8* const m_rec = pc_.rec.data();
    fill4(m_qp, x0, y0, n, n, u8(i8(q)));
    fill4(m_done, x0, y0, n, n, 1);
    fill4(m_rec, x0, y0, n, n, 1);
    fill4(m_pcm, x0, y0, n, n, u8(pcm));
    qp_last_ = q;
    first_qg_ = false;
  }

  int part_mode(bool intra, int log2, int want) {
    if (intra) return bin(kCtxPartMode, want == 0) ? 0 : 3;
    if (bin(kCtxPartMode, want == 0)) return 0;
    const bool min = log2 == sps_.log2_min_cb;
    const bool amp = sps_.amp && !min;
    const bool hor = want == 1 || want == 4 || want == 5;  // 2NxN family
    if (bin(kCtxPartMode + 1, hor)) {                      // 2NxN / 2NxnU / 2NxnD
      if (!amp) return 1;
      if (bin(kCtxPartMode + 3, want == 1)) return 1;
      return byp(want == 5) ? 5 : 4;
    }
    if (min) {
      if (log2 == 3) return 2;  // inter NxN is not allowed for 8x8 CUs
      return bin(kCtxPartMode + 2, want == 2) ? 2 : 3;
    }
    if (!amp) return 2;
    if (bin(kCtxPartMode + 3, want == 2)) return 2;
    return byp(want == 7) ? 7 : 6;
  }

  // -------------------------------------------------------------------- PCM
  void pcm_sample(int x0, int y0, int log2, const u16* want) {
    // pcm_sample_luma / chroma: u(PcmBitDepth) each, MSB first, byte aligned; the sample is the
    // value << (BitDepth - PcmBitDepth) (§8.4.4.1)
    const int n = 1 << log2, nc = n / 2;
    HostSurface& s = *pc_.s;
    const int pby = sps_.pcm_bit_depth_luma, pbc = sps_.pcm_bit_depth_chroma;
    VEP_CHECK(pby >= 1 && pbc >= 1 && pby <= pc_.bd_y && pbc <= pc_.bd_c, "PCM bit depth above the sample bit depth");
    const size_t nl = size_t(n) * n, ns = nl + 2 * size_t(nc) * nc;
    const size_t bytes = (nl * size_t(pby) + (ns - nl) * size_t(pbc)) / 8;  // (n >= 8: whole bytes)
    u16 v[64 * 64 + 2 * 32 * 32];
    if constexpr (kWrite) {
      std::vector<u8> packed(bytes, 0);
      size_t bit = 0;
      for (size_t k = 0; k < ns; ++k) {
        const int nb = k < nl ? pby : pbc;
        for (int b = nb - 1; b >= 0; --b, ++bit)
          if ((want[k] >> b) & 1) packed[bit >> 3] |= u8(0x80u >> (bit & 7));
      }
      wr->align_zero();
      wr->raw_bytes(packed.data(), bytes);
      wr->start();
      for (size_t k = 0; k < ns; ++k) v[k] = u16(want[k] << (k < nl ? pc_.bd_y - pby : pc_.bd_c - pbc));
    } else {
      const size_t pos = rd->aligned_bytepos();
      VEP_CHECK(pos + bytes <= data_n, "PCM samples past the end of the slice");
      const u8* src = data + pos;
      rd->start(pos + bytes);
      size_t bit = 0;
      for (size_t k = 0; k < ns; ++k) {
        const int nb = k < nl ? pby : pbc;
        u32 x = 0;
        for (int b = 0; b < nb; ++b, ++bit) x = (x << 1) | ((src[bit >> 3] >> (7 - (bit & 7))) & 1u);
        v[k] = u16(x << (k < nl ? pc_.bd_y - pby : pc_.bd_c - pbc));
      }
      if (GpuPicture* g = g_) {  // records mode: the GPU copies the samples (level 0)
        GpuTu t{};
        t.x = u16(x0);
        t.y = u16(y0);
        t.log2 = u8(log2);
        t.flags = kTuPcm;
        if (g->wide()) {  // u16 samples (2-byte aligned)
          if (g->pcm.size() & 1) g->pcm.push_back(0);
          t.data = u32(g->pcm.size());
          const u8* b = reinterpret_cast<const u8*>(v);
          g->pcm.insert(g->pcm.end(), b, b + 2 * ns);
        } else {
          t.data = u32(g->pcm.size());
          for (size_t k = 0; k < ns; ++k) g->pcm.push_back(u8(v[k]));
        }
        g->tus.push_back(t);
        return;
      }
    }
    for (int y = 0; y < n; ++y)
      for (int x = 0; x < n; ++x) s.set(0, x0 + x, y0 + y, v[size_t(y) * n + x]);
    const u16* cb = v + nl;
    const u16* cr = cb + size_t(nc) * nc;
    for (int y = 0; y < nc; ++y)
      for (int x = 0; x < nc; ++x) {
        s.set(1, x0 / 2 + x, y0 / 2 + y, cb[y * nc + x]);
        s.set(2, x0 / 2 + x, y0 / 2 + y, cr[y * nc + x]);
      }
  }

  // -------------------------------------------------------------------- intra modes (§8.4.2)
  void mpm_list(int x, int y, int cand[3]) {
    auto nb = [&](int xn, int yn, bool above) {
      if (!pc_.avail(x, y, xn, yn, pc_.done)) return 1;
      const size_t k = pc_.i4(xn, yn);
      if (!pc_.intra[k] || pc_.pcm[k]) return 1;
      if (above && yn < ((y >> sps_.log2_ctb) << sps_.log2_ctb)) return 1;
      return int(pc_.ipm[k]);
    };
    const int a = nb(x - 1, y, false), b = nb(x, y - 1, true);
    if (a == b) {
      if (a < 2) {
        cand[0] = 0, cand[1] = 1, cand[2] = 26;
      } else {
        cand[0] = a;
        cand[1] = 2 + ((a + 29) % 32);
        cand[2] = 2 + ((a - 2 + 1) % 32);
      }
    } else {
      cand[0] = a;
      cand[1] = b;
      cand[2] = (a != 0 && b != 0) ? 0 : (a != 1 && b != 1) ? 1 : 26;
    }
  }

  void intra_modes(int x0, int y0, int log2, int part, const CuDesc& want) {
    const int n = 1 << log2;
    const int np = part == 3 ? 4 : 1, pb = part == 3 ? n / 2 : n;
    int flag[4] = {0, 0, 0, 0}, idx[4] = {0, 0, 0, 0}, rem[4] = {0, 0, 0, 0};
    auto set_mode = [&](int k, int m) {
      const int x = x0 + (k & 1) * pb, y = y0 + (k >> 1) * pb;
      for4(x, y, pb, pb, [&](size_t i) {
        pc_.ipm[i] = u8(m);
        pc_.done[i] = 1;
      });
      cu_.ipm[k] = m;
    };
    if constexpr (kWrite) {  // the flags of all partitions come first: derive them in order
      for (int k = 0; k < np; ++k) {
        int c[3];
        mpm_list(x0 + (k & 1) * pb, y0 + (k >> 1) * pb, c);
        const int m = want.luma_mode[k];
        flag[k] = 0;
        for (int i = 0; i < 3; ++i)
          if (c[i] == m) flag[k] = 1, idx[k] = i;
        if (!flag[k]) {
          std::sort(c, c + 3);
          int r = m;
          for (int i = 2; i >= 0; --i)
            if (m > c[i]) --r;
          rem[k] = r;
        }
        set_mode(k, m);
      }
      for (int k = 0; k < np; ++k) {  // restore: the decoder sees the flags before any mode
        const int x = x0 + (k & 1) * pb, y = y0 + (k >> 1) * pb;
        for4(x, y, pb, pb, [&](size_t i) { pc_.done[i] = 0; });
      }
    }
    for (int k = 0; k < np; ++k) flag[k] = int(bin(kCtxPrevIntra, flag[k]));
    for (int k = 0; k < np; ++k) {
      int c[3];
      mpm_list(x0 + (k & 1) * pb, y0 + (k >> 1) * pb, c);
      int m;
      if (flag[k]) {
        int v = 0;  // mpm_idx: TR cMax 2, bypass
        while (v < 2 && byp(idx[k] > v)) ++v;
        m = c[v];
      } else {
        const int r = int(fl(5, u32(rem[k])));
        std::sort(c, c + 3);
        m = r;
        for (int i = 0; i < 3; ++i)
          if (m >= c[i]) ++m;
      }
      set_mode(k, m);
    }
    // intra_chroma_pred_mode: "0" -> 4 (DM), "1" + 2 bits -> 0..3
    const int wc = want.chroma_mode;
    int cm = 4;
    if (bin(kCtxChromaMode, wc != 4)) cm = int(fl(2, u32(wc & 3)));
    static constexpr int kMap[4] = {0, 26, 10, 1};
    const int luma0 = cu_.ipm[0];
    cu_.ipmc = cm == 4 ? luma0 : (kMap[cm] == luma0 ? 34 : kMap[cm]);
  }

  // -------------------------------------------------------------------- prediction unit
  void prediction_unit(int x, int y, int w, int h, int partIdx, int part, const CuDesc::Pu& want, bool skip) {
    MvField m;
    bool merge = skip;
    if (!skip) merge = bin(kCtxMergeFlag, want.merge) != 0;
    const int maxc = sh_.max_num_merge_cand;
    if (merge) {
      int idx = 0;
      if (maxc > 1) {  // merge_idx: TR cMax MaxNumMergeCand - 1, bin 0 context, rest bypass
        const int wv = want.merge_idx;
        if (bin(kCtxMergeIdx, wv > 0)) {
          idx = 1;
          while (idx < maxc - 1 && byp(wv > idx)) ++idx;
        }
      }
      MergeCand c[5];
      const int nc = merge_candidates(pc_, si_, cu_.x0, cu_.y0, 1 << cu_.log2, x, y, w, h, partIdx, part, c);
      VEP_CHECK(idx < nc, "merge_idx out of range");
      m.pred = c[idx].pred;
      for (int l = 0; l < 2; ++l) {
        m.ref[l] = c[idx].ref[l];
        m.mv[l][0] = c[idx].mv[l][0];
        m.mv[l][1] = c[idx].mv[l][1];
      }
      ++st_->merge;
      if (partIdx == 0) cu_.merge0 = true;
    } else {
      int dir = 1;
      if (sh_.slice_type == kB) {
        const int wd = want.dir;
        if (w + h != 12) {
          const int ctdepth = pc_.depth[pc_.i4(cu_.x0, cu_.y0)];
          if (bin(kCtxInterPred + ctdepth, wd == 3)) dir = 3;
          else dir = bin(kCtxInterPred + 4, wd == 2) ? 2 : 1;
        } else {
          dir = bin(kCtxInterPred + 4, wd == 2) ? 2 : 1;
        }
      }
      i16 mvd[2][2] = {{0, 0}, {0, 0}};
      int ref[2] = {-1, -1}, mvpf[2] = {0, 0};
      i16 mvp_cand[2][2][2];
      for (int l = 0; l < 2; ++l) {
        if (!((dir >> l) & 1)) continue;
        const int nref = l == 0 ? sh_.num_ref_idx_l0 : sh_.num_ref_idx_l1;
        ref[l] = 0;
        if (nref > 1) {  // ref_idx: TR cMax nref - 1, bins 0..1 context, rest bypass
          const int wr = want.ref[l];
          int v = 0;
          while (v < nref - 1) {
            const bool b = v < 2 ? bin(kCtxRefIdx + v, wr > v) : byp(wr > v);
            if (!b) break;
            ++v;
          }
          ref[l] = v;
        }
        VEP_CHECK(size_t(ref[l]) < sl_.list[l].size(), "ref_idx outside the list");
        if constexpr (kWrite) {
          amvp_candidates(pc_, si_, cu_.x0, cu_.y0, 1 << cu_.log2, x, y, w, h, partIdx, l, ref[l], mvp_cand[l]);
          const int f = want.mvp[l];
          for (int c = 0; c < 2; ++c) mvd[l][c] = i16(want.mv[l][c] - mvp_cand[l][f][c]);
        }
        if (l == 1 && sh_.mvd_l1_zero && dir == 3) {
          mvd[1][0] = mvd[1][1] = 0;
        } else {
          mvd_coding(mvd[l]);
        }
        mvpf[l] = int(bin(kCtxMvpFlag, want.mvp[l]));
      }
      m.pred = u8(dir);
      for (int l = 0; l < 2; ++l) {
        if (!((dir >> l) & 1)) continue;
        if constexpr (!kWrite)
          amvp_candidates(pc_, si_, cu_.x0, cu_.y0, 1 << cu_.log2, x, y, w, h, partIdx, l, ref[l], mvp_cand[l]);
        m.ref[l] = i8(ref[l]);
        for (int c = 0; c < 2; ++c) {
          const int u = (mvp_cand[l][mvpf[l]][c] + mvd[l][c] + 65536) & 0xFFFF;
          m.mv[l][c] = i16(u >= 32768 ? u - 65536 : u);
        }
      }
      if (dir == 3) ++st_->bi;
    }
    {
      MvField* const m_mf = pc_.mf.data();
      u8* const m_done = pc_.done.data();
      u8* const m_edge = pc_.edge.data();
      for4(x, y, w, h, [=](size_t k) {
        m_mf[k] = m;
        m_done[k] = 1;
      });
      for4(x, y, 4, h, [=](size_t k) { m_edge[k] |= kEdgePuV; });
      for4(x, y, w, 4, [=](size_t k) { m_edge[k] |= kEdgePuH; });
    }
    cu_.pus[cu_.npu][0] = x, cu_.pus[cu_.npu][1] = y, cu_.pus[cu_.npu][2] = w, cu_.pus[cu_.npu][3] = h;
    ++cu_.npu;
  }

  void mvd_coding(i16 mvd[2]) {  // §7.3.8.9
    const int a[2] = {std::abs(int(mvd[0])), std::abs(int(mvd[1]))};
    bool g0[2], g1[2] = {false, false};
    for (int c = 0; c < 2; ++c) g0[c] = bin(kCtxMvdGt0, a[c] > 0) != 0;
    for (int c = 0; c < 2; ++c)
      if (g0[c]) g1[c] = bin(kCtxMvdGt1, a[c] > 1) != 0;
    for (int c = 0; c < 2; ++c) {
      if (!g0[c]) {
        mvd[c] = 0;
        continue;
      }
      int v = 1;
      if (g1[c]) v = 2 + egk(1, a[c] - 2);
      const bool neg = byp(mvd[c] < 0) != 0;
      mvd[c] = i16(neg ? -v : v);
    }
  }

  // Records mode: index + 1 of the explicit weighting of a PU in the picture's weight table
  // (entries are shared by every PU with the same weights / offsets / shifts).
  u8 gpu_wp_index(const MvField& m) {
    const GpuWp e = explicit_weights(sh_, m, pc_.bd_y, pc_.bd_c);
    std::vector<GpuWp>& tab = g_->wp;
    for (size_t i = 0; i < tab.size(); ++i)
      if (std::memcmp(&tab[i], &e, sizeof e) == 0) return u8(i + 1);
    VEP_CHECK(tab.size() < 255, "HEVC: more than 255 distinct prediction weights in one picture");
    tab.push_back(e);
    return u8(tab.size());
  }

  void predict_inter_cu() {
    if (GpuPicture* g = g_) {  // records mode: one record per prediction block
      for (int k = 0; k < cu_.npu; ++k) {
        const int x = cu_.pus[k][0], y = cu_.pus[k][1];
        const MvField& m = pc_.mf[pc_.i4(x, y)];
        GpuPu u{};
        u.x = u16(x);
        u.y = u16(y);
        u.w = u8(cu_.pus[k][2]);
        u.h = u8(cu_.pus[k][3]);
        u.pred = m.pred;
        u.wp = sh_.weighted ? gpu_wp_index(m) : 0;
        for (int l = 0; l < 2; ++l) {
          u.slot[l] = -1;
          if ((m.pred >> l) & 1) {
            VEP_CHECK(m.ref[l] >= 0 && size_t(m.ref[l]) < sl_.list[l].size(), "reference index outside the list");
            u.slot[l] = i8(sl_.list[l][size_t(m.ref[l])]->slot);
          }
          u.mv[l][0] = m.mv[l][0];
          u.mv[l][1] = m.mv[l][1];
        }
        g->pus.push_back(u);
      }
      return;
    }
    HostSurface& s = *pc_.s;
    for (int k = 0; k < cu_.npu; ++k) {
      const int x = cu_.pus[k][0], y = cu_.pus[k][1], w = cu_.pus[k][2], h = cu_.pus[k][3];
      std::vector<u16> py(size_t(w) * h), pcb(size_t(w / 2) * (h / 2)), pcr(pcb.size());
      predict_pu(pc_, si_, x, y, w, h, pc_.mf[pc_.i4(x, y)], py.data(), w, pcb.data(), pcr.data(), w / 2);
      for (int j = 0; j < h; ++j)
        for (int i = 0; i < w; ++i) s.set(0, x + i, y + j, py[size_t(j) * w + i]);
      for (int j = 0; j < h / 2; ++j)
        for (int i = 0; i < w / 2; ++i) {
          s.set(1, x / 2 + i, y / 2 + j, pcb[size_t(j) * (w / 2) + i]);
          s.set(2, x / 2 + i, y / 2 + j, pcr[size_t(j) * (w / 2) + i]);
        }
    }
  }

  // -------------------------------------------------------------------- transform tree
  // Write mode: a dry run over the CU's transform tree first computes every transform block's
  // levels (prediction -> encoder callback -> reconstruction, in decoding order), then the CU's
  // samples are restored and the tree is written with those levels (cbf flags and rqt_root_cbf
  // follow from them, so they are known before the blocks they cover).
  struct TuKey {
    int c, x, y;
    bool operator<(const TuKey& o) const { return c != o.c ? c < o.c : (x != o.x ? x < o.x : y < o.y); }
  };
  struct TuLevels {
    std::vector<int> lv;
    bool tskip = false;
    bool any = false;
  };

  bool plan_residual(const CuDesc& want) {
    const int n = 1 << cu_.log2;
    HostSurface& s = *pc_.s;
    // save the CU's samples and availability (the dry run reconstructs into them)
    std::vector<u16> sy(size_t(n) * n), suv(size_t(n) * n / 2);
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i) sy[size_t(j) * n + i] = u16(s.get(0, cu_.x0 + i, cu_.y0 + j));
    for (int j = 0; j < n / 2; ++j)
      for (int i = 0; i < n / 2; ++i) {
        suv[size_t(j) * n + 2 * i] = u16(s.get(1, cu_.x0 / 2 + i, cu_.y0 / 2 + j));
        suv[size_t(j) * n + 2 * i + 1] = u16(s.get(2, cu_.x0 / 2 + i, cu_.y0 / 2 + j));
      }
    std::vector<u8> srec;
    for4(cu_.x0, cu_.y0, n, n, [&](size_t k) { srec.push_back(pc_.rec[k]); });
    levels_.clear();
    dry_ = true;
    cu_.max_trafo_depth = cu_.intra ? sps_.max_th_depth_intra + (cu_.part == 3 ? 1 : 0) : sps_.max_th_depth_inter;
    cu_.tu_target = want.tu_log2;
    const int saved_delta = cu_qp_delta_;
    const bool saved_coded = qg_coded_;
    dry_qp_delta_ = want.qp_delta;
    dry_tskip_ = want.tskip;
    transform_tree(cu_.x0, cu_.y0, cu_.x0, cu_.y0, cu_.log2, 0, 0, true, true);
    dry_ = false;
    cu_qp_delta_ = saved_delta;
    qg_coded_ = saved_coded;
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i) s.set(0, cu_.x0 + i, cu_.y0 + j, sy[size_t(j) * n + i]);
    for (int j = 0; j < n / 2; ++j)
      for (int i = 0; i < n / 2; ++i) {
        s.set(1, cu_.x0 / 2 + i, cu_.y0 / 2 + j, suv[size_t(j) * n + 2 * i]);
        s.set(2, cu_.x0 / 2 + i, cu_.y0 / 2 + j, suv[size_t(j) * n + 2 * i + 1]);
      }
    size_t i = 0;
    for4(cu_.x0, cu_.y0, n, n, [&](size_t k) { pc_.rec[k] = srec[i++]; });
    bool any = false;
    for (auto& kv : levels_) any |= kv.second.any;
    return any;
  }

  bool any_levels(int c, int x0, int y0, int n) const {  // any coded block of component c inside
    if (c) x0 >>= 1, y0 >>= 1, n >>= 1;                   // (chroma keys are in chroma samples)
    for (auto& kv : levels_)
      if (kv.first.c == c && kv.first.x >= x0 && kv.first.y >= y0 && kv.first.x < x0 + n && kv.first.y < y0 + n &&
          kv.second.any)
        return true;
    return false;
  }

  void transform_tree(int x0, int y0, int xb, int yb, int log2, int depth, int blk, bool pcb, bool pcr) {
    const bool intra_split = cu_.intra && cu_.part == 3;
    const bool inter_split = sps_.max_th_depth_inter == 0 && !cu_.intra && cu_.part != 0 && depth == 0;
    bool split;
    const bool coded = log2 <= sps_.log2_max_tb && log2 > sps_.log2_min_tb && depth < cu_.max_trafo_depth &&
                       !(intra_split && depth == 0);
    const int target = std::clamp(cu_.tu_target, sps_.log2_min_tb, sps_.log2_max_tb);
    if (coded) {
      const bool want = log2 > target;
      split = dry_ ? want : bin(kCtxSplitTransform + 5 - log2, want) != 0;
    } else {
      split = log2 > sps_.log2_max_tb || (intra_split && depth == 0) || inter_split;
    }
    bool cb = false, cr = false;
    const int n = 1 << log2;
    if (log2 > 2) {
      if (depth == 0 || pcb) {
        const bool w = !dry_ && kWrite && any_levels(1, x0, y0, n);
        cb = dry_ ? true : bin(kCtxCbfChroma + depth, w) != 0;
      }
      if (depth == 0 || pcr) {
        const bool w = !dry_ && kWrite && any_levels(2, x0, y0, n);
        cr = dry_ ? true : bin(kCtxCbfChroma + depth, w) != 0;
      }
    } else {
      cb = pcb;
      cr = pcr;
    }
    if (split) {
      const int h = n >> 1;
      for (int k = 0; k < 4; ++k)
        transform_tree(x0 + (k & 1) * h, y0 + (k >> 1) * h, x0, y0, log2 - 1, depth + 1, k, cb, cr);
      return;
    }
    bool cl = true;
    if (cu_.intra || depth != 0 || cb || cr) {
      const bool w = !dry_ && kWrite && any_levels(0, x0, y0, n);
      cl = dry_ ? true : bin(kCtxCbfLuma + (depth == 0 ? 1 : 0), w) != 0;
    }
    transform_unit(x0, y0, xb, yb, log2, depth, blk, cl, cb, cr);
  }

  void transform_unit(int x0, int y0, int xb, int yb, int log2, int depth, int blk, bool cl, bool cb, bool cr) {
    (void)depth;
    const int n = 1 << log2;
    const bool chroma_here = log2 > 2;
    const bool chroma_at_parent = !chroma_here && blk == 3;
    const int xc = chroma_here ? x0 : xb, yc = chroma_here ? y0 : yb, log2c = chroma_here ? log2 - 1 : 2;
    // TU edges (deblocking) and the luma cbf map
    {
      u8* const m_edge = pc_.edge.data();
      for4(x0, y0, 4, n, [=](size_t k) { m_edge[k] |= kEdgeTuV; });
      for4(x0, y0, n, 4, [=](size_t k) { m_edge[k] |= kEdgeTuH; });
    }
    const bool chroma_coded = cb || cr;  // (4x4 luma blocks: the parent's chroma flags, all four)
    if (dry_) {
      // quantisation parameter as the real pass will see it: the CU's delta is coded at the
      // first coded block (the encoder's delta; blocks before it have no levels)
      if (pps_.cu_qp_delta && !qg_coded_) {
        cu_qp_delta_ = dry_qp_delta_;
        qg_coded_ = true;
      }
    } else if ((cl || chroma_coded) && pps_.cu_qp_delta && !qg_coded_) {
      int v = cu_qp_delta_;
      if constexpr (kWrite) v = want_delta_for_write();
      // cu_qp_delta_abs: prefix TU cMax 5 (bin 0 context 0, bins 1-4 context 1), suffix EG0
      const int a = std::abs(v);
      int p = 0;
      while (p < 5 && bin(kCtxQpDelta + (p == 0 ? 0 : 1), a > p)) ++p;
      int abs = p;
      if (p == 5) abs += egk(0, a - 5);
      int d = abs;
      if (abs) d = byp(v < 0) ? -abs : abs;
      VEP_CHECK(d >= -(26 + pc_.qp_off_y / 2) && d <= 25 + pc_.qp_off_y / 2, "cu_qp_delta out of range");
      cu_qp_delta_ = d;
      qg_coded_ = true;
    }
    const int qp = qp_y();
    // luma (Qp'Y = QpY + QpBdOffsetY)
    if (cu_.intra) intra_pred_block(0, x0, y0, log2);
    residual_block(0, x0, y0, log2, cl, qp + pc_.qp_off_y);
    {
      u8* const m_cbf = pc_.cbf.data();
      u8* const m_rec = pc_.rec.data();
      const u8 cbfv = u8(cl && !dry_ ? cbf_nonzero_ : 0);
      const bool intra = cu_.intra;
      for4(x0, y0, n, n, [=](size_t k) {
        m_cbf[k] = cbfv;
        if (intra) m_rec[k] = 1;
      });
    }
    // chroma
    if (chroma_here || chroma_at_parent) {
      // qPiCb / Cr = Clip3(-QpBdOffsetC, 57, QpY + offsets); Qp'C = table(qPi) + QpBdOffsetC
      const int oc = pc_.qp_off_c;
      const int qpi_cb = std::clamp(qp + pps_.cb_qp_offset + sh_.cb_qp_offset, -oc, 57);
      const int qpi_cr = std::clamp(qp + pps_.cr_qp_offset + sh_.cr_qp_offset, -oc, 57);
      for (int c = 1; c <= 2; ++c) {
        if (cu_.intra) intra_pred_block(c, xc / 2, yc / 2, log2c);
        residual_block(c, xc / 2, yc / 2, log2c, c == 1 ? cb : cr, hevc_chroma_qp(c == 1 ? qpi_cb : qpi_cr) + oc);
      }
    }
  }

  int want_delta_for_write() const { return dry_qp_delta_; }

  // -------------------------------------------------------------------- intra prediction
  void intra_pred_block(int c, int x0, int y0, int log2) {
    // x0, y0 in the component's samples
    if (g_) {
      gpu_intra_refs(c, x0, y0, log2);
      return;
    }
    HostSurface& s = *pc_.s;
    const int n = 1 << log2, sub = c ? 1 : 0;
    const int bd = c ? pc_.bd_c : pc_.bd_y;
    const int mode = c == 0 ? cu_.ipm[cu_.part == 3 ? ((y0 - cu_.y0 >= (1 << cu_.log2) / 2) ? 2 : 0) +
                                                          ((x0 - cu_.x0 >= (1 << cu_.log2) / 2) ? 1 : 0)
                                                    : 0]
                            : cu_.ipmc;
    int top[129], left[128];
    bool av_t[129], av_l[128];
    const int lx = x0 << sub, ly = y0 << sub;  // luma location of the block
    auto sample = [&](int x, int y) -> int { return s.get(c, x, y); };
    auto avail = [&](int x, int y) {  // component location
      const int xl = x << sub, yl = y << sub;
      if (!pc_.avail(lx, ly, xl, yl, pc_.rec)) return false;
      if (pps_.constrained_intra_pred && !pc_.intra[pc_.i4(xl, yl)]) return false;
      return true;
    };
    int navail = 0;
    av_t[0] = avail(x0 - 1, y0 - 1);
    if (av_t[0]) top[0] = sample(x0 - 1, y0 - 1), ++navail;
    for (int i = 0; i < 2 * n; ++i) {
      av_t[i + 1] = avail(x0 + i, y0 - 1);
      if (av_t[i + 1]) top[i + 1] = sample(x0 + i, y0 - 1), ++navail;
      av_l[i] = avail(x0 - 1, y0 + i);
      if (av_l[i]) left[i] = sample(x0 - 1, y0 + i), ++navail;
    }
    if (!navail) {
      for (int i = 0; i <= 2 * n; ++i) top[i] = 1 << (bd - 1);
      for (int i = 0; i < 2 * n; ++i) left[i] = 1 << (bd - 1);
    } else {
      // substitution (§8.4.4.2.2): scan from p[-1][2n-1] up to p[-1][-1], then p[0..2n-1][-1]
      auto get = [&](int k) -> int& { return k < 2 * n ? left[2 * n - 1 - k] : top[k - 2 * n]; };
      auto av = [&](int k) { return k < 2 * n ? av_l[2 * n - 1 - k] : av_t[k - 2 * n]; };
      const int total = 4 * n + 1;
      if (!av(0)) {
        int k = 1;
        while (!av(k)) ++k;
        get(0) = get(k);
      }
      for (int k = 1; k < total; ++k)
        if (!av(k)) get(k) = get(k - 1);
    }
    if (c == 0) filter_intra_refs(top, left, log2, mode, sps_.strong_intra_smoothing, bd);
    u16 pred[32 * 32];
    intra_predict(top, left, log2, mode, c == 0, pred, n, true, bd);
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i) s.set(c, x0 + i, y0 + j, pred[j * n + i]);
  }

  // Records mode: which reference units of the block are available (hk_prepare_refs mask) and
  // the block's intra dependency level (1 + the highest level among the intra blocks it reads).
  void gpu_intra_refs(int c, int x0, int y0, int log2) {
    const int n = 1 << log2, sub = c ? 1 : 0, g = c ? 2 : 4;
    const int lx = x0 << sub, ly = y0 << sub;
    std::vector<u16>& lvl = c ? pc_.lvl_c : pc_.lvl_y;
    u64 mask = 0, pend = 0;
    int level = 0;
    auto probe = [&](int x, int y, int bit) {  // component location of the unit's first sample
      const int xl = x << sub, yl = y << sub;
      if (!pc_.avail(lx, ly, xl, yl, pc_.rec)) return;
      if (pps_.constrained_intra_pred && !pc_.intra[pc_.i4(xl, yl)]) return;
      mask |= u64(1) << bit;
      const int l = int(lvl[pc_.i4(xl, yl)]);
      if (l > 0) pend |= u64(1) << bit;  // written by an intra block of the same launch
      level = std::max(level, l);
    };
    probe(x0 - 1, y0 - 1, 0);
    for (int k = 0; k < 2 * n / g; ++k) {
      probe(x0 - 1, y0 + k * g, 1 + k);
      probe(x0 + k * g, y0 - 1, 17 + k);
    }
    gpu_avail_ = mask;
    gpu_pend_ = pend;
    gpu_level_ = level + 1;
  }

  // -------------------------------------------------------------------- residual
  int scan_idx(int c, int log2) const {
    if (!cu_.intra) return 0;
    if (!(log2 == 2 || (log2 == 3 && c == 0))) return 0;
    const int m = c == 0 ? block_luma_mode_ : cu_.ipmc;
    if (m >= 6 && m <= 14) return 2;
    if (m >= 22 && m <= 30) return 1;
    return 0;
  }

  // Reads / writes one block's levels and adds its residual to the prediction in the surface.
  void residual_block(int c, int x0, int y0, int log2, bool coded, int qp) {
    cbf_nonzero_ = false;
    const int n = 1 << log2;
    if (c == 0 && cu_.intra) {
      const int half = (1 << cu_.log2) / 2;
      block_luma_mode_ = cu_.ipm[cu_.part == 3 ? ((y0 - cu_.y0 >= half) ? 2 : 0) + ((x0 - cu_.x0 >= half) ? 1 : 0) : 0];
    }
    HostSurface& s = *pc_.s;
    const int bd = c ? pc_.bd_c : pc_.bd_y;
    if (lvbuf_.size() < 1024) lvbuf_.assign(1024, 0);
    int* lv = lvbuf_.data();
    const int nn = n * n;
    if (kWrite) std::fill(lv, lv + nn, 0);  // (read mode: residual_coding clears what it reads)
    bool tskip = false;
    int nnz = 0;  // read mode: non-zero levels, raster positions in nzbuf_
    const TuKey key{c, x0, y0};
    if (dry_) {
      if constexpr (kWrite) {
        std::vector<u16> pred(size_t(n) * n);
        for (int j = 0; j < n; ++j)
          for (int i = 0; i < n; ++i) pred[size_t(j) * n + i] = u16(s.get(c, x0 + i, y0 + j));
        const bool ts_ok = pps_.transform_skip && log2 == 2 && !cu_.bypass;
        bool ts = dry_tskip_ && ts_ok;
        dec_->residual(c, x0, y0, log2, pred.data(), n, qp, ts_ok, cu_.intra, lv, ts);
        tskip = ts && ts_ok;
        if (pps_.sign_data_hiding && !cu_.bypass) hide_signs(lv, log2, scan_idx(c, log2));
        TuLevels& t = levels_[key];
        t.lv.assign(lv, lv + nn);
        t.tskip = tskip;
        t.any = std::any_of(lv, lv + nn, [](int v) { return v != 0; });
      }
    } else if (coded) {
      if constexpr (kWrite) {
        const TuLevels& t = levels_[key];
        std::copy(t.lv.begin(), t.lv.end(), lv);
        tskip = t.tskip;
      }
      if constexpr (kWrite) {
        residual_coding(c, log2, lv, tskip);
      } else {
        // lv is all zeros between TUs (the read levels are cleared again by position when this
        // TU is done, below); a decode that threw leaves it dirty and the next one clears it all
        if (lv_dirty_) std::fill(lv, lv + lvbuf_.size(), 0);
        lv_dirty_ = true;
        nnz = residual_coding_rd(c, log2, lv, tskip, nzbuf_);
      }
      if (tskip) ++st_->tskip;
    }
    struct LvClear {  // (read mode) the levels of this TU back to zero on every way out
      int* lv;
      const u16* pos;
      const int& n;
      bool& dirty;
      bool armed;
      ~LvClear() {
        if (!armed) return;
        for (int j = 0; j < n; ++j) lv[pos[j]] = 0;
        dirty = false;
      }
    } lv_clear{lv, nzbuf_, nnz, lv_dirty_, !kWrite && coded && !dry_};
    bool nz = false;
    if constexpr (kWrite) {
      if (coded || dry_)
        for (int k = 0; k < nn; ++k) nz |= lv[k] != 0;
    } else {
      nz = nnz > 0;
    }
    if (GpuPicture* g = g_) {  // records mode: the GPU predicts / transforms / adds
      if (nz) cbf_nonzero_ = true;
      if (!nz && !cu_.intra) return;
      GpuTu t{};
      t.x = u16(x0);
      t.y = u16(y0);
      t.log2 = u8(log2);
      t.c = u8(c);
      if (cu_.intra) {
        t.flags |= kTuIntra;
        t.mode = u8(c == 0 ? block_luma_mode_ : cu_.ipmc);
        t.avail = gpu_avail_;
        t.pend = gpu_pend_;
        t.level = u16(gpu_level_);
        if (sps_.strong_intra_smoothing) t.flags |= kTuStrong;
        if (c == 0 && log2 == 2) t.flags |= kTuDst;
        // the block's samples are level `gpu_level_` output from here on
        const int sub = c ? 1 : 0;
        std::vector<u16>& lvl = c ? pc_.lvl_c : pc_.lvl_y;
        for4(x0 << sub, y0 << sub, n << sub, n << sub, [&](size_t k) { lvl[k] = u16(gpu_level_); });
      }
      if (tskip) t.flags |= kTuSkip;
      if (cu_.bypass) t.flags |= kTuBypass;
      if (nz) {  // sparse: mask words + the non-zero levels' dequantised values (hk_sparse_store)
        t.flags |= kTuCoef;
        t.data = u32(g->coefs.size());
        int ex = 0, ey = 0;
        const u8* m = scale_matrix(c, log2);
        const bool byp = cu_.bypass;
        int np = 0;
        auto put = [&](int k) {
          nzpos_[np] = u16(k);
          nzval_[np++] =
              byp ? i16(std::clamp(lv[k], -32768, 32767)) : i16(dequant_level(lv[k], qp, log2, m ? m[k] : 16, bd));
          ex = std::max(ex, k & (n - 1));
          ey = std::max(ey, k >> log2);
        };
        if constexpr (kWrite) {
          for (int k = 0; k < nn; ++k)
            if (lv[k]) put(k);
        } else {
          for (int j = 0; j < nnz; ++j) put(nzbuf_[j]);
        }
        const size_t off = g->coefs.size();
        g->coefs.resize(off + size_t(hk_sparse_words(log2) + np));
        hk_sparse_store(log2, nzpos_, nzval_, np, g->coefs.data() + off);
        t.ext_x = u8(ex);
        t.ext_y = u8(ey);
      }
      g->tus.push_back(t);
      return;
    }
    if (!nz) return;
    cbf_nonzero_ = true;
    std::vector<i32> d(size_t(n) * n), r(size_t(n) * n);
    if (cu_.bypass) {  // §8.6.2: the residual is the coded levels themselves
      for (size_t k = 0; k < d.size(); ++k) r[k] = lv[k];
    } else {
      const u8* m = scale_matrix(c, log2);
      for (size_t k = 0; k < d.size(); ++k) d[k] = lv[k] ? dequant_level(lv[k], qp, log2, m ? m[k] : 16, bd) : 0;
      inverse_transform(d.data(), log2, c == 0 && log2 == 2 && cu_.intra, tskip, r.data(), bd);
    }
    const int hi = (1 << bd) - 1;
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i) s.set(c, x0 + i, y0 + j, std::clamp(s.get(c, x0 + i, y0 + j) + r[size_t(j) * n + i], 0, hi));
  }

  // ScalingFactor of the block (raster n x n) or null when scaling lists are off (m = 16)
  const u8* scale_matrix(int c, int log2) const {
    if (!pc_.scaling) return nullptr;
    return pc_.sf[log2 - 2][(cu_.intra ? 0 : 3) + c].data();
  }

  // scan position k of a 4x4 sub-block / the sub-block grid
  static void scan_pos(int scan, int log2sb, int k, int& x, int& y) {
    if (scan == 0) {
      const int p = kScanDiag.s[log2sb][k];
      x = p & 7, y = p >> 3;
    } else if (scan == 1) {  // horizontal: row by row
      x = k & ((1 << log2sb) - 1), y = k >> log2sb;
    } else {                 // vertical: column by column
      y = k & ((1 << log2sb) - 1), x = k >> log2sb;
    }
  }

  // Sign data hiding in write mode: make each hiding sub-block's level parity carry the sign of
  // its first coefficient (the decoder infers it), by moving one magnitude by 1.
  void hide_signs(int* lv, int log2, int scan) {
    const int n = 1 << log2, nsb = log2 - 2;
    for (int i = 0; i < (1 << (2 * nsb)); ++i) {
      int xs, ys;
      scan_pos(scan, nsb, i, xs, ys);
      int first = -1, last = -1, sum = 0;
      for (int k = 0; k < 16; ++k) {
        const int p = kScan4.s[scan][k];
        const int v = lv[((ys << 2) + (p >> 2)) * n + (xs << 2) + (p & 3)];
        if (v) {
          if (first < 0) first = k;
          last = k;
          sum += std::abs(v);
        }
      }
      if (first < 0 || last - first <= 3) continue;
      const int pf = kScan4.s[scan][first];
      int& vf = lv[((ys << 2) + (pf >> 2)) * n + (xs << 2) + (pf & 3)];
      const bool neg = vf < 0;
      if ((sum & 1) != int(neg)) vf += vf > 0 ? 1 : -1;  // flips the parity, keeps the sign
    }
  }

  void residual_coding(int c, int log2, int* lv, bool& tskip) {
    const int n = 1 << log2;
    if (pps_.transform_skip && log2 == 2 && !cu_.bypass) tskip = bin(kCtxTransformSkip + (c ? 1 : 0), tskip) != 0;
    const int scan = scan_idx(c, log2);
    const int nsb = log2 - 2;
    // last significant position (write: the last non-zero level in scan order)
    int last_sb = 0, last_pos = 0, lx = 0, ly = 0;
    if constexpr (kWrite) {
      for (int i = (1 << (2 * nsb)) - 1; i >= 0 && !(lx | ly | last_sb | last_pos); --i) {
        int xs, ys;
        scan_pos(scan, nsb, i, xs, ys);
        for (int k = 15; k >= 0; --k) {
          const int p = kScan4.s[scan][k];
          const int x = (xs << 2) + (p & 3), y = (ys << 2) + (p >> 2);
          if (lv[y * n + x]) {
            last_sb = i, last_pos = k, lx = x, ly = y;
            goto found;
          }
        }
      }
    found:;
    }
    // last_sig_coeff_{x,y}_{prefix,suffix}; vertical scan codes the swapped coordinates
    int cx = lx, cy = ly;
    if (scan == 2) std::swap(cx, cy);
    const int off = c ? 15 : 3 * (log2 - 2) + ((log2 - 1) >> 2), shift = c ? log2 - 2 : (log2 + 1) >> 2;
    const int cmax = (log2 << 1) - 1;
    auto prefix_of = [](int v) {
      if (v < 4) return v;
      int k = 31 - __builtin_clz(u32(v));  // v in [2^k, 2^(k+1))
      return 2 * k + ((v >> (k - 1)) & 1);
    };
    int pre[2] = {prefix_of(cx), prefix_of(cy)};
    for (int a = 0; a < 2; ++a) {
      const int base = a == 0 ? kCtxLastX : kCtxLastY;
      int v = 0;
      while (v < cmax && bin(base + off + (v >> shift), pre[a] > v)) ++v;
      pre[a] = v;
    }
    int pos[2] = {pre[0], pre[1]};
    const int want[2] = {cx, cy};
    for (int a = 0; a < 2; ++a)
      if (pre[a] > 3) {
        const int nb = (pre[a] >> 1) - 1;
        const int base = (1 << nb) * (2 + (pre[a] & 1));
        pos[a] = base + int(fl(nb, u32(want[a] - base)));
      }
    if (scan == 2) std::swap(pos[0], pos[1]);
    lx = pos[0], ly = pos[1];
    VEP_CHECK(lx < n && ly < n, "last significant coefficient outside the block");
    if constexpr (!kWrite) {  // locate the last sub-block / position in scan order
      bool ok = false;
      for (int i = (1 << (2 * nsb)) - 1; i >= 0 && !ok; --i) {
        int xs, ys;
        scan_pos(scan, nsb, i, xs, ys);
        if (xs != (lx >> 2) || ys != (ly >> 2)) continue;
        for (int k = 15; k >= 0; --k) {
          const int p = kScan4.s[scan][k];
          if ((xs << 2) + (p & 3) == lx && (ys << 2) + (p >> 2) == ly) {
            last_sb = i, last_pos = k, ok = true;
            break;
          }
        }
      }
      std::fill(lv, lv + n * n, 0);
    }
    u8 csbf[8][8] = {};
    int greater1_ctx = 1;  // c1 carried between sub-blocks
    bool first_sb = true;
    for (int i = last_sb; i >= 0; --i) {
      int xs, ys;
      scan_pos(scan, nsb, i, xs, ys);
      auto at = [&](int k) -> int& {
        const int p = kScan4.s[scan][k];
        return lv[((ys << 2) + (p >> 2)) * n + (xs << 2) + (p & 3)];
      };
      bool infer_dc = false;
      bool sb_coded = true;
      if (i < last_sb && i > 0) {
        const int right = xs + 1 < (1 << nsb) ? csbf[xs + 1][ys] : 0;
        const int below = ys + 1 < (1 << nsb) ? csbf[xs][ys + 1] : 0;
        const int inc = std::min(right + below, 1) + (c ? 2 : 0);
        bool w = false;
        if constexpr (kWrite)
          for (int k = 0; k < 16; ++k) w |= at(k) != 0;
        sb_coded = bin(kCtxCsbf + inc, w) != 0;
        infer_dc = true;
      }
      csbf[xs][ys] = u8(sb_coded);
      bool sig[16] = {};
      if (i == last_sb) sig[last_pos] = true;
      const int start = i == last_sb ? last_pos - 1 : 15;
      const int prev_csbf = (xs + 1 < (1 << nsb) ? csbf[xs + 1][ys] : 0) | ((ys + 1 < (1 << nsb) ? csbf[xs][ys + 1] : 0) << 1);
      for (int k = start; k >= 0; --k) {
        if (!sb_coded) break;
        const int p = kScan4.s[scan][k];
        const int xc = (xs << 2) + (p & 3), yc = (ys << 2) + (p >> 2);
        if (k > 0 || !infer_dc) {
          const bool w = kWrite && at(k) != 0;
          sig[k] = bin(kCtxSig + sig_ctx(c, log2, scan, xc, yc, xs, ys, prev_csbf), w) != 0;
          if (sig[k]) infer_dc = false;
        } else {
          sig[k] = true;  // DC of a coded sub-block with no other significant coefficient
        }
      }
      if (!sb_coded) continue;
      // levels: greater1 (first 8), greater2 (first greater1), signs, remaining
      int first_sig = 16, last_sig = -1, ngt1 = 0, last_gt1 = -1;
      bool gt1[16] = {}, gt2[16] = {};
      int ctx_set = (i == 0 || c > 0) ? 0 : 2;
      if (!first_sb && greater1_ctx == 0) ++ctx_set;
      first_sb = false;
      greater1_ctx = 1;
      for (int k = 15; k >= 0; --k) {
        if (!sig[k]) continue;
        if (ngt1 < 8) {
          const int inc = ctx_set * 4 + greater1_ctx + (c ? 16 : 0);
          gt1[k] = bin(kCtxGt1 + inc, kWrite && std::abs(at(k)) > 1) != 0;
          ++ngt1;
          if (gt1[k]) {
            greater1_ctx = 0;
            if (last_gt1 < 0) last_gt1 = k;
          } else if (greater1_ctx > 0 && greater1_ctx < 3) {
            ++greater1_ctx;
          }
        }
        if (last_sig < 0) last_sig = k;
        first_sig = k;
      }
      const bool hidden = pps_.sign_data_hiding && !cu_.bypass && last_sig - first_sig > 3;
      if (last_gt1 >= 0)
        gt2[last_gt1] = bin(kCtxGt2 + ctx_set + (c ? 4 : 0), kWrite && std::abs(at(last_gt1)) > 2) != 0;
      bool neg[16] = {};
      for (int k = 15; k >= 0; --k)
        if (sig[k] && (!hidden || k != first_sig)) neg[k] = byp(kWrite && at(k) < 0) != 0;
      int nsig = 0, sum = 0, rice = 0;
      for (int k = 15; k >= 0; --k) {
        if (!sig[k]) continue;
        const int base = 1 + gt1[k] + gt2[k];
        int absv = base;
        if (base == ((nsig < 8) ? ((k == last_gt1) ? 3 : 2) : 1)) {
          const int rem = coeff_remaining(rice, kWrite ? std::abs(at(k)) - base : 0);
          absv = base + rem;
          if (absv > 3 * (1 << rice)) rice = std::min(rice + 1, 4);
        }
        int v = neg[k] ? -absv : absv;
        sum += absv;
        if (hidden && k == first_sig && (sum & 1)) v = -v;
        if constexpr (!kWrite) at(k) = v;
        ++nsig;
      }
      if constexpr (kWrite) {  // hidden sign: the written parity must reproduce the level's sign
        if (hidden) {
          const int v = at(first_sig);
          VEP_CHECK((v < 0) == bool(sum & 1), "sign hiding parity not prepared");
        }
      }
    }
  }

  // Decoder direction of residual_coding (the parse hot spot of coded pictures): the same bins
  // and context selection as the generic body above, with the arithmetic decoder held in a local
  // copy (registers across the context updates, see cabac.h), the significance context of a
  // position from per-sub-block tables, and the non-zero levels listed (raster positions in
  // `nzp`) so the caller never scans the whole block. Returns the number of non-zero levels.
  int residual_coding_rd(int c, int log2, int* lv, bool& tskip, u16* nzp) {
    // sigCtx patterns by coded_sub_block_flag of the right / lower sub-blocks (prev_csbf) at
    // position p = x | y << 2 inside a sub-block, and the 4x4-TU map (§9.3.4.2.5)
    static constexpr u8 kPat[4][16] = {{2, 1, 1, 0, 1, 1, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0},
                                       {2, 2, 2, 2, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0},
                                       {2, 1, 0, 0, 2, 1, 0, 0, 2, 1, 0, 0, 2, 1, 0, 0},
                                       {2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2}};
    static constexpr u8 kMap4[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
    cabac::Ctx* const ctx = e_.c;
    cabac::Decoder d = e_.d;
    auto bits = [&d](int nb) {  // fixed length, bypass, MSB first
      u32 r = 0;
      for (int i = nb - 1; i >= 0; --i) r |= d.bypass() << i;
      return int(r);
    };
    const int n = 1 << log2;
    tskip = false;
    if (pps_.transform_skip && log2 == 2 && !cu_.bypass) tskip = d.decision(ctx[kCtxTransformSkip + (c ? 1 : 0)]) != 0;
    const int scan = scan_idx(c, log2);
    const int nsb = log2 - 2;
    const int off = c ? 15 : 3 * (log2 - 2) + ((log2 - 1) >> 2), shift = c ? log2 - 2 : (log2 + 1) >> 2;
    const int cmax = (log2 << 1) - 1;
    int pre[2], pos[2];
    for (int a = 0; a < 2; ++a) {  // both prefixes, then both suffixes
      cabac::Ctx* const base = ctx + (a == 0 ? kCtxLastX : kCtxLastY) + off;
      int v = 0;
      while (v < cmax && d.decision(base[v >> shift])) ++v;
      pre[a] = pos[a] = v;
    }
    for (int a = 0; a < 2; ++a)
      if (pre[a] > 3) {
        const int nb = (pre[a] >> 1) - 1;
        pos[a] = (1 << nb) * (2 + (pre[a] & 1)) + bits(nb);
      }
    if (scan == 2) std::swap(pos[0], pos[1]);
    const int lx = pos[0], ly = pos[1];
    VEP_CHECK(lx < n && ly < n, "last significant coefficient outside the block");
    // the sub-block and position of the last coefficient, by the inverse scans
    const int xs0 = lx >> 2, ys0 = ly >> 2;
    const int last_sb = scan == 0 ? kScanDiagInv.s[nsb][xs0 | ys0 << 3] : (scan == 1 ? (ys0 << nsb | xs0) : (xs0 << nsb | ys0));
    const int last_pos = kScan4Inv.s[scan][(lx & 3) | ((ly & 3) << 2)];
    // (lv arrives all zeros: the caller's invariant; only the non-zero levels are written)
    const u8* const sc4 = kScan4.s[scan];
    const int cofs = c ? 27 : 0;
    u8 csbf[8][8] = {};
    int greater1_ctx = 1;  // c1 carried between sub-blocks
    bool first_sb = true;
    int nnz = 0;
    for (int i = last_sb; i >= 0; --i) {
      int xs, ys;
      scan_pos(scan, nsb, i, xs, ys);
      const int right = xs + 1 < (1 << nsb) ? csbf[xs + 1][ys] : 0;
      const int below = ys + 1 < (1 << nsb) ? csbf[xs][ys + 1] : 0;
      bool infer_dc = false, sb_coded = true;
      if (i < last_sb && i > 0) {
        sb_coded = d.decision(ctx[kCtxCsbf + std::min(right + below, 1) + (c ? 2 : 0)]) != 0;
        infer_dc = true;
      }
      csbf[xs][ys] = u8(sb_coded);
      if (!sb_coded) continue;
      // significance: ctxInc = sig_off + pattern[p] (the DC of a larger TU: cofs; 4x4 TU: map)
      const u8* pat = log2 == 2 ? kMap4 : kPat[right | (below << 1)];
      const int sig_off = log2 == 2 ? cofs
                          : cofs + (c == 0 ? ((xs | ys) ? 3 : 0) + (log2 == 3 ? (scan == 0 ? 9 : 15) : 21)
                                           : (log2 == 3 ? 9 : 12));
      cabac::Ctx* const sigc = ctx + kCtxSig + sig_off;
      const bool dc_sb = log2 > 2 && i == 0;
      u32 sig = i == last_sb ? 1u << last_pos : 0u;
      for (int k = i == last_sb ? last_pos - 1 : 15; k >= 0; --k) {
        if (k > 0 || !infer_dc) {
          const int p = sc4[k];
          cabac::Ctx& cx = (dc_sb && p == 0) ? ctx[kCtxSig + cofs] : sigc[pat[p]];
          if (d.decision(cx)) {
            sig |= 1u << k;
            infer_dc = false;
          }
        } else {
          sig |= 1u;  // DC of a coded sub-block with no other significant coefficient
        }
      }
      // levels: greater1 (first 8), greater2 (first greater1), signs, remaining
      int ctx_set = (i == 0 || c > 0) ? 0 : 2;
      if (!first_sb && greater1_ctx == 0) ++ctx_set;
      first_sb = false;
      greater1_ctx = 1;
      if (!sig) continue;  // (the DC sub-block of a larger TU may have no significant level)
      cabac::Ctx* const g1c = ctx + kCtxGt1 + ctx_set * 4 + (c ? 16 : 0);
      u32 gt1 = 0;
      int ngt1 = 0, last_gt1 = -1;
      const int last_sig = 31 - __builtin_clz(sig), first_sig = __builtin_ctz(sig);
      for (u32 w = sig; w && ngt1 < 8; ++ngt1) {
        const int k = 31 - __builtin_clz(w);
        w &= ~(1u << k);
        if (d.decision(g1c[greater1_ctx])) {
          gt1 |= 1u << k;
          greater1_ctx = 0;
          if (last_gt1 < 0) last_gt1 = k;
        } else if (greater1_ctx > 0 && greater1_ctx < 3) {
          ++greater1_ctx;
        }
      }
      const bool hidden = pps_.sign_data_hiding && !cu_.bypass && last_sig - first_sig > 3;
      const bool gt2 = last_gt1 >= 0 && d.decision(ctx[kCtxGt2 + ctx_set + (c ? 4 : 0)]);
      u32 neg = 0;
      for (u32 w = sig; w;) {
        const int k = 31 - __builtin_clz(w);
        w &= ~(1u << k);
        if ((!hidden || k != first_sig) && d.bypass()) neg |= 1u << k;
      }
      int nsig = 0, sum = 0, rice = 0;
      for (u32 w = sig; w; ++nsig) {
        const int k = 31 - __builtin_clz(w);
        w &= ~(1u << k);
        const int base = 1 + int((gt1 >> k) & 1) + (gt2 && k == last_gt1 ? 1 : 0);
        int absv = base;
        if (base == ((nsig < 8) ? ((k == last_gt1) ? 3 : 2) : 1)) {  // coeff_abs_level_remaining
          int prefix = 0;
          while (d.bypass()) {
            ++prefix;
            VEP_CHECK(prefix < 32, "coeff_abs_level_remaining prefix too long");
          }
          const int rem = prefix < 3 ? (prefix << rice) + bits(rice)
                                     : (((1 << (prefix - 3)) + 2) << rice) + bits(prefix - 3 + rice);
          absv = base + rem;
          if (absv > 3 * (1 << rice)) rice = std::min(rice + 1, 4);
        }
        int v = (neg >> k) & 1 ? -absv : absv;
        sum += absv;
        if (hidden && k == first_sig && (sum & 1)) v = -v;
        const int p = sc4[k];
        const int r = ((ys << 2) + (p >> 2)) * n + (xs << 2) + (p & 3);
        lv[r] = v;
        nzp[nnz++] = u16(r);
      }
    }
    e_.d = d;
    return nnz;
  }

  int coeff_remaining(int rice, int v) {  // §9.3.3.11 (prefix threshold 3, suffix EG(rice + 1))
    int prefix = 0;
    if constexpr (kWrite) {
      const int q = v >> rice;
      const int pf = q < 3 ? q : 3 + (31 - __builtin_clz(u32(((v - (3 << rice)) >> rice) + 1)));
      for (int k = 0; k < pf; ++k) byp(1);
      byp(0);
      if (pf < 3) {
        fl(rice, u32(v - (pf << rice)));
      } else {
        const int nb = pf - 3 + rice;
        fl(nb, u32(v - (((1 << (pf - 3)) + 2) << rice)));
      }
      return v;
    } else {
      while (byp(0)) {
        ++prefix;
        VEP_CHECK(prefix < 32, "coeff_abs_level_remaining prefix too long");
      }
      if (prefix < 3) return (prefix << rice) + int(fl(rice, 0));
      const int nb = prefix - 3 + rice;
      return (((1 << (prefix - 3)) + 2) << rice) + int(fl(nb, 0));
    }
  }

  int sig_ctx(int c, int log2, int scan, int xc, int yc, int xs, int ys, int prev_csbf) const {
    int sig;
    if (log2 == 2) {
      static constexpr u8 kMap[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
      sig = kMap[(yc << 2) + xc];
    } else if (xc + yc == 0) {
      sig = 0;
    } else {
      const int xp = xc & 3, yp = yc & 3;
      if (prev_csbf == 0) sig = (xp + yp == 0) ? 2 : (xp + yp < 3) ? 1 : 0;
      else if (prev_csbf == 1) sig = (yp == 0) ? 2 : (yp == 1) ? 1 : 0;
      else if (prev_csbf == 2) sig = (xp == 0) ? 2 : (xp == 1) ? 1 : 0;
      else sig = 2;
      if (c == 0) {
        if (xs > 0 || ys > 0) sig += 3;
        sig += log2 == 3 ? (scan == 0 ? 9 : 15) : 21;
      } else {
        sig += log2 == 3 ? 9 : 12;
      }
    }
    return c == 0 ? sig : 27 + sig;
  }

  struct CuState {
    int x0 = 0, y0 = 0, log2 = 3;
    bool intra = false, merge0 = false, bypass = false;
    int part = 0;
    int ipm[4] = {1, 1, 1, 1}, ipmc = 1;
    int npu = 0;
    int pus[4][4] = {};
    int max_trafo_depth = 0, tu_target = 5;
  };

  PicCtx& pc_;
  int si_;
  SliceInfo& sl_;
  const SliceHeader& sh_;
  const Sps& sps_;
  const Pps& pps_;
  E& e_;
  CtuDecider* dec_;
  CuState cu_;
  int slice_qp_ = 26, qp_last_ = 26, qp_prev_ = 26, qp_pred_ = 26, cu_qp_delta_ = 0;
  int qg_x_ = 0, qg_y_ = 0, log2_min_qg_ = 6;
  bool qg_coded_ = false, first_qg_ = true;
  bool last_read_ = false;
  bool dry_ = false;
  int dry_qp_delta_ = 0;
  bool dry_tskip_ = false;
  u16 nzbuf_[1024];  // read mode: raster positions of a block's non-zero levels
  u16 nzpos_[1024];  // the block's stored coefficients (raster positions, dequantised values)
  i16 nzval_[1024];
  bool cbf_nonzero_ = false;
  int block_luma_mode_ = 1;
  u64 gpu_avail_ = 0;
  u64 gpu_pend_ = 0;  // reference units the GPU reads from the intra blocks' edge exchange
  std::vector<int> lvbuf_;  // one transform block's levels
  bool lv_dirty_ = true;    // (read mode) lvbuf_ may hold non-zero levels
  int gpu_level_ = 1;
  std::map<TuKey, TuLevels> levels_;
  GpuPicture* g_;         // records (the picture's, or the slice shard's)
  Decoder::Stats* st_;
  bool* bypass_;
};

void init_ctx(cabac::Ctx* ctx, const SliceHeader& sh, int qp) {
  int type = 0;
  if (sh.slice_type == kP) type = sh.cabac_init ? 2 : 1;
  else if (sh.slice_type == kB) type = sh.cabac_init ? 1 : 2;
  for (int i = 0; i < kCtxCount; ++i) ctx[i].init(kCtxInit[type][i], qp);
}

// Context variables at the start of the CTU at `rs` (§9.3.1, §9.3.2.1): initialised at a tile
// start; WPP rows synchronise from the storage after the 2nd CTB of the row above when its
// top-right CTB is available; a dependent slice segment continues from the previous segment.
// The qPY_PREV reset (§8.6.1) follows the same boundaries.
template <class L>
void start_ctu_state(PicCtx& pc, const SliceInfo& sl, cabac::Ctx* ctx, L& layer, int rs, bool segment_start) {
  const bool wpp = pc.pps->entropy_coding_sync;
  if (pc.first_ctb_in_tile(rs)) {
    init_ctx(ctx, sl.sh, sl.qp);
    layer.reset_qp_prediction();
    return;
  }
  if (wpp && pc.ctb_row_start(rs)) {
    const int rx = rs % pc.wctb, ry = rs / pc.wctb;
    const int tr = rs - pc.wctb + 1;
    const bool avail = ry > 0 && rx + 1 < pc.wctb && pc.slice[size_t(tr)] != 0xFFFF &&
                       pc.sord[size_t(tr)] == sl.ord && pc.tile[size_t(tr)] == pc.tile[size_t(rs)];
    if (avail && pc.wpp_sync) {  // rows in parallel: the row above's storage, once it exists
      pc.wpp_sync->wait(tr);
      const cabac::Ctx* src = pc.wpp_sync->rows.data() + size_t(ry - 1) * kCtxCount;
      std::copy(src, src + kCtxCount, ctx);
    } else if (avail) {
      std::copy(pc.wpp_ctx, pc.wpp_ctx + kCtxCount, ctx);
    }
    else init_ctx(ctx, sl.sh, sl.qp);
    layer.reset_qp_prediction();
    return;
  }
  if (segment_start && sl.sh.dependent) {
    std::copy(pc.ds_ctx, pc.ds_ctx + kCtxCount, ctx);
    layer.continue_qp_prediction(pc.ds_qp);
    return;
  }
  if (segment_start) init_ctx(ctx, sl.sh, sl.qp);
}

// After the CTU at `rs`: WPP storage and the end-of-segment storage (dependent segments).
template <class L>
void end_ctu_state(PicCtx& pc, const cabac::Ctx* ctx, const L& layer, int rs, bool segment_end) {
  if (pc.pps->entropy_coding_sync && rs % pc.wctb == pc.tile_col_start(rs % pc.wctb) + 1)
    std::copy(ctx, ctx + kCtxCount,
              pc.wpp_sync ? pc.wpp_sync->rows.data() + size_t(rs / pc.wctb) * kCtxCount : pc.wpp_ctx);
  if (segment_end && pc.pps->dependent_slice_segments) {
    std::copy(ctx, ctx + kCtxCount, pc.ds_ctx);
    pc.ds_qp = layer.qp_last();
  }
}

// The next CTU starts a new substream (new tile, or new CTB row of a tile with WPP).
bool substream_boundary(const PicCtx& pc, int rs, int next_rs) {
  return (pc.pps->tiles && pc.tile[size_t(next_rs)] != pc.tile[size_t(rs)]) ||
         (pc.pps->entropy_coding_sync && pc.ctb_row_start(next_rs));
}

}  // namespace

int decode_slice_data(PicCtx& pc, int slice_idx, const u8* data, size_t n, size_t bytepos, SliceShard* shard) {
  SliceInfo& sl = pc.slices[size_t(slice_idx)];
  cabac::Ctx ctx[kCtxCount];
  cabac::Decoder dec(data, n, bytepos);
  RD e{dec, ctx};
  CtuLayer<RD> L(pc, slice_idx, e, nullptr);
  if (shard) L.use_shard(*shard);
  L.rd = &dec;
  L.data = data;
  L.data_n = n;
  const int total = pc.wctb * pc.hctb;
  int ts = pc.rs2ts[size_t(sl.sh.segment_address)];
  int ctus = 0;
  start_ctu_state(pc, sl, ctx, L, sl.sh.segment_address, true);
  for (;;) {
    const int rs = pc.ts2rs[size_t(ts)];
    // (prefilled: the CTU must lie in this segment's range, filled in before the slices ran)
    VEP_CHECK(pc.prefilled ? pc.slice[size_t(rs)] == u16(slice_idx) : pc.slice[size_t(rs)] == 0xFFFF,
              "HEVC: CTU decoded twice");
    L.ctu(rs, false);
    ++ctus;
    const bool end = L.end_of_slice();
    end_ctu_state(pc, ctx, L, rs, end);
    if (end) break;
    VEP_CHECK(dec.bitpos() <= n * 8 + 16, "slice data overrun");
    ++ts;
    VEP_CHECK(ts < total, "slice data past the last CTU");
    const int next = pc.ts2rs[size_t(ts)];
    if (substream_boundary(pc, rs, next)) {
      VEP_CHECK(dec.terminate() == 1, "HEVC: end_of_subset_one_bit must be 1");
      dec.start(dec.aligned_bytepos());  // byte_alignment(), then a new arithmetic decoder
      start_ctu_state(pc, sl, ctx, L, next, false);
    }
  }
  if (shard) shard->ctus = ctus;
  cabac::bins_decoded().fetch_add(dec.bins(), std::memory_order_relaxed);
  return ctus;
}

void WppSync::wait(int rs) const {
  for (u32 spin = 0; !done[size_t(rs)].load(std::memory_order_acquire); ++spin) {
    if (abort.load(std::memory_order_relaxed)) throw Error("HEVC: a wavefront row failed");
    if (spin > 64) std::this_thread::yield();
  }
}

int decode_substream(PicCtx& pc, int slice_idx, const u8* data, size_t n, size_t bytepos, int first_ts, int end_ts,
                     bool last, SliceShard* shard) {
  SliceInfo& sl = pc.slices[size_t(slice_idx)];
  VEP_CHECK(pc.prefilled && first_ts < end_ts && bytepos < n, "HEVC: bad substream");
  cabac::Ctx ctx[kCtxCount];
  cabac::Decoder dec(data, n, bytepos);
  RD e{dec, ctx};
  CtuLayer<RD> L(pc, slice_idx, e, nullptr);
  if (shard) L.use_shard(*shard);
  L.rd = &dec;
  L.data = data;
  L.data_n = n;
  const int first_rs = pc.ts2rs[size_t(first_ts)];
  // the segment's first substream starts with the segment's state; a later one is a tile start
  start_ctu_state(pc, sl, ctx, L, first_rs, first_rs == sl.sh.segment_address);
  int ctus = 0;
  WppSync* ws = pc.wpp_sync;
  for (int ts = first_ts; ts < end_ts; ++ts) {
    const int rs = pc.ts2rs[size_t(ts)];
    VEP_CHECK(pc.slice[size_t(rs)] == u16(slice_idx), "HEVC: CTU outside the substream's slice");
    if (ws && rs >= pc.wctb) {  // wavefront: the CTBs above-left, above and above-right it may read
      const int rx = rs % pc.wctb;
      for (int dx = -1; dx <= 1; ++dx) {
        const int nx = rx + dx, nrs = rs - pc.wctb + dx;
        if (nx >= 0 && nx < pc.wctb && pc.sord[size_t(nrs)] == pc.sord[size_t(rs)]) ws->wait(nrs);
      }
    }
    L.ctu(rs, false);
    ++ctus;
    const bool end = L.end_of_slice();
    end_ctu_state(pc, ctx, L, rs, end);
    if (ws) ws->done[size_t(rs)].store(1, std::memory_order_release);
    VEP_CHECK(dec.bitpos() <= n * 8 + 16, "slice data overrun");
    if (ts + 1 == end_ts) {
      VEP_CHECK(end == last, last ? "HEVC: slice segment longer than its CTUs" : "HEVC: substream ends the slice early");
      if (!last) VEP_CHECK(dec.terminate() == 1, "HEVC: end_of_subset_one_bit must be 1");
    } else {
      VEP_CHECK(!end, "HEVC: slice segment ends inside a substream");
      VEP_CHECK(!substream_boundary(pc, rs, pc.ts2rs[size_t(ts) + 1]), "HEVC: substream spans a tile boundary");
    }
  }
  if (shard) shard->ctus = ctus;
  cabac::bins_decoded().fetch_add(dec.bins(), std::memory_order_relaxed);
  return ctus;
}

void encode_slice_data(PicCtx& pc, int slice_idx, std::vector<u8>& out, CtuDecider& dec, int first_ts, int end_ts,
                       std::vector<size_t>* substreams) {
  SliceInfo& sl = pc.slices[size_t(slice_idx)];
  cabac::Ctx ctx[kCtxCount];
  cabac::Encoder enc(out);
  WR e{enc, ctx};
  CtuLayer<WR> L(pc, slice_idx, e, &dec);
  L.wr = &enc;
  start_ctu_state(pc, sl, ctx, L, pc.ts2rs[size_t(first_ts)], true);
  for (int ts = first_ts; ts < end_ts; ++ts) {
    const int rs = pc.ts2rs[size_t(ts)];
    const bool last = ts + 1 == end_ts;
    L.ctu(rs, last);
    end_ctu_state(pc, ctx, L, rs, last);
    if (last) break;
    const int next = pc.ts2rs[size_t(ts) + 1];
    if (substream_boundary(pc, rs, next)) {
      enc.terminate(1);  // end_of_subset_one_bit
      enc.align_zero();  // byte_alignment() (the flush wrote its 1 bit)
      if (substreams) substreams->push_back(out.size());
      enc.start();
      start_ctu_state(pc, sl, ctx, L, next, false);
    }
  }
  enc.align_zero();
}

}  // namespace vep::hevc
