// Closed-loop synthetic H.264 Main / High-profile encoder: CABAC or CAVLC, I / P / B pictures
// with B-pyramids, 8x8 transform + Intra_8x8, spatial or temporal direct prediction, explicit
// and implicit weighted prediction, optional scaling matrices. See avc.h (AvcHighEncoder).
//
// Every macroblock goes through the decoder's own macroblock layer in write mode
// (SliceWriter, avc_mb.cpp): the syntax, its context selection, motion-vector prediction, direct
// derivation, dequantisation and the per-MB records are the decoder's code, and each MB is then
// reconstructed with the decoder's reconstruction (cpu_reconstruct_mb), so the encoder's
// reference pictures are by construction what a conforming decoder of the emitted stream
// reconstructs. Mode decision is SAD-driven with a motion search seeded by the scene's known
// object motion; `coverage` randomises every decision (all MB / sub-MB types, prediction
// modes, reference indices, motion phases, transform sizes, levels) for decoder coverage.
#include <cmath>
#include <deque>
#include <map>

#include "avc.h"
#include "avc_internal.h"
#include "avc_scene.h"
#include "h264.h"

namespace vep::avc {

namespace {

// Exact 1-D 8x8 inverse transform matrix (idct8_1d on unit vectors) and its inverse: the 8x8
// quantiser inverts the decoder's transform numerically, so levels reconstruct to the residual.
struct Idct8Inverse {
  double inv[8][8];
  Idct8Inverse() {
    double m[8][8];
    for (int k = 0; k < 8; ++k) {
      int x[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      x[k] = 1024;
      idct8_1d(x);
      for (int i = 0; i < 8; ++i) m[i][k] = x[i] / 1024.0;
    }
    double a[8][16];
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 16; ++j) a[i][j] = j < 8 ? m[i][j] : (j - 8 == i ? 1.0 : 0.0);
    for (int c = 0; c < 8; ++c) {
      int piv = c;
      for (int r = c + 1; r < 8; ++r)
        if (std::fabs(a[r][c]) > std::fabs(a[piv][c])) piv = r;
      for (int j = 0; j < 16; ++j) std::swap(a[c][j], a[piv][j]);
      const double d = a[c][c];
      for (int j = 0; j < 16; ++j) a[c][j] /= d;
      for (int r = 0; r < 8; ++r) {
        if (r == c) continue;
        const double f = a[r][c];
        for (int j = 0; j < 16; ++j) a[r][j] -= f * a[c][j];
      }
    }
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 8; ++j) inv[i][j] = a[i][8 + j];
  }
};
const Idct8Inverse kInv8;

// Levels (8x8 scan order) of residual x (raster 8x8) at qp with flat matrices.
void quant8x8(const int* x, int qp, bool intra, int* lv, const u8* scan = kZigzag8x8) {
  double t[64], d[64];
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) {
      double s = 0;
      for (int k = 0; k < 8; ++k) s += kInv8.inv[i][k] * x[k * 8 + j];
      t[i * 8 + j] = s;
    }
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) {
      double s = 0;
      for (int k = 0; k < 8; ++k) s += t[i * 8 + k] * kInv8.inv[j][k];
      d[i * 8 + j] = s * 64.0;  // coefficient d with r = (M d M^T) / 64
    }
  const double f = intra ? 1.0 / 3 : 1.0 / 6;
  for (int k = 0; k < 64; ++k) {
    const int pos = scan[k], i = pos >> 3, j = pos & 7;
    const double step = 16.0 * norm_adjust8(qp % 6, i, j) * std::ldexp(1.0, qp / 6) / 64.0;
    const double v = d[pos] / step;
    const int a = int(std::fabs(v) + f);
    lv[k] = v < 0 ? -std::min(a, 2047) : std::min(a, 2047);
  }
}

// Decoder-exact 8x8 dequantisation + inverse transform (flat matrices): residual samples.
void recon8x8(const int* lv, int qp, int* r, const u8* scan = kZigzag8x8) {
  i16 d[64] = {};
  for (int k = 0; k < 64; ++k) {
    if (!lv[k]) continue;
    const int pos = scan[k];
    const int ls = 16 * norm_adjust8(qp % 6, pos >> 3, pos & 7);
    const int v = qp >= 36 ? (lv[k] * ls) * (1 << (qp / 6 - 6)) : (lv[k] * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
    d[pos] = sat16(v);
  }
  idct8x8(d, r);
}

}  // namespace

struct AvcHighEncoder::Impl {
  AvcHighConfig cfg;
  Rng rng;
  Scene scene;
  h264::Sps sps;
  h264::Pps pps;
  std::vector<u8> sps_nal, pps_nal;
  int W = 0, H = 0, wpx = 0, hpx = 0, max_fn = 1 << 16;
  std::vector<HostSurface> slots;
  struct Ref {
    int slot, frame_num, poc;
    u32 uid;
    std::shared_ptr<const ColMotion> col;
    // field coding: the frame's reference fields (bit 0 top, bit 1 bottom), their POCs / uids
    u8 fields = 3;
    int poc_f[2] = {0, 0};
    u32 uid_f[2] = {0, 0};
    std::shared_ptr<const ColMotion> col_f[2];
    bool long_term = false;  // (frame pictures, cfg.marking)
    int lt_idx = 0;
    u8 lt_fields = 0;        // (field pictures: long-term fields; `fields` are the short-term ones)
  };
  int max_lt_idx = -1;  // MaxLongTermFrameIdx (-1: no long-term frame indices)
  std::vector<Ref> dpb;
  struct Job {
    i64 disp;
    int type;  // h264::kI / kP / kB
    bool ref;
    bool idr;
    int parity = -1;  // field coding: 0 top / 1 bottom field of the frame (-1: frame picture)
  };
  std::deque<Job> plan;
  std::map<i64, HostSurface> sources;
  i64 next_disp = 0, gop_start = 0, rendered = -1, coded = 0;
  int prev_ref_fn = 0, idr_id = -1;
  u32 next_uid = 1;
  Picture pic;
  MbNeighbours nb;
  HostSurface recon, src_out;
  i64 last_disp = 0, last_pts = 0;
  char last_type = 'I';
  const HostSurface* cur_src = nullptr;
  // field coding (cfg.fields): slots are fields (2 per frame), ph = field height in pixels
  bool fields = false;
  int ph = 0;
  HostSurface field_src;
  int pair_slot = -1, pair_fn = 0;
  int bd = 8, qpbd = 0;  // sample bit depth, QpBdOffset (High 10)
  int cf = 1;            // chroma format (2: 4:2:2)
  const u8* scan4 = kZigzag4x4;  // 4x4 level scan of the current picture (field pictures: field scan)
  const u8* scan8 = kZigzag8x8;

  explicit Impl(const AvcHighConfig& c) : cfg(c), rng{c.seed * 0x9E3779B97F4A7C15ull + 777} {
    VEP_CHECK(c.width >= 16 && c.height >= 16 && c.width % 2 == 0 && c.height % 2 == 0,
              "encoder size must be even and >= 16");
    VEP_CHECK(c.bframes >= 0 && c.bframes <= 4 && c.refs >= 1 && c.refs <= 8, "bframes 0..4, refs 1..8");
    VEP_CHECK(c.bit_depth >= 8 && c.bit_depth <= 10 && (c.bit_depth == 8 || !c.fields),
              "bit_depth 8..10 (High 10: frame pictures)");
    bd = c.bit_depth;
    qpbd = 6 * (bd - 8);
    VEP_CHECK(c.chroma_format == 1 || (c.chroma_format == 2 && !c.fields && !c.mono),
              "chroma_format 1 or 2 (4:2:2: frame pictures, not 4:0:0)");
    cf = c.chroma_format;
    VEP_CHECK(c.qp >= -qpbd && c.qp <= 51 && c.gop >= 1, "bad encoder config");
    VEP_CHECK(!c.fields || (c.interlaced && !c.cabac), "field coding: interlaced CAVLC only");
    fields = c.fields;
    W = (c.width + 15) / 16;
    H = (c.height + 15) / 16;
    if (c.interlaced) H = (H + 1) & ~1;  // (frame height in MB pairs: map units of 2 MB rows)
    wpx = W * 16;
    hpx = H * 16;
    sps.profile_idc = cf == 2 ? 122 : bd > 8 ? 110 : (c.t8x8 || c.scaling || c.mono) ? 100 : 77;
    sps.chroma_format_idc = c.mono ? 0 : cf;
    sps.bit_depth_luma = sps.bit_depth_chroma = bd;
    VEP_CHECK(!c.mono || (!c.weighted_p && c.weighted_b != 1), "4:0:0 encoder: explicit weighted prediction is not emitted");
    sps.constraint_flags = 0;
    sps.level_idc = W * H > 8192 ? 51 : 40;
    sps.log2_max_frame_num = 16;
    sps.poc_type = 0;
    sps.log2_max_poc_lsb = 16;
    const int pyr = c.pyramid && c.bframes >= 2 && !c.fields ? 1 : 0;  // (field pairs: B non-reference)
    sps.max_num_ref_frames = std::max(c.refs, c.bframes > 0 ? 2 : 1) + pyr;
    sps.width_mbs = W;
    sps.frame_mbs_only = !c.interlaced;
    sps.mbaff = false;
    sps.direct_8x8 = true;
    sps.height_map_units = c.interlaced ? H / 2 : H;
    sps.crop_right = wpx - c.width;
    sps.crop_bottom = hpx - c.height;
    sps.timing_info = true;
    sps.num_units_in_tick = 1;
    sps.time_scale = u32(2 * c.fps);
    sps.max_num_reorder_frames = c.bframes > 0 ? (pyr ? 2 : 1) : 0;
    sps.max_dec_frame_buffering = sps.max_num_ref_frames;
    sps.scaling_matrix_present = c.scaling;
    if (c.scaling) {  // non-flat matrices, coded explicitly: the defaults perturbed per entry
      for (int l = 0; l < 6; ++l)
        for (int k = 0; k < 16; ++k) sps.scaling.l4[l][k] = u8(h264::kDefault4x4[l >= 3][k] + rng.uni(9) - 4);
      for (int l = 0; l < 2; ++l)
        for (int k = 0; k < 64; ++k) sps.scaling.l8[l][k] = u8(h264::kDefault8x8[l][k] + rng.uni(9) - 4);
    } else {
      sps.scaling.flat();
    }
    pps.cabac = c.cabac;
    pps.bottom_field_pic_order = c.interlaced;
    pps.weighted_pred = c.weighted_p;
    pps.weighted_bipred_idc = c.weighted_b;
    pps.chroma_qp_index_offset = c.chroma_qp_offset;
    pps.second_chroma_qp_index_offset = c.second_chroma_qp_offset;
    pps.deblocking_filter_control = true;
    pps.transform_8x8_mode = c.t8x8;
    pps.scaling.flat();
    auto nal = [](const std::vector<u8>& rbsp, std::vector<u8>& out) { rbsp_to_ebsp(rbsp.data(), rbsp.size(), out); };
    nal(h264::write_sps(sps), sps_nal);
    nal(h264::write_pps(pps), pps_nal);
    ph = fields ? hpx / 2 : hpx;
    slots.resize((size_t(sps.max_num_ref_frames) + 2) * (fields ? 2 : 1));
    for (auto& s : slots) s.alloc(wpx, ph, bd, cf);
    scene.make(SceneConfig{c.width, c.height, wpx, hpx, c.objects, c.noise, c.temporal_noise, c.seed}, rng);
  }

  bool is_idr_pos(i64 d) const { return d == 0 || (d + cfg.idr_phase) % cfg.gop == 0; }

  const HostSurface& source_of(i64 d) {
    while (rendered < d) {
      ++rendered;
      if (rendered > 0) scene.advance();
      scene.render();
      scene.add_sensor_noise(rendered);
      if (bd > 8 || cf == 2) {
        // High 10 source: the 8-bit scene << 2 plus a position / time dither in the low bits;
        // 4:2:2: the scene's chroma rows interpolated to full height
        HostSurface& w = sources[rendered];
        const HostSurface& s8 = scene.src;
        w.alloc(s8.coded_w, s8.coded_h, bd, cf);
        const int sh = bd - 8;
        auto lo = [&](size_t i) {
          return sh ? int(u16((i * 2654435761u + u64(rendered) * 40503u) >> 29) & ((1u << sh) - 1)) : 0;
        };
        const size_t cw = size_t(s8.coded_w), crows = size_t(s8.coded_h / 2);
        for (size_t i = 0; i < size_t(s8.coded_w) * size_t(s8.coded_h); ++i) w.set(0, int(i % cw), int(i / cw), s8.y[i] << sh | lo(i));
        for (size_t r = 0; r < size_t(w.chroma_rows()); ++r)
          for (size_t x = 0; x < cw; ++x) {
            int v;
            if (cf == 2) {
              const size_t r0 = r >> 1, r1 = std::min(crows - 1, r0 + (r & 1));
              v = (s8.uv[r0 * cw + x] + s8.uv[r1 * cw + x] + 1) >> 1;
            } else {
              v = s8.uv[r * cw + x];
            }
            w.set(1 + int(x & 1), int(x >> 1), int(r), v << sh | lo(r * cw + x + 7));
          }
      } else {
        sources[rendered] = scene.src;
      }
    }
    return sources.at(d);
  }

  void plan_next() {
    if (fields) {  // every frame a field pair: I / P (IDR frames), P / P anchors, non-reference
                   // B / B pairs between them (coding order: the anchor pair, then the B pairs)
      if (is_idr_pos(next_disp)) {
        gop_start = next_disp;
        plan.push_back({next_disp, h264::kI, true, true, 0});
        plan.push_back({next_disp, h264::kP, true, false, 1});
        ++next_disp;
        return;
      }
      i64 next_idr = next_disp + 1;
      while (!is_idr_pos(next_idr)) ++next_idr;
      const i64 anchor = std::min<i64>(next_disp + cfg.bframes, next_idr - 1);
      plan.push_back({anchor, h264::kP, true, false, 0});
      plan.push_back({anchor, h264::kP, true, false, 1});
      for (i64 d = next_disp; d < anchor; ++d) {
        plan.push_back({d, h264::kB, false, false, 0});
        plan.push_back({d, h264::kB, false, false, 1});
      }
      next_disp = anchor + 1;
      return;
    }
    if (is_idr_pos(next_disp)) {
      plan.push_back({next_disp, h264::kI, true, true});
      gop_start = next_disp;
      ++next_disp;
      return;
    }
    i64 next_idr = next_disp + 1;
    while (!is_idr_pos(next_idr)) ++next_idr;
    const i64 anchor = std::min<i64>(next_disp + cfg.bframes, next_idr - 1);
    const int nb_ = int(anchor - next_disp);
    plan.push_back({anchor, h264::kP, true, false});
    const bool pyr = cfg.pyramid && nb_ >= 2;
    const i64 mid = next_disp + nb_ / 2;
    if (pyr) plan.push_back({mid, h264::kB, true, false});
    for (i64 d = next_disp; d < anchor; ++d)
      if (!(pyr && d == mid)) plan.push_back({d, h264::kB, false, false});
    next_disp = anchor + 1;
  }

  // ---------------------------------------------------------------- reference lists
  int wrap_of(const Ref& r, int frame_num) const { return r.frame_num > frame_num ? r.frame_num - max_fn : r.frame_num; }

  // Initial lists of a frame picture (§8.2.4.2.1 / §8.2.4.2.3): short-term (P: FrameNumWrap
  // descending; B: by POC around the current one), then long-term by LongTermFrameIdx.
  void init_lists(const SliceHdr& sh, int cur_poc, std::vector<const Ref*>* init) const {
    std::vector<const Ref*> st, lt;
    for (const Ref& r : dpb) (r.long_term ? lt : st).push_back(&r);
    std::sort(lt.begin(), lt.end(), [](const Ref* a, const Ref* b) { return a->lt_idx < b->lt_idx; });
    init[0].clear();
    init[1].clear();
    if (sh.type() == h264::kP) {
      std::sort(st.begin(), st.end(), [&](const Ref* a, const Ref* b) { return wrap_of(*a, sh.frame_num) > wrap_of(*b, sh.frame_num); });
      init[0] = st;
      init[0].insert(init[0].end(), lt.begin(), lt.end());
    } else if (sh.type() == h264::kB) {
      std::vector<const Ref*> before, after;
      for (const Ref* r : st) (r->poc < cur_poc ? before : after).push_back(r);
      std::sort(before.begin(), before.end(), [](const Ref* a, const Ref* b) { return a->poc > b->poc; });
      std::sort(after.begin(), after.end(), [](const Ref* a, const Ref* b) { return a->poc < b->poc; });
      init[0] = before;
      init[0].insert(init[0].end(), after.begin(), after.end());
      init[0].insert(init[0].end(), lt.begin(), lt.end());
      init[1] = after;
      init[1].insert(init[1].end(), before.begin(), before.end());
      init[1].insert(init[1].end(), lt.begin(), lt.end());
      if (init[1].size() > 1 && init[1] == init[0]) std::swap(init[1][0], init[1][1]);
    }
  }

  // ref_pic_list_modification (cfg.marking): up to two random pictures of the initial list moved
  // to the front, coded relative to picNumPred (short-term) or by LongTermPicNum.
  void choose_mods(SliceHdr& sh, int cur_poc) {
    std::vector<const Ref*> init[2];
    init_lists(sh, cur_poc, init);
    for (int l = 0; l < (sh.type() == h264::kB ? 2 : 1); ++l) {
      sh.ref_mods[l].clear();
      if (init[l].size() < 2 || rng.uni(100) >= 40) continue;
      int pred = sh.frame_num;  // picNumLXPred (CurrPicNum)
      const int n = 1 + rng.uni(2);
      const Ref* last = nullptr;
      for (int k = 0; k < n; ++k) {
        const Ref* r = init[l][size_t(rng.uni(int(init[l].size())))];
        if (r == last) continue;
        last = r;
        if (r->long_term) {
          sh.ref_mods[l].push_back({2, r->lt_idx});
          continue;
        }
        const int pic_num = wrap_of(*r, sh.frame_num);
        const int nowrap = pic_num < 0 ? pic_num + max_fn : pic_num;
        if (nowrap == pred) continue;  // (abs_diff_pic_num 0 is not codable)
        sh.ref_mods[l].push_back({nowrap < pred ? 0 : 1, std::abs(nowrap - pred) - 1});
        pred = nowrap;
      }
    }
  }

  // The modifications applied (§8.2.4.3): each named picture inserted at the next index, its
  // later occurrence removed.
  void apply_mods(const SliceHdr& sh, int l, std::vector<const Ref*>& list) const {
    int pred = sh.frame_num;
    size_t idx = 0;
    for (const auto& m : sh.ref_mods[l]) {
      const Ref* pick = nullptr;
      if (m.idc < 2) {
        int nw = m.idc == 0 ? pred - (m.val + 1) : pred + (m.val + 1);
        if (nw < 0) nw += max_fn;
        if (nw >= max_fn) nw -= max_fn;
        pred = nw;
        const int pic_num = nw > sh.frame_num ? nw - max_fn : nw;
        for (const Ref& r : dpb)
          if (!r.long_term && wrap_of(r, sh.frame_num) == pic_num) pick = &r;
      } else {
        for (const Ref& r : dpb)
          if (r.long_term && r.lt_idx == m.val) pick = &r;
      }
      VEP_CHECK(pick != nullptr, "encoder: list modification names a missing picture");
      list.insert(list.begin() + long(std::min(idx, list.size())), pick);
      for (size_t k = idx + 1; k < list.size(); ++k)
        if (list[k] == pick) {
          list.erase(list.begin() + long(k));
          break;
        }
      ++idx;
    }
  }

  void build_lists(const SliceHdr& sh, int cur_poc, std::vector<ListEntry>* lists) {
    std::vector<const Ref*> init[2];
    init_lists(sh, cur_poc, init);
    for (int l = 0; l < 2; ++l) {
      apply_mods(sh, l, init[l]);
      lists[l].clear();
      for (int i = 0; i < sh.num_ref_idx[l] && i < int(init[l].size()); ++i) {
        const Ref& r = *init[l][size_t(i)];
        lists[l].push_back(ListEntry{r.slot, r.poc, r.long_term, r.uid, r.col.get()});
      }
    }
  }

  // MMCOs of a reference frame picture (cfg.marking): a full DPB frees a frame (MMCO 1 or 2);
  // then at random MMCO 4 (MaxLongTermFrameIdx), 6 (this picture long-term), 3 (a short-term
  // picture long-term), 2 / 1 (a long-term / short-term picture unused). With B pictures the two
  // newest pictures (the anchors the next B pictures predict from) are left as they are.
  void choose_mmcos(SliceHdr& sh, bool anchor_with_bs) {
    sh.mmcos.clear();
    std::vector<const Ref*> all;
    for (const Ref& r : dpb) all.push_back(&r);
    std::sort(all.begin(), all.end(), [&](const Ref* a, const Ref* b) { return wrap_of(*a, sh.frame_num) < wrap_of(*b, sh.frame_num); });
    const size_t keep = std::min(all.size(), size_t(cfg.bframes > 0 ? 2 : 0));  // newest pictures kept
    int kept_lt = -1;  // highest LongTermFrameIdx among the kept pictures
    u32 kept_mask = 0;  // their indices (not reassigned: MMCO 3 / 6 would drop the kept picture)
    for (size_t k = all.size() - keep; k < all.size(); ++k)
      if (all[k]->long_term) {
        kept_lt = std::max(kept_lt, all[k]->lt_idx);
        kept_mask |= 1u << all[k]->lt_idx;
      }
    auto free_idx = [&](int max_idx) {  // a random LongTermFrameIdx <= max_idx not kept, or -1
      std::vector<int> c;
      for (int i = 0; i <= max_idx; ++i)
        if (!((kept_mask >> i) & 1)) c.push_back(i);
      return c.empty() ? -1 : c[size_t(rng.uni(int(c.size())))];
    };
    std::vector<const Ref*> lt, free_st;
    for (size_t k = 0; k + keep < all.size(); ++k) (all[k]->long_term ? lt : free_st).push_back(all[k]);
    auto op1 = [&](const Ref* r) { sh.mmcos.push_back({1, sh.frame_num - wrap_of(*r, sh.frame_num) - 1, 0}); };
    int n_frames = int(dpb.size());
    if (n_frames >= std::max(1, sps.max_num_ref_frames)) {  // room for this picture
      if (!free_st.empty()) {
        op1(free_st.front());
        free_st.erase(free_st.begin());
      } else if (!lt.empty()) {
        sh.mmcos.push_back({2, lt.front()->lt_idx, 0});
        lt.erase(lt.begin());
      } else {
        return;  // (sliding window instead)
      }
      --n_frames;
    }
    const int r = rng.uni(100);
    int max_lt = max_lt_idx;
    if (cfg.bframes == 0 && r >= 93) {  // MMCO 5 alone (POC and frame_num restart; no B pictures
      sh.mmcos.assign(1, {5, 0, 0});   // to reorder around it)
      sh.adaptive_marking = true;
      return;
    }
    if (r < 20) {
      max_lt = std::max(kept_lt, rng.uni(3) - 1);  // max_long_term_frame_idx_plus1 0..2
      sh.mmcos.push_back({4, max_lt + 1, 0});
      std::vector<const Ref*> kept;
      for (const Ref* x : lt)
        if (x->lt_idx <= max_lt) kept.push_back(x);
      lt = kept;
    } else if (r < 40 && free_idx(max_lt) >= 0 && !anchor_with_bs) {
      sh.mmcos.push_back({6, free_idx(max_lt), 0});
    } else if (r < 60 && free_idx(max_lt) >= 0 && !free_st.empty()) {
      const Ref* x = free_st[size_t(rng.uni(int(free_st.size())))];
      sh.mmcos.push_back({3, sh.frame_num - wrap_of(*x, sh.frame_num) - 1, free_idx(max_lt)});
    } else if (r < 75 && !lt.empty()) {
      sh.mmcos.push_back({2, lt[size_t(rng.uni(int(lt.size())))]->lt_idx, 0});
    } else if (r < 90 && !free_st.empty()) {
      op1(free_st[size_t(rng.uni(int(free_st.size())))]);
    }
    if (!sh.mmcos.empty()) sh.adaptive_marking = true;
  }

  // Marking of the current reference frame picture (the decoder's mark_references): MMCOs in
  // order, else the sliding window; returns the entry's long-term state.
  void mark_frame(const SliceHdr& sh, Ref cur) {
    auto erase_if = [&](auto pred) { dpb.erase(std::remove_if(dpb.begin(), dpb.end(), pred), dpb.end()); };
    if (sh.idr()) {
      dpb.clear();
      max_lt_idx = sh.long_term_reference ? 0 : -1;
      cur.long_term = sh.long_term_reference;
      cur.lt_idx = 0;
      dpb.push_back(cur);
      return;
    }
    if (sh.adaptive_marking) {
      for (const auto& m : sh.mmcos) {
        switch (m.op) {
          case 1: erase_if([&](const Ref& r) { return !r.long_term && wrap_of(r, sh.frame_num) == sh.frame_num - (m.a + 1); }); break;
          case 2: erase_if([&](const Ref& r) { return r.long_term && r.lt_idx == m.a; }); break;
          case 3:
            erase_if([&](const Ref& r) { return r.long_term && r.lt_idx == m.b; });
            for (Ref& r : dpb)
              if (!r.long_term && wrap_of(r, sh.frame_num) == sh.frame_num - (m.a + 1)) {
                r.long_term = true;
                r.lt_idx = m.b;
              }
            break;
          case 4:
            max_lt_idx = m.a - 1;
            erase_if([&](const Ref& r) { return r.long_term && r.lt_idx > max_lt_idx; });
            break;
          case 5:  // every reference unused; this picture becomes frame_num 0, POC 0
            dpb.clear();
            max_lt_idx = -1;
            cur.frame_num = 0;
            cur.poc = 0;
            break;
          case 6:
            erase_if([&](const Ref& r) { return r.long_term && r.lt_idx == m.a; });
            cur.long_term = true;
            cur.lt_idx = m.a;
            break;
          default: break;
        }
      }
    } else if (int(dpb.size()) >= std::max(1, sps.max_num_ref_frames)) {  // sliding window (§8.2.5.3)
      int n_short = 0;
      for (const Ref& r : dpb) n_short += !r.long_term;
      if (n_short > 0) {
        auto it = std::min_element(dpb.begin(), dpb.end(), [&](const Ref& a, const Ref& b) {
          if (a.long_term != b.long_term) return !a.long_term;
          return wrap_of(a, sh.frame_num) < wrap_of(b, sh.frame_num);
        });
        dpb.erase(it);
      }
    }
    dpb.push_back(cur);
    VEP_CHECK(int(dpb.size()) <= std::max(1, sps.max_num_ref_frames), "encoder: DPB overflow after marking");
  }

  // Field picture numbers (the decoder's field_pic_num / field_lt_pic_num, §8.2.4.1).
  int fpic_num(const Ref& r, int par, int cur_par, int fn) const { return 2 * wrap_of(r, fn) + (par == cur_par ? 1 : 0); }
  static int flt_pic_num(const Ref& r, int par, int cur_par) { return 2 * r.lt_idx + (par == cur_par ? 1 : 0); }
  static ListEntry fentry(const Ref& r, int par, bool lt) {
    return ListEntry{2 * r.slot + par, r.poc_f[par], lt, r.uid_f[par], r.col_f[par].get()};
  }

  // Initial lists of a P / B field: the decoder's field list initialisation
  // (Decoder::build_field_lists): reference frames (P: FrameNumWrap descending; B: by POC around
  // the current field's, a frame's POC the lowest of its short-term fields'), then long-term by
  // index, split into fields alternating from the current parity.
  void init_field_lists(const SliceHdr& sh, int cur_poc, std::vector<ListEntry>* all) const {
    all[0].clear();
    all[1].clear();
    if (sh.type() == h264::kI) return;
    std::vector<const Ref*> st, lt;
    for (const Ref& r : dpb) {
      if (r.fields & 3) st.push_back(&r);
      if (r.lt_fields & 3) lt.push_back(&r);
    }
    std::sort(lt.begin(), lt.end(), [](const Ref* a, const Ref* b) { return a->lt_idx < b->lt_idx; });
    auto st_poc = [](const Ref* r) {
      return (r->fields & 1) ? ((r->fields & 2) ? std::min(r->poc_f[0], r->poc_f[1]) : r->poc_f[0]) : r->poc_f[1];
    };
    std::vector<const Ref*> init[2];
    if (sh.type() == h264::kP) {
      std::sort(st.begin(), st.end(), [&](const Ref* a, const Ref* b) { return wrap_of(*a, sh.frame_num) > wrap_of(*b, sh.frame_num); });
      init[0] = st;
    } else {
      std::vector<const Ref*> before, after;
      for (const Ref* r : st) (st_poc(r) <= cur_poc ? before : after).push_back(r);
      std::sort(before.begin(), before.end(), [&](const Ref* a, const Ref* b) { return st_poc(a) > st_poc(b); });
      std::sort(after.begin(), after.end(), [&](const Ref* a, const Ref* b) { return st_poc(a) < st_poc(b); });
      init[0] = before;
      init[0].insert(init[0].end(), after.begin(), after.end());
      init[1] = after;
      init[1].insert(init[1].end(), before.begin(), before.end());
    }
    const int same = sh.bottom_field ? 1 : 0;
    const int nl = sh.type() == h264::kB ? 2 : 1;
    for (int l = 0; l < nl; ++l)
      for (int part = 0; part < 2; ++part) {  // short-term frames, then long-term
        std::vector<ListEntry> f[2];
        for (const Ref* r : part == 0 ? init[l] : lt)
          for (int k = 0; k < 2; ++k) {
            const int par = k == 0 ? same : 1 - same;
            if (((part == 0 ? r->fields : r->lt_fields) >> par) & 1) f[k].push_back(fentry(*r, par, part == 1));
          }
        size_t i[2] = {0, 0};
        for (int k = 0; i[0] < f[0].size() || i[1] < f[1].size(); k ^= 1) {
          const int from = i[k] < f[k].size() ? k : k ^ 1;
          all[l].push_back(f[from][i[from]++]);
        }
      }
    if (nl == 2 && all[1].size() > 1) {
      bool same_lists = all[0].size() == all[1].size();
      for (size_t k = 0; same_lists && k < all[0].size(); ++k)
        same_lists = all[0][k].slot == all[1][k].slot && all[0][k].long_term == all[1][k].long_term;
      if (same_lists) std::swap(all[1][0], all[1][1]);
    }
  }

  // Field list modifications (cfg.marking): up to two random fields moved to the front.
  void choose_field_mods(SliceHdr& sh, int cur_poc) {
    std::vector<ListEntry> all[2];
    init_field_lists(sh, cur_poc, all);
    const int cur = sh.bottom_field ? 1 : 0, max_pic = 2 * max_fn;
    for (int l = 0; l < (sh.type() == h264::kB ? 2 : 1); ++l) {
      sh.ref_mods[l].clear();
      if (all[l].size() < 2 || rng.uni(100) >= 40) continue;
      int pred = 2 * sh.frame_num + 1;  // CurrPicNum
      const int n = 1 + rng.uni(2);
      for (int k = 0; k < n; ++k) {
        const ListEntry& e = all[l][size_t(rng.uni(int(all[l].size())))];
        const Ref* r = nullptr;
        for (const Ref& x : dpb)
          if (x.slot == e.slot >> 1) r = &x;
        const int par = e.slot & 1;
        if (e.long_term) {
          sh.ref_mods[l].push_back({2, flt_pic_num(*r, par, cur)});
          continue;
        }
        const int pn = fpic_num(*r, par, cur, sh.frame_num);
        const int nowrap = pn < 0 ? pn + max_pic : pn;
        if (nowrap == pred) continue;
        sh.ref_mods[l].push_back({nowrap < pred ? 0 : 1, std::abs(nowrap - pred) - 1});
        pred = nowrap;
      }
    }
  }

  void build_field_lists(const SliceHdr& sh, int cur_poc, std::vector<ListEntry>* lists) {
    std::vector<ListEntry> all[2];
    init_field_lists(sh, cur_poc, all);
    const int cur = sh.bottom_field ? 1 : 0, cur_pic_num = 2 * sh.frame_num + 1, max_pic = 2 * max_fn;
    for (int l = 0; l < 2; ++l) {
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
          for (const Ref& r : dpb)
            for (int par = 0; par < 2; ++par)
              if (((r.fields >> par) & 1) && fpic_num(r, par, cur, sh.frame_num) == pic_num) {
                pick = fentry(r, par, false);
                found = true;
              }
        } else {
          for (const Ref& r : dpb)
            for (int par = 0; par < 2; ++par)
              if (((r.lt_fields >> par) & 1) && flt_pic_num(r, par, cur) == m.val) {
                pick = fentry(r, par, true);
                found = true;
              }
        }
        VEP_CHECK(found, "encoder: field list modification names a missing field");
        list.insert(list.begin() + long(std::min(idx, list.size())), pick);
        for (size_t k = idx + 1; k < list.size(); ++k)
          if (list[k].slot == pick.slot && list[k].long_term == pick.long_term) {
            list.erase(list.begin() + long(k));
            break;
          }
        ++idx;
      }
      lists[l].clear();
      for (int k = 0; k < sh.num_ref_idx[l] && k < int(list.size()); ++k) lists[l].push_back(list[size_t(k)]);
    }
  }

  // MMCOs of a reference field (cfg.marking): room for a new frame (its first field) frees the
  // oldest unprotected frame's fields (MMCO 1 / 2); then at random MMCO 4, 6 (a first field
  // long-term: its second field follows), 3 (a short-term field of an all-short-term frame
  // long-term), 2 / 1 (a long-term / short-term field unused). The current frame and, with B
  // pictures, the two newest frames are left as they are.
  void choose_field_mmcos(SliceHdr& sh, int parity, bool anchor_with_bs) {
    sh.mmcos.clear();
    const int cur = parity;
    std::vector<const Ref*> all;
    for (const Ref& r : dpb) all.push_back(&r);
    std::sort(all.begin(), all.end(), [&](const Ref* a, const Ref* b) { return wrap_of(*a, sh.frame_num) < wrap_of(*b, sh.frame_num); });
    std::vector<const Ref*> prot;  // frames left alone
    const size_t keep = cfg.bframes > 0 ? 2 : 0;
    for (size_t k = all.size() >= keep ? all.size() - keep : 0; k < all.size(); ++k) prot.push_back(all[k]);
    if (parity == 1)
      for (const Ref* r : all)
        if (r->slot == pair_slot && r->frame_num == sh.frame_num) prot.push_back(r);
    auto is_prot = [&](const Ref* r) { return std::find(prot.begin(), prot.end(), r) != prot.end(); };
    u32 kept_mask = 0;
    int kept_lt = -1;
    for (const Ref* r : prot)
      if (r->lt_fields & 3) {
        kept_mask |= 1u << r->lt_idx;
        kept_lt = std::max(kept_lt, r->lt_idx);
      }
    auto free_idx = [&](int max_idx) {
      std::vector<int> c;
      for (int i = 0; i <= max_idx; ++i)
        if (!((kept_mask >> i) & 1)) c.push_back(i);
      return c.empty() ? -1 : c[size_t(rng.uni(int(c.size())))];
    };
    auto op1 = [&](const Ref* r, int par) { sh.mmcos.push_back({1, 2 * sh.frame_num + 1 - fpic_num(*r, par, cur, sh.frame_num) - 1, 0}); };
    auto op2 = [&](const Ref* r, int par) { sh.mmcos.push_back({2, flt_pic_num(*r, par, cur), 0}); };
    std::vector<const Ref*> freed;
    if (parity == 0 && int(dpb.size()) >= std::max(1, sps.max_num_ref_frames)) {  // room for this frame
      const Ref* victim = nullptr;
      for (const Ref* r : all)
        if (!is_prot(r)) {
          victim = r;
          break;
        }
      if (!victim) return;  // (sliding window instead)
      for (int par = 0; par < 2; ++par) {
        if ((victim->fields >> par) & 1) op1(victim, par);
        if ((victim->lt_fields >> par) & 1) op2(victim, par);
      }
      freed.push_back(victim);
    }
    std::vector<std::pair<const Ref*, int>> st_f, lt_f;  // unprotected fields
    for (const Ref* r : all) {
      if (is_prot(r) || std::find(freed.begin(), freed.end(), r) != freed.end()) continue;
      for (int par = 0; par < 2; ++par) {
        if (((r->fields >> par) & 1) && !(r->lt_fields & 3)) st_f.push_back({r, par});
        if ((r->lt_fields >> par) & 1) lt_f.push_back({r, par});
      }
    }
    const int rr = rng.uni(100);
    int max_lt = max_lt_idx;
    if (parity == 0 && cfg.bframes == 0 && rr >= 94) {  // MMCO 5 alone, in a first field
      sh.mmcos.assign(1, {5, 0, 0});
      sh.adaptive_marking = true;
      return;
    }
    if (rr < 15) {
      max_lt = std::max(kept_lt, rng.uni(3) - 1);
      sh.mmcos.push_back({4, max_lt + 1, 0});
    } else if (rr < 30 && parity == 0 && !anchor_with_bs && free_idx(max_lt) >= 0) {
      sh.mmcos.push_back({6, free_idx(max_lt), 0});
    } else if (rr < 45 && free_idx(max_lt) >= 0 && !st_f.empty()) {
      const auto [r, par] = st_f[size_t(rng.uni(int(st_f.size())))];
      sh.mmcos.push_back({3, 2 * sh.frame_num + 1 - fpic_num(*r, par, cur, sh.frame_num) - 1, free_idx(max_lt)});
    } else if (rr < 55 && !lt_f.empty()) {
      const auto [r, par] = lt_f[size_t(rng.uni(int(lt_f.size())))];
      op2(r, par);
    } else if (rr < 70 && !st_f.empty()) {
      const auto [r, par] = st_f[size_t(rng.uni(int(st_f.size())))];
      op1(r, par);
    }
    if (!sh.mmcos.empty()) sh.adaptive_marking = true;
  }

  // Marking of the current reference field: Decoder::mark_field, mirrored.
  void mark_field_enc(const SliceHdr& sh, int slot, int poc, u32 uid, bool second, std::shared_ptr<const ColMotion> col) {
    const int par = sh.bottom_field ? 1 : 0;
    const int max_refs = std::max(1, sps.max_num_ref_frames);
    const int cur_pic_num = 2 * sh.frame_num + 1;
    auto cur_entry = [&]() -> Ref* {
      if (!second) return nullptr;
      for (Ref& r : dpb)
        if (r.slot == slot && r.frame_num == sh.frame_num && ((r.fields | r.lt_fields) & 3)) return &r;
      return nullptr;
    };
    bool cur_long = false, mmco5 = false;
    int cur_lt = 0;
    if (sh.idr() && !second) {
      dpb.clear();
      max_lt_idx = sh.long_term_reference ? 0 : -1;
      cur_long = sh.long_term_reference;
    } else if (sh.adaptive_marking) {
      const Ref* self = cur_entry();
      for (const auto& m : sh.mmcos) {
        switch (m.op) {
          case 1:
            for (Ref& r : dpb)
              for (int p = 0; p < 2; ++p)
                if (((r.fields >> p) & 1) && fpic_num(r, p, par, sh.frame_num) == cur_pic_num - (m.a + 1)) r.fields &= u8(~(1 << p));
            break;
          case 2:
            for (Ref& r : dpb)
              for (int p = 0; p < 2; ++p)
                if (((r.lt_fields >> p) & 1) && flt_pic_num(r, p, par) == m.a) r.lt_fields &= u8(~(1 << p));
            break;
          case 3: {
            Ref* f = nullptr;
            int fp = 0;
            for (Ref& r : dpb)
              for (int p = 0; p < 2; ++p)
                if (((r.fields >> p) & 1) && fpic_num(r, p, par, sh.frame_num) == cur_pic_num - (m.a + 1)) {
                  f = &r;
                  fp = p;
                }
            if (!f) break;
            for (Ref& r : dpb)
              if (&r != f && (r.lt_fields & 3) && r.lt_idx == m.b) r.lt_fields = 0;
            f->fields &= u8(~(1 << fp));
            f->lt_fields |= u8(1 << fp);
            f->lt_idx = m.b;
            break;
          }
          case 4:
            max_lt_idx = m.a - 1;
            for (Ref& r : dpb)
              if ((r.lt_fields & 3) && r.lt_idx > max_lt_idx) r.lt_fields = 0;
            break;
          case 5:  // (first fields only, see choose_field_mmcos)
            for (Ref& r : dpb) r.fields = r.lt_fields = 0;
            max_lt_idx = -1;
            mmco5 = true;
            break;
          case 6:
            for (Ref& r : dpb)
              if (&r != self && (r.lt_fields & 3) && r.lt_idx == m.a) r.lt_fields = 0;
            cur_long = true;
            cur_lt = m.a;
            break;
          default: break;
        }
      }
    } else if (!second) {  // sliding window on frames
      int frames = 0, n_short = 0;
      for (const Ref& r : dpb) {
        frames += ((r.fields | r.lt_fields) & 3) ? 1 : 0;
        n_short += (r.fields & 3) ? 1 : 0;
      }
      if (frames >= max_refs && n_short > 0) {
        Ref* oldest = nullptr;
        for (Ref& r : dpb)
          if ((r.fields & 3) && (!oldest || wrap_of(r, sh.frame_num) < wrap_of(*oldest, sh.frame_num))) oldest = &r;
        oldest->fields = 0;
      }
    }
    if (!cur_long && second)
      if (const Ref* f = cur_entry(); f && (f->lt_fields & 3)) {
        cur_long = true;
        cur_lt = f->lt_idx;
      }
    dpb.erase(std::remove_if(dpb.begin(), dpb.end(), [](const Ref& r) { return !((r.fields | r.lt_fields) & 3); }), dpb.end());
    if (mmco5) poc = 0;
    Ref* e = cur_entry();
    if (!e) {
      dpb.push_back(Ref{slot, mmco5 ? 0 : sh.frame_num, poc, uid, nullptr});
      e = &dpb.back();
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
    VEP_CHECK(int(dpb.size()) <= max_refs, "encoder: DPB overflow after field marking");
  }

  int pick_slot() const {
    if (fields) {  // a frame slot (both of its field slots free)
      for (int s = 0; 2 * s + 1 < int(slots.size()); ++s) {
        bool used = false;
        for (const Ref& r : dpb) used |= r.slot == s;
        if (!used) return s;
      }
      throw Error("vep: encoder DPB overflow");
    }
    for (int s = 0; s < int(slots.size()); ++s) {
      bool used = false;
      for (const Ref& r : dpb) used |= r.slot == s;
      if (!used) return s;
    }
    throw Error("vep: encoder DPB overflow");
  }

  // ---------------------------------------------------------------- slice header
  void write_header(BitWriter& bw, const SliceHdr& sh) {
    bw.u(8, u32(sh.nal_ref_idc) << 5 | u32(sh.nal_type));
    bw.ue(u32(sh.first_mb));
    bw.ue(u32(sh.slice_type));
    bw.ue(0);
    bw.u(sps.log2_max_frame_num, u32(sh.frame_num));
    if (!sps.frame_mbs_only) {
      bw.u1(sh.field_pic);
      if (sh.field_pic) bw.u1(sh.bottom_field);
    }
    if (sh.idr()) bw.ue(u32(sh.idr_pic_id));
    bw.u(sps.log2_max_poc_lsb, u32(sh.poc_lsb));
    // delta_pic_order_cnt_bottom (frame pictures): top field first
    if (pps.bottom_field_pic_order && !sh.field_pic) bw.se(1);
    const int st = sh.type();
    if (st == h264::kB) bw.u1(sh.direct_spatial);
    if (st != h264::kI) {
      bw.u1(1);  // num_ref_idx_active_override_flag
      bw.ue(u32(sh.num_ref_idx[0] - 1));
      if (st == h264::kB) bw.ue(u32(sh.num_ref_idx[1] - 1));
      for (int l = 0; l < (st == h264::kB ? 2 : 1); ++l) {  // ref_pic_list_modification()
        bw.u1(!sh.ref_mods[l].empty());
        if (sh.ref_mods[l].empty()) continue;
        for (const auto& m : sh.ref_mods[l]) {
          bw.ue(u32(m.idc));
          bw.ue(u32(m.val));
        }
        bw.ue(3);
      }
    }
    if (sh.explicit_wp) {
      bw.ue(u32(sh.luma_lwd));
      bw.ue(u32(sh.chroma_lwd));
      for (int l = 0; l < (st == h264::kB ? 2 : 1); ++l)
        for (const auto& w : sh.wt[l]) {
          const bool lf = w.w[0] != (1 << sh.luma_lwd) || w.o[0] != 0;
          bw.u1(lf);
          if (lf) {
            bw.se(w.w[0]);
            bw.se(w.o[0]);
          }
          const bool cf = w.w[1] != (1 << sh.chroma_lwd) || w.o[1] != 0 || w.w[2] != (1 << sh.chroma_lwd) || w.o[2] != 0;
          bw.u1(cf);
          if (cf)
            for (int c = 1; c < 3; ++c) {
              bw.se(w.w[c]);
              bw.se(w.o[c]);
            }
        }
    }
    if (sh.nal_ref_idc != 0) {  // dec_ref_pic_marking()
      if (sh.idr()) {
        bw.u1(0);
        bw.u1(sh.long_term_reference);
      } else {
        bw.u1(sh.adaptive_marking);
        if (sh.adaptive_marking) {
          for (const auto& m : sh.mmcos) {
            bw.ue(u32(m.op));
            if (m.op == 1 || m.op == 3) bw.ue(u32(m.a));
            if (m.op == 2) bw.ue(u32(m.a));
            if (m.op == 3) bw.ue(u32(m.b));
            if (m.op == 6) bw.ue(u32(m.a));
            if (m.op == 4) bw.ue(u32(m.a));
          }
          bw.ue(0);
        }
      }
    }
    if (pps.cabac && st != h264::kI) bw.ue(0);  // cabac_init_idc
    bw.se(sh.qp - pps.pic_init_qp);
    bw.ue(u32(sh.disable_deblocking));
    if (sh.disable_deblocking != 1) {
      bw.se(sh.alpha_off / 2);
      bw.se(sh.beta_off / 2);
    }
  }

  // ---------------------------------------------------------------- helpers
  int S(int x, int y) const { return cur_src->get(0, x, y); }
  int SC(int x, int y, int c) const { return cur_src->get(1 + c, x, y); }
  // reconstructed luma sample of the current picture (u8 or u16 surface)
  int ty(int x, int y) { return T().get(0, x, y); }
  void set_ty(int x, int y, int v) { T().set(0, x, y, v); }
  HostSurface& T() { return slots[size_t(pic.target)]; }

  // Neighbour MB (dx, dy) of `mb` coded in the current slice (intra availability).
  bool avail(int mb, int dx, int dy) const {
    const int mx = mb % W + dx, my = mb / W + dy;
    if (mx < 0 || mx >= W || my < 0) return false;
    const int n = my * W + mx;
    return n < mb && pic.mbs[size_t(n)].slice == cur_slice;
  }
  int cur_slice = 0;

  // Luma / chroma residual levels of a prediction into `d` (t8: 8x8 transform), cbp returned.
  // (qp = QP'Y = QPY + QpBdOffsetY)
  int code_residual(int mb, const int* py, const int (*pc)[128], bool intra, bool t8, bool i16, int qp, MbDesc& d) {
    const int mx = mb % W, my = mb / W;
    int cl = 0;
    if (t8) {
      for (int q = 0; q < 4; ++q) {
        int x[64];
        for (int i = 0; i < 8; ++i)
          for (int j = 0; j < 8; ++j) {
            const int yy = (q >> 1) * 8 + i, xx = (q & 1) * 8 + j;
            x[i * 8 + j] = S(mx * 16 + xx, my * 16 + yy) - py[yy * 16 + xx];
          }
        quant8x8(x, qp, intra, d.l8[q], scan8);
        for (int k = 0; k < 64; ++k)
          if (d.l8[q][k]) cl |= 1 << q;
      }
    } else {
      int dcw[16];
      for (int r = 0; r < 16; ++r) {
        const int bx = r & 3, by = r >> 2;
        int x[16], w[16];
        for (int i = 0; i < 4; ++i)
          for (int j = 0; j < 4; ++j)
            x[i * 4 + j] = S(mx * 16 + bx * 4 + j, my * 16 + by * 4 + i) - py[(by * 4 + i) * 16 + bx * 4 + j];
        fwd4x4(x, w);
        dcw[r] = w[0];
        for (int k = i16 ? 1 : 0; k < 16; ++k) {
          const int pos = scan4[k];
          const int l = quant(w[pos], qp, mf_class(pos), intra);
          d.ac[r][i16 ? k - 1 : k] = l;
          if (l) cl |= 1 << (raster_to_blk(r) >> 2);
        }
      }
      if (i16) {
        int f[16], g[16];
        for (int i = 0; i < 4; ++i) {
          const int a = dcw[i * 4], b = dcw[i * 4 + 1], c = dcw[i * 4 + 2], e = dcw[i * 4 + 3];
          f[i * 4] = a + b + c + e;
          f[i * 4 + 1] = a + b - c - e;
          f[i * 4 + 2] = a - b - c + e;
          f[i * 4 + 3] = a - b + c - e;
        }
        for (int j = 0; j < 4; ++j) {
          const int a = f[j], b = f[4 + j], c = f[8 + j], e = f[12 + j];
          g[j] = a + b + c + e;
          g[4 + j] = a + b - c - e;
          g[8 + j] = a - b - c + e;
          g[12 + j] = a - b + c - e;
        }
        for (int k = 0; k < 16; ++k) d.dc[k] = quant(g[scan4[k]] / 2, qp, 0, true, 1);
        cl = cl ? 15 : 0;
      }
    }
    int cc = 0;
    const int qpc[2] = {chroma_qp_bd(qp - qpbd, pps.chroma_qp_index_offset, qpbd) + qpbd,
                        chroma_qp_bd(qp - qpbd, pps.second_chroma_qp_index_offset, qpbd) + qpbd};
    const int nbc = cf == 2 ? 8 : 4, ch = cf == 2 ? 16 : 8;  // chroma 4x4 blocks / MB height
    for (int c = 0; c < (cfg.mono ? 0 : 2); ++c) {  // (4:0:0: no chroma residual)
      int cw[8];
      for (int b = 0; b < nbc; ++b) {
        const int bx = (b & 1) * 4, by = (b >> 1) * 4;
        int x[16], w[16];
        for (int i = 0; i < 4; ++i)
          for (int j = 0; j < 4; ++j)
            x[i * 4 + j] = SC(mx * 8 + bx + j, my * ch + by + i, c) - pc[c][(by + i) * 8 + bx + j];
        fwd4x4(x, w);
        cw[b] = w[0];
        for (int k = 1; k < 16; ++k) {
          const int pos = scan4[k];
          d.cac[c][b][k - 1] = quant(w[pos], qpc[c], mf_class(pos), intra);
          if (d.cac[c][b][k - 1]) cc = 2;
        }
      }
      if (cf == 2) {  // 2x4 DC: the decoder's transform (self-inverse up to scale), levels at QP'C + 3,
                      // in the 4:2:2 chroma DC scan order
        int f[8];
        for (int x = 0; x < 2; ++x) {
          const int c0 = cw[x], c1 = cw[2 + x], c2 = cw[4 + x], c3 = cw[6 + x];
          f[x] = c0 + c1 + c2 + c3;
          f[2 + x] = c0 + c1 - c2 - c3;
          f[4 + x] = c0 - c1 - c2 + c3;
          f[6 + x] = c0 - c1 + c2 - c3;
        }
        for (int y = 0; y < 4; ++y) {
          const int a = f[2 * y], b = f[2 * y + 1];
          f[2 * y] = a + b;
          f[2 * y + 1] = a - b;
        }
        for (int k = 0; k < 8; ++k) {
          d.cdc[c][k] = quant(f[kChroma422DcScanToRaster[k]], qpc[c] + 3, 0, intra, 1);
          if (d.cdc[c][k]) cc = std::max(cc, 1);
        }
        continue;
      }
      const int f[4] = {cw[0] + cw[1] + cw[2] + cw[3], cw[0] - cw[1] + cw[2] - cw[3],
                        cw[0] + cw[1] - cw[2] - cw[3], cw[0] - cw[1] - cw[2] + cw[3]};
      for (int b = 0; b < 4; ++b) {
        d.cdc[c][b] = quant(f[b], qpc[c], 0, intra, 1);
        if (d.cdc[c][b]) cc = std::max(cc, 1);
      }
    }
    if (cc < 2)
      for (auto& c : d.cac)
        for (auto& b : c)
          for (int& v : b) v = 0;
    return cl | cc << 4;
  }

  int sad_pred(int mb, const int* py) const {
    const int mx = mb % W, my = mb / W;
    int s = 0;
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) s += std::abs(S(mx * 16 + x, my * 16 + y) - py[y * 16 + x]);
    return s;
  }

  // Inter prediction of a whole MB from per-8x8 list entries and per-4x4 motion.
  void predict(const SliceEnv& env, int mb, const int r0[4], const int r1[4], const i16 (*mv)[16][2], int* py,
               int (*pc)[128], bool weighted) {
    MbRec m{};
    bool l1 = false;
    WpEntry wp[4];
    for (int k = 0; k < 4; ++k) {
      m.ref[k] = r0[k] >= 0 ? u8((*env.list[0])[size_t(r0[k])].slot) : u8(0xFF);
      m.ref1[k] = r1[k] >= 0 ? u8((*env.list[1])[size_t(r1[k])].slot) : u8(0xFF);
      l1 |= r1[k] >= 0;
      if (weighted) wp[k] = wp_entry(env, r0[k], r1[k]);
    }
    predict_inter(slots, m, &mv[0][0][0], l1 ? &mv[1][0][0] : nullptr, weighted ? wp : nullptr, mb % W, mb / W, py, pc,
                  pic.structure);
  }

  // 16x16 motion search in one list for reference r: candidates (zero, predictor, the scene's
  // object motion) refined by full-, half- and quarter-sample steps.
  void search(const SliceEnv& env, int mb, int list, int r, const int pmv[2], int best[2], int& best_sad) {
    const ListEntry& e = (*env.list[list])[size_t(r)];
    const HostSurface& R = slots[size_t(e.slot)];
    const double dist = (e.poc - env.cur_poc) / 2.0;  // display frames from here to the reference
    const int mx = mb % W, my = mb / W;
    auto cost = [&](int vx, int vy) {
      int s = 0;
      for (int i = 0; i < 16; i += 2)
        for (int j = 0; j < 16; j += 2) {
          const int x = mx * 16 + j, y = my * 16 + i;
          const int p = bd > 8 ? luma_qpel(R.y16.data(), wpx, wpx, ph, x + (vx >> 2), y + (vy >> 2), vx & 3, vy & 3, bd)
                               : luma_qpel(R.y.data(), wpx, wpx, ph, x + (vx >> 2), y + (vy >> 2), vx & 3, vy & 3);
          s += std::abs(S(x, y) - p);
        }
      return s * 4 + 4 * (std::abs(vx - pmv[0]) + std::abs(vy - pmv[1]));
    };
    std::vector<std::pair<int, int>> cand = {{0, 0}, {pmv[0], pmv[1]}};
    const double ys = fields ? 0.5 : 1.0;  // (a field has half the frame's rows)
    for (const Scene::Obj& o : scene.objs) {
      if (o.x > mx * 16 + 24 || o.x + o.w < mx * 16 - 8 || o.y * ys > my * 16 + 24 || (o.y + o.h) * ys < my * 16 - 8)
        continue;
      cand.push_back({int(std::lround(o.vx * 4 * dist)), int(std::lround(o.vy * ys * 4 * dist))});
    }
    best_sad = 1 << 30;
    for (auto [vx, vy] : cand) {
      const int c = cost(vx, vy);
      if (c < best_sad) {
        best_sad = c;
        best[0] = vx;
        best[1] = vy;
      }
    }
    for (int step : {4, 2, 1}) {
      bool moved = true;
      for (int it = 0; moved && it < 4; ++it) {
        moved = false;
        const int cx = best[0], cy = best[1];
        for (int k = 0; k < 8; ++k) {
          static const int dx[8] = {-1, 1, 0, 0, -1, -1, 1, 1}, dy[8] = {0, 0, -1, 1, -1, 1, -1, 1};
          const int vx = cx + dx[k] * step, vy = cy + dy[k] * step;
          if (std::abs(vx) > 2048 || std::abs(vy) > 512) continue;
          const int c = cost(vx, vy);
          if (c < best_sad) {
            best_sad = c;
            best[0] = vx;
            best[1] = vy;
            moved = true;
          }
        }
      }
    }
  }

  // ---------------------------------------------------------------- intra decisions
  // Intra_16x16 (no 8x8 transform) or Intra_8x8 with per-block closed-loop mode choice.
  void decide_intra(int mb, int qp, MbDesc& d, int& sad) {
    const int mx = mb % W, my = mb / W;
    const bool A = avail(mb, -1, 0), B = avail(mb, 0, -1), D = avail(mb, -1, -1);
    const int itype_base = 0;
    (void)itype_base;
    int cp[2][128];
    {  // chroma: DC
      for (int c = 0; c < 2; ++c) {
        IntraChromaNb n;
        chroma_neighbours(pic, mb, c, T(), n);
        for (int y = 0; y < (cf == 2 ? 16 : 8); ++y)
          for (int x = 0; x < 8; ++x) cp[c][y * 8 + x] = chroma_pred(n, PredConst{0, 0, 0, 0}, 0, x, y, bd, cf);
      }
      d.chroma_mode = 0;
    }
    if (cfg.t8x8) {
      // Intra_8x8: each block predicted from the (closed-loop) reconstruction of the previous ones
      int py[256];
      HostSurface& t = T();
      sad = 0;
      for (int q = 0; q < 4; ++q) {
        int f[25];
        bool top, left;
        intra8x8_neighbours(pic, mb, q, t, f, top, left);
        const int bx = q & 1, by = q >> 1;
        const bool tl = (bx > 0 && by > 0) || (bx == 0 && by == 0 ? D : bx == 0 ? A : B);
        int best = 2, best_s = 1 << 30;
        for (int mode = 0; mode < 9; ++mode) {
          const bool ok = mode == 2 || ((mode == 0 || mode == 3 || mode == 7) && top) || ((mode == 1 || mode == 8) && left) ||
                          ((mode >= 4 && mode <= 6) && top && left && tl);
          if (!ok) continue;
          int s = 0;
          for (int i = 0; i < 8; ++i)
            for (int j = 0; j < 8; ++j)
              s += std::abs(S(mx * 16 + bx * 8 + j, my * 16 + by * 8 + i) - intra8x8_pred(f, top, left, mode, j, i, bd));
          if (s < best_s) {
            best_s = s;
            best = mode;
          }
        }
        d.ipred[q] = u8(best);
        int x[64], pb[64];
        for (int i = 0; i < 8; ++i)
          for (int j = 0; j < 8; ++j) {
            pb[i * 8 + j] = intra8x8_pred(f, top, left, best, j, i, bd);
            py[(by * 8 + i) * 16 + bx * 8 + j] = pb[i * 8 + j];
            x[i * 8 + j] = S(mx * 16 + bx * 8 + j, my * 16 + by * 8 + i) - pb[i * 8 + j];
          }
        quant8x8(x, qp, true, d.l8[q], scan8);
        int r[64];
        recon8x8(d.l8[q], qp, r, scan8);
        for (int i = 0; i < 8; ++i)
          for (int j = 0; j < 8; ++j)
            t.set(0, mx * 16 + bx * 8 + j, my * 16 + by * 8 + i, clip1(pb[i * 8 + j] + r[i * 8 + j], bd));
        sad += best_s;
      }
      MbDesc tmp;
      const int cbp = code_residual(mb, py, cp, true, true, false, qp, tmp);
      for (int c = 0; c < 2; ++c) {  // keep the closed-loop luma levels, take the chroma ones
        std::memcpy(d.cdc[c], tmp.cdc[c], sizeof d.cdc[c]);
        std::memcpy(d.cac[c], tmp.cac[c], sizeof d.cac[c]);
      }
      int cl = 0;
      for (int q = 0; q < 4; ++q)
        for (int k = 0; k < 64; ++k)
          if (d.l8[q][k]) cl |= 1 << q;
      d.t8x8 = true;
      d.cbp = cl | (cbp & 0x30);
      d.mb_type = 0;  // I_NxN (+ transform_size_8x8_flag)
      return;
    }
    Intra16Nb n;
    intra16_neighbours(pic, mb, T(), n);
    int best = 2, best_s = 1 << 30;
    int py[256];
    for (int mode = 0; mode < 4; ++mode) {
      if ((mode == 0 && !B) || (mode == 1 && !A) || (mode == 3 && !(A && B && D))) continue;
      const PredConst k = intra16x16_const(n, mode, bd);
      int s = 0;
      for (int y = 0; y < 16; ++y)
        for (int x = 0; x < 16; ++x) s += std::abs(S(mx * 16 + x, my * 16 + y) - intra16x16_pred(n, k, mode, x, y, bd));
      if (s < best_s) {
        best_s = s;
        best = mode;
      }
    }
    const PredConst k = intra16x16_const(n, best, bd);
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) py[y * 16 + x] = intra16x16_pred(n, k, best, x, y, bd);
    const int cbp = code_residual(mb, py, cp, true, false, true, qp, d);
    d.mb_type = 1 + best + 4 * (cbp >> 4) + 12 * ((cbp & 15) ? 1 : 0);
    if (!(cbp & 15))
      for (auto& b : d.ac)
        for (int& v : b) v = 0;
    sad = best_s;
  }

  // ---------------------------------------------------------------- coverage decisions
  void random_levels(MbDesc& d, bool t8, bool i16) {
    auto lvl = [&]() {
      const int r = rng.uni(100);
      if (r < 70) return 0;
      int a = r < 95 ? 1 + rng.uni(3) : 1 + rng.uni(r < 99 ? 40 : 600);
      return rng.uni(2) ? a : -a;
    };
    if (t8)
      for (auto& b : d.l8)
        for (int k = 0; k < 64; ++k) b[k] = k < 20 ? lvl() : (rng.chance(5) ? lvl() : 0);
    else
      for (auto& b : d.ac)
        for (int k = 0; k < (i16 ? 15 : 16); ++k) b[k] = lvl();
    if (i16)
      for (int& v : d.dc) v = lvl();
    for (auto& c : d.cdc)
      for (int& v : c) v = lvl();
    for (auto& c : d.cac)
      for (auto& b : c)
        for (int& v : b) v = rng.chance(30) ? lvl() : 0;
  }

  void random_intra(int mb, bool islice_pcm_ok, MbDesc& d, int& base_type) {
    const bool A = avail(mb, -1, 0), B = avail(mb, 0, -1), D = avail(mb, -1, -1);
    const int r = rng.uni(100);
    auto chroma = [&]() {
      int m;
      do m = rng.uni(4);
      while ((m == 1 && !A) || (m == 2 && !B) || (m == 3 && !(A && B && D)));
      return m;
    };
    if (islice_pcm_ok && r < 5 && bd > 8) {  // (High 10: u16 samples of bd bits)
      static thread_local u16 pcm16[kPcmMaxSamples];
      for (auto& p : pcm16) p = u16(rng.uni(1 << bd));
      if (cfg.mono)
        for (size_t i = 256; i < kPcmMbBytes; ++i) pcm16[i] = u16(1 << (bd - 1));
      d.pcm = reinterpret_cast<const u8*>(pcm16);
      base_type = 25;
      return;
    }
    if (islice_pcm_ok && r < 5) {
      static thread_local u8 pcm[kPcmMaxSamples];  // (4:2:2: 512 samples)
      for (auto& p : pcm) p = u8(16 + rng.uni(220));
      if (cfg.mono) std::memset(pcm + 256, 128, kPcmMbBytes - 256);  // (the grey the decoder fills)
      d.pcm = pcm;
      base_type = 25;
      return;
    }
    d.chroma_mode = cfg.mono ? 0 : chroma();
    if (r < 40) {  // Intra_16x16
      int m;
      do m = rng.uni(4);
      while ((m == 0 && !B) || (m == 1 && !A) || (m == 3 && !(A && B && D)));
      random_levels(d, false, true);
      const int cl = rng.chance(50) ? 15 : 0, cc = cfg.mono ? 0 : rng.uni(3);
      if (!cl)
        for (auto& b : d.ac)
          for (int& v : b) v = 0;
      if (cc < 2)
        for (auto& c : d.cac)
          for (auto& b : c)
            for (int& v : b) v = 0;
      if (cc < 1)
        for (auto& c : d.cdc)
          for (int& v : c) v = 0;
      base_type = 1 + m + 4 * cc + 12 * (cl ? 1 : 0);
      return;
    }
    base_type = 0;
    d.t8x8 = cfg.t8x8 && rng.chance(50);
    const int mx = mb % W, my = mb / W;
    (void)mx;
    (void)my;
    if (d.t8x8) {
      for (int q = 0; q < 4; ++q) {
        const int bx = q & 1, by = q >> 1;
        const bool top = by > 0 || B, left = bx > 0 || A;
        const bool tl = (bx > 0 && by > 0) || (bx == 0 && by == 0 ? D : bx == 0 ? A : B);
        int m;
        do m = rng.uni(9);
        while (!(m == 2 || ((m == 0 || m == 3 || m == 7) && top) || ((m == 1 || m == 8) && left) ||
                 ((m >= 4 && m <= 6) && top && left && tl)));
        d.ipred[q] = u8(m);
      }
    } else {
      for (int rb = 0; rb < 16; ++rb) {
        const int bx = rb & 3, by = rb >> 2;
        const bool top = by > 0 || B, left = bx > 0 || A;
        const bool tl = (bx > 0 && by > 0) || (bx == 0 && by == 0 ? D : bx == 0 ? A : B);
        int m;
        do m = rng.uni(9);
        while (!(m == 2 || ((m == 0 || m == 3 || m == 7) && top) || ((m == 1 || m == 8) && left) ||
                 ((m >= 4 && m <= 6) && top && left && tl)));
        d.ipred[rb] = u8(m);
      }
    }
    random_levels(d, d.t8x8, false);
    d.cbp = rng.uni(16) | (cfg.mono ? 0 : rng.uni(3) << 4);
  }

  // ---------------------------------------------------------------- picture
  std::shared_ptr<AccessUnit> encode(const Job& job) {
    cur_src = &source_of(job.disp);
    const bool fld = job.parity >= 0;
    if (fld) {  // the field's rows of the frame
      const HostSurface& f = *cur_src;
      if (field_src.coded_w != wpx || field_src.coded_h != ph) field_src.alloc(wpx, ph);
      for (int r = 0; r < ph; ++r)
        std::memcpy(&field_src.y[size_t(r) * wpx], &f.y[size_t(2 * r + job.parity) * wpx], size_t(wpx));
      for (int r = 0; r < ph / 2; ++r)
        std::memcpy(&field_src.uv[size_t(r) * wpx], &f.uv[size_t(2 * r + job.parity) * wpx], size_t(wpx));
      cur_src = &field_src;
    }
    scan4 = fld ? kFieldScan4x4 : kZigzag4x4;
    scan8 = fld ? kFieldScan8x8 : kZigzag8x8;
    const bool idr = job.idr;
    if (idr) {
      dpb.clear();
      ++idr_id;
    }
    SliceHdr sh;
    sh.nal_type = idr ? h264::kNalIdr : h264::kNalSlice;
    sh.nal_ref_idc = job.ref ? (job.type == h264::kB ? 2 : 3) : 0;
    sh.slice_type = job.type;
    sh.frame_num = job.parity == 1 ? pair_fn : idr ? 0 : (prev_ref_fn + 1) % max_fn;
    sh.field_pic = fld;
    sh.bottom_field = job.parity == 1;
    sh.idr_pic_id = idr_id & 0xFFFF;
    const int poc = int(2 * (job.disp - gop_start)) + (fld ? job.parity : 0);  // top 2k, bottom 2k + 1
    sh.poc_lsb = poc & ((1 << sps.log2_max_poc_lsb) - 1);
    sh.direct_spatial = cfg.direct_spatial;
    int n0 = 0, n1 = 0;
    if (job.type == h264::kP && !fld) n0 = std::min<int>(cfg.refs, int(dpb.size()));
    if (job.type == h264::kP && fld) {  // reference fields (the first field of this frame included)
      int nf = 0;
      for (const Ref& r : dpb) nf += (r.fields & 1) + ((r.fields >> 1) & 1) + (r.lt_fields & 1) + ((r.lt_fields >> 1) & 1);
      n0 = std::min(2 * cfg.refs, nf);
    }
    if (job.type == h264::kB && fld) {  // reference fields on both sides (every one in list 0)
      int before = 0, after = 0, nf = 0;
      for (const Ref& r : dpb)
        for (int par = 0; par < 2; ++par)
          if (((r.fields | r.lt_fields) >> par) & 1) {
            ++nf;
            (r.poc_f[par] < poc ? before : after) += 1;
          }
      n0 = nf;
      n1 = std::min<int>(cfg.coverage ? 2 : 1, nf);
      VEP_CHECK(before > 0 && after > 0, "B field without reference fields on both sides");
    }
    if (job.type == h264::kB && !fld) {
      int before = 0, after = 0;
      for (const Ref& r : dpb) (r.poc < poc ? before : after) += 1;
      // every reference in list 0: temporal direct needs the colocated picture's references
      n0 = int(dpb.size());
      n1 = std::min<int>(cfg.coverage ? 2 : 1, int(dpb.size()));
      VEP_CHECK(before > 0 && after > 0, "B picture without references on both sides");
    }
    sh.num_ref_idx[0] = std::max(1, n0);
    sh.num_ref_idx[1] = std::max(1, n1);
    const bool wp_p = job.type == h264::kP && cfg.weighted_p;
    const bool wp_b = job.type == h264::kB && cfg.weighted_b == 1;
    sh.explicit_wp = wp_p || wp_b;
    if (sh.explicit_wp) {
      sh.luma_lwd = 5;
      sh.chroma_lwd = 4;
      for (int l = 0; l < (job.type == h264::kB ? 2 : 1); ++l) {
        sh.wt[l].resize(size_t(sh.num_ref_idx[l]));
        for (auto& w : sh.wt[l]) {
          w.w[0] = i16(32 + (cfg.coverage ? rng.uni(9) - 4 : 1));
          w.o[0] = i16(cfg.coverage ? rng.uni(9) - 4 : -2);
          w.w[1] = w.w[2] = i16(16);
          w.o[1] = w.o[2] = i16(cfg.coverage ? rng.uni(5) - 2 : 0);
        }
      }
    }
    if (cfg.marking && !fld) {  // reference marking / list modification coverage
      if (idr) {
        sh.long_term_reference = rng.uni(100) < 30;
      } else {
        if (job.type != h264::kI) choose_mods(sh, poc);
        if (job.ref) choose_mmcos(sh, job.type == h264::kP && cfg.bframes > 0);
      }
    }
    if (cfg.marking && fld) {
      if (idr) {
        sh.long_term_reference = rng.uni(100) < 30;
      } else {
        if (job.type != h264::kI) choose_field_mods(sh, poc);
        if (job.ref) choose_field_mmcos(sh, job.parity, job.type == h264::kP && cfg.bframes > 0);
      }
    }
    sh.cabac_init_idc = 0;
    sh.qp = std::clamp(cfg.qp + (job.type == h264::kB ? (job.ref ? 1 : 2) : 0), -qpbd, 51);
    sh.disable_deblocking = cfg.deblock_idc;
    const bool weighted = sh.explicit_wp || (job.type == h264::kB && cfg.weighted_b == 2);

    const int Hp = fld ? H / 2 : H;  // MB rows of the picture
    pic = Picture{};
    pic.wmbs = W;
    pic.hmbs = Hp;
    pic.mbs.assign(size_t(W) * Hp, MbRec{});
    pic.coefs.reserve(size_t(W) * Hp * 64);
    pic.mvs.reserve(size_t(W) * Hp * 64);
    pic.dpb_slots = int(slots.size());
    pic.structure = fld ? 1 + job.parity : 0;
    pic.bd = bd;
    pic.qp_bias = pic.qpc_bias = qpbd;
    pic.cf = cf;
    pic.target = fld ? 2 * (job.parity == 1 ? pair_slot : pick_slot()) + job.parity : pick_slot();
    if (job.parity == 0) {  // the pair's frame_num and frame slot, for its second field
      pair_fn = sh.frame_num;
      pair_slot = pic.target >> 1;
    }
    pic.idr = idr;
    pic.poc = poc;
    nb.reset(W, Hp);
    std::vector<ListEntry> lists[2];
    auto au = std::make_shared<AccessUnit>();
    au->codec = Codec::kH264;
    au->keyframe = idr;
    // decoding timestamps run `reorder depth` frames behind the display timestamps
    const i64 dur = 90000 / std::max(1, cfg.fps);
    au->pts = (job.disp + std::max(0, sps.max_num_reorder_frames)) * dur;
    au->dts = fld ? coded * dur / 2 : coded * dur;
    au->duration = dur;
    au->seq = u64(coded);
    last_pts = au->pts;
    last_type = job.type == h264::kI ? 'I' : job.type == h264::kP ? 'P' : 'B';
    if (idr) {
      au->add_nal(sps_nal.data(), sps_nal.size());
      au->add_nal(pps_nal.data(), pps_nal.size());
    }
    std::vector<std::array<std::vector<u32>, 2>> slice_uids;
    const int nslices = std::max(1, std::min(cfg.slices, Hp));
    for (int si = 0; si < nslices; ++si) {
      const int row0 = si * Hp / nslices, row1 = (si + 1) * Hp / nslices;
      sh.first_mb = row0 * W;
      if (fld) build_field_lists(sh, poc, lists);
      else build_lists(sh, poc, lists);
      std::array<std::vector<u32>, 2> uids;
      for (int l = 0; l < 2; ++l)
        for (const auto& e : lists[l]) uids[size_t(l)].push_back(e.uid);
      slice_uids.push_back(uids);
      SliceEnv env;
      env.sh = &sh;
      env.sps = &sps;
      env.pps = &pps;
      env.slice = si;
      env.list[0] = &lists[0];
      env.list[1] = &lists[1];
      env.cur_poc = poc;
      env.scaling = h264::resolve_scaling(sps, pps);
      env.field = fld;
      BitWriter bw;
      write_header(bw, sh);
      SliceWriter sw(nb, pic, env, bw);
      cur_slice = si;
      for (int mb = row0 * W; mb < row1 * W; ++mb) {
        pic.mbs[size_t(mb)].slice = decltype(MbRec::slice)(si);  // intra availability of this MB
        MbDesc d;
        decide(env, sw, mb, job, sh, weighted, d);
        sw.write_mb(mb, d);
        cpu_reconstruct_mb(pic, mb, slots);
      }
      sw.finish();
      std::vector<u8> nal;
      rbsp_to_ebsp(bw.buf().data(), bw.buf().size(), nal);
      au->add_nal(nal.data(), nal.size());
    }
    if (pic.deblock) cpu_deblock(pic, T());
    if (job.ref && fld) {  // a frame entry holding its reference fields
      mark_field_enc(sh, pic.target >> 1, poc, next_uid, job.parity == 1,
                     build_col_motion(nb, W, Hp, slice_uids, sps.direct_8x8));
      prev_ref_fn = sh.frame_num;
      if (sh.has_mmco5()) {  // the pair continues with frame_num 0; POCs count from this frame
        prev_ref_fn = pair_fn = 0;
        gop_start = job.disp;
      }
    } else if (job.ref) {
      mark_frame(sh, Ref{pic.target, sh.frame_num, poc, next_uid, build_col_motion(nb, W, H, slice_uids, sps.direct_8x8)});
      prev_ref_fn = sh.frame_num;
      if (sh.has_mmco5()) {  // the picture now counts as frame_num 0, POC 0 (§8.2.1)
        prev_ref_fn = 0;
        gop_start = job.disp;
      }
    }
    ++next_uid;
    if (!fld) {
      recon = T();
      src_out = *cur_src;
    } else if (job.parity == 1) {  // the frame is complete: its two fields woven
      weave_fields(slots[size_t(2 * pair_slot)], slots[size_t(2 * pair_slot + 1)], recon);
      src_out = source_of(job.disp);
    }
    last_disp = job.disp;
    ++coded;
    // sources of pictures coded and no longer needed
    if (job.parity != 0) sources.erase(job.disp);
    return au;
  }

  void decide(const SliceEnv& env, SliceWriter& sw, int mb, const Job& job, const SliceHdr& sh, bool weighted,
              MbDesc& d) {
    const int qp = sh.qp + qpbd;  // QP'Y
    const int t = job.type;
    if (cfg.coverage) {
      decide_random(env, sw, mb, t, d);
      return;
    }
    if (t == h264::kI) {
      int sad;
      decide_intra(mb, qp, d, sad);
      return;
    }
    const int mx = mb % W, my = mb / W;
    (void)mx;
    (void)my;
    MbState skip;
    sw.skip_motion(mb, skip);
    int r0[4], r1[4];
    for (int k = 0; k < 4; ++k) {
      r0[k] = skip.ref[0][k];
      r1[k] = skip.ref[1][k];
    }
    int py[256], pc[2][128];
    predict(env, mb, r0, r1, skip.mv, py, pc, weighted);
    const int skip_sad = sad_pred(mb, py);
    MbDesc sd;
    const int skip_cbp = code_residual(mb, py, pc, false, cfg.t8x8, false, qp, sd);
    if (skip_cbp == 0 && skip_sad < 256 * 6) {
      d.skip = true;
      return;
    }
    // 16x16 motion search: list 0 (P: the first two references) and list 1 (B: reference 0)
    int best[2][2] = {{0, 0}, {0, 0}}, bsad[2] = {1 << 30, 1 << 30}, bref[2] = {0, 0};
    for (int l = 0; l < (t == h264::kB ? 2 : 1); ++l) {
      const int nr = t == h264::kP ? std::min(2, int(env.list[l]->size())) : 1;
      for (int r = 0; r < nr; ++r) {
        int pmv[2], mv[2], s;
        nb.pred_mv(mb, 0, 0, 4, 4, l, r, 0, 0, pmv);
        search(env, mb, l, r, pmv, mv, s);
        if (s < bsad[l]) {
          bsad[l] = s;
          best[l][0] = mv[0];
          best[l][1] = mv[1];
          bref[l] = r;
        }
      }
    }
    // candidate predictions: 0 L0, 1 L1, 2 Bi (B) ; direct (with residual)
    int cands = t == h264::kB ? 3 : 1;
    int best_c = -1, best_cost = skip_sad + 256 * 2;  // direct / skip-motion with residual
    int cpy[3][256], cpc[3][2][128];
    for (int c = 0; c < cands; ++c) {
      int a0[4], a1[4];
      i16 mv[2][16][2];
      for (int k = 0; k < 4; ++k) {
        a0[k] = (c == 0 || c == 2) ? bref[0] : -1;
        a1[k] = (c == 1 || c == 2) ? bref[1] : -1;
      }
      for (int l = 0; l < 2; ++l)
        for (int b = 0; b < 16; ++b) {
          mv[l][b][0] = i16(best[l][0]);
          mv[l][b][1] = i16(best[l][1]);
        }
      predict(env, mb, a0, a1, mv, cpy[c], cpc[c], weighted);
      const int s = sad_pred(mb, cpy[c]);
      if (s < best_cost) {
        best_cost = s;
        best_c = c;
      }
    }
    // intra fallback
    if (best_cost > 256 * 22) {
      MbDesc id;
      int isad;
      HostSurface& T0 = T();
      std::vector<int> save;
      (void)T0;
      if (cfg.t8x8) {  // decide_intra's closed loop writes samples: keep them to undo
        save.resize(16 * 16);
        for (int y = 0; y < 16; ++y)
          for (int x = 0; x < 16; ++x) save[size_t(y) * 16 + x] = ty(mb % W * 16 + x, mb / W * 16 + y);
      }
      decide_intra(mb, qp, id, isad);
      if (isad + 256 * 4 < best_cost) {
        d = id;
        d.mb_type += t == h264::kP ? 5 : 23;
        return;
      }
      if (cfg.t8x8)
        for (int y = 0; y < 16; ++y)
          for (int x = 0; x < 16; ++x) set_ty(mb % W * 16 + x, mb / W * 16 + y, save[size_t(y) * 16 + x]);
    }
    if (best_c < 0) {  // the skip / direct motion with residual
      if (t == h264::kP) {
        d.mb_type = 0;
        d.ref[0][0] = 0;
        for (int b = 0; b < 16; ++b) {
          d.mv[0][b][0] = skip.mv[0][b][0];
          d.mv[0][b][1] = skip.mv[0][b][1];
        }
      } else {
        d.mb_type = 0;  // B_Direct_16x16
      }
      d.t8x8 = cfg.t8x8 && (t == h264::kP || sps.direct_8x8);
      const int cbp = code_residual(mb, py, pc, false, d.t8x8, false, qp, d);
      d.cbp = cbp;
      return;
    }
    d.mb_type = t == h264::kP ? 0 : 1 + best_c;  // P_L0_16x16 / B_L0, B_L1, B_Bi _16x16
    for (int l = 0; l < 2; ++l) {
      d.ref[l][0] = bref[l];
      for (int b = 0; b < 16; ++b) {
        d.mv[l][b][0] = i16(best[l][0]);
        d.mv[l][b][1] = i16(best[l][1]);
      }
    }
    d.t8x8 = cfg.t8x8;
    d.cbp = code_residual(mb, cpy[best_c], cpc[best_c], false, d.t8x8, false, qp, d);
  }

  void decide_random(const SliceEnv& env, SliceWriter& sw, int mb, int t, MbDesc& d) {
    (void)sw;
    const int r = rng.uni(100);
    auto rmv = [&]() { return i16(rng.uni(100) < 20 ? 0 : rng.uni(161) - 80); };
    if (t == h264::kI || r < 12) {
      int base;
      random_intra(mb, true, d, base);
      d.mb_type = base + (t == h264::kI ? 0 : (t == h264::kP ? 5 : 23));
      if (base > 0 && base < 25) d.cbp = 0;
      d.qp_delta = rng.chance(20) ? rng.uni(9) - 4 : 0;
      return;
    }
    if (r < 25) {
      d.skip = true;
      return;
    }
    const bool b = t == h264::kB;
    const int n0 = sh_num(env, 0), n1 = sh_num(env, 1);
    int mbt;
    if (b) mbt = rng.uni(23);
    else mbt = rng.uni(4);
    d.mb_type = mbt;
    for (int l = 0; l < 2; ++l)
      for (int k = 0; k < 4; ++k) d.ref[l][k] = rng.uni(l == 0 ? n0 : n1);
    for (int l = 0; l < 2; ++l)
      for (int k = 0; k < 16; ++k) {
        d.mv[l][k][0] = rmv();
        d.mv[l][k][1] = rmv();
      }
    // sub-macroblock shapes: 0 8x8, 1 8x4, 2 4x8, 3 4x4 (B_Direct_8x8 counts as 8x8: the SPS
    // sets direct_8x8_inference)
    static const u8 kBShape[13] = {0, 0, 0, 0, 1, 2, 1, 2, 1, 2, 3, 3, 3};
    bool small = false;
    const bool eight = (!b && mbt == 3) || (b && mbt == 22);
    if (eight)
      for (int i = 0; i < 4; ++i) {
        d.sub[i] = b ? rng.uni(13) : rng.uni(4);
        small |= (b ? kBShape[d.sub[i]] : d.sub[i]) != 0;
      }
    // uniform motion inside each partition (the layer reads the partition's top-left block)
    auto fill = [&](int l, int x4, int y4, int w4, int h4) {
      const i16 vx = d.mv[l][y4 * 4 + x4][0], vy = d.mv[l][y4 * 4 + x4][1];
      for (int y = y4; y < y4 + h4; ++y)
        for (int x = x4; x < x4 + w4; ++x) {
          d.mv[l][y * 4 + x][0] = vx;
          d.mv[l][y * 4 + x][1] = vy;
        }
    };
    for (int l = 0; l < 2; ++l) {
      if (!eight) {
        const int shape = (!b ? mbt : (mbt <= 3 ? 0 : ((mbt & 1) ? 2 : 1)));
        if (shape == 0) fill(l, 0, 0, 4, 4);
        else if (shape == 1) {
          fill(l, 0, 0, 4, 2);
          fill(l, 0, 2, 4, 2);
        } else {
          fill(l, 0, 0, 2, 4);
          fill(l, 2, 0, 2, 4);
        }
      } else {
        for (int i = 0; i < 4; ++i) {
          const int x8 = (i & 1) * 2, y8 = (i >> 1) * 2;
          const int shape = b ? kBShape[d.sub[i]] : d.sub[i];
          if (shape == 0) fill(l, x8, y8, 2, 2);
          else if (shape == 1) {
            fill(l, x8, y8, 2, 1);
            fill(l, x8, y8 + 1, 2, 1);
          } else if (shape == 2) {
            fill(l, x8, y8, 1, 2);
            fill(l, x8 + 1, y8, 1, 2);
          }
        }
      }
    }
    const bool direct16 = b && mbt == 0;
    const bool t8_ok = cfg.t8x8 && !small && (!direct16 || sps.direct_8x8);
    d.t8x8 = t8_ok && rng.chance(50);
    random_levels(d, d.t8x8, false);
    d.cbp = rng.uni(16) | (cfg.mono ? 0 : rng.uni(3) << 4);
    d.qp_delta = rng.chance(20) ? rng.uni(9) - 4 : 0;
  }

  static int sh_num(const SliceEnv& env, int l) { return std::max(1, int(env.list[l]->size())); }

  std::shared_ptr<AccessUnit> next() {
    if (plan.empty()) plan_next();
    const Job j = plan.front();
    plan.pop_front();
    return encode(j);
  }
};

AvcHighEncoder::AvcHighEncoder(const AvcHighConfig& cfg) : cfg_(cfg), p_(std::make_unique<Impl>(cfg)) {}
AvcHighEncoder::~AvcHighEncoder() = default;
std::shared_ptr<AccessUnit> AvcHighEncoder::next() { return p_->next(); }
const HostSurface& AvcHighEncoder::reconstruction() const { return p_->recon; }
const HostSurface& AvcHighEncoder::source() const { return p_->src_out; }
i64 AvcHighEncoder::last_display_index() const { return p_->last_disp; }
i64 AvcHighEncoder::last_pts() const { return p_->last_pts; }
char AvcHighEncoder::last_type() const { return p_->last_type; }
const std::vector<u8>& AvcHighEncoder::sps_nal() const { return p_->sps_nal; }
const std::vector<u8>& AvcHighEncoder::pps_nal() const { return p_->pps_nal; }

}  // namespace vep::avc
