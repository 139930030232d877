// Closed-loop synthetic H.265 Main encoder over the shared CTU layer (hevc_ctu.cpp, write mode):
// the layer writes the CABAC syntax for the decisions made here and reconstructs exactly like
// the decoder, so the decoder must reproduce `reconstruction()` bit for bit.
//
// Two decision modes: `coverage` randomises every decision the syntax allows (CU / TU trees,
// all partition modes incl. AMP, the 35 intra modes and 5 chroma modes, PCM, merge indices, AMVP
// predictors and vectors, bi-prediction, transform skip, QP deltas, SAO types and offsets,
// per-slice deblocking / SAO / CABAC-init / merge-list settings), which is what the round-trip
// tests run; otherwise a simple camera encoder (16x16 CUs, SAD motion search seeded with the
// scene's object motion, skip / merge / AMVP / intra choice) for the synthetic camera farm.
#include <cmath>
#include <deque>

#include "avc_scene.h"
#include "bits.h"
#include "hevc_ctu.h"
#include "hevc_recon.h"

namespace vep::hevc {

namespace {

using avc::Rng;
using avc::Scene;
using avc::SceneConfig;

// Orthonormal basis rows of the n-point transform used by the encoder's forward transform.
struct Basis {
  double u[32][32];
};
const Basis& dct_basis(int log2) {
  struct Table {
    Basis b[4];
    Table() {
      for (int l = 0; l < 4; ++l) {
        const int n = 4 << l, step = 32 / n;
        const double s = 1.0 / (64.0 * std::sqrt(double(n)));
        for (int k = 0; k < n; ++k)
          for (int j = 0; j < n; ++j) b[l].u[k][j] = kDct.m[k * step][j] * s;
      }
    }
  };
  static const Table t;  // (thread-safe one-time initialisation: encoders run on many threads)
  return t.b[log2 - 2];
}

// Forward transform + dead-zone quantisation (level = C / Qstep, Qstep = 2^((qp - 4) / 6), times
// m / 16 with a scaling matrix m).
void quantise(const int* res, int log2, bool dst, bool tskip, int qp, bool intra, int* lv, const u8* m) {
  const int n = 1 << log2;
  const double qstep = std::pow(2.0, (qp - 4) / 6.0);
  const double f = intra ? 1.0 / 3 : 1.0 / 6;
  std::vector<double> c(size_t(n) * n);
  if (tskip) {
    for (int k = 0; k < n * n; ++k) c[size_t(k)] = res[k];
  } else {
    double u[32][32];
    if (dst) {
      for (int k = 0; k < 4; ++k)
        for (int j = 0; j < 4; ++j) u[k][j] = kDst4[k][j] / 128.0;
    } else {
      const Basis& b = dct_basis(log2);
      for (int k = 0; k < n; ++k)
        for (int j = 0; j < n; ++j) u[k][j] = b.u[k][j];
    }
    std::vector<double> t(size_t(n) * n);
    for (int k = 0; k < n; ++k)  // t = U R (columns)
      for (int x = 0; x < n; ++x) {
        double a = 0;
        for (int y = 0; y < n; ++y) a += u[k][y] * res[y * n + x];
        t[size_t(k) * n + x] = a;
      }
    for (int k = 0; k < n; ++k)  // C = t U^T (rows: vertical frequency k, horizontal m)
      for (int m = 0; m < n; ++m) {
        double a = 0;
        for (int x = 0; x < n; ++x) a += t[size_t(k) * n + x] * u[m][x];
        c[size_t(k) * n + m] = a;
      }
  }
  for (int k = 0; k < n * n; ++k) {
    const double a = std::fabs(c[size_t(k)]) / (qstep * (m ? m[k] / 16.0 : 1.0)) + f;
    int l = int(std::min(a, 32767.0));
    lv[k] = c[size_t(k)] < 0 ? -l : l;
  }
}

}  // namespace

struct HevcEncoder::Impl : CtuDecider {
  HevcEncConfig cfg;
  Rng rng;
  Scene scene;
  Vps vps;
  Sps sps;
  Pps pps;
  std::vector<u8> vps_nal, sps_nal, pps_nal;
  int W = 0, H = 0;  // coded size
  struct Job {
    i64 disp;
    int type;
    bool ref, idr;
    bool cra = false, rasl = false;  // (open GOPs)
  };
  std::deque<Job> plan;
  std::map<i64, HostSurface> sources;
  i64 next_disp = 0, rendered = -1, coded = 0, idr_disp = 0;
  int cra_poc = -1;  // open GOP: POC of the last CRA until its first trailing picture drops the older anchors
  std::vector<FramePtr> anchors;  // kept reference pictures (coding order)
  int keep_refs = 2;
  PicCtx pc;
  FramePtr cur;
  const HostSurface* cur_src = nullptr;
  int cur_slice = 0, cur_type = kI, cur_qp = 30;
  i64 last_pts = 0;
  char last_type = 'I';
  HostSurface recon_out, src_out;
  std::vector<u16> pcm_buf;
  int bd = 8;                // sample bit depth (Main10: 10)
  FramePtr lt_pic;         // long_term: the GOP's IDR, referenced as a long-term picture
  bool cur_bypass = false; // the CU being coded is lossless (transquant bypass)

  explicit Impl(const HevcEncConfig& c) : cfg(c), rng{c.seed * 0x9E3779B97F4A7C15ull + 4242} {
    VEP_CHECK(c.width >= 16 && c.height >= 16 && c.width % 2 == 0 && c.height % 2 == 0,
              "encoder size must be even and >= 16");
    VEP_CHECK(c.log2_ctb >= 4 && c.log2_ctb <= 6 && c.log2_min_cb == 3, "log2_ctb 4..6, log2_min_cb 3");
    VEP_CHECK(c.bframes >= 0 && c.bframes <= 4 && c.qp >= 0 && c.qp <= 51 && c.gop >= 1, "bad encoder config");
    VEP_CHECK(c.bit_depth >= 8 && c.bit_depth <= 10, "encoder bit depth 8..10");
    VEP_CHECK(!(c.open_gop && c.long_term), "open_gop: the long-term IDR would precede every CRA");
    bd = c.bit_depth;
    W = (c.width + 7) & ~7;
    H = (c.height + 7) & ~7;
    const bool cov = c.coverage;
    sps.width = W;
    sps.height = H;
    sps.conf_right = W - c.width;
    sps.conf_bottom = H - c.height;
    sps.log2_max_poc_lsb = 8;
    sps.log2_ctb = c.log2_ctb;
    sps.log2_min_cb = 3;
    sps.log2_min_tb = 2;
    sps.log2_max_tb = std::min(5, c.log2_ctb);
    sps.max_th_depth_inter = cov ? rng.uni(4) : 1;
    sps.max_th_depth_intra = cov ? rng.uni(4) : 1;
    sps.amp = c.amp;
    sps.sao = c.sao;
    sps.pcm = c.pcm;
    sps.log2_min_pcm = 3;
    sps.log2_max_pcm = std::min(5, c.log2_ctb);
    sps.pcm_loop_filter_disabled = cov ? rng.chance(50) : true;
    sps.bit_depth_luma = sps.bit_depth_chroma = bd;
    sps.pcm_bit_depth_luma = sps.pcm_bit_depth_chroma = 8;
    if (bd > 8) {  // Main10 (general_profile_idc 2); PCM below the sample bit depth in coverage
      sps.ptl.profile_idc = vps.ptl.profile_idc = 2;
      sps.ptl.compat_flags = vps.ptl.compat_flags = 1u << 29;  // general_profile_compatibility_flag[2]
      sps.pcm_bit_depth_luma = cov ? 6 + rng.uni(bd - 5) : bd;
      sps.pcm_bit_depth_chroma = cov ? 6 + rng.uni(bd - 5) : bd;
    }
    sps.temporal_mvp = c.tmvp;
    sps.strong_intra_smoothing = true;
    keep_refs = 2;
    sps.max_dec_pic_buffering = keep_refs + 2;
    sps.max_num_reorder = c.bframes > 0 ? 1 : 0;
    sps.vui = true;
    sps.timing_info = true;
    sps.num_units_in_tick = 1;
    sps.time_scale = u32(c.fps);
    vps.timing_info = true;
    vps.num_units_in_tick = 1;
    vps.time_scale = u32(c.fps);
    pps.sign_data_hiding = c.sign_hiding;
    pps.cabac_init_present = true;
    pps.init_qp = c.qp;
    pps.constrained_intra_pred = cov ? rng.chance(30) : false;
    pps.transform_skip = c.tskip;
    pps.cu_qp_delta = c.cu_qp_delta;
    pps.diff_cu_qp_delta_depth = c.cu_qp_delta ? std::min(1, c.log2_ctb - 3) : 0;
    pps.cb_qp_offset = cov ? rng.uni(7) - 3 : 0;
    pps.cr_qp_offset = cov ? rng.uni(7) - 3 : 0;
    pps.slice_chroma_qp_offsets_present = cov;
    pps.loop_filter_across_slices = true;
    pps.deblocking_override_enabled = cov;
    pps.deblocking_disabled = !c.deblock;
    pps.beta_offset = cov ? 2 * (rng.uni(5) - 2) : 0;
    pps.tc_offset = cov ? 2 * (rng.uni(5) - 2) : 0;
    pps.log2_parallel_merge_level = cov && rng.chance(40) ? 3 : 2;
    setup_tools(c);
    auto nal = [](const std::vector<u8>& rbsp, std::vector<u8>& out) { rbsp_to_ebsp(rbsp.data(), rbsp.size(), out); };
    nal(write_vps(vps), vps_nal);
    nal(write_sps(sps), sps_nal);
    nal(write_pps(pps), pps_nal);
    scene.make(SceneConfig{c.width, c.height, W, H, c.objects, c.noise, c.temporal_noise, c.seed}, rng);
    residual = [this](int ci, int x0, int y0, int log2, const u16* pred, int ps, int qp, bool ts_ok, bool intra, int* lv,
                      bool& ts) { this->make_residual(ci, x0, y0, log2, pred, ps, qp, ts_ok, intra, lv, ts); };
  }

  // Tiles, WPP, dependent segments, scaling lists, weighted prediction, long-term references,
  // transquant bypass (HevcEncConfig); coverage randomises their parameters.
  void setup_tools(const HevcEncConfig& c) {
    const bool cov = c.coverage;
    const int ctb = 1 << c.log2_ctb;
    const int wct = (W + ctb - 1) / ctb, hct = (H + ctb - 1) / ctb;
    pps.tile_cols = std::clamp(c.tile_cols, 1, wct);
    pps.tile_rows = std::clamp(c.tile_rows, 1, hct);
    pps.tiles = pps.tile_cols * pps.tile_rows > 1;
    if (pps.tiles) {
      pps.uniform_spacing = !cov || rng.chance(50);
      if (!pps.uniform_spacing) {
        auto sizes = [&](int count, int total) {
          std::vector<int> v(size_t(count), total / count);
          v.back() += total % count;
          for (int k = 0; k < 2 * count; ++k) {  // move single CTB columns / rows around
            const int a = rng.uni(count), b = rng.uni(count);
            if (a != b && v[size_t(a)] > 1) --v[size_t(a)], ++v[size_t(b)];
          }
          v.pop_back();  // (the last size is implied)
          return v;
        };
        pps.col_width = sizes(pps.tile_cols, wct);
        pps.row_height = sizes(pps.tile_rows, hct);
      }
      pps.loop_filter_across_tiles = !cov || rng.chance(50);
    }
    pps.entropy_coding_sync = c.wpp;
    pps.dependent_slice_segments = c.segments > 1;
    pps.weighted_pred = pps.weighted_bipred = c.weighted;
    pps.transquant_bypass = c.lossless;
    if (c.scaling_lists) {
      sps.scaling_list = true;
      if (cov) {
        auto custom = [&](ScalingList& sl) {
          for (int si = 0; si < 4; ++si)
            for (int m = 0; m < 6; ++m) {
              const int base = 8 + rng.uni(16);
              for (int i = 0; i < 64; ++i) sl.list[si][m][i] = u8(std::clamp(base + i / 3 + rng.uni(9) - 4, 1, 255));
              sl.dc[si][m] = u8(8 + rng.uni(24));
            }
          for (int m = 0; m < 6; ++m)  // (the 32x32 chroma lists are not coded for 4:2:0)
            if (m % 3) std::memcpy(sl.list[3][m], sl.list[2][m], 64), sl.dc[3][m] = sl.dc[2][m];
        };
        sps.scaling_list_data = rng.chance(50);
        if (sps.scaling_list_data) custom(sps.sl);
        pps.scaling_list = rng.chance(50);
        if (pps.scaling_list) custom(pps.sl);
      }
    }
    if (c.long_term) {
      sps.long_term_refs = true;
      if (cov) {  // an SPS candidate list: the IDR (POC 0) and an unused entry
        sps.lt_poc_lsb_sps = {0, 5};
        sps.lt_used_sps = {true, false};
      }
      sps.num_long_term_ref_pics_sps = int(sps.lt_poc_lsb_sps.size());
      sps.max_dec_pic_buffering += 1;
    }
  }

  bool is_idr_pos(i64 d) const { return d == 0 || (d + cfg.idr_phase) % cfg.gop == 0; }

  const HostSurface& source_of(i64 d) {
    while (rendered < d) {
      ++rendered;
      if (rendered > 0) scene.advance();
      scene.render();
      scene.add_sensor_noise(rendered);
      if (bd > 8) {  // 10-bit source: the 8-bit scene << 2 plus a position / time dither in the low bits
        HostSurface& w = sources[rendered];
        w.alloc(scene.src.coded_w, scene.src.coded_h, bd);
        const int sh = bd - 8;
        auto lo = [&](size_t i) { return u16((i * 2654435761u + u64(rendered) * 40503u) >> 29) & ((1u << sh) - 1); };
        for (size_t i = 0; i < w.y16.size(); ++i) w.y16[i] = u16(scene.src.y[i] << sh | lo(i));
        for (size_t i = 0; i < w.uv16.size(); ++i) w.uv16[i] = u16(scene.src.uv[i] << sh | lo(i + 7));
      } else {
        sources[rendered] = scene.src;
      }
    }
    return sources.at(d);
  }

  void plan_next() {
    if (is_idr_pos(next_disp)) {  // (open GOPs: only the stream's first IRAP is an IDR)
      const bool cra = cfg.open_gop && next_disp > 0;
      plan.push_back({next_disp, kI, true, !cra, cra, false});
      ++next_disp;
      return;
    }
    i64 next_idr = next_disp + 1;
    while (!is_idr_pos(next_idr)) ++next_idr;
    if (cfg.open_gop && next_idr - next_disp <= cfg.bframes) {
      // the mini-GOP ends at the next IRAP: a CRA anchors it, and the B pictures before it in
      // display order follow it in decoding order (RASL)
      plan.push_back({next_idr, kI, true, false, true, false});
      for (i64 d = next_disp; d < next_idr; ++d) plan.push_back({d, kB, false, false, false, true});
      next_disp = next_idr + 1;
      return;
    }
    const i64 anchor = std::min<i64>(next_disp + cfg.bframes, next_idr - 1);
    plan.push_back({anchor, kP, true, false});
    for (i64 d = next_disp; d < anchor; ++d) plan.push_back({d, kB, false, false});
    next_disp = anchor + 1;
  }

  // ------------------------------------------------------------------ decisions (CtuDecider)
  bool split(int x0, int y0, int log2) override {
    (void)x0, (void)y0;
    if (cfg.coverage) return rng.chance(log2 == 6 ? 80 : 50);
    return log2 > 4;
  }

  void sao(int rx, int ry, SaoParams& p, bool& ml, bool& mu) override {
    (void)rx, (void)ry;
    p = SaoParams{};
    ml = cfg.coverage && rng.chance(20);
    mu = cfg.coverage && rng.chance(20);
    if (!cfg.coverage) return;
    for (int c = 0; c < 3; ++c) {
      p.type[c] = u8(c == 2 ? p.type[1] : rng.uni(3));
      p.band[c] = u8(rng.uni(32));
      p.eo[c] = u8(c == 2 ? p.eo[1] : rng.uni(4));
      for (int i = 0; i < 4; ++i) {
        const int a = rng.uni(bd > 8 ? 32 : 8);  // (SAO offsets up to 31 at 10 bits)
        p.off[c][i] = i8(p.type[c] == 1 && rng.chance(50) ? -a : a);
      }
    }
  }

  int sad_block(const HostSurface& ref, int x0, int y0, int n, int mvx, int mvy) const {
    int s = 0;
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i) {
        const int rx = std::clamp(x0 + i + mvx, 0, W - 1), ry = std::clamp(y0 + j + mvy, 0, H - 1);
        s += std::abs(cur_src->get(0, x0 + i, y0 + j) - ref.get(0, rx, ry));
      }
    return s;
  }

  void cu(int x0, int y0, int log2, CuDesc& d) override {
    d = CuDesc{};
    const int n = 1 << log2;
    const SliceInfo& sl = pc.slices[size_t(cur_slice)];
    const SliceHeader& sh = sl.sh;
    if (cfg.coverage) {
      coverage_cu(x0, y0, log2, d, sl);
      d.bypass = pps.transquant_bypass && rng.chance(15);
      cur_bypass = d.bypass;
      return;
    }
    cur_bypass = false;
    d.tu_log2 = log2;
    d.chroma_mode = 4;
    d.luma_mode[0] = 0;  // planar
    if (sh.slice_type == kI) {
      d.intra = true;
      return;
    }
    // merge candidates first (skip), then a small motion search per list
    MergeCand mc[5];
    const int nm = merge_candidates(pc, cur_slice, x0, y0, n, x0, y0, n, n, 0, 0, mc);
    int best = INT32_MAX, best_m = -1;
    for (int k = 0; k < nm; ++k) {
      int s = 0;
      if (mc[k].pred == 3) continue;
      const int l = mc[k].pred == 1 ? 0 : 1;
      if (mc[k].mv[l][0] & 3 || mc[k].mv[l][1] & 3) continue;
      s = sad_block(sl.list[l][size_t(mc[k].ref[l])]->s, x0, y0, n, mc[k].mv[l][0] >> 2, mc[k].mv[l][1] >> 2);
      if (s < best) best = s, best_m = k;
    }
    const double qstep = std::pow(2.0, (cur_qp + pc.qp_off_y - 4) / 6.0);  // (SADs at the bit depth)
    if (best_m >= 0 && best < int(n * n * std::max(1.5 * (1 << (bd - 8)), qstep * 0.15))) {
      d.skip = true;
      d.pu[0].merge = true;
      d.pu[0].merge_idx = best_m;
      return;
    }
    int bl = 0, bmv[2] = {0, 0}, bs = INT32_MAX;
    const int nl = sh.slice_type == kB ? 2 : 1;
    for (int l = 0; l < nl; ++l) {
      const HevcFrame& rf = *sl.list[l][0];
      const int dist = pc.poc - rf.poc;
      std::vector<std::pair<int, int>> cands = {{0, 0}};
      for (const Scene::Obj& o : scene.objs) cands.push_back({-int(std::lround(o.vx * dist)), -int(std::lround(o.vy * dist))});
      for (auto [cx, cy] : cands)
        for (int dy = -1; dy <= 1; ++dy)
          for (int dx = -1; dx <= 1; ++dx) {
            const int s = sad_block(rf.s, x0, y0, n, cx + dx, cy + dy);
            if (s < bs) bs = s, bl = l, bmv[0] = cx + dx, bmv[1] = cy + dy;
          }
    }
    if (best_m >= 0 && best <= bs) {
      d.pu[0].merge = true;
      d.pu[0].merge_idx = best_m;
      d.tu_log2 = std::min(log2, 4);
      return;
    }
    if (bs > n * n * (40 << (bd - 8))) {  // nothing matches: intra
      d.intra = true;
      return;
    }
    d.pu[0].dir = bl + 1;
    d.pu[0].ref[bl] = 0;
    d.pu[0].mv[bl][0] = i16(bmv[0] * 4);
    d.pu[0].mv[bl][1] = i16(bmv[1] * 4);
    d.tu_log2 = std::min(log2, 4);
  }

  void coverage_cu(int x0, int y0, int log2, CuDesc& d, const SliceInfo& sl) {
    const SliceHeader& sh = sl.sh;
    const int n = 1 << log2;
    d.tu_log2 = 2 + rng.uni(log2 - 1);
    d.qp_delta = rng.uni(7) - 3;
    d.tskip = rng.chance(30);
    d.chroma_mode = rng.uni(5);
    for (int k = 0; k < 4; ++k) d.luma_mode[k] = rng.uni(35);
    const bool inter_slice = sh.slice_type != kI;
    if (inter_slice && rng.chance(15)) {
      d.skip = true;
      d.pu[0].merge = true;
      d.pu[0].merge_idx = rng.uni(sh.max_num_merge_cand);
      return;
    }
    d.intra = !inter_slice || rng.chance(25);
    if (d.intra) {
      d.part = (log2 == sps.log2_min_cb && rng.chance(40)) ? 3 : 0;
      if (d.part == 0 && sps.pcm && log2 >= sps.log2_min_pcm && log2 <= sps.log2_max_pcm && rng.chance(6)) {
        d.pcm = true;
        pcm_buf.clear();
        const int shy = bd - sps.pcm_bit_depth_luma, shc = bd - sps.pcm_bit_depth_chroma;
        for (int j = 0; j < n; ++j)
          for (int i = 0; i < n; ++i) pcm_buf.push_back(u16(cur_src->get(0, x0 + i, y0 + j) >> shy));
        for (int c = 0; c < 2; ++c)
          for (int j = 0; j < n / 2; ++j)
            for (int i = 0; i < n / 2; ++i) pcm_buf.push_back(u16(cur_src->get(1 + c, x0 / 2 + i, y0 / 2 + j) >> shc));
        d.pcm_samples = pcm_buf.data();
      }
      return;
    }
    // inter partition
    const bool min = log2 == sps.log2_min_cb;
    int opts[8], no = 0;
    opts[no++] = 0;
    opts[no++] = 1;
    opts[no++] = 2;
    if (sps.amp && !min)
      for (int p = 4; p < 8; ++p) opts[no++] = p;
    d.part = opts[rng.uni(no)];
    const int npu = d.part == 0 ? 1 : (d.part == 3 ? 4 : 2);
    const int w = n, h = n;
    for (int k = 0; k < npu; ++k) {
      CuDesc::Pu& p = d.pu[k];
      int pw = w, ph = h;
      if (d.part == 1) ph = h / 2;
      if (d.part == 2) pw = w / 2;
      if (d.part >= 4 && d.part <= 5) ph = (k == 0) == (d.part == 4) ? h / 4 : 3 * h / 4;
      if (d.part >= 6) pw = (k == 0) == (d.part == 6) ? w / 4 : 3 * w / 4;
      p.merge = rng.chance(35);
      p.merge_idx = rng.uni(sh.max_num_merge_cand);
      p.dir = 1;
      if (sh.slice_type == kB) p.dir = (pw + ph == 12) ? 1 + rng.uni(2) : 1 + rng.uni(3);
      for (int l = 0; l < 2; ++l) {
        const int nref = l == 0 ? sh.num_ref_idx_l0 : sh.num_ref_idx_l1;
        p.ref[l] = nref > 0 ? rng.uni(nref) : 0;
        p.mvp[l] = rng.uni(2);
        const Scene::Obj* o = scene.objs.empty() ? nullptr : &scene.objs[size_t(rng.uni(int(scene.objs.size())))];
        const int base_x = o ? int(-o->vx * 4) : 0, base_y = o ? int(-o->vy * 4) : 0;
        p.mv[l][0] = i16(rng.chance(20) ? rng.uni(513) - 256 : base_x + rng.uni(17) - 8);
        p.mv[l][1] = i16(rng.chance(20) ? rng.uni(257) - 128 : base_y + rng.uni(17) - 8);
      }
    }
  }

  // qp: Qp' of the component (QpBdOffset included: the level scale is then bit-depth free)
  void make_residual(int c, int x0, int y0, int log2, const u16* pred, int ps, int qp, bool ts_ok, bool intra, int* lv,
                     bool& ts) {
    const int n = 1 << log2;
    std::vector<int> res(size_t(n) * n);
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i) res[size_t(j) * n + i] = cur_src->get(c, x0 + i, y0 + j) - int(pred[size_t(j) * ps + i]);
    if (cur_bypass) {  // lossless CU: the levels are the residual
      ts = false;
      for (int k = 0; k < n * n; ++k) lv[k] = res[size_t(k)];
      return;
    }
    if (!cfg.coverage) ts = false;
    ts = ts && ts_ok;
    const u8* m = pc.scaling ? pc.sf[log2 - 2][(intra ? 0 : 3) + c].data() : nullptr;
    quantise(res.data(), log2, c == 0 && log2 == 2 && intra, ts, qp, intra, lv, m);
  }

  // ------------------------------------------------------------------ pictures
  // Slice ranges in tile scan: one slice per tile, or slices within the picture (CTB-row
  // aligned with WPP, as §7.4.7.1 requires of a slice that does not start a row).
  std::vector<std::pair<int, int>> plan_slices(int nctb) {
    std::vector<std::pair<int, int>> out;
    if (pps.tiles) {
      if (cfg.slices > 1 || (cfg.coverage && rng.chance(50))) {
        int a = 0;
        for (int ts = 1; ts <= nctb; ++ts)
          if (ts == nctb || pc.first_ctb_in_tile(pc.ts2rs[size_t(ts)])) {
            out.push_back({a, ts});
            a = ts;
          }
      } else {
        out.push_back({0, nctb});
      }
      return out;
    }
    if (pps.entropy_coding_sync) {
      const int nsl = std::clamp(cfg.slices, 1, pc.hctb);
      for (int s = 0; s < nsl; ++s) out.push_back({s * pc.hctb / nsl * pc.wctb, (s + 1) * pc.hctb / nsl * pc.wctb});
      return out;
    }
    const int nsl = std::clamp(cfg.slices, 1, nctb);
    for (int s = 0; s < nsl; ++s) out.push_back({s * nctb / nsl, (s + 1) * nctb / nsl});
    return out;
  }

  // Slice segments of the slice [a, b): the first independent, the others dependent. A segment
  // spanning several tiles holds whole tiles; with WPP segments start at CTB rows.
  std::vector<std::pair<int, int>> plan_segments(int a, int b) {
    const bool multi_tile = pps.tiles && pc.tile[size_t(pc.ts2rs[size_t(a)])] != pc.tile[size_t(pc.ts2rs[size_t(b - 1)])];
    std::vector<int> cand;
    for (int ts = a + 1; ts < b; ++ts) {
      const int rs = pc.ts2rs[size_t(ts)];
      if (multi_tile ? pc.first_ctb_in_tile(rs) : (!pps.entropy_coding_sync || pc.ctb_row_start(rs))) cand.push_back(ts);
    }
    const int k = std::min(cfg.segments - 1, int(cand.size()));
    std::vector<std::pair<int, int>> out;
    int prev = a;
    for (int i = 1; i <= k; ++i) {
      const int cut = cand[size_t(i * int(cand.size()) / (k + 1))];
      if (cut <= prev) continue;
      out.push_back({prev, cut});
      prev = cut;
    }
    out.push_back({prev, b});
    return out;
  }

  void make_weights(SliceHeader& sh) {
    const bool cov = cfg.coverage;
    PredWeights& w = sh.pwt;
    w = PredWeights{};
    w.luma_log2_denom = cov ? rng.uni(8) : 6;
    w.chroma_log2_denom = cov ? rng.uni(8) : 6;
    for (int l = 0; l < (sh.slice_type == kB ? 2 : 1); ++l) {
      const int nref = l == 0 ? sh.num_ref_idx_l0 : sh.num_ref_idx_l1;
      for (int i = 0; i < nref; ++i) {
        w.luma_flag[l][i] = !cov || rng.chance(70);
        w.chroma_flag[l][i] = !cov || rng.chance(60);
        const int dl = w.luma_log2_denom, dc = w.chroma_log2_denom;
        w.w[l][i][0] = (1 << dl) + (w.luma_flag[l][i] && cov ? rng.uni(25) - 12 : 0);
        w.o[l][i][0] = w.luma_flag[l][i] && cov ? rng.uni(21) - 10 : 0;
        for (int c = 1; c <= 2; ++c) {
          int wc = (1 << dc) + (w.chroma_flag[l][i] && cov ? rng.uni(17) - 8 : 0);
          const int oc = w.chroma_flag[l][i] && cov ? rng.uni(11) - 5 : 0;
          const int doff = oc - 128 + ((128 * wc) >> dc);
          if (doff < -512 || doff > 511) wc = 1 << dc;  // keep delta_chroma_offset codable
          w.w[l][i][c] = wc;
          w.o[l][i][c] = oc;
        }
      }
    }
  }

  // Emulation-prevented NAL of a slice segment: header (with entry points) + data. The entry
  // point offsets count emulation prevention bytes (§7.4.7.1), which depend on the header: the
  // offsets are iterated to a fixed point.
  std::vector<u8> segment_nal(SliceHeader& sh, const std::vector<u8>& data, const std::vector<size_t>& subs) {
    std::vector<u32> ep;
    for (size_t k = 0; k < subs.size(); ++k) ep.push_back(u32(subs[k] - (k ? subs[k - 1] : 0)));
    std::vector<u8> ebsp;
    for (int iter = 0; iter < 8; ++iter) {
      sh.entry_points = ep;
      BitWriter bw;
      write_slice_header_full(bw, sh, sps, pps);
      std::vector<u8> rb = std::move(bw.buf());
      const size_t hdr = rb.size();
      rb.insert(rb.end(), data.begin(), data.end());
      ebsp.clear();
      std::vector<size_t> pos(rb.size() + 1);
      int zeros = 0;
      for (size_t i = 0; i < rb.size(); ++i) {
        if (zeros >= 2 && rb[i] <= 3) {
          ebsp.push_back(3);
          zeros = 0;
        }
        pos[i] = ebsp.size();
        ebsp.push_back(rb[i]);
        zeros = rb[i] == 0 ? zeros + 1 : 0;
      }
      pos[rb.size()] = ebsp.size();
      std::vector<u32> ep2;
      size_t prev = pos[hdr];
      for (size_t k = 0; k < subs.size(); ++k) {
        const size_t at = pos[hdr + subs[k]];
        ep2.push_back(u32(at - prev));
        prev = at;
      }
      if (ep2 == ep) return ebsp;
      ep = ep2;
    }
    VEP_CHECK(false, "entry point offsets did not converge");
    return ebsp;
  }

  std::shared_ptr<AccessUnit> encode(const Job& job) {
    const int dur = 90000 / std::max(1, cfg.fps);
    if (job.idr) {
      idr_disp = job.disp;
      anchors.clear();
      lt_pic = nullptr;
    }
    const int poc = int(job.disp - idr_disp);
    if (job.cra) cra_poc = poc;
    if (cra_poc >= 0 && !job.cra && !job.rasl) {  // a trailing picture references nothing before its CRA
      anchors.erase(std::remove_if(anchors.begin(), anchors.end(), [&](const FramePtr& f) { return f->poc < cra_poc; }),
                    anchors.end());
      cra_poc = -1;
    }
    cur_src = &source_of(job.disp);
    cur_type = job.type;
    cur = std::make_shared<HevcFrame>();
    cur->s.alloc(W, H, bd);
    cur->poc = poc;
    cur->is_ref = job.ref;
    // reference picture set: every kept anchor; used = the ones this picture predicts from
    std::vector<FramePtr> before, after;
    for (const FramePtr& f : anchors) (f->poc < poc ? before : after).push_back(f);
    std::sort(before.begin(), before.end(), [](const FramePtr& a, const FramePtr& b) { return a->poc > b->poc; });
    std::sort(after.begin(), after.end(), [](const FramePtr& a, const FramePtr& b) { return a->poc < b->poc; });
    ShortTermRps rps;
    rps.num_negative = int(before.size());
    rps.num_positive = int(after.size());
    for (size_t i = 0; i < before.size(); ++i) rps.delta_poc[i] = before[i]->poc - poc, rps.used[i] = true;
    for (size_t i = 0; i < after.size(); ++i)
      rps.delta_poc[before.size() + i] = after[i]->poc - poc, rps.used[before.size() + i] = true;
    if (job.cra)  // an IRAP predicts from nothing: its RPS only keeps the anchors its RASL pictures use
      for (int i = 0; i < rps.num_delta(); ++i) rps.used[i] = false;
    const bool cov = cfg.coverage;
    // the GOP's long-term picture (used unless coverage leaves it in LtFoll for a while)
    std::vector<FramePtr> lt;
    SliceHeader lth;  // long-term fields shared by the picture's slices
    if (lt_pic && !job.idr) {
      const bool used = rps.num_delta() == 0 || !cov || rng.chance(75);
      if (used) lt.push_back(lt_pic);
      const int max_lsb = 1 << sps.log2_max_poc_lsb;
      lth.num_long_term = 1;
      lth.lt_poc_lsb[0] = lt_pic->poc & (max_lsb - 1);
      lth.lt_used[0] = used;
      if (cov && used && sps.num_long_term_ref_pics_sps > 0 && rng.chance(50) &&
          sps.lt_poc_lsb_sps[0] == lth.lt_poc_lsb[0]) {
        lth.num_long_term_sps = 1;
        lth.lt_idx_sps[0] = 0;
      }
      lth.lt_msb_present[0] = cov && rng.chance(50);
      lth.lt_msb_cycle[0] = lth.lt_msb_present[0] ? ((poc - (poc & (max_lsb - 1))) - (lt_pic->poc - lth.lt_poc_lsb[0])) / max_lsb : 0;
    }
    const int total = rps.num_delta() + int(lt.size());
    // slices
    pc.init(sps, pps, &cur->s);
    pc.poc = poc;
    auto au = std::make_shared<AccessUnit>();
    au->codec = Codec::kH265;
    if (job.idr || job.cra) {
      au->add_nal(vps_nal.data(), vps_nal.size());
      au->add_nal(sps_nal.data(), sps_nal.size());
      au->add_nal(pps_nal.data(), pps_nal.size());
    }
    const int nctb = pc.wctb * pc.hctb;
    const std::vector<std::pair<int, int>> slice_ranges = plan_slices(nctb);
    if (slice_ranges.size() > 1) pc.multi = true;
    const int pic_qp = cov ? std::clamp(cfg.qp + rng.uni(21) - 10, 5, 51) : cfg.qp;
    for (size_t s = 0; s < slice_ranges.size(); ++s) {
      const auto [first_ts, end_ts] = slice_ranges[s];
      SliceHeader sh = lth;
      sh.nal_type = job.idr ? kIdrWRadl : job.cra ? kCra : job.rasl ? kRaslN : (job.ref ? kTrailR : kTrailN);
      sh.first_slice_in_pic = s == 0;
      sh.segment_address = pc.ts2rs[size_t(first_ts)];
      sh.slice_type = job.type;
      sh.poc_lsb = poc & 255;
      sh.rps = rps;
      sh.temporal_mvp = sps.temporal_mvp && job.type != kI;
      sh.sao_luma = sps.sao && (!cov || rng.chance(70));
      sh.sao_chroma = sps.sao && (!cov || rng.chance(70));
      if (!cov) sh.sao_luma = sh.sao_chroma = false;
      if (job.type != kI) {
        sh.num_ref_idx_l0 = cov ? 1 + rng.uni(std::max(1, std::min(total, 3))) : 1;
        sh.num_ref_idx_l1 = job.type == kB ? (cov ? 1 + rng.uni(2) : 1) : 0;
        sh.mvd_l1_zero = job.type == kB && cov && rng.chance(30);
        sh.cabac_init = cov && rng.chance(50);
        sh.collocated_from_l0 = job.type != kB || !cov || rng.chance(50);
        const int ncol = sh.collocated_from_l0 ? sh.num_ref_idx_l0 : sh.num_ref_idx_l1;
        sh.collocated_ref_idx = cov ? rng.uni(ncol) : 0;
        sh.max_num_merge_cand = cov ? 1 + rng.uni(5) : 5;
        sh.weighted = pps.weighted_pred;  // (weighted_bipred is set alike)
        if (sh.weighted) make_weights(sh);
      }
      sh.qp_delta = pic_qp - pps.init_qp;
      sh.cb_qp_offset = cov ? rng.uni(5) - 2 : 0;
      sh.cr_qp_offset = cov ? rng.uni(5) - 2 : 0;
      sh.deblocking_disabled = pps.deblocking_disabled;
      sh.beta_offset = pps.beta_offset;
      sh.tc_offset = pps.tc_offset;
      if (cov && pps.deblocking_override_enabled && rng.chance(40)) {
        sh.deblocking_disabled = rng.chance(30);
        sh.beta_offset = sh.deblocking_disabled ? pps.beta_offset : 2 * (rng.uni(13) - 6);
        sh.tc_offset = sh.deblocking_disabled ? pps.tc_offset : 2 * (rng.uni(13) - 6);
      }
      sh.loop_filter_across_slices = !cov || rng.chance(50);
      if (!(pps.loop_filter_across_slices && (sh.sao_luma || sh.sao_chroma || !sh.deblocking_disabled)))
        sh.loop_filter_across_slices = pps.loop_filter_across_slices;
      SliceInfo si;
      si.sh = sh;
      si.qp = pic_qp;
      si.ord = int(s);
      si.addr_rs = sh.segment_address;
      if (job.type != kI) build_lists(sh, before, after, lt, si);
      for (const auto& [sa, sb] : plan_segments(first_ts, end_ts)) {
        SliceInfo seg = si;
        seg.sh.dependent = sa != first_ts;
        seg.sh.segment_address = pc.ts2rs[size_t(sa)];
        seg.sh.first_slice_in_pic = s == 0 && sa == first_ts;
        pc.slices.push_back(seg);
        cur_slice = int(pc.slices.size()) - 1;
        cur_qp = pic_qp;
        std::vector<u8> data;
        std::vector<size_t> subs;
        encode_slice_data(pc, cur_slice, data, *this, sa, sb, &subs);
        const std::vector<u8> nal = segment_nal(pc.slices.back().sh, data, subs);
        au->add_nal(nal.data(), nal.size());
      }
    }
    bool deblock = false, sao_on = false;
    for (const SliceInfo& s : pc.slices) {
      deblock |= !s.sh.deblocking_disabled;
      sao_on |= s.sh.sao_luma || s.sh.sao_chroma;
    }
    if (deblock) deblock_picture(pc);
    if (sao_on) sao_picture(pc);
    if (sps.temporal_mvp) cur->col = build_col(pc, cur->col_w);
    if (job.ref) {
      if (cfg.long_term && job.idr) {
        lt_pic = cur;
      } else {
        anchors.push_back(cur);
        if (int(anchors.size()) > keep_refs) anchors.erase(anchors.begin());
      }
    }
    au->pts = job.disp * dur;
    au->dts = coded * dur - (cfg.bframes > 0 ? dur : 0);
    au->duration = dur;
    au->keyframe = job.idr || job.cra;
    ++coded;
    last_pts = au->pts;
    last_type = job.type == kI ? 'I' : job.type == kP ? 'P' : 'B';
    recon_out = cur->s;
    src_out = *cur_src;
    // sources no longer needed
    while (!sources.empty() && sources.begin()->first < job.disp - 8) sources.erase(sources.begin());
    return au;
  }

  void build_lists(const SliceHeader& sh, const std::vector<FramePtr>& before, const std::vector<FramePtr>& after,
                   const std::vector<FramePtr>& lt, SliceInfo& si) {
    const int total = int(before.size() + after.size() + lt.size());
    VEP_CHECK(total > 0, "inter picture without references");
    for (int l = 0; l < (sh.slice_type == kB ? 2 : 1); ++l) {
      const int nref = l == 0 ? sh.num_ref_idx_l0 : sh.num_ref_idx_l1;
      std::vector<std::pair<FramePtr, bool>> temp;
      const auto& a = l == 0 ? before : after;
      const auto& b = l == 0 ? after : before;
      while (int(temp.size()) < std::max(nref, total)) {
        for (const FramePtr& f : a) temp.push_back({f, false});
        for (const FramePtr& f : b) temp.push_back({f, false});
        for (const FramePtr& f : lt) temp.push_back({f, true});
      }
      for (int i = 0; i < nref; ++i) {
        si.list[l].push_back(temp[size_t(i)].first);
        si.list_poc[l].push_back(temp[size_t(i)].first->poc);
        si.list_lt[l].push_back(u8(temp[size_t(i)].second));
      }
    }
  }

  std::shared_ptr<AccessUnit> next() {
    if (plan.empty()) plan_next();
    const Job j = plan.front();
    plan.pop_front();
    return encode(j);
  }
};

HevcEncoder::HevcEncoder(const HevcEncConfig& cfg) : p_(std::make_unique<Impl>(cfg)) {}
HevcEncoder::~HevcEncoder() = default;
std::shared_ptr<AccessUnit> HevcEncoder::next() { return p_->next(); }
const HostSurface& HevcEncoder::reconstruction() const { return p_->recon_out; }
const HostSurface& HevcEncoder::source() const { return p_->src_out; }
i64 HevcEncoder::last_pts() const { return p_->last_pts; }
char HevcEncoder::last_type() const { return p_->last_type; }
const std::vector<u8>& HevcEncoder::vps_nal() const { return p_->vps_nal; }
const std::vector<u8>& HevcEncoder::sps_nal() const { return p_->sps_nal; }
const std::vector<u8>& HevcEncoder::pps_nal() const { return p_->pps_nal; }

}  // namespace vep::hevc
