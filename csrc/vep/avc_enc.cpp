// Closed-loop synthetic H.264 encoder (CAVLC, I and P slices). See avc.h.
//
// Mode decision is deliberately simple (SAD costs, seeded motion search from the scene's known
// object motion); reconstruction reuses the decoder's own dequantisation, prediction and
// deblocking (avc.cpp), so the encoder's reference pictures are exactly what a decoder of the
// emitted bitstream reconstructs. With `coverage` the decisions are randomised so every
// macroblock type, partition shape, prediction mode, reference index and sub-sample motion
// phase the decoder supports is exercised.
#include <cmath>

#include "avc.h"
#include "avc_cavlc.h"
#include "avc_scene.h"
#include "h264.h"

namespace vep::avc {

namespace {

}  // namespace

struct AvcEncoder::Impl {
  AvcEncConfig cfg;
  Rng rng;
  h264::Sps sps;
  std::vector<u8> sps_nal, pps_nal;
  int W = 0, H = 0, wpx = 0, hpx = 0;
  Scene scene;
  const HostSurface& src = scene.src;
  std::vector<HostSurface> slots;
  struct Ref {
    int slot;
    int frame_num;
  };
  std::vector<Ref> refs;  // most recent first (= list 0 order without modifications)
  Picture pic;
  MbNeighbours nb;
  i64 frame = -1;
  int next_fn = 0, idr_id = -1, gop_pos = 0;
  // per-slice state
  BitWriter* bw = nullptr;
  int slice = 0, qp_run = 0, skip_run = 0, nref = 0;
  bool is_p = false;

  explicit Impl(const AvcEncConfig& c) : cfg(c), rng{c.seed * 0x9E3779B97F4A7C15ull + 12345} {
    VEP_CHECK(c.width >= 16 && c.height >= 16 && c.width % 2 == 0 && c.height % 2 == 0,
              "encoder size must be even and >= 16");
    VEP_CHECK(c.refs >= 1 && c.refs <= 16, "refs must be 1..16");
    VEP_CHECK(c.qp >= 0 && c.qp <= 51, "qp out of range");
    W = (c.width + 15) / 16;
    H = (c.height + 15) / 16;
    wpx = W * 16;
    hpx = H * 16;
    sps.profile_idc = 66;
    sps.constraint_flags = 0xC0;  // constrained baseline
    sps.level_idc = W * H > 8192 ? 51 : 40;
    sps.log2_max_frame_num = 16;
    sps.poc_type = 0;
    sps.log2_max_poc_lsb = 16;
    sps.max_num_ref_frames = c.refs;
    sps.width_mbs = W;
    sps.height_map_units = H;
    sps.crop_right = wpx - c.width;
    sps.crop_bottom = hpx - c.height;
    sps.timing_info = true;
    sps.num_units_in_tick = 1;
    sps.time_scale = u32(2 * c.fps);
    const std::vector<u8> sps_rbsp = h264::write_sps(sps);
    rbsp_to_ebsp(sps_rbsp.data(), sps_rbsp.size(), sps_nal);
    BitWriter pw;
    pw.u(8, 0x68);
    pw.ue(0);
    pw.ue(0);
    pw.u1(0);  // CAVLC
    pw.u1(0);
    pw.ue(0);  // one slice group
    pw.ue(0);
    pw.ue(0);
    pw.u1(0);
    pw.u(2, 0);
    pw.se(0);  // pic_init_qp = 26
    pw.se(0);
    pw.se(c.chroma_qp_offset);
    pw.u1(1);  // deblocking_filter_control_present_flag
    pw.u1(c.constrained_intra ? 1u : 0u);
    pw.u1(0);
    pw.trailing();
    rbsp_to_ebsp(pw.buf().data(), pw.buf().size(), pps_nal);
    slots.resize(size_t(c.refs) + 1);
    for (auto& s : slots) s.alloc(wpx, hpx);
    scene.make(SceneConfig{c.width, c.height, wpx, hpx, c.objects, c.noise, c.temporal_noise, c.seed}, rng);
  }

  // ------------------------------------------------------------------ helpers
  int S(int x, int y) const { return src.y[size_t(y) * wpx + x]; }
  int SC(int x, int y, int c) const { return src.uv[size_t(y) * wpx + 2 * x + c]; }
  HostSurface& T() { return slots[size_t(pic.target)]; }

  // Motion-compensated prediction of one MB (exactly Recon::inter's arithmetic).
  void mc(int mb, const int (*mv)[2], const int* slot8, int* py, int (*pc)[64]) {
    const int mx = mb % W, my = mb / W;
    for (int r = 0; r < 16; ++r) {
      const int bx = r & 3, by = r >> 2;
      const HostSurface& R = slots[size_t(slot8[((by >> 1) << 1) | (bx >> 1)])];
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
          py[(by * 4 + i) * 16 + bx * 4 + j] =
              luma_qpel(R.y.data(), wpx, wpx, hpx, mx * 16 + bx * 4 + j + (mv[r][0] >> 2),
                        my * 16 + by * 4 + i + (mv[r][1] >> 2), mv[r][0] & 3, mv[r][1] & 3);
    }
    for (int c = 0; c < 2; ++c)
      for (int y = 0; y < 8; ++y)
        for (int x = 0; x < 8; ++x) {
          const int r = (y >> 1) * 4 + (x >> 1);
          const HostSurface& R = slots[size_t(slot8[((r >> 3) << 1) | ((r & 3) >> 1)])];
          pc[c][y * 8 + x] = chroma_epel(R.uv.data(), wpx, wpx / 2, hpx / 2, c, mx * 8 + x + (mv[r][0] >> 3),
                                         my * 8 + y + (mv[r][1] >> 3), mv[r][0] & 7, mv[r][1] & 7);
        }
  }

  // Cheap SAD estimate of a 16x16 prediction with one motion vector (16 sample points).
  int sampled_sad(int mb, int slot, int mvx, int mvy) {
    const int mx = mb % W, my = mb / W;
    const HostSurface& R = slots[size_t(slot)];
    int sad = 0;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) {
        const int x = mx * 16 + 2 + 4 * j, y = my * 16 + 2 + 4 * i;
        sad += std::abs(S(x, y) - luma_qpel(R.y.data(), wpx, wpx, hpx, x + (mvx >> 2), y + (mvy >> 2), mvx & 3, mvy & 3));
      }
    return sad * 16;
  }

  int sad16(int mb, const int* py) const {
    const int mx = mb % W, my = mb / W;
    int s = 0;
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) s += std::abs(S(mx * 16 + x, my * 16 + y) - py[y * 16 + x]);
    return s;
  }

  // Transform + quantise one MB's luma/chroma residual against predictions (py: 16x16, pc:
  // 2x 8x8) into scan-order levels. i16: Intra16x16 DC path.
  void quantize(int mb, const int* py, const int (*pc)[64], bool intra, bool i16, int qp, int qpc,
                MbLevels& lv) {
    const int mx = mb % W, my = mb / W;
    std::memset(&lv, 0, sizeof lv);
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
        const int pos = kZigzag4x4[k];
        lv.luma[r][k] = quant(w[pos], qp, mf_class(pos), intra);
      }
    }
    if (i16) {
      // 4x4 Hadamard of the DC terms (spatial), halved, quantised with one extra bit
      int f[16];
      for (int i = 0; i < 4; ++i) {
        const int a = dcw[i * 4], b = dcw[i * 4 + 1], c = dcw[i * 4 + 2], d = dcw[i * 4 + 3];
        f[i * 4] = a + b + c + d;
        f[i * 4 + 1] = a + b - c - d;
        f[i * 4 + 2] = a - b - c + d;
        f[i * 4 + 3] = a - b + c - d;
      }
      int g[16];
      for (int j = 0; j < 4; ++j) {
        const int a = f[j], b = f[4 + j], c = f[8 + j], d = f[12 + j];
        g[j] = a + b + c + d;
        g[4 + j] = a + b - c - d;
        g[8 + j] = a - b - c + d;
        g[12 + j] = a - b + c - d;
      }
      for (int k = 0; k < 16; ++k) lv.dc[k] = quant(g[kZigzag4x4[k]] / 2, qp, 0, true, 1);
    }
    for (int c = 0; c < 2; ++c) {
      int cw[4];
      for (int b = 0; b < 4; ++b) {
        const int bx = (b & 1) * 4, by = (b >> 1) * 4;
        int x[16], w[16];
        for (int i = 0; i < 4; ++i)
          for (int j = 0; j < 4; ++j)
            x[i * 4 + j] = SC(mx * 8 + bx + j, my * 8 + by + i, c) - pc[c][(by + i) * 8 + bx + j];
        fwd4x4(x, w);
        cw[b] = w[0];
        for (int k = 1; k < 16; ++k) {
          const int pos = kZigzag4x4[k];
          lv.cac[c][b][k] = quant(w[pos], qpc, mf_class(pos), intra);
        }
      }
      const int f[4] = {cw[0] + cw[1] + cw[2] + cw[3], cw[0] - cw[1] + cw[2] - cw[3],
                        cw[0] + cw[1] - cw[2] - cw[3], cw[0] - cw[1] - cw[2] + cw[3]};
      for (int b = 0; b < 4; ++b) lv.cdc[c][b] = quant(f[b], qpc, 0, intra, 1);
    }
  }

  static int cbp_of(const MbLevels& lv, bool i16, int& luma, int& chroma) {
    luma = 0;
    for (int r = 0; r < 16; ++r)
      for (int k = i16 ? 1 : 0; k < 16; ++k)
        if (lv.luma[r][k]) luma |= 1 << (raster_to_blk(r) >> 2);
    if (i16 && luma) luma = 15;
    chroma = 0;
    for (int c = 0; c < 2; ++c)
      for (int b = 0; b < 4; ++b) {
        if (lv.cdc[c][b]) chroma = std::max(chroma, 1);
        for (int k = 1; k < 16; ++k)
          if (lv.cac[c][b][k]) chroma = 2;
      }
    return luma | (chroma << 4);
  }

  // Drop levels the chosen coded_block_pattern does not transmit.
  static void apply_cbp(MbLevels& lv, bool i16, int luma, int chroma) {
    for (int r = 0; r < 16; ++r)
      if (!((luma >> (raster_to_blk(r) >> 2)) & 1))
        for (int k = i16 ? 1 : 0; k < 16; ++k) lv.luma[r][k] = 0;
    if (chroma < 2)
      for (auto& c : lv.cac)
        for (auto& b : c)
          for (int& v : b) v = 0;
    if (chroma < 1)
      for (auto& c : lv.cdc)
        for (int& v : c) v = 0;
  }

  void write_residual(int mb, MbState& s, const MbLevels& lv, int cbp_luma, int cbp_chroma) {
    if (s.kind == kI16x16) {
      write_residual_block(*bw, nb.nc_luma(mb, 0), 16, lv.dc);
      for (int idx = 0; idx < 16; ++idx) {
        const int r = blk_to_raster(idx);
        if (cbp_luma) s.tc[r] = u8(write_residual_block(*bw, nb.nc_luma(mb, r), 15, lv.luma[r] + 1));
      }
    } else {
      for (int idx = 0; idx < 16; ++idx) {
        const int r = blk_to_raster(idx);
        if ((cbp_luma >> (idx >> 2)) & 1)
          s.tc[r] = u8(write_residual_block(*bw, nb.nc_luma(mb, r), 16, lv.luma[r]));
      }
    }
    if (cbp_chroma) {
      for (int c = 0; c < 2; ++c) {
        int dc[16] = {lv.cdc[c][0], lv.cdc[c][1], lv.cdc[c][2], lv.cdc[c][3]};
        write_residual_block(*bw, -1, 4, dc);
      }
      if (cbp_chroma & 2)
        for (int c = 0; c < 2; ++c)
          for (int b = 0; b < 4; ++b)
            s.tcc[c][b] = u8(write_residual_block(*bw, nb.nc_chroma(mb, c, b), 15, lv.cac[c][b] + 1));
    }
  }

  MbRec base_rec(const MbState& s) const {
    MbRec m{};
    m.kind = s.kind;
    m.slice = u16(slice);
    m.dbk = u8(cfg.deblock_idc == 1 ? 1 : cfg.deblock_idc == 2 ? 2 : 0);
    m.alpha_off = i8(2 * cfg.alpha_off);
    m.beta_off = i8(2 * cfg.beta_off);
    std::fill(std::begin(m.ref), std::end(m.ref), u8(0xFF));
    std::fill(std::begin(m.ref1), std::end(m.ref1), u8(0xFF));
    return m;
  }

  void finish_mb(int mb, MbRec m, MbState& s, const MbLevels* lv, bool i16, int qp, const u8* pcm) {
    m.qp = m.kind == kIPcm ? 0 : u8(qp);
    m.qpc = u8(chroma_qp(m.qp, cfg.chroma_qp_offset));
    m.qpc2 = m.qpc;
    s.qp = u8(qp);
    MbResidual res;
    if (lv) {
      MbLevels l = *lv;
      l.update_masks();
      dequantize_mb(l, i16, qp, chroma_qp(qp, cfg.chroma_qp_offset), res);
    }
    for (int r = 0; r < 16; ++r) m.i4[r >> 1] |= u8((m.kind == kI4x4 ? s.i4[r] : 0) << ((r & 1) * 4));
    m.nz = 0;
    for (int r = 0; r < 16; ++r) m.nz |= u16(s.tc[r] ? 1u << r : 0u);
    store_mb(pic, mb, m, s, lv ? &res : nullptr, pcm);
    cpu_reconstruct_mb(pic, mb, slots);
  }

  // QP for a coded MB (coverage: random mb_qp_delta).
  int pick_qp() {
    if (!cfg.coverage || !rng.chance(30)) return qp_run;
    return std::min(51, std::max(0, qp_run + rng.uni(9) - 4));
  }

  void write_qp_delta(int qp) {
    int d = qp - qp_run;
    if (d > 25) d -= 52;
    if (d < -26) d += 52;
    bw->se(d);
    qp_run = qp;
  }

  // ------------------------------------------------------------------ intra
  void encode_pcm(int mb, MbState& s) {
    const int mx = mb % W, my = mb / W;
    s.kind = kIPcm;
    std::fill(std::begin(s.tc), std::end(s.tc), u8(16));
    for (auto& c : s.tcc) std::fill(std::begin(c), std::end(c), u8(16));
    u8 raw[kPcmMbBytes];
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) raw[y * 16 + x] = u8(S(mx * 16 + x, my * 16 + y));
    for (int c = 0; c < 2; ++c)
      for (int y = 0; y < 8; ++y)
        for (int x = 0; x < 8; ++x) raw[256 + c * 64 + y * 8 + x] = u8(SC(mx * 8 + x, my * 8 + y, c));
    bw->ue(is_p ? 5 + 25 : 25);
    bw->align_zero();
    bw->bytes(raw, kPcmMbBytes);
    MbRec m = base_rec(s);
    finish_mb(mb, m, s, nullptr, false, qp_run, raw);
  }

  int chroma_mode_for(int mb, bool top, bool left, bool tl, int (*pc)[64]) {
    const int mx = mb % W, my = mb / W;
    int best = 0, best_cost = INT32_MAX;
    const int order[4] = {0, 1, 2, 3};
    int pick = -1;
    if (cfg.coverage) {
      int valid[4], n = 0;
      for (int m : order)
        if (m == 0 || (m == 1 && left) || (m == 2 && top) || (m == 3 && top && left && tl)) valid[n++] = m;
      pick = valid[rng.uni(n)];
    }
    for (int mode : order) {
      if ((mode == 1 && !left) || (mode == 2 && !top) || (mode == 3 && !(top && left && tl))) continue;
      if (pick >= 0 && mode != pick) continue;
      int cost = 0;
      int tmp[2][64];
      for (int c = 0; c < 2; ++c) {
        IntraChromaNb n;
        chroma_neighbours(pic, mb, c, T(), n);
        const PredConst k = mode == 3 ? chroma_plane_const(n) : PredConst{0, 0, 0, 0};
        for (int y = 0; y < 8; ++y)
          for (int x = 0; x < 8; ++x) {
            tmp[c][y * 8 + x] = chroma_pred(n, k, mode, x, y);
            cost += std::abs(SC(mx * 8 + x, my * 8 + y, c) - tmp[c][y * 8 + x]);
          }
      }
      if (cost < best_cost) {
        best_cost = cost;
        best = mode;
        std::memcpy(pc, tmp, sizeof tmp);
      }
    }
    return best;
  }

  // Intra MB (I16x16 or I4x4) decision + coding. Returns after the MB is stored/reconstructed.
  void encode_intra(int mb, MbState& s) {
    const int mx = mb % W, my = mb / W;
    MbRec& cur = pic.mbs[size_t(mb)];
    cur = MbRec{};
    cur.slice = u16(slice);
    cur.kind = kI16x16;
    // ---- Intra 16x16 candidates
    Intra16Nb n16;
    intra16_neighbours(pic, mb, T(), n16);
    int best16 = -1, cost16 = INT32_MAX;
    int py16[256];
    int modes16[4], nm = 0;
    for (int mode = 0; mode < 4; ++mode) {
      if ((mode == 0 && !n16.has_top) || (mode == 1 && !n16.has_left) ||
          (mode == 3 && !(n16.has_top && n16.has_left && n16.has_tl)))
        continue;
      modes16[nm++] = mode;
    }
    const int pick16 = cfg.coverage ? modes16[rng.uni(nm)] : -1;
    for (int k = 0; k < nm; ++k) {
      const int mode = modes16[k];
      if (pick16 >= 0 && mode != pick16) continue;
      const PredConst pk = intra16x16_const(n16, mode);
      int py[256];
      for (int y = 0; y < 16; ++y)
        for (int x = 0; x < 16; ++x) py[y * 16 + x] = intra16x16_pred(n16, pk, mode, x, y);
      const int c = sad16(mb, py);
      if (c < cost16) {
        cost16 = c;
        best16 = mode;
        std::memcpy(py16, py, sizeof py);
      }
    }
    const int qp = pick_qp();
    bool use4 = cfg.coverage ? rng.chance(50) : false;
    // ---- Intra 4x4 (sequential: each block predicts from reconstructed earlier blocks)
    MbLevels lv4;
    std::memset(&lv4, 0, sizeof lv4);
    u8 modes4[16];
    int cost4 = 0;
    if (use4 || !cfg.coverage) {
      cur.kind = kI4x4;
      s.kind = kI4x4;
      for (int idx = 0; idx < 16; ++idx) {
        const int r = blk_to_raster(idx), bx = r & 3, by = r >> 2;
        const int x0 = mx * 16 + bx * 4, y0 = my * 16 + by * 4;
        Intra4Nb n;
        intra4x4_neighbours(pic, mb, idx, T(), n);
        int valid[9], nv = 0;
        for (int mode = 0; mode < 9; ++mode) {
          const bool need_top = mode == 0 || mode == 3 || mode == 7;
          const bool need_left = mode == 1 || mode == 8;
          const bool need_all = mode >= 4 && mode <= 6;
          if ((need_top && !n.has_top) || (need_left && !n.has_left) ||
              (need_all && !(n.has_top && n.has_left && n.has_tl)))
            continue;
          valid[nv++] = mode;
        }
        int best = 2, bc = INT32_MAX, bp[16] = {};
        const int pick = cfg.coverage ? valid[rng.uni(nv)] : -1;
        for (int k = 0; k < nv; ++k) {
          const int mode = valid[k];
          if (pick >= 0 && mode != pick) continue;
          int p[16], c = 0;
          for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
              p[i * 4 + j] = intra4x4_pred(n, mode, j, i);
              c += std::abs(S(x0 + j, y0 + i) - p[i * 4 + j]);
            }
          if (c < bc) {
            bc = c;
            best = mode;
            std::memcpy(bp, p, sizeof p);
          }
        }
        modes4[r] = u8(best);
        cost4 += bc;
        // transform/quantise this block and reconstruct it into the surface right away
        int x[16], w[16];
        for (int i = 0; i < 4; ++i)
          for (int j = 0; j < 4; ++j) x[i * 4 + j] = S(x0 + j, y0 + i) - bp[i * 4 + j];
        fwd4x4(x, w);
        i16 d[16];
        for (int k = 0; k < 16; ++k) {
          const int pos = kZigzag4x4[k];
          lv4.luma[r][k] = quant(w[pos], qp, mf_class(pos), true);
          d[pos] = i16(lv4.luma[r][k] ? dequant4x4(lv4.luma[r][k], qp, pos >> 2, pos & 3) : 0);
        }
        int res[16];
        idct4x4(d, res);
        HostSurface& t = T();
        for (int i = 0; i < 4; ++i)
          for (int j = 0; j < 4; ++j) t.y[size_t(y0 + i) * wpx + x0 + j] = u8(clip1(bp[i * 4 + j] + res[i * 4 + j]));
      }
      cost4 += 6 * 16;  // mode signalling
    }
    if (!cfg.coverage) use4 = cost4 < cost16;
    s.kind = use4 ? kI4x4 : kI16x16;
    cur.kind = s.kind;
    int pc[2][64];
    const int chroma_mode = chroma_mode_for(mb, n16.has_top, n16.has_left, n16.has_tl, pc);
    MbLevels lv;
    if (use4) {
      // luma levels were fixed block by block; chroma residual against its prediction
      MbLevels tmp;
      int dummy[256] = {};
      quantize(mb, dummy, pc, true, false, qp, chroma_qp(qp, cfg.chroma_qp_offset), tmp);
      lv = lv4;
      std::memcpy(lv.cdc, tmp.cdc, sizeof lv.cdc);
      std::memcpy(lv.cac, tmp.cac, sizeof lv.cac);
      for (int r = 0; r < 16; ++r) s.i4[r] = modes4[r];
    } else {
      quantize(mb, py16, pc, true, true, qp, chroma_qp(qp, cfg.chroma_qp_offset), lv);
      std::fill(std::begin(s.i4), std::end(s.i4), u8(2));
    }
    int cl, cc;
    cbp_of(lv, !use4, cl, cc);
    apply_cbp(lv, !use4, cl, cc);
    // ---- syntax
    const int mbt_base = is_p ? 5 : 0;
    if (use4) {
      bw->ue(u32(mbt_base));
      for (int idx = 0; idx < 16; ++idx) {
        const int r = blk_to_raster(idx);
        const int pred = nb.pred_intra4x4(mb, r, cfg.constrained_intra);
        if (s.i4[r] == pred) {
          bw->u1(1);
        } else {
          bw->u1(0);
          bw->u(3, u32(s.i4[r] < pred ? s.i4[r] : s.i4[r] - 1));
        }
      }
      bw->ue(u32(chroma_mode));
      int me = 0;
      while (kCbpIntra[me] != (cl | (cc << 4))) ++me;
      bw->ue(u32(me));
    } else {
      bw->ue(u32(mbt_base + 1 + best16 + 4 * cc + (cl ? 12 : 0)));
      bw->ue(u32(chroma_mode));
    }
    const bool send_qp = !use4 || cl || cc;
    const int qp_used = send_qp ? qp : qp_run;
    if (send_qp) write_qp_delta(qp);
    else if (qp != qp_run) {  // no delta transmitted: levels are all zero, QP unchanged
      std::memset(&lv, 0, sizeof lv);
    }
    write_residual(mb, s, lv, cl, cc);
    MbRec m = base_rec(s);
    m.i16_mode = u8(use4 ? 0 : best16);
    m.chroma_mode = u8(chroma_mode);
    finish_mb(mb, m, s, &lv, !use4, qp_used, nullptr);
  }

  // ------------------------------------------------------------------ inter
  struct Part {
    int x4, y4, w4, h4, shape, ref;
    int mv[2];
  };

  void candidates(int mb, int ref, std::vector<std::pair<int, int>>& out) {
    const int mx = mb % W, my = mb / W;
    out.clear();
    out.push_back({0, 0});
    int p[2];
    nb.pred_mv(mb, 0, 0, 4, 4, 0, ref, 0, 0, p);
    out.push_back({p[0], p[1]});
    for (const Scene::Obj& o : scene.objs) {
      if (o.x > mx * 16 + 16 || o.x + o.w < mx * 16 || o.y > my * 16 + 16 || o.y + o.h < my * 16) continue;
      const int k = ref + 1;  // reference k pictures back (ref pictures are consecutive)
      out.push_back({int(std::lround(-o.vx * 4 * k)), int(std::lround(-o.vy * 4 * k))});
    }
  }

  void encode_inter(int mb, MbState& s) {
    MbRec& cur = pic.mbs[size_t(mb)];
    cur = MbRec{};
    cur.slice = u16(slice);
    cur.kind = kInter;
    s.kind = kInter;
    // ---- motion search (16x16, per reference)
    int best_ref = 0, best_mv[2] = {0, 0}, best_cost = INT32_MAX;
    std::vector<std::pair<int, int>> cand;
    for (int ref = 0; ref < nref; ++ref) {
      const int slot = refs[size_t(ref)].slot;
      candidates(mb, ref, cand);
      for (auto [cx, cy] : cand) {
        const int c = sampled_sad(mb, slot, cx, cy) + 4 * (std::abs(cx) + std::abs(cy)) / 4 + 32 * ref;
        if (c < best_cost) {
          best_cost = c;
          best_ref = ref;
          best_mv[0] = cx;
          best_mv[1] = cy;
        }
      }
      if (!cfg.coverage) break;  // one reference keeps the bench encode fast
    }
    for (int it = 0; it < 2; ++it) {  // +-1 quarter-sample refinement
      int bx = best_mv[0], by = best_mv[1];
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          if (!dx && !dy) continue;
          const int c = sampled_sad(mb, refs[size_t(best_ref)].slot, bx + dx, by + dy) + 32 * best_ref;
          if (c < best_cost) {
            best_cost = c;
            best_mv[0] = bx + dx;
            best_mv[1] = by + dy;
          }
        }
    }
    // ---- partition layout
    int mbt = 0, sub[4] = {0, 0, 0, 0};
    Part parts[16];
    int np = 0;
    int ref8[4] = {best_ref, best_ref, best_ref, best_ref};
    auto jitter = [&](int v) { return cfg.coverage ? v + rng.uni(13) - 6 : v; };
    if (cfg.coverage) {
      mbt = rng.uni(4);
      for (int& r : ref8) r = rng.uni(nref);
    }
    if (mbt == 0) {
      ref8[1] = ref8[2] = ref8[3] = ref8[0];
      parts[np++] = {0, 0, 4, 4, 0, ref8[0], {jitter(best_mv[0]), jitter(best_mv[1])}};
    } else if (mbt == 1) {
      ref8[1] = ref8[0];
      ref8[3] = ref8[2];
      for (int i = 0; i < 2; ++i) parts[np++] = {0, 2 * i, 4, 2, 1, ref8[2 * i], {jitter(best_mv[0]), jitter(best_mv[1])}};
    } else if (mbt == 2) {
      ref8[2] = ref8[0];
      ref8[3] = ref8[1];
      for (int i = 0; i < 2; ++i) parts[np++] = {2 * i, 0, 2, 4, 2, ref8[i], {jitter(best_mv[0]), jitter(best_mv[1])}};
    } else {
      for (int i = 0; i < 4; ++i) {
        sub[i] = rng.uni(4);
        const int x8 = (i & 1) * 2, y8 = (i >> 1) * 2;
        const int cnt = sub[i] == 0 ? 1 : sub[i] == 3 ? 4 : 2;
        for (int j = 0; j < cnt; ++j) {
          Part p{0, 0, 0, 0, 0, ref8[i], {jitter(best_mv[0]), jitter(best_mv[1])}};
          switch (sub[i]) {
            case 0: p.x4 = x8, p.y4 = y8, p.w4 = 2, p.h4 = 2; break;
            case 1: p.x4 = x8, p.y4 = y8 + j, p.w4 = 2, p.h4 = 1; break;
            case 2: p.x4 = x8 + j, p.y4 = y8, p.w4 = 1, p.h4 = 2; break;
            default: p.x4 = x8 + (j & 1), p.y4 = y8 + (j >> 1), p.w4 = 1, p.h4 = 1; break;
          }
          parts[np++] = p;
        }
      }
    }
    // ---- motion vectors in decoding order (predictors depend on earlier partitions)
    for (int i = 0; i < 4; ++i) s.ref[0][i] = i8(ref8[i]);
    int mvd[16][2];
    u16 done = 0;
    int mvs[16][2];
    for (int i = 0; i < np; ++i) {
      Part& p = parts[i];
      int mvp[2];
      nb.pred_mv(mb, p.x4, p.y4, p.w4, p.h4, 0, p.ref, done, p.shape, mvp);
      mvd[i][0] = p.mv[0] - mvp[0];
      mvd[i][1] = p.mv[1] - mvp[1];
      for (int y = p.y4; y < p.y4 + p.h4; ++y)
        for (int x = p.x4; x < p.x4 + p.w4; ++x) {
          s.mv[0][y * 4 + x][0] = i16(p.mv[0]);
          s.mv[0][y * 4 + x][1] = i16(p.mv[1]);
          mvs[y * 4 + x][0] = p.mv[0];
          mvs[y * 4 + x][1] = p.mv[1];
          done |= u16(1u << (y * 4 + x));
        }
    }
    int slot8[4];
    for (int i = 0; i < 4; ++i) slot8[i] = refs[size_t(ref8[i])].slot;
    int py[256], pc[2][64];
    mc(mb, mvs, slot8, py, pc);
    const int qp = pick_qp();
    MbLevels lv;
    quantize(mb, py, pc, false, false, qp, chroma_qp(qp, cfg.chroma_qp_offset), lv);
    int cl, cc;
    cbp_of(lv, false, cl, cc);
    // ---- P_Skip: 16x16, reference 0, the skip predictor, nothing coded
    int skmv[2];
    nb.pskip_mv(mb, skmv);
    const bool skip = mbt == 0 && ref8[0] == 0 && parts[0].mv[0] == skmv[0] && parts[0].mv[1] == skmv[1] &&
                      cl == 0 && cc == 0;
    // ---- intra fallback when the motion search failed badly (occlusions / new content)
    const int inter_sad = sad16(mb, py);
    if (!skip && (cfg.coverage ? rng.chance(10) : inter_sad > 256 * 24)) {
      s = MbState{};
      s.slice = u16(slice);
      bw->ue(u32(skip_run));
      skip_run = 0;
      if (cfg.coverage && rng.chance(cfg.pcm_rate)) encode_pcm(mb, s);
      else encode_intra(mb, s);
      return;
    }
    if (skip) {
      s.kind = kSkip;
      cur.kind = kSkip;
      ++skip_run;
      MbRec m = base_rec(s);
      for (int i = 0; i < 4; ++i) m.ref[i] = u8(slot8[i]);
      finish_mb(mb, m, s, nullptr, false, qp_run, nullptr);
      return;
    }
    apply_cbp(lv, false, cl, cc);
    bw->ue(u32(skip_run));
    skip_run = 0;
    bw->ue(u32(mbt));
    auto write_ref = [&](int r) {
      if (nref == 2) bw->u1(r ? 0u : 1u);
      else if (nref > 2) bw->ue(u32(r));
    };
    if (mbt <= 2) {
      for (int i = 0; i < np; ++i) write_ref(parts[i].ref);
      for (int i = 0; i < np; ++i) {
        bw->se(mvd[i][0]);
        bw->se(mvd[i][1]);
      }
    } else {
      for (int i = 0; i < 4; ++i) bw->ue(u32(sub[i]));
      for (int i = 0; i < 4; ++i) write_ref(ref8[i]);
      for (int i = 0; i < np; ++i) {
        bw->se(mvd[i][0]);
        bw->se(mvd[i][1]);
      }
    }
    int me = 0;
    while (kCbpInter[me] != (cl | (cc << 4))) ++me;
    bw->ue(u32(me));
    int qp_used = qp_run;
    if (cl || cc) {
      write_qp_delta(qp);
      qp_used = qp;
    } else if (qp != qp_run) {
      std::memset(&lv, 0, sizeof lv);
    }
    write_residual(mb, s, lv, cl, cc);
    MbRec m = base_rec(s);
    for (int i = 0; i < 4; ++i) m.ref[i] = u8(slot8[i]);
    finish_mb(mb, m, s, &lv, false, qp_used, nullptr);
  }

  // ------------------------------------------------------------------ picture
  std::shared_ptr<AccessUnit> next() {
    ++frame;
    if (frame > 0) scene.advance();
    scene.render();
    scene.add_sensor_noise(frame);
    const bool idr = frame == 0 || (frame + cfg.idr_phase) % std::max(1, cfg.gop) == 0;
    gop_pos = idr ? 1 : gop_pos + 1;
    if (idr) {
      refs.clear();
      next_fn = 0;
      ++idr_id;
    }
    is_p = !idr;
    const bool ref_pic = idr || !(cfg.coverage && rng.chance(cfg.nonref_rate));
    const int frame_num = next_fn;
    if (ref_pic) next_fn = (next_fn + 1) & 0xFFFF;
    nref = int(refs.size());
    // target slot: one no reference occupies
    int target = 0;
    for (int sl = 0; sl < int(slots.size()); ++sl) {
      bool used = false;
      for (const Ref& r : refs) used |= r.slot == sl;
      if (!used) {
        target = sl;
        break;
      }
    }
    pic = Picture{};
    pic.wmbs = W;
    pic.hmbs = H;
    pic.mbs.assign(size_t(W) * H, MbRec{});
    pic.target = target;
    pic.dpb_slots = int(slots.size());
    pic.constrained_intra = cfg.constrained_intra;
    nb.reset(W, H);
    auto au = std::make_shared<AccessUnit>();
    au->codec = Codec::kH264;
    if (idr) {
      au->add_nal(sps_nal.data(), sps_nal.size());
      au->add_nal(pps_nal.data(), pps_nal.size());
    }
    const int nslices = std::max(1, std::min(cfg.slices, H));
    for (int sidx = 0; sidx < nslices; ++sidx) {
      const int r0 = sidx * H / nslices, r1 = (sidx + 1) * H / nslices;
      BitWriter w;
      bw = &w;
      slice = sidx;
      skip_run = 0;
      qp_run = cfg.qp;
      w.u(8, (ref_pic ? 3u << 5 : 0u) | (idr ? 5u : 1u));
      w.ue(u32(r0 * W));
      w.ue(is_p ? 0u : 2u);
      w.ue(0);
      w.u(16, u32(frame_num));
      if (idr) w.ue(u32(idr_id & 0xFFFF));
      w.u(16, u32((2 * (gop_pos - 1)) & 0xFFFF));
      if (is_p) {
        w.u1(1);  // num_ref_idx_active_override_flag
        w.ue(u32(nref - 1));
        w.u1(0);  // no reference list modification
      }
      if (ref_pic) {
        if (idr) {
          w.u1(0);
          w.u1(0);
        } else {
          w.u1(0);  // sliding window
        }
      }
      w.se(cfg.qp - 26);
      w.ue(u32(cfg.deblock_idc));
      if (cfg.deblock_idc != 1) {
        w.se(cfg.alpha_off);
        w.se(cfg.beta_off);
      }
      for (int mb = r0 * W; mb < r1 * W; ++mb) {
        MbState& s = nb.at(mb);
        s = MbState{};
        s.slice = u16(slice);
        nb.begin(mb);
        if (!is_p) {
          if (cfg.coverage && rng.chance(cfg.pcm_rate)) encode_pcm(mb, s);
          else encode_intra(mb, s);
        } else {
          encode_inter(mb, s);
        }
      }
      if (is_p && skip_run > 0) w.ue(u32(skip_run));
      w.trailing();
      std::vector<u8> e;
      rbsp_to_ebsp(w.buf().data(), w.buf().size(), e);
      au->add_nal(e.data(), e.size());
      bw = nullptr;
    }
    if (pic.deblock) cpu_deblock(pic, T());
    if (ref_pic) {
      if (int(refs.size()) >= cfg.refs) refs.pop_back();  // sliding window: drop the oldest
      refs.insert(refs.begin(), Ref{target, frame_num});
    }
    last_target = target;
    const i64 dur = 90000 / std::max(1, cfg.fps);
    au->pts = au->dts = frame * dur;
    au->duration = dur;
    au->keyframe = idr;
    au->seq = u64(frame);
    return au;
  }
  int last_target = 0;
};

AvcEncoder::AvcEncoder(const AvcEncConfig& cfg) : cfg_(cfg), p_(std::make_unique<Impl>(cfg)) {}
AvcEncoder::~AvcEncoder() = default;
std::shared_ptr<AccessUnit> AvcEncoder::next() { return p_->next(); }
const HostSurface& AvcEncoder::reconstruction() const { return p_->slots[size_t(p_->last_target)]; }
const HostSurface& AvcEncoder::source() const { return p_->src; }
i64 AvcEncoder::last_pts() const { return p_->frame * (90000 / std::max(1, cfg_.fps)); }
const std::vector<u8>& AvcEncoder::sps_nal() const { return p_->sps_nal; }
const std::vector<u8>& AvcEncoder::pps_nal() const { return p_->pps_nal; }

}  // namespace vep::avc
