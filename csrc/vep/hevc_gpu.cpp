// HEVC reconstruction records (hevc_kern.h): assembly of a picture's loop-filter inputs after
// parsing in records mode, and the CPU mirror that executes a picture's records with the GPU
// kernels' per-sample functions, in the kernels' pass order. The mirror is the CPU backend of
// the records path and the oracle the kernels are checked against.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>

#include "hevc_ctu.h"
#include "hevc_recon.h"

namespace vep::hevc {

void finish_gpu_picture(PicCtx& pc) {
  GpuPicture& g = *pc.gpu;
  g.width = pc.W;
  g.height = pc.H;
  g.log2ctb = pc.log2ctb;
  g.wctb = pc.wctb;
  g.hctb = pc.hctb;
  g.cb_qp_offset = pc.pps->cb_qp_offset;
  g.cr_qp_offset = pc.pps->cr_qp_offset;
  g.constrained_intra = pc.pps->constrained_intra_pred;
  g.deblock = g.sao = false;
  g.slices.clear();
  for (const SliceInfo& s : pc.slices) {  // one entry per slice (its segments share the fields)
    if (s.ord < int(g.slices.size())) continue;
    g.deblock |= !s.sh.deblocking_disabled;
    g.sao |= s.sh.sao_luma || s.sh.sao_chroma;
    GpuSlice gs{};
    gs.beta_offset = i8(s.sh.beta_offset);
    gs.tc_offset = i8(s.sh.tc_offset);
    gs.across = u8(s.sh.loop_filter_across_slices);
    gs.sao_luma = u8(s.sh.sao_luma);
    gs.sao_chroma = u8(s.sh.sao_chroma);
    g.slices.push_back(gs);
  }
  if (g.deblock) deblock_strengths(pc, g.bs_v, g.bs_h);
  g.qp.assign(pc.qp.begin(), pc.qp.end());
  // samples the loop filters leave alone: PCM (pcm_loop_filter_disabled) and lossless CUs
  g.pcm_nofilter = pc.sps->pcm_loop_filter_disabled || pc.any_bypass;
  g.pcm_map.resize(pc.pcm.size());
  for (size_t k = 0; k < pc.pcm.size(); ++k) g.pcm_map[k] = u8(pc.nofilter(k));
  g.ctb_slice.assign(pc.sord.begin(), pc.sord.end());
  g.ctb_tile.assign(pc.tile.begin(), pc.tile.end());
  g.tiles_block_sao = (pc.col_bd.size() > 2 || pc.row_bd.size() > 2) && !pc.pps->loop_filter_across_tiles;
  g.sao_params.resize(pc.sao.size());
  for (size_t k = 0; k < pc.sao.size(); ++k) {
    const SaoParams& p = pc.sao[k];
    GpuSao& q = g.sao_params[k];
    for (int c = 0; c < 3; ++c) {
      q.type[c] = p.type[c];
      q.band[c] = p.band[c];
      q.eo[c] = p.eo[c];
      for (int i = 0; i < 4; ++i) q.off[c][i] = p.off[c][i];
    }
  }
  // level order: inter residual / PCM (0) first, then the intra levels
  std::stable_sort(g.tus.begin(), g.tus.end(), [](const GpuTu& a, const GpuTu& b) { return a.level < b.level; });
  const int levels = g.tus.empty() ? 0 : g.tus.back().level + 1;
  g.level_begin.assign(size_t(levels) + 1, u32(g.tus.size()));
  for (size_t i = g.tus.size(); i-- > 0;) g.level_begin[g.tus[i].level] = u32(i);
  for (int l = levels - 1; l >= 0; --l)  // empty levels start where the next one does
    if (g.level_begin[size_t(l)] > g.level_begin[size_t(l) + 1]) g.level_begin[size_t(l)] = g.level_begin[size_t(l) + 1];
}

namespace {

// One transform block: residual into `res` (n x n raster).
void tu_residual(const GpuPicture& p, const GpuTu& t, int* res, int bd) {
  const int log2 = t.log2, n = 1 << log2;
  i16 d[32 * 32];
  hk_sparse_expand(p.coefs.data() + t.data, log2, d);
  if (t.flags & kTuBypass) {
    for (int k = 0; k < n * n; ++k) res[k] = d[k];
    return;
  }
  if (t.flags & kTuSkip) {
    for (int k = 0; k < n * n; ++k) res[k] = hk_tskip(d[k], bd);
    return;
  }
  const int mx = t.ext_x, my = t.ext_y;
  const bool dst = t.flags & kTuDst;
  int g[32 * 32];
  for (int y = 0; y < n; ++y)
    for (int x = 0; x <= mx; ++x) g[y * n + x] = hk_itx_col(d, log2, dst, y, x, my);
  for (int y = 0; y < n; ++y)
    for (int x = 0; x < n; ++x) res[y * n + x] = hk_itx_row(g + y * n, log2, dst, x, mx, bd);
}

// the planes of a surface as the sample type of the picture
template <class P> P* yplane(HostSurface& s);
template <class P> P* uvplane(HostSurface& s);
template <> u8* yplane<u8>(HostSurface& s) { return s.y.data(); }
template <> u8* uvplane<u8>(HostSurface& s) { return s.uv.data(); }
template <> u16* yplane<u16>(HostSurface& s) { return s.y16.data(); }
template <> u16* uvplane<u16>(HostSurface& s) { return s.uv16.data(); }

}  // namespace

u64 exchange_violations(const GpuPicture& p) {
  auto key = [](int c, int x, int y) { return u64(c) << 40 | u64(u32(y)) << 20 | u64(u32(x)); };
  std::unordered_map<u64, int> col, row;  // edge word -> level of the block publishing it
  for (const GpuTu& t : p.tus) {
    if (!(t.flags & kTuIntra) || (t.flags & kTuPcm)) continue;
    const int n = 1 << t.log2;
    for (int k = 0; k < n; ++k) {
      col[key(t.c, t.x + n - 1, t.y + k)] = t.level;
      row[key(t.c, t.x + k, t.y + n - 1)] = t.level;
    }
  }
  u64 bad = 0;
  for (const GpuTu& t : p.tus) {
    if (!(t.flags & kTuIntra) || (t.flags & kTuPcm) || !t.pend) continue;
    const int n = 1 << t.log2, g = t.c == 0 ? 4 : 2;
    auto need = [&](const std::unordered_map<u64, int>& m, int x, int y) {
      auto it = m.find(key(t.c, x, y));
      if (it == m.end() || it->second >= t.level) {
        if (bad < 8 && std::getenv("VEP_XG_DEBUG"))
          std::fprintf(stderr, "tu c%d (%d,%d) n%d lvl%d mode%d pend=%llx avail=%llx: word (%d,%d) %s %s lvl %d\n",
                       t.c, t.x, t.y, n, t.level, t.mode, (unsigned long long)t.pend, (unsigned long long)t.avail, x, y,
                       &m == &col ? "col" : "row", it == m.end() ? "missing" : "late", it == m.end() ? -1 : it->second);
        ++bad;
      }
    };
    if (t.pend & 1) {  // the corner: on the covering block's right column or bottom row
      auto a = col.find(key(t.c, t.x - 1, t.y - 1)), b = row.find(key(t.c, t.x - 1, t.y - 1));
      const bool ok = (a != col.end() && a->second < t.level) || (b != row.end() && b->second < t.level);
      if (!ok) need(col, t.x - 1, t.y - 1);
    }
    for (int k = 0; k < 2 * n; ++k) {
      if ((t.pend >> (1 + k / g)) & 1) need(col, t.x - 1, t.y + k);
      if ((t.pend >> (17 + k / g)) & 1) need(row, t.x + k, t.y - 1);
    }
  }
  return bad;
}

template <class P>
static void execute_planes(const GpuPicture& p, std::vector<HostSurface>& slots) {
  HostSurface& s = slots[size_t(p.target)];
  P* const SY = yplane<P>(s);
  P* const SUV = uvplane<P>(s);
  const int bdy = p.bd_y, bdc = p.bd_c;
  const int stride = s.coded_w, W = p.width, H = p.height;
  // pass 1: motion compensation
  for (const GpuPu& u : p.pus) {
    const bool bi = u.pred == 3;
    const GpuWp* wp = u.wp ? &p.wp[size_t(u.wp) - 1] : nullptr;
    const int ul = (u.pred & 1) ? 0 : 1;
    auto fin = [&](int c, int p0, int p1) {
      const int bd = c ? bdc : bdy;
      return P(wp ? hk_weight_explicit(*wp, c, p0, p1, bi, ul, bd) : hk_weight(p0, p1, bi, bd));
    };
    for (int j = 0; j < u.h; ++j)
      for (int i = 0; i < u.w; ++i) {
        int v[2] = {0, 0}, nv = 0;
        for (int l = 0; l < 2; ++l) {
          if (!((u.pred >> l) & 1)) continue;
          const P* r = yplane<P>(slots[size_t(u.slot[l])]);
          v[nv++] = hk_luma_mc(r, stride, W, H, u.x + i + (u.mv[l][0] >> 2), u.y + j + (u.mv[l][1] >> 2),
                               u.mv[l][0] & 3, u.mv[l][1] & 3, bdy);
        }
        SY[size_t(u.y + j) * stride + size_t(u.x + i)] = fin(0, v[0], v[1]);
      }
    for (int c = 0; c < 2; ++c)
      for (int j = 0; j < u.h / 2; ++j)
        for (int i = 0; i < u.w / 2; ++i) {
          int v[2] = {0, 0}, nv = 0;
          for (int l = 0; l < 2; ++l) {
            if (!((u.pred >> l) & 1)) continue;
            const P* r = uvplane<P>(slots[size_t(u.slot[l])]);
            v[nv++] = hk_chroma_mc(r, stride, W / 2, H / 2, c, u.x / 2 + i + (u.mv[l][0] >> 3),
                                   u.y / 2 + j + (u.mv[l][1] >> 3), u.mv[l][0] & 7, u.mv[l][1] & 7, bdc);
          }
          SUV[size_t(u.y / 2 + j) * stride + size_t(u.x + 2 * i + c)] = fin(1 + c, v[0], v[1]);
        }
  }
  // pass 2+: transform blocks by level (0: inter residual and PCM; then intra levels)
  int res[32 * 32];
  for (const GpuTu& t : p.tus) {
    if (t.flags & kTuPcm) {
      const int n = 1 << t.log2, nc = n / 2;
      const P* src = reinterpret_cast<const P*>(p.pcm.data() + t.data);
      for (int y = 0; y < n; ++y)
        for (int x = 0; x < n; ++x) SY[size_t(t.y + y) * stride + t.x + x] = src[y * n + x];
      const P* cb = src + n * n;
      const P* cr = cb + nc * nc;
      for (int y = 0; y < nc; ++y)
        for (int x = 0; x < nc; ++x) {
          SUV[size_t(t.y / 2 + y) * stride + size_t(t.x + 2 * x)] = cb[y * nc + x];
          SUV[size_t(t.y / 2 + y) * stride + size_t(t.x + 2 * x + 1)] = cr[y * nc + x];
        }
      continue;
    }
    const int n = 1 << t.log2;
    P* plane = t.c == 0 ? SY : SUV + (t.c - 1);
    const int step = t.c == 0 ? 1 : 2;
    const int bd = t.c == 0 ? bdy : bdc;
    if (t.flags & kTuIntra) {
      int top[129], left[128];
      hk_prepare_refs(plane, stride, step, t.x, t.y, t.log2, t.c == 0, t.avail, t.mode, t.flags & kTuStrong, top, left,
                      bd);
      for (int y = 0; y < n; ++y)
        for (int x = 0; x < n; ++x)
          plane[(t.y + y) * stride + (t.x + x) * step] = P(hk_intra_sample(top, left, t.log2, t.mode, t.c == 0, x, y, bd));
    }
    if (t.flags & kTuCoef) {
      tu_residual(p, t, res, bd);
      for (int y = 0; y < n; ++y)
        for (int x = 0; x < n; ++x) {
          P& q = plane[(t.y + y) * stride + (t.x + x) * step];
          q = P(hk_clip(int(q) + res[y * n + x], bd));
        }
    }
  }
  // deblocking: every vertical edge, then every horizontal edge
  if (p.deblock) {
    const int w4 = p.w4();
    auto ctb = [&](int x, int y) { return (y >> p.log2ctb) * p.wctb + (x >> p.log2ctb); };
    for (int dir = 0; dir < 2; ++dir) {
      const std::vector<u8>& bs = dir == 0 ? p.bs_v : p.bs_h;
      for (int y = 0; y < H; y += 4)
        for (int x = 0; x < W; x += 4) {
          const int b = bs[size_t(y >> 2) * w4 + size_t(x >> 2)];
          if (!b) continue;
          const int xp = dir == 0 ? x - 1 : x, yp = dir == 0 ? y : y - 1;
          const size_t kp = size_t(yp >> 2) * w4 + size_t(xp >> 2), kq = size_t(y >> 2) * w4 + size_t(x >> 2);
          const GpuSlice& sl = p.slices[p.ctb_slice[size_t(ctb(x, y))]];
          const bool nfp = p.pcm_nofilter && p.pcm_map[kp], nfq = p.pcm_nofilter && p.pcm_map[kq];
          HkLumaEdgeT<P> e{&SY[size_t(y) * stride + size_t(x)], dir == 0 ? stride : 1, dir == 0 ? 1 : stride};
          hk_deblock_luma(e, b, (p.qp[kp] + p.qp[kq] + 1) >> 1, sl.beta_offset, sl.tc_offset, nfp, nfq, bdy);
        }
      for (int y = 0; y < H; y += 4)
        for (int x = 0; x < W; x += 4) {
          if ((dir == 0 ? x : y) % 16 != 0) continue;
          const int b = bs[size_t(y >> 2) * w4 + size_t(x >> 2)];
          if (b != 2) continue;
          const int xp = dir == 0 ? x - 1 : x, yp = dir == 0 ? y : y - 1;
          const size_t kp = size_t(yp >> 2) * w4 + size_t(xp >> 2), kq = size_t(y >> 2) * w4 + size_t(x >> 2);
          const GpuSlice& sl = p.slices[p.ctb_slice[size_t(ctb(x, y))]];
          const bool nfp = p.pcm_nofilter && p.pcm_map[kp], nfq = p.pcm_nofilter && p.pcm_map[kq];
          for (int c = 0; c < 2; ++c) {
            P* q = &SUV[size_t(y / 2) * stride + size_t(x + c)];
            hk_deblock_chroma(q, dir == 0 ? stride : 2, dir == 0 ? 2 : stride, p.qp[kp], p.qp[kq],
                              c == 0 ? p.cb_qp_offset : p.cr_qp_offset, sl.tc_offset, nfp, nfq, bdc);
          }
        }
    }
  }
  // SAO from a copy of the deblocked picture
  if (p.sao) {
    HostSurface src = s;
    const int ctbs = 1 << p.log2ctb;
    for (int ry = 0; ry < p.hctb; ++ry)
      for (int rx = 0; rx < p.wctb; ++rx) {
        const int ci = ry * p.wctb + rx;
        const GpuSao& sp = p.sao_params[size_t(ci)];
        const int si = p.ctb_slice[size_t(ci)];
        const GpuSlice& sl = p.slices[size_t(si)];
        for (int c = 0; c < 3; ++c) {
          if (!sp.type[c] || (c == 0 ? !sl.sao_luma : !sl.sao_chroma)) continue;
          const int sub = c ? 1 : 0, step = c ? 2 : 1;
          const P* splane = c == 0 ? yplane<P>(src) : uvplane<P>(src) + (c - 1);
          P* dplane = c == 0 ? SY : SUV + (c - 1);
          const int bd = c ? bdc : bdy;
          const int pw = W >> sub, ph = H >> sub;
          const int x0 = (rx * ctbs) >> sub, y0 = (ry * ctbs) >> sub;
          const int x1 = std::min(x0 + (ctbs >> sub), pw), y1 = std::min(y0 + (ctbs >> sub), ph);
          for (int y = y0; y < y1; ++y)
            for (int x = x0; x < x1; ++x) {
              if (p.pcm_nofilter && p.pcm_map[size_t((y << sub) >> 2) * p.w4() + size_t((x << sub) >> 2)]) continue;
              auto nb_ok = [&](int nx, int ny) {
                if (nx < 0 || ny < 0 || nx >= pw || ny >= ph) return false;
                const size_t nci = size_t((((ny << sub) >> p.log2ctb) * p.wctb) + ((nx << sub) >> p.log2ctb));
                if (p.tiles_block_sao && p.ctb_tile[nci] != p.ctb_tile[size_t(ci)]) return false;
                const int nsi = p.ctb_slice[nci];
                if (nsi == si) return true;
                return nsi > si ? bool(p.slices[size_t(nsi)].across) : bool(sl.across);
              };
              dplane[y * stride + x * step] = P(hk_sao_sample(splane, stride, step, sp, c, x, y, nb_ok, bd));
            }
        }
      }
  }
}

void cpu_execute(const GpuPicture& p, std::vector<HostSurface>& slots) {
  HostSurface& s = slots[size_t(p.target)];
  const int bd = std::max(p.bd_y, p.bd_c);
  for (HostSurface& h : slots)  // (a CVS with another bit depth: the camera's surfaces follow it)
    if (h.bd != bd) h.alloc(s.coded_w, s.coded_h, bd);
  if (p.wide()) execute_planes<u16>(p, slots);
  else execute_planes<u8>(p, slots);
}

}  // namespace vep::hevc
