// HEVC sample reconstruction (CPU reference): intra prediction (§8.4.4.2), motion compensation
// (§8.5.3.3), dequantisation + inverse transforms (§8.6), merge / AMVP candidates (§8.5.3.2),
// the deblocking filter (§8.7.2) and SAO (§8.7.3). See hevc_dec.h.
#include <algorithm>
#include <cstring>

#include "hevc_ctu.h"
#include "hevc_recon.h"

namespace vep::hevc {

// ------------------------------------------------------------------------------ transforms
void inverse_transform(const i32* d, int log2, bool dst, bool tskip, i32* r, int bd) {
  const int n = 1 << log2;
  const int bsh = 20 - bd;  // the final bdShift
  if (tskip) {  // §8.6.4.2: r = d << 7, then bdShift
    for (int k = 0; k < n * n; ++k) r[k] = ((d[k] << 7) + (1 << (bsh - 1))) >> bsh;
    return;
  }
  // basis rows (frequency j, sample i): the n-point DCT is every (32 / n)-th row of the 32-point
  // matrix; |coef| <= 90 and |d| < 2^15, so 32-term sums fit in 32 bits
  const i8* basis[32];
  for (int j = 0; j < n; ++j) basis[j] = dst ? kDst4[j] : kDct.m[j << (5 - log2)];
  // the coded coefficients sit in the top-left corner: bound the work by their extent
  int mx = -1, my = -1;
  for (int y = 0; y < n; ++y)
    for (int x = 0; x < n; ++x)
      if (d[y * n + x]) {
        mx = std::max(mx, x);
        my = y;
      }
  if (mx < 0) {
    std::fill(r, r + n * n, 0);
    return;
  }
  i32 g[32 * 32];
  // first stage (vertical): g[y][x] = clip((sum_j basis[j][y] * d[j][x] + 64) >> 7), columns <= mx
  for (int y = 0; y < n; ++y)
    for (int x = 0; x <= mx; ++x) {
      i32 s = 0;
      for (int j = 0; j <= my; ++j) s += basis[j][y] * d[j * n + x];
      g[y * n + x] = std::clamp((s + 64) >> 7, -32768, 32767);
    }
  // second stage (horizontal): r[y][x] = (sum_j basis[j][x] * g[y][j] + 2^(bsh - 1)) >> bsh
  for (int y = 0; y < n; ++y) {
    const i32* gr = g + y * n;
    for (int x = 0; x < n; ++x) {
      i32 s = 0;
      for (int j = 0; j <= mx; ++j) s += basis[j][x] * gr[j];
      r[y * n + x] = (s + (1 << (bsh - 1))) >> bsh;
    }
  }
}

int dequant_level(int level, int qp, int log2, int m, int bit_depth) {
  static constexpr int kLevelScale[6] = {40, 45, 51, 57, 64, 72};
  const int bd = bit_depth + log2 - 5;  // bdShift
  const i64 v = ((i64(level) * m * kLevelScale[qp % 6]) << (qp / 6)) + (i64(1) << (bd - 1));
  return int(std::clamp<i64>(v >> bd, -32768, 32767));
}

// ------------------------------------------------------------------------------ intra
void intra_predict(const int* top, const int* left, int log2, int mode, bool luma, u16* out, int stride,
                   bool filter_edges, int bd) {
  const int hi = (1 << bd) - 1;
  // top[x + 1] = p[x][-1] (x = -1 .. 2n-1), left[y] = p[-1][y] (y = 0 .. 2n-1)
  const int n = 1 << log2;
  auto P = [&](int x, int y) -> int { return y < 0 ? top[x + 1] : left[y]; };
  if (mode == 0) {  // planar
    for (int y = 0; y < n; ++y)
      for (int x = 0; x < n; ++x)
        out[y * stride + x] = u16(((n - 1 - x) * P(-1, y) + (x + 1) * P(n, -1) + (n - 1 - y) * P(x, -1) +
                                  (y + 1) * P(-1, n) + n) >> (log2 + 1));
    return;
  }
  if (mode == 1) {  // DC
    int sum = n;
    for (int k = 0; k < n; ++k) sum += P(k, -1) + P(-1, k);
    const int dc = sum >> (log2 + 1);
    for (int y = 0; y < n; ++y)
      for (int x = 0; x < n; ++x) out[y * stride + x] = u16(dc);
    if (luma && n < 32 && filter_edges) {
      out[0] = u16((P(-1, 0) + 2 * dc + P(0, -1) + 2) >> 2);
      for (int x = 1; x < n; ++x) out[x] = u16((P(x, -1) + 3 * dc + 2) >> 2);
      for (int y = 1; y < n; ++y) out[y * stride] = u16((P(-1, y) + 3 * dc + 2) >> 2);
    }
    return;
  }
  const int angle = kIntraAngle[mode - 2];
  int refbuf[3 * 64 + 1];
  int* ref = refbuf + 64;  // ref[-n .. 2n]
  if (mode >= 18) {
    for (int x = 0; x <= n; ++x) ref[x] = P(-1 + x, -1);
    if (angle < 0) {
      const int inv = kInvAngle[mode - 11];
      if ((n * angle) >> 5 < -1)
        for (int x = (n * angle) >> 5; x <= -1; ++x) ref[x] = P(-1, -1 + ((x * inv + 128) >> 8));
    } else {
      for (int x = n + 1; x <= 2 * n; ++x) ref[x] = P(-1 + x, -1);
    }
    for (int y = 0; y < n; ++y) {
      const int idx = ((y + 1) * angle) >> 5, fact = ((y + 1) * angle) & 31;
      for (int x = 0; x < n; ++x)
        out[y * stride + x] = u16(fact ? ((32 - fact) * ref[x + idx + 1] + fact * ref[x + idx + 2] + 16) >> 5
                                      : ref[x + idx + 1]);
    }
    if (mode == 26 && luma && n < 32 && filter_edges)
      for (int y = 0; y < n; ++y) out[y * stride] = u16(std::clamp(P(0, -1) + ((P(-1, y) - P(-1, -1)) >> 1), 0, hi));
  } else {
    for (int x = 0; x <= n; ++x) ref[x] = P(-1, -1 + x);
    if (angle < 0) {
      const int inv = kInvAngle[mode - 11];
      if ((n * angle) >> 5 < -1)
        for (int x = (n * angle) >> 5; x <= -1; ++x) ref[x] = P(-1 + ((x * inv + 128) >> 8), -1);
    } else {
      for (int x = n + 1; x <= 2 * n; ++x) ref[x] = P(-1, -1 + x);
    }
    for (int x = 0; x < n; ++x) {
      const int idx = ((x + 1) * angle) >> 5, fact = ((x + 1) * angle) & 31;
      for (int y = 0; y < n; ++y)
        out[y * stride + x] = u16(fact ? ((32 - fact) * ref[y + idx + 1] + fact * ref[y + idx + 2] + 16) >> 5
                                      : ref[y + idx + 1]);
    }
    if (mode == 10 && luma && n < 32 && filter_edges)
      for (int x = 0; x < n; ++x) out[x] = u16(std::clamp(P(-1, 0) + ((P(x, -1) - P(-1, -1)) >> 1), 0, hi));
  }
}

void filter_intra_refs(int* top, int* left, int log2, int mode, bool strong_enabled, int bd) {
  const int lim = 1 << (bd - 5);
  const int n = 1 << log2;
  if (mode == 1 || n == 4) return;
  const int dist = std::min(std::abs(mode - 26), std::abs(mode - 10));
  const int thres = n == 8 ? 7 : n == 16 ? 1 : 0;
  if (!(dist > thres)) return;
  // p[-1][-1] = top[0]; p[x][-1] = top[x + 1]; p[-1][y] = left[y]
  int t[65], l[64];
  const int tl = top[0];
  if (strong_enabled && n == 32 && std::abs(tl + top[2 * n] - 2 * top[n]) < lim &&
      std::abs(tl + left[2 * n - 1] - 2 * left[n - 1]) < lim) {
    t[0] = tl;
    for (int y = 0; y < 63; ++y) l[y] = ((63 - y) * tl + (y + 1) * left[63] + 32) >> 6;
    l[63] = left[63];
    for (int x = 0; x < 63; ++x) t[x + 1] = ((63 - x) * tl + (x + 1) * top[64] + 32) >> 6;
    t[64] = top[64];
  } else {
    t[0] = (left[0] + 2 * tl + top[1] + 2) >> 2;
    for (int y = 0; y < 2 * n - 1; ++y) l[y] = ((y == 0 ? tl : left[y - 1]) + 2 * left[y] + left[y + 1] + 2) >> 2;
    l[2 * n - 1] = left[2 * n - 1];
    for (int x = 0; x < 2 * n - 1; ++x) t[x + 1] = ((x == 0 ? tl : top[x]) + 2 * top[x + 1] + top[x + 2] + 2) >> 2;
    t[2 * n] = top[2 * n];
  }
  std::memcpy(top, t, sizeof(int) * size_t(2 * n + 1));
  std::memcpy(left, l, sizeof(int) * size_t(2 * n));
}

// ------------------------------------------------------------------------------ inter
// 14-bit intermediate prediction samples of one reference sample position (spec form, tests).
int luma_inter_sample(const HostSurface& r, int xi, int yi, int fx, int fy) {
  if (r.wide()) return hk_luma_mc(r.y16.data(), r.coded_w, r.coded_w, r.coded_h, xi, yi, fx, fy, r.bd);
  return hk_luma_mc(r.y.data(), r.coded_w, r.coded_w, r.coded_h, xi, yi, fx, fy);
}
int chroma_inter_sample(const HostSurface& r, int c, int xi, int yi, int fx, int fy) {
  if (r.wide()) return hk_chroma_mc(r.uv16.data(), r.coded_w, r.coded_w / 2, r.coded_h / 2, c, xi, yi, fx, fy, r.bd);
  return hk_chroma_mc(r.uv.data(), r.coded_w, r.coded_w / 2, r.coded_h / 2, c, xi, yi, fx, fy);
}

// 14-bit intermediate prediction of a w x h luma block at integer position (x0, y0) with
// fraction (fx, fy), separable (§8.5.3.3.3.1; shift1 = bd - 8): the (w + 7) x (h + 7) source
// window is read in place when it lies inside the picture, else gathered with edge clamping.
template <class P>
static void mc_luma(const P* plane, int W, int H, int x0, int y0, int w, int h, int fx, int fy, i16* dst, int bd) {
  P win[71 * 71];
  const P* src;
  int ss;
  if (x0 - 3 >= 0 && y0 - 3 >= 0 && x0 + w + 4 <= W && y0 + h + 4 <= H) {
    src = &plane[size_t(y0 - 3) * W + size_t(x0 - 3)];
    ss = W;
  } else {
    ss = w + 7;
    for (int j = 0; j < h + 7; ++j) {
      const size_t row = size_t(std::clamp(y0 - 3 + j, 0, H - 1)) * W;
      for (int i = 0; i < w + 7; ++i) win[j * ss + i] = plane[row + size_t(std::clamp(x0 - 3 + i, 0, W - 1))];
    }
    src = win;
  }
  const int sh1 = bd - 8;
  const i8* fh = kLumaFilter[fx];
  const i8* fv = kLumaFilter[fy];
  if (!fx && !fy) {
    for (int j = 0; j < h; ++j)
      for (int i = 0; i < w; ++i) dst[j * w + i] = i16(src[(j + 3) * ss + i + 3] << (14 - bd));
  } else if (!fy) {
    for (int j = 0; j < h; ++j) {
      const P* p = src + (j + 3) * ss;
      for (int i = 0; i < w; ++i) {
        int s = 0;
        for (int k = 0; k < 8; ++k) s += fh[k] * p[i + k];
        dst[j * w + i] = i16(s >> sh1);
      }
    }
  } else if (!fx) {
    for (int j = 0; j < h; ++j)
      for (int i = 0; i < w; ++i) {
        int s = 0;
        for (int k = 0; k < 8; ++k) s += fv[k] * src[(j + k) * ss + i + 3];
        dst[j * w + i] = i16(s >> sh1);
      }
  } else {
    i16 tmp[71 * 64];
    for (int j = 0; j < h + 7; ++j) {
      const P* p = src + j * ss;
      for (int i = 0; i < w; ++i) {
        int s = 0;
        for (int k = 0; k < 8; ++k) s += fh[k] * p[i + k];
        tmp[j * w + i] = i16(s >> sh1);
      }
    }
    for (int j = 0; j < h; ++j)
      for (int i = 0; i < w; ++i) {
        int s = 0;
        for (int k = 0; k < 8; ++k) s += fv[k] * tmp[(j + k) * w + i];
        dst[j * w + i] = i16(s >> 6);
      }
  }
}

// Same for one chroma component (4-tap, eighth-sample fraction) of the NV12 plane (`uv` of a
// luma-wide stride).
template <class P>
static void mc_chroma(const P* uv, int st, int W, int H, int c, int x0, int y0, int w, int h, int fx, int fy, i16* dst,
                      int bd) {
  P win[35 * 35];
  const int ss = w + 3;
  for (int j = 0; j < h + 3; ++j) {
    const size_t row = size_t(std::clamp(y0 - 1 + j, 0, H - 1)) * st;
    if (x0 - 1 >= 0 && x0 + w + 2 <= W) {
      const P* p = &uv[row + 2 * size_t(x0 - 1) + size_t(c)];
      for (int i = 0; i < w + 3; ++i) win[j * ss + i] = p[2 * i];
    } else {
      for (int i = 0; i < w + 3; ++i) win[j * ss + i] = uv[row + 2 * size_t(std::clamp(x0 - 1 + i, 0, W - 1)) + size_t(c)];
    }
  }
  const int sh1 = bd - 8;
  const i8* fh = kChromaFilter[fx];
  const i8* fv = kChromaFilter[fy];
  if (!fx && !fy) {
    for (int j = 0; j < h; ++j)
      for (int i = 0; i < w; ++i) dst[j * w + i] = i16(win[(j + 1) * ss + i + 1] << (14 - bd));
  } else if (!fy) {
    for (int j = 0; j < h; ++j)
      for (int i = 0; i < w; ++i) {
        const P* p = win + (j + 1) * ss + i;
        dst[j * w + i] = i16((fh[0] * p[0] + fh[1] * p[1] + fh[2] * p[2] + fh[3] * p[3]) >> sh1);
      }
  } else if (!fx) {
    for (int j = 0; j < h; ++j)
      for (int i = 0; i < w; ++i) {
        const P* p = win + j * ss + i + 1;
        dst[j * w + i] = i16((fv[0] * p[0] + fv[1] * p[ss] + fv[2] * p[2 * ss] + fv[3] * p[3 * ss]) >> sh1);
      }
  } else {
    i16 tmp[35 * 32];
    for (int j = 0; j < h + 3; ++j)
      for (int i = 0; i < w; ++i) {
        const P* p = win + j * ss + i;
        tmp[j * w + i] = i16((fh[0] * p[0] + fh[1] * p[1] + fh[2] * p[2] + fh[3] * p[3]) >> sh1);
      }
    for (int j = 0; j < h; ++j)
      for (int i = 0; i < w; ++i) {
        const i16* p = tmp + j * w + i;
        dst[j * w + i] = i16((fv[0] * p[0] + fv[1] * p[w] + fv[2] * p[2 * w] + fv[3] * p[3 * w]) >> 6);
      }
  }
}

static void mc_luma(const HostSurface& r, int x0, int y0, int w, int h, int fx, int fy, i16* dst) {
  if (r.wide()) mc_luma(r.y16.data(), r.coded_w, r.coded_h, x0, y0, w, h, fx, fy, dst, r.bd);
  else mc_luma(r.y.data(), r.coded_w, r.coded_h, x0, y0, w, h, fx, fy, dst, 8);
}
static void mc_chroma(const HostSurface& r, int c, int x0, int y0, int w, int h, int fx, int fy, i16* dst) {
  if (r.wide())
    mc_chroma(r.uv16.data(), r.coded_w, r.coded_w / 2, r.coded_h / 2, c, x0, y0, w, h, fx, fy, dst, r.bd);
  else mc_chroma(r.uv.data(), r.coded_w, r.coded_w / 2, r.coded_h / 2, c, x0, y0, w, h, fx, fy, dst, 8);
}

// Explicit weighting record of one PU (§8.5.3.3.4.3) for the components' bit depths: log2WD =
// denom + 14 - bd, offsets << (bd - 8) (the GPU records carry the same, hevc_ctu.cpp).
GpuWp explicit_weights(const SliceHeader& sh, const MvField& m, int bd_y, int bd_c) {
  GpuWp e{};
  for (int c = 0; c < 3; ++c) {
    const int bd = c ? bd_c : bd_y;
    e.shift[c] = u8(sh.pwt.log2_denom(c) + 14 - bd);
    for (int l = 0; l < 2; ++l)
      if ((m.pred >> l) & 1) {
        e.w[l][c] = i16(sh.pwt.w[l][m.ref[l]][c]);
        e.o[l][c] = i16(sh.pwt.o[l][m.ref[l]][c] * (1 << (bd - 8)));
      }
  }
  return e;
}

void predict_pu(const PicCtx& pc, int si, int xPb, int yPb, int w, int h, const MvField& m, u16* y, int ys, u16* cb,
                u16* cr, int cs) {
  const SliceInfo& sl = pc.slices[size_t(si)];
  const HostSurface* r[2] = {nullptr, nullptr};
  for (int l = 0; l < 2; ++l)
    if (m.pred & (1 << l)) {
      VEP_CHECK(m.ref[l] >= 0 && size_t(m.ref[l]) < sl.list[l].size() && sl.list[l][size_t(m.ref[l])],
                "reference index outside the list");
      r[l] = &sl.list[l][size_t(m.ref[l])]->s;
      VEP_CHECK(r[l]->bd == pc.s->bd, "reference picture of another bit depth");
    }
  const bool bi = r[0] && r[1];
  // explicit weighted prediction (§8.5.3.3.4.3): the slice's weights of the PU's references
  const bool wt = sl.sh.weighted;
  const GpuWp e = wt ? explicit_weights(sl.sh, m, pc.bd_y, pc.bd_c) : GpuWp{};
  const int ul = r[0] ? 0 : 1;  // the list of a uni-predicted PU
  auto fin = [&](int c, int p0, int p1) -> u16 {
    const int bd = c ? pc.bd_c : pc.bd_y;
    return u16(wt ? hk_weight_explicit(e, c, p0, p1, bi, ul, bd) : hk_weight(p0, p1, bi, bd));
  };
  if (!bi && !wt) {  // uni-prediction with a full-sample vector inside the picture: a plain copy
    const int l = r[0] ? 0 : 1;
    const HostSurface& s = *r[l];
    const int mx = m.mv[l][0], my = m.mv[l][1];
    const int xi = xPb + (mx >> 2), yi = yPb + (my >> 2);
    if (!(mx & 7) && !(my & 7) && xi >= 0 && yi >= 0 && xi + w <= s.coded_w && yi + h <= s.coded_h) {
      for (int j = 0; j < h; ++j)
        for (int i = 0; i < w; ++i) y[j * ys + i] = u16(s.get(0, xi + i, yi + j));
      for (int j = 0; j < h / 2; ++j)
        for (int i = 0; i < w / 2; ++i) {
          cb[j * cs + i] = u16(s.get(1, xi / 2 + i, yi / 2 + j));
          cr[j * cs + i] = u16(s.get(2, xi / 2 + i, yi / 2 + j));
        }
      return;
    }
  }
  i16 p[2][64 * 64];
  int np = 0;
  for (int l = 0; l < 2; ++l)
    if (r[l]) mc_luma(*r[l], xPb + (m.mv[l][0] >> 2), yPb + (m.mv[l][1] >> 2), w, h, m.mv[l][0] & 3, m.mv[l][1] & 3, p[np++]);
  for (int j = 0; j < h; ++j)
    for (int i = 0; i < w; ++i) y[j * ys + i] = fin(0, p[0][j * w + i], bi ? p[1][j * w + i] : 0);
  const int xc = xPb / 2, yc = yPb / 2, wc = w / 2, hc = h / 2;
  for (int c = 0; c < 2; ++c) {
    np = 0;
    for (int l = 0; l < 2; ++l)
      if (r[l])
        mc_chroma(*r[l], c, xc + (m.mv[l][0] >> 3), yc + (m.mv[l][1] >> 3), wc, hc, m.mv[l][0] & 7, m.mv[l][1] & 7,
                  p[np++]);
    u16* out = c == 0 ? cb : cr;
    for (int j = 0; j < hc; ++j)
      for (int i = 0; i < wc; ++i) out[j * cs + i] = fin(1 + c, p[0][j * wc + i], bi ? p[1][j * wc + i] : 0);
  }
}

// ------------------------------------------------------------------------------ MV prediction
static bool same_motion(const MvField& a, const MvField& b) {
  if (a.pred != b.pred) return false;
  for (int l = 0; l < 2; ++l)
    if ((a.pred >> l) & 1)
      if (a.ref[l] != b.ref[l] || a.mv[l][0] != b.mv[l][0] || a.mv[l][1] != b.mv[l][1]) return false;
  return true;
}

static i16 scale_mv(int mv, int td, int tb) {
  td = std::clamp(td, -128, 127);
  tb = std::clamp(tb, -128, 127);
  const int tx = (16384 + (std::abs(td) >> 1)) / td;
  const int dsf = std::clamp((tb * tx + 32) >> 6, -4096, 4095);
  const int p = dsf * mv;
  const int v = p >= 0 ? (p + 127) >> 8 : -((-p + 127) >> 8);
  return i16(std::clamp(v, -32768, 32767));
}

// Prediction-block availability (§6.4.2) + not intra.
static bool pb_avail(const PicCtx& pc, int xCb, int yCb, int nCbS, int xPb, int yPb, int nPbW, int nPbH, int partIdx,
                     int xN, int yN) {
  const bool same_cb = xCb <= xN && yCb <= yN && xCb + nCbS > xN && yCb + nCbS > yN;
  bool a;
  if (!same_cb) {
    a = pc.avail(xPb, yPb, xN, yN, pc.done);
  } else {
    a = !((nPbW << 1) == nCbS && (nPbH << 1) == nCbS && partIdx == 1 && yCb + nPbH <= yN && xCb + nPbW > xN);
    if (a) a = pc.done[pc.i4(xN, yN)] != 0;
  }
  if (a && pc.intra[pc.i4(xN, yN)]) a = false;
  return a;
}

// Temporal candidate (§8.5.3.2.8): mv for list X with target refIdx; returns availability.
static bool temporal_mv(const PicCtx& pc, int si, int xPb, int yPb, int nPbW, int nPbH, int X, int refIdx, i16 mv[2]) {
  const SliceInfo& sl = pc.slices[size_t(si)];
  const SliceHeader& sh = sl.sh;
  if (!sh.temporal_mvp) return false;
  const int cl = (sh.slice_type == kB && !sh.collocated_from_l0) ? 1 : 0;
  if (size_t(sh.collocated_ref_idx) >= sl.list[cl].size()) return false;
  const FramePtr& col = sl.list[cl][size_t(sh.collocated_ref_idx)];
  if (!col || !col->col) return false;
  auto fetch = [&](int x, int y, ColMv& out) {
    const size_t k = size_t(y >> 4) * size_t(col->col_w) + size_t(x >> 4);
    if (k >= col->col->size()) return false;
    out = (*col->col)[k];
    return out.pred != 0;
  };
  ColMv c{};
  bool ok = false;
  const int xBr = xPb + nPbW, yBr = yPb + nPbH;
  if ((yPb >> pc.log2ctb) == (yBr >> pc.log2ctb) && yBr < pc.H && xBr < pc.W)
    ok = fetch((xBr >> 4) << 4, (yBr >> 4) << 4, c);
  if (!ok) {
    const int xC = xPb + (nPbW >> 1), yC = yPb + (nPbH >> 1);
    ok = fetch((xC >> 4) << 4, (yC >> 4) << 4, c);
  }
  if (!ok) return false;
  int lc;
  if (!(c.pred & 1)) lc = 1;
  else if (!(c.pred & 2)) lc = 0;
  else {
    bool no_backward = true;  // every reference picture precedes the current one
    for (int l = 0; l < 2; ++l)
      for (int p : sl.list_poc[l]) no_backward &= p <= pc.poc;
    lc = no_backward ? X : (sh.collocated_from_l0 ? 1 : 0);
  }
  // LongTermRefPic of the target and of the collocated vector's reference must agree; a
  // long-term target takes the vector unscaled (§8.5.3.2.8)
  const bool cur_lt = sl.list_lt[X][size_t(refIdx)] != 0;
  if (cur_lt != (((c.lt >> lc) & 1) != 0)) return false;
  const int col_diff = col->poc - c.poc[lc];
  const int cur_diff = pc.poc - sl.list_poc[X][size_t(refIdx)];
  if (cur_lt || col_diff == cur_diff || col_diff == 0) {
    mv[0] = c.mv[lc][0];
    mv[1] = c.mv[lc][1];
  } else {
    mv[0] = scale_mv(c.mv[lc][0], col_diff, cur_diff);
    mv[1] = scale_mv(c.mv[lc][1], col_diff, cur_diff);
  }
  return true;
}

int merge_candidates(const PicCtx& pc, int si, int xCb, int yCb, int nCbS, int xPb, int yPb, int nPbW, int nPbH,
                     int partIdx, int part_mode, MergeCand* out) {
  const SliceInfo& sl = pc.slices[size_t(si)];
  const SliceHeader& sh = sl.sh;
  const int par = pc.pps->log2_parallel_merge_level;
  const int orig_w = nPbW, orig_h = nPbH;
  if (par > 2 && nCbS == 8) {  // single merge candidate list for the whole 8x8 CU
    xPb = xCb;
    yPb = yCb;
    nPbW = nPbH = nCbS;
    partIdx = 0;
  }
  const int maxc = sh.max_num_merge_cand;
  int n = 0;
  MvField cand[5];
  bool loc[5], flg[5];  // availableN (location), availableFlagN (after pruning)
  const int xs[5] = {xPb - 1, xPb + nPbW - 1, xPb + nPbW, xPb - 1, xPb - 1};
  const int ys[5] = {yPb + nPbH - 1, yPb - 1, yPb - 1, yPb + nPbH, yPb - 1};
  for (int k = 0; k < 5; ++k) {  // A1, B1, B0, A0, B2
    loc[k] = false;
    if ((xPb >> par) == (xs[k] >> par) && (yPb >> par) == (ys[k] >> par)) continue;
    if (!pb_avail(pc, xCb, yCb, nCbS, xPb, yPb, nPbW, nPbH, partIdx, xs[k], ys[k])) continue;
    if (k == 0 && partIdx == 1 && (part_mode == 2 || part_mode == 6 || part_mode == 7)) continue;
    if (k == 1 && partIdx == 1 && (part_mode == 1 || part_mode == 4 || part_mode == 5)) continue;
    cand[k] = pc.mf[pc.i4(xs[k], ys[k])];
    loc[k] = true;
  }
  flg[0] = loc[0];
  flg[1] = loc[1] && !(loc[0] && same_motion(cand[0], cand[1]));
  flg[2] = loc[2] && !(loc[1] && same_motion(cand[1], cand[2]));
  flg[3] = loc[3] && !(loc[0] && same_motion(cand[0], cand[3]));
  flg[4] = loc[4] && !(loc[0] && same_motion(cand[0], cand[4])) && !(loc[1] && same_motion(cand[1], cand[4])) &&
           !(flg[0] && flg[1] && flg[2] && flg[3]);
  for (int k = 0; k < 5 && n < maxc; ++k)
    if (flg[k]) {
      out[n] = MergeCand{{{cand[k].mv[0][0], cand[k].mv[0][1]}, {cand[k].mv[1][0], cand[k].mv[1][1]}},
                         {cand[k].ref[0], cand[k].ref[1]}, cand[k].pred};
      ++n;
    }
  if (n > 4) n = 4;  // at most four spatial candidates
  if (n < maxc && sh.temporal_mvp) {
    MergeCand t{{{0, 0}, {0, 0}}, {-1, -1}, 0};
    i16 mv[2];
    if (temporal_mv(pc, si, xPb, yPb, nPbW, nPbH, 0, 0, mv)) {
      t.pred |= 1;
      t.ref[0] = 0;
      t.mv[0][0] = mv[0];
      t.mv[0][1] = mv[1];
    }
    if (sh.slice_type == kB && temporal_mv(pc, si, xPb, yPb, nPbW, nPbH, 1, 0, mv)) {
      t.pred |= 2;
      t.ref[1] = 0;
      t.mv[1][0] = mv[0];
      t.mv[1][1] = mv[1];
    }
    if (t.pred) out[n++] = t;
  }
  const int orig = n;
  if (sh.slice_type == kB && orig > 1 && orig < maxc) {  // combined bi-predictive candidates
    static constexpr u8 k0[12] = {0, 1, 0, 2, 1, 2, 0, 3, 1, 3, 2, 3};
    static constexpr u8 k1[12] = {1, 0, 2, 0, 2, 1, 3, 0, 3, 1, 3, 2};
    for (int c = 0; c < orig * (orig - 1) && n < maxc; ++c) {
      const MergeCand& a = out[k0[c]];
      const MergeCand& b = out[k1[c]];
      if (!(a.pred & 1) || !(b.pred & 2)) continue;
      const bool differ = sl.list[0][size_t(a.ref[0])] != sl.list[1][size_t(b.ref[1])] ||
                          a.mv[0][0] != b.mv[1][0] || a.mv[0][1] != b.mv[1][1];
      if (!differ) continue;
      out[n++] = MergeCand{{{a.mv[0][0], a.mv[0][1]}, {b.mv[1][0], b.mv[1][1]}}, {a.ref[0], b.ref[1]}, 3};
    }
  }
  const int nref = sh.slice_type == kP ? sh.num_ref_idx_l0 : std::min(sh.num_ref_idx_l0, sh.num_ref_idx_l1);
  for (int z = 0; n < maxc; ++z) {
    const i8 r = i8(z < nref ? z : 0);
    out[n++] = sh.slice_type == kP ? MergeCand{{{0, 0}, {0, 0}}, {r, -1}, 1} : MergeCand{{{0, 0}, {0, 0}}, {r, r}, 3};
  }
  if (orig_w + orig_h == 12)  // 8x4 / 4x8: uni-prediction only
    for (int k = 0; k < n; ++k)
      if (out[k].pred == 3) {
        out[k].pred = 1;
        out[k].ref[1] = -1;
      }
  return n;
}

void amvp_candidates(const PicCtx& pc, int si, int xCb, int yCb, int nCbS, int xPb, int yPb, int nPbW, int nPbH,
                     int partIdx, int X, int refIdx, i16 out[2][2]) {
  const SliceInfo& sl = pc.slices[size_t(si)];
  const int Y = 1 - X;
  const FramePtr& target = sl.list[X][size_t(refIdx)];
  const int tpoc = sl.list_poc[X][size_t(refIdx)];
  auto first_pass = [&](const MvField& m, i16 mv[2]) {
    if ((m.pred >> X) & 1 && sl.list[X][size_t(m.ref[X])] == target) {
      mv[0] = m.mv[X][0];
      mv[1] = m.mv[X][1];
      return true;
    }
    if ((m.pred >> Y) & 1 && sl.list[Y][size_t(m.ref[Y])] == target) {
      mv[0] = m.mv[Y][0];
      mv[1] = m.mv[Y][1];
      return true;
    }
    return false;
  };
  const bool tlt = sl.list_lt[X][size_t(refIdx)] != 0;
  auto second_pass = [&](const MvField& m, i16 mv[2]) {
    // a neighbour vector qualifies when its reference's LongTermRefPic equals the target's;
    // only short-term pairs are scaled (§8.5.3.2.7 steps 7 / 8)
    int l = -1;
    if ((m.pred >> X) & 1 && (sl.list_lt[X][size_t(m.ref[X])] != 0) == tlt) l = X;
    else if ((m.pred >> Y) & 1 && (sl.list_lt[Y][size_t(m.ref[Y])] != 0) == tlt) l = Y;
    if (l < 0) return false;
    const int rpoc = sl.list_poc[l][size_t(m.ref[l])];
    if (tlt || rpoc == tpoc) {
      mv[0] = m.mv[l][0];
      mv[1] = m.mv[l][1];
    } else {
      mv[0] = scale_mv(m.mv[l][0], pc.poc - rpoc, pc.poc - tpoc);
      mv[1] = scale_mv(m.mv[l][1], pc.poc - rpoc, pc.poc - tpoc);
    }
    return true;
  };
  // A: A0, A1
  const int ax[2] = {xPb - 1, xPb - 1}, ay[2] = {yPb + nPbH, yPb + nPbH - 1};
  bool availA[2];
  for (int k = 0; k < 2; ++k) availA[k] = pb_avail(pc, xCb, yCb, nCbS, xPb, yPb, nPbW, nPbH, partIdx, ax[k], ay[k]);
  const bool scaled_flag = availA[0] || availA[1];
  i16 mvA[2] = {0, 0}, mvB[2] = {0, 0};
  bool fA = false, fB = false;
  for (int k = 0; k < 2 && !fA; ++k)
    if (availA[k]) fA = first_pass(pc.mf[pc.i4(ax[k], ay[k])], mvA);
  for (int k = 0; k < 2 && !fA; ++k)
    if (availA[k]) fA = second_pass(pc.mf[pc.i4(ax[k], ay[k])], mvA);
  // B: B0, B1, B2
  const int bx[3] = {xPb + nPbW, xPb + nPbW - 1, xPb - 1}, by[3] = {yPb - 1, yPb - 1, yPb - 1};
  bool availB[3];
  for (int k = 0; k < 3; ++k) availB[k] = pb_avail(pc, xCb, yCb, nCbS, xPb, yPb, nPbW, nPbH, partIdx, bx[k], by[k]);
  for (int k = 0; k < 3 && !fB; ++k)
    if (availB[k]) fB = first_pass(pc.mf[pc.i4(bx[k], by[k])], mvB);
  if (!scaled_flag && fB) {
    mvA[0] = mvB[0];
    mvA[1] = mvB[1];
    fA = true;
  }
  if (!scaled_flag) {
    fB = false;
    for (int k = 0; k < 3 && !fB; ++k)
      if (availB[k]) fB = second_pass(pc.mf[pc.i4(bx[k], by[k])], mvB);
  }
  int n = 0;
  i16 list[3][2];
  if (fA) {
    list[n][0] = mvA[0];
    list[n++][1] = mvA[1];
  }
  if (fB && !(fA && mvA[0] == mvB[0] && mvA[1] == mvB[1])) {
    list[n][0] = mvB[0];
    list[n++][1] = mvB[1];
  }
  if (n < 2) {
    i16 t[2];
    if (temporal_mv(pc, si, xPb, yPb, nPbW, nPbH, X, refIdx, t)) {
      list[n][0] = t[0];
      list[n++][1] = t[1];
    }
  }
  while (n < 2) {
    list[n][0] = list[n][1] = 0;
    ++n;
  }
  for (int k = 0; k < 2; ++k) {
    out[k][0] = list[k][0];
    out[k][1] = list[k][1];
  }
}

std::shared_ptr<std::vector<ColMv>> build_col(const PicCtx& pc, int& col_w) {
  col_w = (pc.W + 15) >> 4;
  const int col_h = (pc.H + 15) >> 4;
  auto col = std::make_shared<std::vector<ColMv>>(size_t(col_w) * size_t(col_h));
  for (int y = 0; y < col_h; ++y)
    for (int x = 0; x < col_w; ++x) {
      ColMv& c = (*col)[size_t(y) * size_t(col_w) + size_t(x)];
      const int px = x << 4, py = y << 4;
      const MvField& m = pc.mf[pc.i4(px, py)];
      c = ColMv{{{0, 0}, {0, 0}}, {0, 0}, 0, 0};
      if (pc.intra[pc.i4(px, py)] || !m.pred) continue;
      const int si = pc.slice[size_t(pc.ctb_of(px, py))];
      if (si >= int(pc.slices.size())) continue;
      const SliceInfo& sl = pc.slices[size_t(si)];
      c.pred = m.pred;
      for (int l = 0; l < 2; ++l)
        if ((m.pred >> l) & 1) {
          c.mv[l][0] = m.mv[l][0];
          c.mv[l][1] = m.mv[l][1];
          c.poc[l] = sl.list_poc[l][size_t(m.ref[l])];
          if (sl.list_lt[l][size_t(m.ref[l])]) c.lt |= u8(1 << l);
        }
    }
  return col;
}

// ------------------------------------------------------------------------------ deblocking
static int bs_of(const PicCtx& pc, int xp, int yp, int xq, int yq, bool tu_edge, bool one_slice) {
  const size_t p = pc.i4(xp, yp), q = pc.i4(xq, yq);
  if (pc.intra[p] || pc.intra[q]) return 2;
  if (tu_edge && (pc.cbf[p] || pc.cbf[q])) return 1;
  const MvField& a = pc.mf[p];
  const MvField& b = pc.mf[q];
  // the same motion in one slice segment (same lists): same pictures and vectors
  const int slp = one_slice ? 0 : pc.slice[size_t(pc.ctb_of(xp, yp))];
  const int slq = one_slice ? 0 : pc.slice[size_t(pc.ctb_of(xq, yq))];
  if (std::memcmp(&a, &b, sizeof(MvField)) == 0 && slp == slq) return 0;
  const SliceInfo& sa = pc.slices[size_t(slp)];
  const SliceInfo& sb = pc.slices[size_t(slq)];
  const HevcFrame* ra[2] = {nullptr, nullptr};
  const HevcFrame* rb[2] = {nullptr, nullptr};
  int na = 0, nb = 0;
  for (int l = 0; l < 2; ++l) {
    if ((a.pred >> l) & 1) ra[na++] = sa.list[l][size_t(a.ref[l])].get();
    if ((b.pred >> l) & 1) rb[nb++] = sb.list[l][size_t(b.ref[l])].get();
  }
  if (na != nb) return 1;
  auto far = [](const i16* u, const i16* v) { return std::abs(u[0] - v[0]) >= 4 || std::abs(u[1] - v[1]) >= 4; };
  const i16* ma[2];
  const i16* mb[2];
  {
    int k = 0;
    for (int l = 0; l < 2; ++l)
      if ((a.pred >> l) & 1) ma[k++] = a.mv[l];
    k = 0;
    for (int l = 0; l < 2; ++l)
      if ((b.pred >> l) & 1) mb[k++] = b.mv[l];
  }
  if (na == 1) {
    if (ra[0] != rb[0]) return 1;
    return far(ma[0], mb[0]) ? 1 : 0;
  }
  if (!((ra[0] == rb[0] && ra[1] == rb[1]) || (ra[0] == rb[1] && ra[1] == rb[0]))) return 1;
  if (ra[0] != ra[1]) {
    if (ra[0] == rb[0]) return (far(ma[0], mb[0]) || far(ma[1], mb[1])) ? 1 : 0;
    return (far(ma[0], mb[1]) || far(ma[1], mb[0])) ? 1 : 0;
  }
  return ((far(ma[0], mb[0]) || far(ma[1], mb[1])) && (far(ma[0], mb[1]) || far(ma[1], mb[0]))) ? 1 : 0;
}

void deblock_strengths(const PicCtx& pc, std::vector<u8>& bsv, std::vector<u8>& bsh) {
  const int W = pc.W, H = pc.H;
  bsv.assign(size_t(pc.w4) * pc.h4, 0);
  bsh.assign(size_t(pc.w4) * pc.h4, 0);
  // single-slice, single-tile pictures (the common case) skip every per-edge slice lookup
  const bool one = !pc.multi && pc.slices.size() == 1;
  if (one && pc.slices[0].sh.deblocking_disabled) return;
  const bool tile_edges = pc.col_bd.size() > 2 || pc.row_bd.size() > 2;
  const bool across_tiles = pc.pps->loop_filter_across_tiles;
  // edges lie on the 8x8 grid: vertical ones in every 8th column, horizontal ones in every 8th row
  for (int dir = 0; dir < 2; ++dir) {
    const u8 tu_flag = dir == 0 ? kEdgeTuV : kEdgeTuH, pu_flag = dir == 0 ? kEdgePuV : kEdgePuH;
    std::vector<u8>& out = dir == 0 ? bsv : bsh;
    for (int y = dir == 0 ? 0 : 8; y < H; y += dir == 0 ? 4 : 8) {
      const size_t row = size_t(y >> 2) * size_t(pc.w4);
      const u8* erow = pc.edge.data() + row;
      for (int x = dir == 0 ? 8 : 0; x < W; x += dir == 0 ? 8 : 4) {
        const u8 e = erow[x >> 2];
        if (!(e & (tu_flag | pu_flag))) continue;
        const int xp = dir == 0 ? x - 1 : x, yp = dir == 0 ? y : y - 1;
        if (!one) {
          const size_t cq = size_t(pc.ctb_of(x, y)), cp = size_t(pc.ctb_of(xp, yp));
          const SliceHeader& sh = pc.slices[size_t(pc.slice[cq])].sh;
          if (sh.deblocking_disabled) continue;
          // slice boundary: the current (q) slice's flag decides (§8.7.2.3)
          if (pc.sord[cp] != pc.sord[cq] && !sh.loop_filter_across_slices) continue;
          if (tile_edges && !across_tiles && pc.tile[cp] != pc.tile[cq]) continue;
        }
        out[row + size_t(x >> 2)] = u8(bs_of(pc, xp, yp, x, y, (e & tu_flag) != 0, one));
      }
    }
  }
}

template <class T>
static void deblock_planes(PicCtx& pc, T* Y, T* UV, const std::vector<u8>& bsv, const std::vector<u8>& bsh) {
  const int stride = pc.s->coded_w;
  const int W = pc.W, H = pc.H;
  const int bdy = pc.bd_y, bdc = pc.bd_c, hiy = (1 << bdy) - 1, hic = (1 << bdc) - 1;
  auto qpc = [&](int qpi, int c) {
    return hevc_chroma_qp(qpi + (c == 0 ? pc.pps->cb_qp_offset : pc.pps->cr_qp_offset));  // (no qPi clipping)
  };
  for (int dir = 0; dir < 2; ++dir) {
    const std::vector<u8>& bs = dir == 0 ? bsv : bsh;
    // luma
    for (int y = 0; y < H; y += 4)
      for (int x = 0; x < W; x += 4) {
        const int b = bs[pc.i4(x, y)];
        if (!b) continue;
        const int xp = dir == 0 ? x - 1 : x, yp = dir == 0 ? y : y - 1;
        const int qpP = pc.qp[pc.i4(xp, yp)], qpQ = pc.qp[pc.i4(x, y)];
        const SliceHeader& sh = pc.slices[pc.slice[size_t(pc.ctb_of(x, y))]].sh;
        const int qpl = (qpP + qpQ + 1) >> 1;
        const int beta = kBetaTable[std::clamp(qpl + sh.beta_offset, 0, 51)] * (1 << (bdy - 8));
        const int tc = kTcTable[std::clamp(qpl + 2 * (b - 1) + sh.tc_offset, 0, 53)] * (1 << (bdy - 8));
        const bool nfp = pc.nofilter(pc.i4(xp, yp));
        const bool nfq = pc.nofilter(pc.i4(x, y));
        // sample access: line k (0..3) along the edge, i = distance from the edge (p: -1-i, q: i)
        auto at = [&](int k, int i) -> T& {
          return dir == 0 ? Y[size_t(y + k) * stride + size_t(x + i)] : Y[size_t(y + i) * stride + size_t(x + k)];
        };
        auto P = [&](int k, int i) { return int(at(k, -1 - i)); };
        auto Q = [&](int k, int i) { return int(at(k, i)); };
        const int dp0 = std::abs(P(0, 2) - 2 * P(0, 1) + P(0, 0)), dp3 = std::abs(P(3, 2) - 2 * P(3, 1) + P(3, 0));
        const int dq0 = std::abs(Q(0, 2) - 2 * Q(0, 1) + Q(0, 0)), dq3 = std::abs(Q(3, 2) - 2 * Q(3, 1) + Q(3, 0));
        const int dpq0 = dp0 + dq0, dpq3 = dp3 + dq3, dp = dp0 + dp3, dq = dq0 + dq3, d = dpq0 + dpq3;
        if (d >= beta) continue;
        auto dsam = [&](int k, int dpq) {
          return 2 * dpq < (beta >> 2) && std::abs(P(k, 3) - P(k, 0)) + std::abs(Q(k, 0) - Q(k, 3)) < (beta >> 3) &&
                 std::abs(P(k, 0) - Q(k, 0)) < ((5 * tc + 1) >> 1);
        };
        const bool strong = dsam(0, dpq0) && dsam(3, dpq3);
        const bool dEp = dp < ((beta + (beta >> 1)) >> 3), dEq = dq < ((beta + (beta >> 1)) >> 3);
        for (int k = 0; k < 4; ++k) {
          const int p0 = P(k, 0), p1 = P(k, 1), p2 = P(k, 2), p3 = P(k, 3);
          const int q0 = Q(k, 0), q1 = Q(k, 1), q2 = Q(k, 2), q3 = Q(k, 3);
          if (strong) {
            if (!nfp) {
              at(k, -1) = T(std::clamp((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3, p0 - 2 * tc, p0 + 2 * tc));
              at(k, -2) = T(std::clamp((p2 + p1 + p0 + q0 + 2) >> 2, p1 - 2 * tc, p1 + 2 * tc));
              at(k, -3) = T(std::clamp((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3, p2 - 2 * tc, p2 + 2 * tc));
            }
            if (!nfq) {
              at(k, 0) = T(std::clamp((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3, q0 - 2 * tc, q0 + 2 * tc));
              at(k, 1) = T(std::clamp((p0 + q0 + q1 + q2 + 2) >> 2, q1 - 2 * tc, q1 + 2 * tc));
              at(k, 2) = T(std::clamp((p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3, q2 - 2 * tc, q2 + 2 * tc));
            }
          } else {
            int delta = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4;
            if (std::abs(delta) >= tc * 10) continue;
            delta = std::clamp(delta, -tc, tc);
            if (!nfp) at(k, -1) = T(std::clamp(p0 + delta, 0, hiy));
            if (!nfq) at(k, 0) = T(std::clamp(q0 - delta, 0, hiy));
            if (dEp && !nfp) {
              const int dlt = std::clamp((((p2 + p0 + 1) >> 1) - p1 + delta) >> 1, -(tc >> 1), tc >> 1);
              at(k, -2) = T(std::clamp(p1 + dlt, 0, hiy));
            }
            if (dEq && !nfq) {
              const int dlt = std::clamp((((q2 + q0 + 1) >> 1) - q1 - delta) >> 1, -(tc >> 1), tc >> 1);
              at(k, 1) = T(std::clamp(q1 + dlt, 0, hiy));
            }
          }
        }
      }
    // chroma: bS 2 edges on the 8x8 chroma grid (16 luma samples)
    for (int y = 0; y < H; y += 4)
      for (int x = 0; x < W; x += 4) {
        if ((dir == 0 ? x : y) % 16 != 0) continue;
        const int b = bs[pc.i4(x, y)];
        if (b != 2) continue;
        const int xp = dir == 0 ? x - 1 : x, yp = dir == 0 ? y : y - 1;
        const int qpP = pc.qp[pc.i4(xp, yp)], qpQ = pc.qp[pc.i4(x, y)];
        const SliceHeader& sh = pc.slices[pc.slice[size_t(pc.ctb_of(x, y))]].sh;
        const bool nfp = pc.nofilter(pc.i4(xp, yp));
        const bool nfq = pc.nofilter(pc.i4(x, y));
        for (int c = 0; c < 2; ++c) {
          const int qc = qpc((qpP + qpQ + 1) >> 1, c);
          const int tc = kTcTable[std::clamp(qc + 2 + sh.tc_offset, 0, 53)] * (1 << (bdc - 8));
          const int xc = x / 2, yc = y / 2;
          for (int k = 0; k < 2; ++k) {  // 4 luma lines = 2 chroma lines
            auto at = [&](int i) -> T& {
              return dir == 0 ? UV[size_t(yc + k) * stride + size_t(2 * (xc + i) + c)]
                              : UV[size_t(yc + i) * stride + size_t(2 * (xc + k) + c)];
            };
            const int p0 = at(-1), p1 = at(-2), q0 = at(0), q1 = at(1);
            const int delta = std::clamp((((q0 - p0) * 4) + p1 - q1 + 4) >> 3, -tc, tc);
            if (!nfp) at(-1) = T(std::clamp(p0 + delta, 0, hic));
            if (!nfq) at(0) = T(std::clamp(q0 - delta, 0, hic));
          }
        }
      }
  }
}

void deblock_picture(PicCtx& pc) {
  // bS for every 4-sample edge segment on the 8x8 grid, both directions, before filtering
  std::vector<u8> bsv, bsh;
  deblock_strengths(pc, bsv, bsh);
  HostSurface& s = *pc.s;
  if (s.wide()) deblock_planes(pc, s.y16.data(), s.uv16.data(), bsv, bsh);
  else deblock_planes(pc, s.y.data(), s.uv.data(), bsv, bsh);
}

// ------------------------------------------------------------------------------ SAO
template <class P>
static void sao_planes(PicCtx& pc, const P* SY, const P* SUV, P* DY, P* DUV) {
  const int stride = pc.s->coded_w;
  const int ctb = 1 << pc.log2ctb;
  static constexpr int kHx[4][2] = {{-1, 1}, {0, 0}, {-1, 1}, {1, -1}};
  static constexpr int kVy[4][2] = {{0, 0}, {-1, 1}, {-1, 1}, {-1, 1}};
  for (int ry = 0; ry < pc.hctb; ++ry)
    for (int rx = 0; rx < pc.wctb; ++rx) {
      const int ci = ry * pc.wctb + rx;
      const SaoParams& sp = pc.sao[size_t(ci)];
      const int si = pc.slice[size_t(ci)];
      if (si == 0xFFFF) continue;
      const SliceHeader& sh = pc.slices[size_t(si)].sh;
      const int so = pc.sord[size_t(ci)];
      const bool tiles_cut = (pc.col_bd.size() > 2 || pc.row_bd.size() > 2) && !pc.pps->loop_filter_across_tiles;
      for (int c = 0; c < 3; ++c) {
        if (!sp.type[c] || (c == 0 ? !sh.sao_luma : !sh.sao_chroma)) continue;
        const int sub = c ? 1 : 0;
        const int x0 = (rx * ctb) >> sub, y0 = (ry * ctb) >> sub;
        const int w = std::min(ctb >> sub, (pc.W >> sub) - x0), h = std::min(ctb >> sub, (pc.H >> sub) - y0);
        const int pw = pc.W >> sub, ph = pc.H >> sub;
        const int bd = c ? pc.bd_c : pc.bd_y;
        auto get = [&](int x, int y) -> int {
          return c == 0 ? SY[size_t(y) * stride + x] : SUV[size_t(y) * stride + 2 * x + (c - 1)];
        };
        auto put = [&](int x, int y, int v) {
          if (c == 0) DY[size_t(y) * stride + x] = P(v);
          else DUV[size_t(y) * stride + 2 * x + (c - 1)] = P(v);
        };
        for (int y = y0; y < y0 + h; ++y)
          for (int x = x0; x < x0 + w; ++x) {
            const int lx = x << sub, ly = y << sub;  // luma location of the sample
            if (pc.nofilter(pc.i4(lx, ly))) continue;
            const int v = get(x, y);
            int off = 0;
            if (sp.type[c] == 1) {
              const int band = v >> (bd - 5);
              const int k = (band - sp.band[c]) & 31;
              if (k < 4) off = sp.off[c][k];
            } else {
              const int e = sp.eo[c];
              bool ok = true;
              int sgn = 0;
              for (int t = 0; t < 2 && ok; ++t) {
                const int nx = x + kHx[e][t], ny = y + kVy[e][t];
                if (nx < 0 || ny < 0 || nx >= pw || ny >= ph) {
                  ok = false;
                  break;
                }
                const size_t nc = size_t(pc.ctb_of(nx << sub, ny << sub));
                const int nso = pc.sord[nc];
                if (nso != so) {
                  // the sample that comes later in decoding order decides by its slice's flag
                  const bool nb_later = nso > so;
                  const bool across = nb_later ? pc.slices[size_t(pc.slice[nc])].sh.loop_filter_across_slices
                                               : sh.loop_filter_across_slices;
                  if (!across) {
                    ok = false;
                    break;
                  }
                }
                if (tiles_cut && pc.tile[nc] != pc.tile[size_t(ci)]) {
                  ok = false;
                  break;
                }
                const int nv = get(nx, ny);
                sgn += (v > nv) - (v < nv);
              }
              if (!ok) continue;
              int edge = 2 + sgn;
              if (edge <= 2) edge = edge == 2 ? 0 : edge + 1;
              if (edge) off = sp.off[c][edge - 1];
            }
            if (off) put(x, y, std::clamp(v + off, 0, (1 << bd) - 1));
          }
      }
    }
}

void sao_picture(PicCtx& pc) {
  HostSurface& s = *pc.s;
  const HostSurface src = s;  // deblocked picture: SAO reads it, writes s
  if (s.wide()) sao_planes(pc, src.y16.data(), src.uv16.data(), s.y16.data(), s.uv16.data());
  else sao_planes(pc, src.y.data(), src.uv.data(), s.y.data(), s.uv.data());
}

}  // namespace vep::hevc
