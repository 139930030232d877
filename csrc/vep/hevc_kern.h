// Per-sample HEVC reconstruction math shared by the gfx950 kernels (gpu_hevc.hip) and their CPU
// mirror (hevc_gpu.cpp): motion-compensated samples, the two inverse-transform stages, intra
// prediction of one sample from prepared references, the deblocking of one 4-line edge segment
// and one SAO sample. The picture-level record format the CPU parser emits for the GPU
// (GpuPicture) is declared here too. Bit-exact with the CPU decoder (hevc_recon.cpp); the
// equivalence is tested through the CPU mirror (tests/test_hevc_gpu_records.py) and on the GPU
// (tests/test_gpu_hevc.py).
#pragma once

#include <cstdint>
#include <memory>
#include <vector>

#include "common.h"
#include "hevc_tables.h"

#ifdef __HIPCC__
#define VEP_HD __host__ __device__ inline
#else
#define VEP_HD inline
#endif

namespace vep::hevc {

// ---------------------------------------------------------------------------- records
struct GpuPu {    // one prediction block
  u16 x, y;       // luma position
  u8 w, h;        // luma size (4..64)
  u8 pred;        // bit 0 list 0, bit 1 list 1
  u8 wp;          // 0: default weighting, else 1 + index into GpuPicture::wp (explicit weights)
  i8 slot[2];     // DPB surface slot per list (-1 unused)
  i16 mv[2][2];   // quarter-sample luma vectors
};
static_assert(sizeof(GpuPu) == 18, "GpuPu layout");

enum : u8 { kTuIntra = 1, kTuDst = 2, kTuSkip = 4, kTuCoef = 8, kTuPcm = 16, kTuStrong = 32, kTuBypass = 64 };

// Explicit weighted sample prediction of one PU (§8.5.3.3.4.3): per list / component weight and
// offset, log2WD per component.
struct GpuWp {
  i16 w[2][3], o[2][3];
  u8 shift[3];
  u8 pad;
};
static_assert(sizeof(GpuWp) == 28, "GpuWp layout");

struct GpuTu {    // one transform block of one component (or one PCM coding block)
  u16 x, y;       // position in the component's samples
  u8 log2;        // 2..5 (PCM: luma log2 of the CU)
  u8 c;           // 0 Y, 1 Cb, 2 Cr (PCM: 0, covers all three)
  u8 flags;       // kTu*
  u8 mode;        // intra prediction mode (component's)
  u32 data;       // kTuCoef: i16 offset of the block's sparse coefficients (hk_sparse_*; kTuBypass:
                  // the residual itself); kTuPcm: byte offset
  u16 level;      // intra dependency level (0: inter residual / PCM)
  u8 ext_x, ext_y;  // kTuCoef: last column / row holding a non-zero coefficient
  u64 avail;      // intra: reference availability, see hk_prepare_refs
  u64 pend;       // intra: the available units another intra block (level >= 1) writes, which
                  // the GPU reads from that block's published edge (same bit layout as avail)
};
static_assert(sizeof(GpuTu) == 32, "GpuTu layout");

struct GpuSlice {  // per-slice loop-filter parameters
  i8 beta_offset, tc_offset;  // *2 values
  u8 across;                  // slice_loop_filter_across_slices_enabled_flag
  u8 sao_luma, sao_chroma;
  u8 pad[3];
};

struct GpuSao {  // per CTB (SaoParams)
  u8 type[3], band[3], eo[3];
  i8 off[3][4];
};

// A picture's reconstruction work in decoding order, produced by hevc::Decoder in GPU mode.
// Sparse transform-block coefficients (GpuTu::data): n*n/16 mask words (u16; word w covers
// raster positions 16w .. 16w + 15, bit set = a stored coefficient), then the stored values in
// raster order. 98% of the dense blocks' entries are zero on the camera streams, which made the
// dense pool 4 MB per 1080p picture (16 MB at 4K) for the parse to zero-fill and the host to copy.
VEP_HD int hk_sparse_words(int log2) { return (1 << (2 * log2)) >> 4; }
// Positions in `pos` (any order, distinct) with their values -> out (words then values); returns
// the entries written. (`pos` / `val` are the non-zero levels of the block.)
inline int hk_sparse_store(int log2, const u16* pos, const i16* val, int n, i16* out) {
  const int nw = hk_sparse_words(log2);
  u16 m[64] = {};
  for (int i = 0; i < n; ++i) m[pos[i] >> 4] |= u16(1u << (pos[i] & 15));
  int before[64];
  for (int w = 0, acc = 0; w < nw; ++w) {
    before[w] = acc;
    acc += __builtin_popcount(u32(m[w]));
    out[w] = i16(m[w]);
  }
  for (int i = 0; i < n; ++i) {
    const int k = pos[i];
    out[nw + before[k >> 4] + __builtin_popcount(u32(m[k >> 4]) & ((1u << (k & 15)) - 1u))] = val[i];
  }
  return nw + n;
}
// The block's coefficients into dense[n * n] (CPU mirror; the GPU expands with the wave).
inline void hk_sparse_expand(const i16* src, int log2, i16* dense) {
  const int nn = 1 << (2 * log2), nw = nn >> 4;
  for (int k = 0; k < nn; ++k) dense[k] = 0;
  const i16* v = src + nw;
  for (int w = 0; w < nw; ++w)
    for (u32 b = u16(src[w]); b; b &= b - 1) dense[16 * w + __builtin_ctz(b)] = *v++;
}

struct GpuPicture {
  int width = 0, height = 0, log2ctb = 4, wctb = 0, hctb = 0;
  int target = 0;                     // DPB slot being reconstructed
  i64 pts = 0, tag = -1;              // of the access unit (output bookkeeping of merged backlogs)
  bool cra = false;                   // a CRA whose RASL pictures predict from earlier pictures
  int cb_qp_offset = 0, cr_qp_offset = 0;
  // sample bit depths (Main10: up to 10; the surfaces then hold one u16 per sample and `pcm`
  // holds the PCM samples as u16, already scaled to the bit depth)
  int bd_y = 8, bd_c = 8;
  bool deblock = false, sao = false, pcm_nofilter = false, constrained_intra = false;
  bool wide() const { return bd_y > 8 || bd_c > 8; }
  std::vector<GpuPu> pus;
  std::vector<GpuTu> tus;             // inter residual / PCM first (level 0), then intra by level
  std::vector<u32> level_begin;       // tus index where each level starts (size levels + 1)
  std::vector<i16> coefs;
  std::vector<u8> pcm;
  // per 4x4 luma block
  std::vector<u8> bs_v, bs_h;         // boundary strength of the left / top edge (0..2)
  std::vector<i8> qp;
  std::vector<u8> pcm_map;            // block whose samples the loop filters must not change
                                      // (PCM with pcm_loop_filter_disabled, transquant bypass)
  std::vector<u8> intra_map;          // (constrained intra prediction) intra block
  std::vector<u8> avail;              // decoded-before flags: see intra reference availability
  std::vector<u16> ctb_slice;         // slice ordinal per CTB
  std::vector<u16> ctb_tile;          // tile id per CTB (SAO across tile boundaries)
  bool tiles_block_sao = false;       // several tiles and loop_filter_across_tiles_enabled_flag 0
  std::vector<GpuSlice> slices;       // per slice ordinal
  std::vector<GpuWp> wp;              // explicit prediction weights (GpuPu::wp)
  std::vector<GpuSao> sao_params;     // per CTB
  int w4() const { return width >> 2; }
  int h4() const { return height >> 2; }
};
using GpuPicturePtr = std::shared_ptr<GpuPicture>;

// ---------------------------------------------------------------------------- inter
// Sample planes are u8 (8-bit streams) or u16 (Main10: one sample per u16, LSB-aligned); `bd` is
// the component's bit depth (8..10). The 8-bit instantiations see bd = 8 as a constant.
// 14-bit intermediate luma sample at integer (xi, yi) + fraction (fx, fy) from a plane with edge
// clamping (§8.5.3.3.3.1): shift1 = bd - 8, shift2 = 6, full samples << (14 - bd).
template <class P>
VEP_HD int hk_luma_at(const P* p, int stride, int W, int H, int x, int y) {
  x = x < 0 ? 0 : (x >= W ? W - 1 : x);
  y = y < 0 ? 0 : (y >= H ? H - 1 : y);
  return p[y * stride + x];
}

template <class P>
VEP_HD int hk_luma_mc(const P* p, int stride, int W, int H, int xi, int yi, int fx, int fy, int bd = 8) {
  const int sh1 = bd - 8;
  if (!fx && !fy) return hk_luma_at(p, stride, W, H, xi, yi) << (14 - bd);
  if (!fy) {
    int s = 0;
    for (int i = 0; i < 8; ++i) s += kLumaFilter[fx][i] * hk_luma_at(p, stride, W, H, xi + i - 3, yi);
    return s >> sh1;
  }
  if (!fx) {
    int s = 0;
    for (int i = 0; i < 8; ++i) s += kLumaFilter[fy][i] * hk_luma_at(p, stride, W, H, xi, yi + i - 3);
    return s >> sh1;
  }
  int s = 0;
  for (int k = 0; k < 8; ++k) {
    int h = 0;
    for (int i = 0; i < 8; ++i) h += kLumaFilter[fx][i] * hk_luma_at(p, stride, W, H, xi + i - 3, yi + k - 3);
    s += kLumaFilter[fy][k] * (h >> sh1);
  }
  return s >> 6;
}

// Chroma component c (0 Cb, 1 Cr) of an NV12 plane (stride = luma width), chroma size W x H.
template <class P>
VEP_HD int hk_chroma_at(const P* uv, int stride, int W, int H, int c, int x, int y) {
  x = x < 0 ? 0 : (x >= W ? W - 1 : x);
  y = y < 0 ? 0 : (y >= H ? H - 1 : y);
  return uv[y * stride + 2 * x + c];
}

template <class P>
VEP_HD int hk_chroma_mc(const P* uv, int stride, int W, int H, int c, int xi, int yi, int fx, int fy, int bd = 8) {
  const int sh1 = bd - 8;
  if (!fx && !fy) return hk_chroma_at(uv, stride, W, H, c, xi, yi) << (14 - bd);
  if (!fy) {
    int s = 0;
    for (int i = 0; i < 4; ++i) s += kChromaFilter[fx][i] * hk_chroma_at(uv, stride, W, H, c, xi + i - 1, yi);
    return s >> sh1;
  }
  if (!fx) {
    int s = 0;
    for (int i = 0; i < 4; ++i) s += kChromaFilter[fy][i] * hk_chroma_at(uv, stride, W, H, c, xi, yi + i - 1);
    return s >> sh1;
  }
  int s = 0;
  for (int k = 0; k < 4; ++k) {
    int h = 0;
    for (int i = 0; i < 4; ++i) h += kChromaFilter[fx][i] * hk_chroma_at(uv, stride, W, H, c, xi + i - 1, yi + k - 1);
    s += kChromaFilter[fy][k] * (h >> sh1);
  }
  return s >> 6;
}

VEP_HD u8 hk_clip8(int v) { return u8(v < 0 ? 0 : (v > 255 ? 255 : v)); }
VEP_HD int hk_clip(int v, int bd) {
  const int hi = (1 << bd) - 1;
  return v < 0 ? 0 : (v > hi ? hi : v);
}

// Final prediction sample from the 14-bit intermediates (§8.5.3.3.4.2): uni (p + off) >> (14 -
// bd), bi (p0 + p1 + off) >> (15 - bd).
VEP_HD int hk_weight(int p0, int p1, bool bi, int bd = 8) {
  const int sh = bi ? 15 - bd : 14 - bd;
  return hk_clip(((bi ? p0 + p1 : p0) + (1 << (sh - 1))) >> sh, bd);
}

// Explicit weighting (§8.5.3.3.4.3) of component c; `l` is the list of a uni-predicted sample
// (p0), ignored for bi-prediction (p0 list 0, p1 list 1). The record carries log2WD (= denom +
// 14 - bd) and the offsets already scaled by 1 << (bd - 8).
VEP_HD int hk_weight_explicit(const GpuWp& e, int c, int p0, int p1, bool bi, int l, int bd = 8) {
  const int sh = e.shift[c];
  if (bi) return hk_clip((p0 * e.w[0][c] + p1 * e.w[1][c] + ((e.o[0][c] + e.o[1][c] + 1) << sh)) >> (sh + 1), bd);
  const int v = sh >= 1 ? ((p0 * e.w[l][c] + (1 << (sh - 1))) >> sh) + e.o[l][c] : p0 * e.w[l][c] + e.o[l][c];
  return hk_clip(v, bd);
}

// ---------------------------------------------------------------------------- transform
VEP_HD int hk_basis(int log2, bool dst, int j, int i) {  // basis j (frequency) at sample i
  return dst ? kDst4[j][i] : kDct.m[j << (5 - log2)][i];
}

// First stage (vertical) of the inverse transform: g[y][x] for one (y, x), coefficients d
// (row-major n x n), rows <= my used.
VEP_HD int hk_itx_col(const i16* d, int log2, bool dst, int y, int x, int my) {
  const int n = 1 << log2;
  int s = 0;
  for (int j = 0; j <= my; ++j) s += hk_basis(log2, dst, j, y) * d[j * n + x];
  s = (s + 64) >> 7;
  return s < -32768 ? -32768 : (s > 32767 ? 32767 : s);
}

// Second stage (horizontal): residual r[y][x] from the first-stage row g (columns <= mx);
// bdShift = 20 - bd.
VEP_HD int hk_itx_row(const int* grow, int log2, bool dst, int x, int mx, int bd = 8) {
  int s = 0;
  for (int j = 0; j <= mx; ++j) s += hk_basis(log2, dst, j, x) * grow[j];
  return (s + (1 << (19 - bd))) >> (20 - bd);
}

VEP_HD int hk_tskip(int d, int bd = 8) { return ((d << 7) + (1 << (19 - bd))) >> (20 - bd); }

// ---------------------------------------------------------------------------- intra
// One predicted sample at (x, y) of an n x n block (n = 1 << log2) from prepared (substituted,
// filtered) references: top[k + 1] = p[k][-1] (k = -1 .. 2n-1), left[k] = p[-1][k] (k = 0 .. 2n-1).
VEP_HD int hk_intra_sample(const int* top, const int* left, int log2, int mode, bool luma, int x, int y, int bd = 8) {
  const int n = 1 << log2;
  if (mode == 0) {  // planar
    return ((n - 1 - x) * left[y] + (x + 1) * top[n + 1] + (n - 1 - y) * top[x + 1] + (y + 1) * left[n] + n) >>
           (log2 + 1);
  }
  if (mode == 1) {  // DC (+ edge filter for luma blocks below 32)
    int sum = n;
    for (int k = 0; k < n; ++k) sum += top[k + 1] + left[k];
    const int dc = sum >> (log2 + 1);
    if (luma && n < 32) {
      if (x == 0 && y == 0) return (left[0] + 2 * dc + top[1] + 2) >> 2;
      if (y == 0) return (top[x + 1] + 3 * dc + 2) >> 2;
      if (x == 0) return (left[y] + 3 * dc + 2) >> 2;
    }
    return dc;
  }
  const int angle = kIntraAngle[mode - 2];
  // main direction: vertical modes read the top row (ref[k] = p[-1 + k][-1]); horizontal modes
  // the left column (ref[k] = p[-1][-1 + k]), mirrored coordinates
  const bool vert = mode >= 18;
  const int u = vert ? x : y, v = vert ? y : x;  // u along the reference, v away from it
  const int idx = ((v + 1) * angle) >> 5, fact = ((v + 1) * angle) & 31;
  auto ref = [&](int k) -> int {  // ref[k], k in [-n, 2n]
    if (k >= 0) return vert ? top[k] : (k == 0 ? top[0] : left[k - 1]);
    const int inv = kInvAngle[mode - 11];
    const int j = -1 + ((k * inv + 128) >> 8);  // projected index on the side reference
    return vert ? (j < 0 ? top[0] : left[j]) : top[j + 1];
  };
  int val = fact ? ((32 - fact) * ref(u + idx + 1) + fact * ref(u + idx + 2) + 16) >> 5 : ref(u + idx + 1);
  if (luma && n < 32) {
    if (mode == 26 && x == 0) val = top[1] + ((left[y] - top[0]) >> 1);
    if (mode == 10 && y == 0) val = left[0] + ((top[x + 1] - top[0]) >> 1);
  }
  return hk_clip(val, bd);
}

// Reference samples of an intra block (§8.4.4.2.2-3) from the picture plane, the availability
// mask and the mode: substitution of unavailable samples, then filtering (luma only).
// Mask: bit 0 the corner p[-1][-1]; bits 1.. the left column and bits 17.. the top row in units
// of g samples (g = 4 luma, 2 chroma: one 4x4 luma block), nearest units first.
// `plane` addresses sample (0, 0) of the component: luma plane, or the NV12 plane offset by c - 1
// (then `step` = 2 between horizontal neighbours).
template <class P>
VEP_HD void hk_prepare_refs(const P* plane, int stride, int step, int x0, int y0, int log2, bool luma, u64 avail,
                            int mode, bool strong, int* top, int* left, int bd = 8) {
  const int n = 1 << log2, g = luma ? 4 : 2;
  auto at = [&](int x, int y) { return int(plane[y * stride + x * step]); };
  // p[-1][2n-1] .. p[-1][-1] .. p[2n-1][-1] as one scan (k = 0 .. 4n)
  int buf[129];
  bool av[129];
  int any = 0;
  for (int k = 0; k <= 4 * n; ++k) {
    bool a;
    int v = 0;
    if (k < 2 * n) {  // left column, bottom to top: y = 2n - 1 - k
      const int y = 2 * n - 1 - k;
      a = (avail >> (1 + y / g)) & 1;
      if (a) v = at(x0 - 1, y0 + y);
    } else if (k == 2 * n) {
      a = avail & 1;
      if (a) v = at(x0 - 1, y0 - 1);
    } else {  // top row, left to right: x = k - 2n - 1
      const int x = k - 2 * n - 1;
      a = (avail >> (17 + x / g)) & 1;
      if (a) v = at(x0 + x, y0 - 1);
    }
    buf[k] = v;
    av[k] = a;
    any |= a ? 1 : 0;
  }
  if (!any) {
    for (int k = 0; k <= 4 * n; ++k) buf[k] = 1 << (bd - 1);
  } else {
    if (!av[0]) {
      int k = 1;
      while (!av[k]) ++k;
      buf[0] = buf[k];
    }
    for (int k = 1; k <= 4 * n; ++k)
      if (!av[k]) buf[k] = buf[k - 1];
  }
  for (int y = 0; y < 2 * n; ++y) left[y] = buf[2 * n - 1 - y];
  for (int x = 0; x <= 2 * n; ++x) top[x] = buf[2 * n + x];
  // filtering (§8.4.4.2.3)
  if (!luma || mode == 1 || n == 4) return;
  const int dm = mode - 26 < 0 ? 26 - mode : mode - 26, dh = mode - 10 < 0 ? 10 - mode : mode - 10;
  const int dist = dm < dh ? dm : dh;
  const int thres = n == 8 ? 7 : (n == 16 ? 1 : 0);
  if (!(dist > thres)) return;
  int t[65], l[64];
  const int tl = top[0];
  auto iabs = [](int v) { return v < 0 ? -v : v; };
  const int lim = 1 << (bd - 5);
  if (strong && n == 32 && iabs(tl + top[2 * n] - 2 * top[n]) < lim && iabs(tl + left[2 * n - 1] - 2 * left[n - 1]) < lim) {
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
  for (int x = 0; x <= 2 * n; ++x) top[x] = t[x];
  for (int y = 0; y < 2 * n; ++y) left[y] = l[y];
}

// ---------------------------------------------------------------------------- deblocking
// Luma filtering of one 4-line segment of an edge (§8.7.2.5.3 / .6-.7). `at(k, i)` addresses line
// k (0..3) at distance i from the edge (p side: i < 0, q side: i >= 0). beta and tC scale by
// 1 << (bd - 8).
template <class P>
struct HkLumaEdgeT {
  P* base;    // sample q0 of line 0
  int along;  // step between lines
  int across; // step across the edge (q direction)
  VEP_HD P& at(int k, int i) const { return base[k * along + i * across]; }
};
using HkLumaEdge = HkLumaEdgeT<u8>;

template <class P>
VEP_HD void hk_deblock_luma(const HkLumaEdgeT<P>& e, int bs, int qpl, int beta_offset, int tc_offset, bool nfp, bool nfq,
                            int bd = 8) {
  const int bi = qpl + beta_offset, ti = qpl + 2 * (bs - 1) + tc_offset;
  const int beta = kBetaTable[bi < 0 ? 0 : (bi > 51 ? 51 : bi)] * (1 << (bd - 8));
  const int tc = kTcTable[ti < 0 ? 0 : (ti > 53 ? 53 : ti)] * (1 << (bd - 8));
  auto P_ = [&](int k, int i) { return int(e.at(k, -1 - i)); };
  auto Q = [&](int k, int i) { return int(e.at(k, i)); };
  auto iabs = [](int v) { return v < 0 ? -v : v; };
  const int dp0 = iabs(P_(0, 2) - 2 * P_(0, 1) + P_(0, 0)), dp3 = iabs(P_(3, 2) - 2 * P_(3, 1) + P_(3, 0));
  const int dq0 = iabs(Q(0, 2) - 2 * Q(0, 1) + Q(0, 0)), dq3 = iabs(Q(3, 2) - 2 * Q(3, 1) + Q(3, 0));
  const int dpq0 = dp0 + dq0, dpq3 = dp3 + dq3, dp = dp0 + dp3, dq = dq0 + dq3, d = dpq0 + dpq3;
  if (d >= beta) return;
  auto dsam = [&](int k, int dpq) {
    return 2 * dpq < (beta >> 2) && iabs(P_(k, 3) - P_(k, 0)) + iabs(Q(k, 0) - Q(k, 3)) < (beta >> 3) &&
           iabs(P_(k, 0) - Q(k, 0)) < ((5 * tc + 1) >> 1);
  };
  const bool strong = dsam(0, dpq0) && dsam(3, dpq3);
  const bool dEp = dp < ((beta + (beta >> 1)) >> 3), dEq = dq < ((beta + (beta >> 1)) >> 3);
  auto clip3 = [](int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); };
  for (int k = 0; k < 4; ++k) {
    const int p0 = P_(k, 0), p1 = P_(k, 1), p2 = P_(k, 2), p3 = P_(k, 3);
    const int q0 = Q(k, 0), q1 = Q(k, 1), q2 = Q(k, 2), q3 = Q(k, 3);
    if (strong) {
      if (!nfp) {
        e.at(k, -1) = P(clip3(p0 - 2 * tc, p0 + 2 * tc, (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3));
        e.at(k, -2) = P(clip3(p1 - 2 * tc, p1 + 2 * tc, (p2 + p1 + p0 + q0 + 2) >> 2));
        e.at(k, -3) = P(clip3(p2 - 2 * tc, p2 + 2 * tc, (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3));
      }
      if (!nfq) {
        e.at(k, 0) = P(clip3(q0 - 2 * tc, q0 + 2 * tc, (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3));
        e.at(k, 1) = P(clip3(q1 - 2 * tc, q1 + 2 * tc, (p0 + q0 + q1 + q2 + 2) >> 2));
        e.at(k, 2) = P(clip3(q2 - 2 * tc, q2 + 2 * tc, (p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3));
      }
    } else {
      int delta = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4;
      if (iabs(delta) >= tc * 10) continue;
      delta = clip3(-tc, tc, delta);
      if (!nfp) e.at(k, -1) = P(hk_clip(p0 + delta, bd));
      if (!nfq) e.at(k, 0) = P(hk_clip(q0 - delta, bd));
      if (dEp && !nfp) e.at(k, -2) = P(hk_clip(p1 + clip3(-(tc >> 1), tc >> 1, (((p2 + p0 + 1) >> 1) - p1 + delta) >> 1), bd));
      if (dEq && !nfq) e.at(k, 1) = P(hk_clip(q1 + clip3(-(tc >> 1), tc >> 1, (((q2 + q0 + 1) >> 1) - q1 - delta) >> 1), bd));
    }
  }
}

VEP_HD int hk_chroma_qp(int qpi) {
  if (qpi < 30) return qpi;
  if (qpi > 43) return qpi - 6;
  const int k[14] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37};
  return k[qpi - 30];
}

// Chroma filtering of the 2 chroma lines of one 4-luma-line segment (bS 2 edges only).
template <class P>
VEP_HD void hk_deblock_chroma(P* base, int along, int across, int qpP, int qpQ, int cqp_offset, int tc_offset,
                              bool nfp, bool nfq, int bd = 8) {
  // §8.7.2.5.5: QpC from Table 8-10 of qPi (no clipping of qPi: that is the CU-level rule)
  const int qpi = ((qpP + qpQ + 1) >> 1) + cqp_offset;
  int ti = hk_chroma_qp(qpi) + 2 + tc_offset;
  const int tc = kTcTable[ti < 0 ? 0 : (ti > 53 ? 53 : ti)] * (1 << (bd - 8));
  for (int k = 0; k < 2; ++k) {
    P* q = base + k * along;
    const int p0 = q[-across], p1 = q[-2 * across], q0 = q[0], q1 = q[across];
    int delta = (((q0 - p0) * 4) + p1 - q1 + 4) >> 3;
    delta = delta < -tc ? -tc : (delta > tc ? tc : delta);
    if (!nfp) q[-across] = P(hk_clip(p0 + delta, bd));
    if (!nfq) q[0] = P(hk_clip(q0 - delta, bd));
  }
}

// ---------------------------------------------------------------------------- SAO
// One SAO output sample of component c (0 luma) at (x, y) (component samples) of the CTB with
// parameters sp, reading the deblocked picture `src` (plane pointer of the component as in
// hk_prepare_refs). `nb_ok(nx, ny)` says whether the neighbour may be used (inside the picture,
// slice-boundary rules). Returns the input sample when no offset applies. Bands are
// 1 << (bd - 5) wide; the offsets (SaoOffsetVal, << (bd - min(bd, 10)) = 0 for bd <= 10) are
// the parsed ones.
template <class P, class NbOk>
VEP_HD int hk_sao_sample(const P* src, int stride, int step, const GpuSao& sp, int c, int x, int y, NbOk nb_ok,
                         int bd = 8) {
  const int v = src[y * stride + x * step];
  const int type = sp.type[c];
  // offset k of component c: a shift out of the component's four offsets as one word (an index
  // into the arrays, varying per GPU lane, would put the parameters in scratch memory)
  u32 ow;
  __builtin_memcpy(&ow, sp.off[c], 4);
  auto off = [&](int k) { return int(i8(u8(ow >> (8 * k)))); };
  if (type == 1) {
    const int k = ((v >> (bd - 5)) - sp.band[c]) & 31;
    return k < 4 ? hk_clip(v + off(k), bd) : v;
  }
  // edge class: 0 horizontal (-1, 0) / (1, 0), 1 vertical (0, -1) / (0, 1), 2 135 degrees
  // (-1, -1) / (1, 1), 3 45 degrees (1, -1) / (-1, 1)
  const int e = sp.eo[c];
  const int dx = e == 1 ? 0 : (e == 3 ? 1 : -1), dy = e == 0 ? 0 : -1;
  int sgn = 0;
  for (int t = 0; t < 2; ++t) {
    const int nx = x + (t ? -dx : dx), ny = y + (t ? -dy : dy);
    if (!nb_ok(nx, ny)) return v;
    const int nv = src[ny * stride + nx * step];
    sgn += (v > nv) - (v < nv);
  }
  int edge = 2 + sgn;
  if (edge <= 2) edge = edge == 2 ? 0 : edge + 1;
  return edge ? hk_clip(v + off(edge - 1), bd) : v;
}

}  // namespace vep::hevc
