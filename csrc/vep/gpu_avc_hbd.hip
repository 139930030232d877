// gfx950 intra prediction + loop filter of H.264 High 10 (9 / 10-bit samples, u16 surfaces) and
// 4:2:2 (High 4:2:2, 8..10 bits, NV16 surfaces) pictures. The 8-bit 4:2:0 wavefront kernels
// (gpu_avc.hip) keep their byte-packed LDS tiles and word-wide filters and skip such pictures;
// avc_inter_kernel handles every depth and chroma format (motion compensation, I_PCM and the intra
// residuals), and this kernel then runs the two ordered passes of every such picture of the
// round:
//
//  * one 512-lane workgroup per picture; both passes walk the MBs in 2-skewed diagonals
//    (step t = x + 2y): every intra neighbour of an MB (left, top-left, top, top-right) and every
//    sample the loop filter of an MB reads or writes that an earlier MB (raster order) also
//    touches belongs to a smaller step, and the MBs of one step touch disjoint samples. A step's
//    MBs are spread over the 8 waves (one MB per wave at a time, its 64 lanes on the MB's
//    samples); a workgroup barrier separates the steps.
//  * intra: the MB and its neighbours (p[-1..23, -1], p[-1, 0..15]; chroma p[-1..7, -1],
//    p[-1, 0..7], 4:2:2 p[-1, 0..15]) in a per-wave LDS tile of ints; Intra_4x4 / Intra_8x8 blocks
//    in decoding order (16 / 64 lanes each), Intra_16x16 and chroma 4 / 2 (4:2:2: 4) samples per
//    lane, then one store.
//  * loop filter: per edge (vertical edges first, left to right, then horizontal ones), lanes
//    0-15 the luma lines and 16-47 the two chroma components' lines, read-modify-write in place;
//    bS from avc_bs_kernel's AvcDbkInfo, thresholds from the records at the picture's depth
//    (alpha / beta / tC0 << (bd - 8), QPs less the QpBdOffset bias). 4:2:2 chroma: 16-row
//    vertical edges at chroma x 0 / 4, horizontal edges at chroma rows 0, 4, 8, 12 (the odd ones
//    inside luma 8x8 transform blocks too: luma skips them, chroma filters them).
//
// All sample arithmetic comes from avc_recon.h (the CPU reconstruction's, avc.cpp cpu_deblock /
// Recon), at the picture's bit depth. High 10 is a coverage feature, not the 8-bit headline's
// path: one workgroup per picture keeps the ordering trivially correct.
//
// Reference parity: replaces libavcodec's High 10 H.264 decoding behind
// /root/reference/python/read_image.py:87 (cv2.VideoCapture).
#define VEP_KERNEL_SOURCE 1
#include "avc_recon.h"
#include "gpu.h"

#include <type_traits>

namespace vep::gpu {

using avc::MbRec;

namespace {

constexpr int kHbdWaves = 8;
constexpr int kTw = 25;  // luma tile row: x = -1..23
constexpr int kCw = 9;   // chroma tile row: x = -1..7

struct HbdIntra {
  int t[17 * kTw];      // luma: row 0 = p[-1..23, -1], row 1 + y = p[-1..23, y] (x > 15 unused)
  int c[2][17 * kCw];   // chroma per component: row 0 = p[-1..7, -1], row 1 + y = p[-1..7, y]
  int f[25];            // Intra_8x8 filtered references of the current 8x8 block
  i16 r[kAvcResSamples];  // the MB's residual (avc_inter_kernel's slot), loaded once
};
constexpr int kDw = 20;   // loop-filter luma tile row: x = -4..15 (rows y = -4..15)
constexpr int kDcw = 10;  // chroma tile row: x = -2..7 (rows y = -2..CH-1)
struct HbdDbk {
  int y[20 * kDw];
  int c[2][18 * kDcw];
  AvcDbkInfo info;  // the MB's bS / thresholds (lane-indexed reads: LDS, not scratch)
};
// A wave's LDS: the intra tile in the first pass, the loop-filter tile in the second (a
// workgroup barrier separates them).
union HbdWave {
  HbdIntra in;
  HbdDbk db;
};

// (The per-MB functions are host-callable too: csrc/tests/hbd_emu.cpp runs them lane by lane on
// the CPU under AddressSanitizer.)
#define VEP_HBD_FN __host__ __device__ inline __attribute__((always_inline))
// Wave-level sync of the LDS tile (both passes keep every dependency inside the wave's tile; the
// picture in global memory is read once per MB before and written once after).
VEP_HBD_FN void wsync() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
#endif
}

// clock64() / "thread 0 of the workgroup" for the phase clocks (0 / false in the host emulation)
VEP_HBD_FN u64 hbd_clock() {
#if defined(__HIP_DEVICE_COMPILE__)
  return clock64();
#else
  return 0;
#endif
}
VEP_HBD_FN bool hbd_thread0() {
#if defined(__HIP_DEVICE_COMPILE__)
  return threadIdx.x == 0;
#else
  return false;
#endif
}

VEP_HBD_FN const MbRec& recd(const AvcDesc& d, int mb) { return static_cast<const MbRec*>(d.mbs)[mb]; }

// avc.cpp intra_avail
VEP_HBD_FN bool avail(const AvcDesc& d, const MbRec& m, int nx, int ny) {
  if (nx < 0 || ny < 0 || nx >= d.wmbs) return false;
  const MbRec& n = recd(d, ny * d.wmbs + nx);
  if (n.slice != m.slice) return false;
  return !(d.constrained && !avc::is_intra(n.kind));
}

// Bound check of a picture index (luma: wpx * hpx samples; chroma plane: wpx * chroma rows): a
// violation is reported in *err (bits 8..15, AvcDesc) and the access skipped, never performed.
VEP_HBD_FN bool oob(const AvcDesc& d, long i, long n, u32 bit) {
  if (i >= 0 && i < n) return false;
#if defined(__HIP_DEVICE_COMPILE__)
  atomicOr(d.err, bit);
#else
  *d.err |= bit;
#endif
  return true;
}
constexpr u32 kOobLumaLoad = 0x100, kOobChromaLoad = 0x200, kOobRes = 0x400, kOobStore = 0x800,
              kOobDbkLuma = 0x1000, kOobDbkChroma = 0x2000;

VEP_HBD_FN int& T(HbdIntra& L, int x, int y) { return L.t[(y + 1) * kTw + x + 1]; }
VEP_HBD_FN int& Cc(HbdIntra& L, int c, int x, int y) { return L.c[c][(y + 1) * kCw + x + 1]; }

template <class P, int CF>
VEP_HBD_FN void intra_mb(const AvcDesc& d, HbdWave& LW, int mb, int lane) {
  HbdIntra& L = LW.in;
  constexpr int CH = CF == 2 ? 16 : 8;  // chroma MB height
  const MbRec m = recd(d, mb);
  if (!avc::is_wave_intra(m.kind)) return;  // (skip / inter / I_PCM: written by the inter kernel)
  const int W = d.wmbs, pitch = W * 16, mx = mb % W, my = mb / W, bd = sizeof(P) == 1 ? 8 : d.bd;
  VEP_DEV P* Y = reinterpret_cast<VEP_DEV P*>(d.y + d.slot_y * u64(d.target));
  VEP_DEV P* UV = reinterpret_cast<VEP_DEV P*>(d.uv + d.slot_uv * u64(d.target));
  const bool A = avail(d, m, mx - 1, my), B = avail(d, m, mx, my - 1), C = avail(d, m, mx + 1, my - 1),
             D = avail(d, m, mx - 1, my - 1);
  const long ny = long(pitch) * d.hmbs * 16, nuv = long(pitch) * d.hmbs * CH;
  if (m.res != avc::kNoRes && oob(d, long(m.res), long(d.nres), kOobRes)) return;
  const bool has_res = m.res != avc::kNoRes;
  // the residual into LDS in one round trip (8 samples a lane): a global load per 4x4 block
  // would sit on the Intra_4x4 chain sixteen times
  if (has_res) {
    static_assert(kAvcResSamples == 64 * 8, "one 16-byte load per lane");
    const VEP_DEV uint4* src = reinterpret_cast<const VEP_DEV uint4*>(d.res + size_t(m.res) * kAvcResSamples);
    reinterpret_cast<uint4*>(L.r)[lane] = src[lane];
  }
  const i16* res = has_res ? L.r : nullptr;
  // ---- neighbours into the tile (128: an unavailable side, as the CPU's neighbour arrays)
  if (lane < 25) {  // top row x = -1..23
    const int x = lane - 1;
    const bool ok = x < 0 ? D : (x < 16 ? B : C);
    const long i = long(my * 16 - 1) * pitch + mx * 16 + x;
    T(L, x, -1) = ok && !oob(d, i, ny, kOobLumaLoad) ? int(Y[i]) : 128;
  } else if (lane < 41) {  // left column
    const int y = lane - 25;
    const long i = long(my * 16 + y) * pitch + mx * 16 - 1;
    T(L, -1, y) = A && !oob(d, i, ny, kOobLumaLoad) ? int(Y[i]) : 128;
  } else if (lane < 59) {  // chroma: row -1 x = -1..7 (9 per component), then the left column
    const int k = lane - 41, c = k / 9, x = k % 9 - 1;
    const bool ok = x < 0 ? D : B;
    const long i = long(my * CH - 1) * pitch + (mx * 8 + x) * 2 + c;
    Cc(L, c, x, -1) = ok && !oob(d, i, nuv, kOobChromaLoad) ? int(UV[i]) : 128;
  }
  if (lane < 2 * CH) {
    const int c = lane / CH, y = lane % CH;
    const long i = long(my * CH + y) * pitch + (mx * 8 - 1) * 2 + c;
    Cc(L, c, -1, y) = A && !oob(d, i, nuv, kOobChromaLoad) ? int(UV[i]) : 128;
  }
  wsync();
  // ---- luma (the predictors read their neighbours straight from the LDS tile, which already
  // holds 128 for an unavailable side: no per-lane neighbour arrays, which would live in
  // scratch when indexed by lane)
  if (m.kind == avc::kI16x16) {
    auto tf = [&](int x) { return T(L, x, -1); };
    auto lf = [&](int y) { return T(L, -1, y); };
    const avc::PredConst k = avc::intra16x16_const_g(tf, lf, B, A, m.i16_mode, bd);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int x = lane & 15, y = (lane >> 4) + 4 * s;
      T(L, x, y) = avc::clip1(avc::intra16x16_pred_g(tf, lf, k, m.i16_mode, x, y, bd) + (res ? int(res[y * 16 + x]) : 0), bd);
    }
  } else if (m.kind == avc::kI4x4) {
    for (int idx = 0; idx < 16; ++idx) {
      const int r = avc::blk_to_raster(idx), bx = r & 3, by = r >> 2;
      if (lane < 16) {
        const int x0 = bx * 4, y0 = by * 4;
        const bool has_top = by > 0 || B, has_left = bx > 0 || A;
        const bool tr = by == 0 ? (bx < 3 ? B : C) : (bx < 3 && avc::raster_to_blk((by - 1) * 4 + bx + 1) < idx);
        // (top-right unavailable: p[3, -1] repeated)
        auto tf = [&](int x) { return T(L, x0 + (x >= 4 && !tr ? 3 : x), y0 - 1); };
        auto lf = [&](int y) { return T(L, x0 - 1, y0 + y); };  // (y = -1: the corner)
        const int j = lane & 3, i = lane >> 2;
        const int v = avc::intra4x4_pred_g(tf, lf, has_top, has_left, avc::i4_mode(m, r), j, i, bd) +
                      (res ? int(res[(y0 + i) * 16 + x0 + j]) : 0);
        T(L, x0 + j, y0 + i) = avc::clip1(v, bd);
      }
      wsync();
    }
  } else {  // Intra_8x8: the 25 filtered references into LDS (a lane each), then the prediction
    for (int q = 0; q < 4; ++q) {
      const int bx = q & 1, by = q >> 1, x0 = bx * 8, y0 = by * 8;
      const bool has_top = by > 0 || B, has_left = bx > 0 || A;
      const bool has_tl = (bx > 0 && by > 0) || (bx == 0 && by == 0 ? D : bx == 0 ? A : B);
      const bool has_tr = by == 0 ? (bx == 0 ? B : C) : (bx == 0);
      if (lane < 25) {
        auto tf = [&](int x) { return T(L, x0 + (x >= 8 && !has_tr ? 7 : x), y0 - 1); };
        auto lf = [&](int y) { return T(L, x0 - 1, y0 + y); };
        L.f[lane] = avc::intra8x8_filter_at(tf, lf, has_top, has_left, has_tl, lane);
      }
      wsync();
      const int j = lane & 7, i = lane >> 3;
      const int v = avc::intra8x8_pred_g([&](int x) { return L.f[1 + x]; },
                                         [&](int y) { return y < 0 ? L.f[0] : L.f[17 + y]; }, has_top, has_left,
                                         avc::i4_mode(m, q), j, i, bd) +
                    (res ? int(res[(y0 + i) * 16 + x0 + j]) : 0);
      T(L, x0 + j, y0 + i) = avc::clip1(v, bd);  // (no sample of the block is its own neighbour)
      wsync();
    }
  }
  // ---- chroma (the whole 8x8 / 8x16 predicted from the neighbours: straight to the picture)
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    auto tf = [&](int x) { return Cc(L, c, x, -1); };
    auto lf = [&](int y) { return Cc(L, c, -1, y); };
    const avc::PredConst k = m.chroma_mode == 3 ? avc::chroma_plane_const_g(tf, lf, CF) : avc::PredConst{0, 0, 0, 0};
#pragma unroll
    for (int h = 0; h < CH / 8; ++h) {
      const int x = lane & 7, y = (lane >> 3) + 8 * h;
      const int v = avc::chroma_pred_g(tf, lf, B, A, k, m.chroma_mode, x, y, bd, CF) +
                    (res ? int(res[256 + c * 8 * CH + y * 8 + x]) : 0);
      const long i = long(my * CH + y) * pitch + (mx * 8 + x) * 2 + c;
      if (!oob(d, i, nuv, kOobStore)) UV[i] = P(avc::clip1(v, bd));
    }
  }
  wsync();
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int x = lane & 15, y = (lane >> 4) + 4 * s;
    const long i = long(my * 16 + y) * pitch + mx * 16 + x;
    if (!oob(d, i, ny, kOobStore)) Y[i] = P(T(L, x, y));
  }
}

// avc.cpp deblock_t for one MB (bS per 4-line segment from avc_bs_kernel), on an LDS tile: the
// MB and the samples its edges reach (luma rows / columns -4..15, chroma -2..) are loaded once,
// the edges run in order, and the tile goes back once. (The MBs of a step touch disjoint
// samples, and every earlier step is complete, so the tile is exact and writing all of it back
// is safe.) NT lanes per MB: a whole wave (64), or half a wave (32, so a wave filters two MBs at
// once; the 48 lines of a 4:2:2 MB's vertical edges take two rounds); `valid` false: this half
// has no MB.
template <class P, int CF, int NT = 64>
VEP_HBD_FN void deblock_mb(const AvcDesc& d, HbdDbk& L, int mb, int lane, bool valid = true) {
  constexpr int CH = CF == 2 ? 16 : 8;
  if (!valid) mb = 0;
  const MbRec q = recd(d, mb);
  // bS and the thresholds (avc_bs_kernel, 8-bit scale) into LDS once per MB: no table lookup on
  // the filters' dependency chain, and the lane-indexed reads stay out of scratch
  const AvcDbkInfo* infos = static_cast<const AvcDbkInfo*>(d.dbk);
  const bool on = valid && !(q.dbk & 1) && infos[mb].any;
  if (NT == 64 && !on) return;  // (whole-wave MB: uniform)
  const AvcDbkInfo& info = L.info;
  if (on && lane < 16) reinterpret_cast<u32*>(&L.info)[lane] = reinterpret_cast<const u32*>(&infos[mb])[lane];
  const int W = d.wmbs, pitch = W * 16, mx = mb % W, my = mb / W, bd = sizeof(P) == 1 ? 8 : d.bd;
  const int sh = bd - 8;
  const bool t8 = (q.flags & avc::kMbT8x8) != 0;
  VEP_DEV P* Y = reinterpret_cast<VEP_DEV P*>(d.y + d.slot_y * u64(d.target));
  VEP_DEV P* UV = reinterpret_cast<VEP_DEV P*>(d.uv + d.slot_uv * u64(d.target));
  // edge class k (0: left MB edge, 1: top MB edge, 2: internal) of component c
  const long ny = long(pitch) * d.hmbs * 16, nuv = long(pitch) * d.hmbs * CH;
  // The tile moves in groups of 4 consecutive picture samples (one 4- or 8-byte access): luma
  // tile row y (-4..15) is 5 groups, columns 4g - 4 .. 4g - 1; a chroma tile row (-2..CH-1) is
  // the 20 interleaved Cb / Cr samples of columns -2..7, 5 groups of 2 columns x 2 components.
  // Group index -> picture index of its first sample (-1: left of / above the picture).
  constexpr int NLG = 20 * 5, NCG = (CH + 2) * 5;
  auto luma_grp = [&](int g) -> long {
    const int y = g / 5 - 4, x = 4 * (g % 5) - 4;
    if (my * 16 + y < 0 || mx * 16 + x < 0) return -1;
    return long(my * 16 + y) * pitch + mx * 16 + x;
  };
  auto chroma_grp = [&](int g) -> long {
    const int y = g / 5 - 2, x = 2 * (g % 5) - 2;
    if (my * CH + y < 0 || mx * 8 + x < 0) return -1;
    return long(my * CH + y) * pitch + (mx * 8 + x) * 2;
  };
  using V4 = typename std::conditional<sizeof(P) == 1, u32, u64>::type;  // 4 samples
  auto get4 = [](V4 v, int k) { return int((v >> (8 * sizeof(P) * k)) & ((V4(1) << (8 * sizeof(P))) - 1)); };
  const bool pf = on && d.prof && hbd_thread0();  // (VEP_AVC_PROF: wave 0's MB phases)
  const u64 c0 = pf ? hbd_clock() : 0;
  // every load of the tile in flight at once: unconditional loads at clamped indices (a
  // conditional load would wait at its join), then the LDS stores
  constexpr int KL = (NLG + NT - 1) / NT, KC = (NCG + NT - 1) / NT;
  V4 lv[KL], cv[KC];
#pragma unroll
  for (int j = 0; j < KL; ++j) {
    const int g = lane + NT * j;
    const long i = on && g < NLG ? luma_grp(g) : -1;
    const bool ok = i >= 0 && i + 3 < ny;
    if (i >= 0 && !ok) oob(d, i, ny, kOobDbkLuma);
    lv[j] = *reinterpret_cast<const VEP_DEV V4*>(Y + (ok ? i : 0));
  }
#pragma unroll
  for (int j = 0; j < KC; ++j) {
    const int g = lane + NT * j;
    const long i = on && g < NCG ? chroma_grp(g) : -1;
    const bool ok = i >= 0 && i + 3 < nuv;
    if (i >= 0 && !ok) oob(d, i, nuv, kOobDbkChroma);
    cv[j] = *reinterpret_cast<const VEP_DEV V4*>(UV + (ok ? i : 0));
  }
#pragma unroll
  for (int j = 0; j < KL; ++j) {
    const int g = lane + NT * j;
    if (g < NLG) {
      int* o = &L.y[(g / 5) * kDw + 4 * (g % 5)];
      for (int k = 0; k < 4; ++k) o[k] = get4(lv[j], k);
    }
  }
#pragma unroll
  for (int j = 0; j < KC; ++j) {
    const int g = lane + NT * j;
    if (g < NCG) {
      const int r = (g / 5) * kDcw + 2 * (g % 5);
      L.c[0][r] = get4(cv[j], 0);
      L.c[1][r] = get4(cv[j], 1);
      L.c[0][r + 1] = get4(cv[j], 2);
      L.c[1][r + 1] = get4(cv[j], 3);
    }
  }
  wsync();
  const u64 c1 = pf ? hbd_clock() : 0;
  auto bs_of = [&](int i) { return int((info.bs[i >> 3] >> (4 * (i & 7))) & 15u); };
  // Per direction, each lane holds one line in registers — lanes 0-15 a luma row (vertical
  // edges) / column (horizontal edges) as 20 samples (positions -4..15), lanes 16.. a chroma row /
  // column of one component at positions -2.. from register 2 — so its register edge r (between
  // registers 4r + 3 and 4r + 4) is luma MB edge r, and chroma edge r is chroma sample 4r (MB edges
  // 0 and 2; 4:2:2 horizontal: all four). The line's four edges then run in order in registers,
  // with one LDS round trip per direction instead of one per edge.
#pragma unroll
  for (int dir = 0; dir < 2; ++dir) {
    const int nlc = dir == 0 ? CH : 8;  // chroma lines per component
    // line slots: 16 luma lines, then 2 x nlc chroma lines, NT at a time (4:2:2 vertical edges
    // with half a wave per MB: two rounds)
    constexpr int kRounds = (16 + 2 * CH + NT - 1) / NT;
#pragma unroll
    for (int rho = 0; rho < kRounds; ++rho) {
    const int slot = lane + NT * rho;
    if (rho > 0 && 16 + 2 * nlc <= NT * rho) break;  // (uniform)
    const bool luma = slot < 16;
    const int cl = slot - 16, c = luma ? 0 : cl / nlc, k = luma ? slot : cl % nlc;
    const bool act = luma || c < 2;
    const bool all4 = luma || (CF == 2 && dir == 1);
    const int comp = luma ? 0 : 1 + c;
    int bsr[4], al[4], be[4], tc[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = all4 ? r : 2 * r;
      int bs = 0;
      if (on && act && e < 4) {
        if (luma) bs = (e & 1) && t8 ? 0 : bs_of(dir * 16 + e * 4 + (k >> 2));  // (4:2:2 t8: chroma only)
        // chroma: bS of the luma line through it (vertical: luma row k, 4:2:0 2k; horizontal: column 2k)
        else bs = bs_of(dir * 16 + e * 4 + (dir == 0 && CF == 2 ? k >> 2 : k >> 1));
      }
      const int pi = (act ? comp : 0) * 3 + (e > 0 ? 2 : dir);
      bsr[r] = bs;
      al[r] = int(info.alpha[pi]) << sh;
      be[r] = int(info.beta[pi]) << sh;
      tc[r] = bs > 0 && bs < 4 ? int(info.tc0[pi][bs - 1]) << sh : 0;
    }
    int* base;
    int stride, off, n;
    if (luma) {
      base = dir == 0 ? &L.y[(k + 4) * kDw] : &L.y[k + 4];
      stride = dir == 0 ? 1 : kDw;
      off = 0;
      n = 20;
    } else {
      base = dir == 0 ? &L.c[act ? c : 0][(k + 2) * kDcw] : &L.c[act ? c : 0][k + 2];
      stride = dir == 0 ? 1 : kDcw;
      off = 2;
      n = act ? (dir == 0 ? kDcw : CH + 2) : 0;
    }
    int v[20];
#pragma unroll
    for (int i = 0; i < 20; ++i) v[i] = i >= off && i - off < n ? base[(i - off) * stride] : 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (!bsr[r]) continue;
      int pp[4] = {v[4 * r + 3], v[4 * r + 2], v[4 * r + 1], v[4 * r]};
      int qq[4] = {v[4 * r + 4], v[4 * r + 5], v[4 * r + 6], v[4 * r + 7]};
      avc::filter_samples_u(pp, qq, bsr[r], al[r], be[r], tc[r], !luma, bd);  // (in place; chroma: p0 / q0)
      v[4 * r + 3] = pp[0];
      v[4 * r + 2] = pp[1];
      v[4 * r + 1] = pp[2];
      v[4 * r + 4] = qq[0];
      v[4 * r + 5] = qq[1];
      v[4 * r + 6] = qq[2];
    }
#pragma unroll
    for (int i = 0; i < 20; ++i)
      if (i >= off && i - off < n) base[(i - off) * stride] = v[i];
    }  // rounds (each lane's lines are its own: no sync between them)
    wsync();
  }
  const u64 c2 = pf ? hbd_clock() : 0;
  auto put4 = [](int a, int b, int c, int e) {
    constexpr int B = 8 * sizeof(P);
    return V4(u32(a)) | V4(u32(b)) << B | V4(u32(c)) << (2 * B) | V4(u32(e)) << (3 * B);
  };
#pragma unroll
  for (int j = 0; j < KL; ++j) {
    const int g = lane + NT * j;
    if (g < NLG) {
      const int* o = &L.y[(g / 5) * kDw + 4 * (g % 5)];
      lv[j] = put4(o[0], o[1], o[2], o[3]);
    }
  }
#pragma unroll
  for (int j = 0; j < KC; ++j) {
    const int g = lane + NT * j;
    if (g < NCG) {
      const int r = (g / 5) * kDcw + 2 * (g % 5);
      cv[j] = put4(L.c[0][r], L.c[1][r], L.c[0][r + 1], L.c[1][r + 1]);
    }
  }
#pragma unroll
  for (int j = 0; j < KL; ++j) {
    const int g = lane + NT * j;
    const long i = on && g < NLG ? luma_grp(g) : -1;
    if (i >= 0 && !oob(d, i + 3, ny, kOobStore)) *reinterpret_cast<VEP_DEV V4*>(Y + i) = lv[j];
  }
#pragma unroll
  for (int j = 0; j < KC; ++j) {
    const int g = lane + NT * j;
    const long i = on && g < NCG ? chroma_grp(g) : -1;
    if (i >= 0 && !oob(d, i + 3, nuv, kOobStore)) *reinterpret_cast<VEP_DEV V4*>(UV + i) = cv[j];
  }
  wsync();  // (the tile is reused by the wave's next MB)
#if defined(__HIP_DEVICE_COMPILE__)
  if (pf) {
    atomicAdd(&d.prof[16], c1 - c0);
    atomicAdd(&d.prof[17], c2 - c1);
    atomicAdd(&d.prof[18], clock64() - c2);
    atomicAdd(&d.prof[19], u64(1));
  }
#endif
}

#ifndef VEP_HBD_EMU  // (csrc/tests/hbd_emu.cpp: the per-MB functions only)
// One instantiation per (sample type, chroma format, pass): each workgroup takes one picture of
// the round and returns at once unless the picture is of its variant. The two passes are
// separate kernels (intra, then the loop filter) so each gets the whole register file.
template <class P, int CF, int PASS>
__global__ __launch_bounds__(64 * kHbdWaves) void avc_hbd_kernel(const AvcDesc* __restrict__ descs, int n) {
  const int pic = int(blockIdx.x);
  if (pic >= n) return;
  const AvcDesc d = descs[pic];
  // (uniform over the workgroup, before any barrier)
  if ((d.bd > 8) != (sizeof(P) == 2) || (d.cf == 2) != (CF == 2)) return;
  if (!(PASS == 0 ? d.intra_mbs > 0 : d.deblock != 0)) return;
  // loop filter: two MBs per wave (half a wave each, a tile each)
  constexpr bool kHalf = PASS == 1;
  constexpr int kTiles = kHalf ? 2 : 1;
  // (per pass its own tile type: the intra tile with the residual is the larger)
  __shared__ typename std::conditional<PASS == 0, HbdWave, HbdDbk>::type lds[kHbdWaves][kTiles];
  const int wave = int(threadIdx.x) >> 6, lane = int(threadIdx.x) & 63;
  const int W = d.wmbs, H = d.hmbs, steps = W + 2 * (H - 1);
  const bool prof = d.prof && threadIdx.x == 0;  // (VEP_AVC_PROF=1: workgroup phase clocks)
  u64 tb = 0;
  const u64 tp = prof ? clock64() : 0;
  // Intra pass: the intra MBs and the diagonal steps that hold any, listed in LDS up front (one
  // parallel scan of the records), so a P / B picture's few intra MBs cost a few steps instead of
  // a record load per MB and a barrier per step of the whole picture.
  constexpr int kMaxMbs = PASS == 0 ? 16384 : 1, kMaxSteps = PASS == 0 ? 1024 : 1;
  __shared__ u8 intra_at[kMaxMbs];
  __shared__ u8 step_has[kMaxSteps];
  const bool listed = PASS == 0 && W * H <= kMaxMbs && steps <= kMaxSteps;
  if (listed) {
    for (int i = int(threadIdx.x); i < steps; i += 64 * kHbdWaves) step_has[i] = 0;
    __syncthreads();
    const MbRec* recs = static_cast<const MbRec*>(d.mbs);
    for (int i = int(threadIdx.x); i < W * H; i += 64 * kHbdWaves) {
      const bool in = avc::is_wave_intra(recs[i].kind);
      intra_at[i] = in ? 1 : 0;
      if (in) step_has[i % W + 2 * (i / W)] = 1;  // (benign race: every writer stores 1)
    }
    __syncthreads();
  }
  for (int t = 0; t < steps; ++t) {
    if (listed && !step_has[t]) continue;  // (uniform: nothing of this step to predict)
    const int ylo = max(0, (t - W + 2) >> 1), yhi = min(H - 1, t >> 1);
    // (the descriptor by reference into global memory: a local copy passed by reference would
    // live in scratch)
    if (listed) {  // this step's intra MBs, dealt round-robin over the waves
      int k = 0;
      for (int y = ylo; y <= yhi; ++y) {
        const int mb = y * W + t - 2 * y;
        if (!intra_at[mb]) continue;
        if constexpr (PASS == 0)
          if (k++ % kHbdWaves == wave) intra_mb<P, CF>(descs[pic], lds[wave][0], mb, lane);
      }
    } else if constexpr (kHalf) {
      const int hh = lane >> 5;
      for (int y0 = ylo + 2 * wave; y0 <= yhi; y0 += 2 * kHbdWaves) {  // (wave-uniform)
        const int y = y0 + hh;
        deblock_mb<P, CF, 32>(descs[pic], lds[wave][hh], y * W + t - 2 * y, lane & 31,
                              y <= yhi);
      }
    } else {
      for (int y = ylo + wave; y <= yhi; y += kHbdWaves) {
        const int mb = y * W + t - 2 * y;
        if constexpr (PASS == 0) intra_mb<P, CF>(descs[pic], lds[wave][0], mb, lane);
        else deblock_mb<P, CF>(descs[pic], lds[wave][0], mb, lane);
      }
    }
    const u64 ts = prof ? clock64() : 0;
    __syncthreads();
    if (prof) tb += clock64() - ts;
  }
  if (prof) {
    atomicAdd(&d.prof[12 + PASS], clock64() - tp);
    atomicAdd(&d.prof[14], tb);
    if (PASS == 1) atomicAdd(&d.prof[15], u64(1));
  }
}

#endif  // VEP_HBD_EMU

}  // namespace

#ifndef VEP_HBD_EMU
void launch_avc_hbd(const AvcDesc* d_descs, int n, bool intra, bool dbk, int variants, hipStream_t s) {
  if (n <= 0 || !(intra || dbk)) return;
  const dim3 grid{unsigned(n)}, block{64 * kHbdWaves};
  if (intra) {
    if (variants & 1) hipLaunchKernelGGL((avc_hbd_kernel<u16, 1, 0>), grid, block, 0, s, d_descs, n);
    if (variants & 2) hipLaunchKernelGGL((avc_hbd_kernel<u8, 2, 0>), grid, block, 0, s, d_descs, n);
    if (variants & 4) hipLaunchKernelGGL((avc_hbd_kernel<u16, 2, 0>), grid, block, 0, s, d_descs, n);
  }
  if (dbk) {
    if (variants & 1) hipLaunchKernelGGL((avc_hbd_kernel<u16, 1, 1>), grid, block, 0, s, d_descs, n);
    if (variants & 2) hipLaunchKernelGGL((avc_hbd_kernel<u8, 2, 1>), grid, block, 0, s, d_descs, n);
    if (variants & 4) hipLaunchKernelGGL((avc_hbd_kernel<u16, 2, 1>), grid, block, 0, s, d_descs, n);
  }
  VEP_HIP(hipGetLastError());
}
#endif  // VEP_HBD_EMU

}  // namespace vep::gpu
