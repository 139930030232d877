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

namespace vep::gpu {

using avc::MbRec;

namespace {

constexpr int kHbdWaves = 8;
constexpr int kTw = 25;  // luma tile row: x = -1..23
constexpr int kCw = 9;   // chroma tile row: x = -1..7

struct HbdWave {
  int t[17 * kTw];      // luma: row 0 = p[-1..23, -1], row 1 + y = p[-1..23, y] (x > 15 unused)
  int c[2][17 * kCw];   // chroma per component: row 0 = p[-1..7, -1], row 1 + y = p[-1..7, y]
};

// (The per-MB functions are host-callable too: csrc/tests/hbd_emu.cpp runs them lane by lane on
// the CPU under AddressSanitizer.)
#define VEP_HBD_FN __host__ __device__
VEP_HBD_FN inline void wsync() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // (global RMW of the filter steps too)
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
#endif
}

VEP_HBD_FN inline const MbRec& recd(const AvcDesc& d, int mb) { return static_cast<const MbRec*>(d.mbs)[mb]; }

// avc.cpp intra_avail
VEP_HBD_FN inline bool avail(const AvcDesc& d, const MbRec& m, int nx, int ny) {
  if (nx < 0 || ny < 0 || nx >= d.wmbs) return false;
  const MbRec& n = recd(d, ny * d.wmbs + nx);
  if (n.slice != m.slice) return false;
  return !(d.constrained && !avc::is_intra(n.kind));
}

// Bound check of a picture index (luma: wpx * hpx samples; chroma plane: wpx * chroma rows): a
// violation is reported in *err (bits 8..15, AvcDesc) and the access skipped, never performed.
VEP_HBD_FN inline bool oob(const AvcDesc& d, long i, long n, u32 bit) {
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

VEP_HBD_FN inline int& T(HbdWave& L, int x, int y) { return L.t[(y + 1) * kTw + x + 1]; }
VEP_HBD_FN inline int& Cc(HbdWave& L, int c, int x, int y) { return L.c[c][(y + 1) * kCw + x + 1]; }

template <class P, int CF>
VEP_HBD_FN void intra_mb(const AvcDesc& d, HbdWave& L, int mb, int lane) {
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
  const VEP_DEV i16* res = m.res == avc::kNoRes ? nullptr : d.res + size_t(m.res) * kAvcResSamples;
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
  // ---- luma
  if (m.kind == avc::kI16x16) {
    avc::Intra16Nb n;
    n.has_left = A;
    n.has_top = B;
    n.has_tl = D;
    n.top[0] = T(L, -1, -1);
    for (int k = 0; k < 16; ++k) {
      n.top[k + 1] = T(L, k, -1);
      n.left[k] = T(L, -1, k);
    }
    const avc::PredConst k = avc::intra16x16_const(n, m.i16_mode, bd);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int x = lane & 15, y = (lane >> 4) + 4 * s;
      T(L, x, y) = avc::clip1(avc::intra16x16_pred(n, k, m.i16_mode, x, y, bd) + (res ? int(res[y * 16 + x]) : 0), bd);
    }
  } else if (m.kind == avc::kI4x4) {
    for (int idx = 0; idx < 16; ++idx) {
      const int r = avc::blk_to_raster(idx), bx = r & 3, by = r >> 2;
      if (lane < 16) {
        const int x0 = bx * 4, y0 = by * 4;
        avc::Intra4Nb n;
        n.has_top = by > 0 || B;
        n.has_left = bx > 0 || A;
        n.has_tl = (bx > 0 && by > 0) || (bx == 0 && by == 0 ? D : bx == 0 ? A : B);
        const bool tr = by == 0 ? (bx < 3 ? B : C) : (bx < 3 && avc::raster_to_blk((by - 1) * 4 + bx + 1) < idx);
        n.t[0] = n.has_tl ? T(L, x0 - 1, y0 - 1) : 128;
        for (int k = 0; k < 4; ++k) {
          n.t[1 + k] = n.has_top ? T(L, x0 + k, y0 - 1) : 128;
          n.l[k] = n.has_left ? T(L, x0 - 1, y0 + k) : 128;
        }
        for (int k = 0; k < 4; ++k) n.t[5 + k] = tr ? T(L, x0 + 4 + k, y0 - 1) : n.t[4];
        const int j = lane & 3, i = lane >> 2;
        const int v = avc::intra4x4_pred(n, avc::i4_mode(m, r), j, i, bd) +
                      (res ? int(res[(y0 + i) * 16 + x0 + j]) : 0);
        T(L, x0 + j, y0 + i) = avc::clip1(v, bd);
      }
      wsync();
    }
  } else {  // Intra_8x8
    for (int q = 0; q < 4; ++q) {
      const int bx = q & 1, by = q >> 1, x0 = bx * 8, y0 = by * 8;
      const bool has_top = by > 0 || B, has_left = bx > 0 || A;
      const bool has_tl = (bx > 0 && by > 0) || (bx == 0 && by == 0 ? D : bx == 0 ? A : B);
      const bool has_tr = by == 0 ? (bx == 0 ? B : C) : (bx == 0);
      int t[17], l[8];
      t[0] = has_tl ? T(L, x0 - 1, y0 - 1) : 128;
      for (int k = 0; k < 8; ++k) {
        t[1 + k] = has_top ? T(L, x0 + k, y0 - 1) : 128;
        l[k] = has_left ? T(L, x0 - 1, y0 + k) : 128;
      }
      for (int k = 8; k < 16; ++k) t[1 + k] = has_tr ? T(L, x0 + k, y0 - 1) : t[8];
      int f[25];
      avc::intra8x8_filter([&](int x) { return t[1 + x]; }, [&](int y) { return l[y]; }, has_top, has_left,
                           has_tl, f);
      const int j = lane & 7, i = lane >> 3;
      const int v = avc::intra8x8_pred(f, has_top, has_left, avc::i4_mode(m, q), j, i, bd) +
                    (res ? int(res[(y0 + i) * 16 + x0 + j]) : 0);
      T(L, x0 + j, y0 + i) = avc::clip1(v, bd);  // (no sample of the block is its own neighbour)
      wsync();
    }
  }
  // ---- chroma (the whole 8x8 / 8x16 predicted from the neighbours: straight to the picture)
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    avc::IntraChromaNb n;
    n.has_left = A;
    n.has_top = B;
    n.has_tl = D;
    n.top[0] = Cc(L, c, -1, -1);
    for (int k = 0; k < 8; ++k) n.top[k + 1] = Cc(L, c, k, -1);
    for (int k = 0; k < CH; ++k) n.left[k] = Cc(L, c, -1, k);
    const avc::PredConst k = m.chroma_mode == 3 ? avc::chroma_plane_const(n, CF) : avc::PredConst{0, 0, 0, 0};
#pragma unroll
    for (int h = 0; h < CH / 8; ++h) {
      const int x = lane & 7, y = (lane >> 3) + 8 * h;
      const int v = avc::chroma_pred(n, k, m.chroma_mode, x, y, bd, CF) +
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

// avc.cpp deblock_t for one MB (bS per 4-line segment from avc_bs_kernel)
template <class P, int CF>
VEP_HBD_FN void deblock_mb(const AvcDesc& d, int mb, int lane) {
  constexpr int CH = CF == 2 ? 16 : 8;
  const MbRec q = recd(d, mb);
  if (q.dbk & 1) return;
  const AvcDbkInfo* infos = static_cast<const AvcDbkInfo*>(d.dbk);
  const AvcDbkInfo& info = infos[mb];
  if (!info.any) return;
  const int W = d.wmbs, pitch = W * 16, mx = mb % W, my = mb / W, bd = sizeof(P) == 1 ? 8 : d.bd;
  const int qb = d.qp_bias, qcb = d.qpc_bias;
  const bool t8 = (q.flags & avc::kMbT8x8) != 0;
  VEP_DEV P* Y = reinterpret_cast<VEP_DEV P*>(d.y + d.slot_y * u64(d.target));
  VEP_DEV P* UV = reinterpret_cast<VEP_DEV P*>(d.uv + d.slot_uv * u64(d.target));
  const MbRec lm = mx > 0 ? recd(d, mb - 1) : q;
  const MbRec tm = my > 0 ? recd(d, mb - W) : q;
  const long ny = long(pitch) * d.hmbs * 16, nuv = long(pitch) * d.hmbs * CH;
  // (a line at index i across an edge with stride st touches i - n * st .. i + (n - 1) * st)
  auto line_ok = [&](long i, long st, int n, long lim, u32 bit) {
    return !oob(d, i - n * st, lim, bit) && !oob(d, i + (n - 1) * st, lim, bit);
  };
  auto bs_of = [&](int i) { return int((info.bs[i >> 3] >> (4 * (i & 7))) & 15u); };
  for (int dir = 0; dir < 2; ++dir)
    for (int e = 0; e < 4; ++e) {
      const MbRec& p = e > 0 ? q : (dir == 0 ? lm : tm);
      if (lane < 16) {
        const int k = lane, bs = (e & 1) && t8 ? 0 : bs_of(dir * 16 + e * 4 + (k >> 2));  // (4:2:2 t8: chroma only)
        if (bs) {
          const avc::EdgeParams ep = avc::edge_params(p.qp - qb, q.qp - qb, q.alpha_off, q.beta_off, bd);
          const long i = dir == 0 ? long(my * 16 + k) * pitch + mx * 16 + 4 * e : long(my * 16 + 4 * e) * pitch + mx * 16 + k;
          const long st = dir == 0 ? 1 : long(pitch);
          if (line_ok(i, st, 4, ny, kOobDbkLuma)) avc::filter_line(Y + i, st, bs, ep, false, bd);
        }
      } else if (lane >= 16 && !(e & 1) || (CF == 2 && dir == 1 && lane >= 16)) {
        // chroma edges at chroma samples 0 and 4 (luma edges 0, 2); 4:2:2: every horizontal edge
        // (chroma rows 4e). Lines: vertical edges CH rows, horizontal edges 8 columns, per component.
        const int nl = dir == 0 ? CH : 8, c = (lane - 16) / nl, k = (lane - 16) % nl;
        // bS of the luma line through the chroma line: vertical edges luma row k (4:2:0: 2k),
        // horizontal edges luma column 2k
        const int bs = c < 2 ? bs_of(dir * 16 + e * 4 + (dir == 0 && CF == 2 ? k >> 2 : k >> 1)) : 0;
        if (bs) {
          const avc::EdgeParams ep = c == 0 ? avc::edge_params(p.qpc - qcb, q.qpc - qcb, q.alpha_off, q.beta_off, bd)
                                            : avc::edge_params(p.qpc2 - qcb, q.qpc2 - qcb, q.alpha_off, q.beta_off, bd);
          const long i = dir == 0 ? long(my * CH + k) * pitch + (mx * 8 + 2 * e) * 2 + c
                                  : long(my * CH + (CF == 2 ? 4 : 2) * e) * pitch + (mx * 8 + k) * 2 + c;
          const long st = dir == 0 ? 2 : long(pitch);
          if (line_ok(i, st, 2, nuv, kOobDbkChroma)) avc::filter_line(UV + i, st, bs, ep, true, bd);
        }
      }
      wsync();
    }
}

#ifndef VEP_HBD_EMU  // (csrc/tests/hbd_emu.cpp: the per-MB functions only)
// One instantiation per (sample type, chroma format): each workgroup takes one picture of the
// round and returns at once unless the picture is of its variant.
template <class P, int CF>
__global__ __launch_bounds__(64 * kHbdWaves) void avc_hbd_kernel(const AvcDesc* __restrict__ descs, int n,
                                                                  int intra, int dbk) {
  const int pic = int(blockIdx.x);
  if (pic >= n) return;
  const AvcDesc d = descs[pic];
  // (uniform over the workgroup, before any barrier)
  if ((d.bd > 8) != (sizeof(P) == 2) || (d.cf == 2) != (CF == 2)) return;
  __shared__ HbdWave lds[kHbdWaves];
  const int wave = int(threadIdx.x) >> 6, lane = int(threadIdx.x) & 63;
  const int W = d.wmbs, H = d.hmbs, steps = W + 2 * (H - 1);
  for (int pass = 0; pass < 2; ++pass) {
    if (!(pass == 0 ? intra : dbk)) continue;
    for (int t = 0; t < steps; ++t) {
      const int ylo = max(0, (t - W + 2) >> 1), yhi = min(H - 1, t >> 1);
      for (int y = ylo + wave; y <= yhi; y += kHbdWaves) {
        const int mb = y * W + t - 2 * y;
        if (pass == 0) intra_mb<P, CF>(d, lds[wave], mb, lane);
        else deblock_mb<P, CF>(d, mb, lane);
      }
      __syncthreads();
    }
  }
}

#endif  // VEP_HBD_EMU

}  // namespace

#ifndef VEP_HBD_EMU
void launch_avc_hbd(const AvcDesc* d_descs, int n, bool intra, bool dbk, int variants, hipStream_t s) {
  if (n <= 0 || !(intra || dbk)) return;
  const dim3 grid{unsigned(n)}, block{64 * kHbdWaves};
  const int in = intra ? 1 : 0, db = dbk ? 1 : 0;
  if (variants & 1) hipLaunchKernelGGL((avc_hbd_kernel<u16, 1>), grid, block, 0, s, d_descs, n, in, db);
  if (variants & 2) hipLaunchKernelGGL((avc_hbd_kernel<u8, 2>), grid, block, 0, s, d_descs, n, in, db);
  if (variants & 4) hipLaunchKernelGGL((avc_hbd_kernel<u16, 2>), grid, block, 0, s, d_descs, n, in, db);
  VEP_HIP(hipGetLastError());
}
#endif  // VEP_HBD_EMU

}  // namespace vep::gpu
