// gfx950 reconstruction kernels of the general H.264 path (records from avc::Decoder).
//
//  * avc_inter_kernel — every skip / inter / I_PCM macroblock of every picture of a round, one
//    256-lane workgroup per MB (lane = luma sample; lanes 0..127 also one chroma sample):
//    quarter-sample luma / eighth-sample chroma motion compensation from the camera's DPB
//    surfaces + 4x4 inverse transform of the dequantised residual. No neighbour dependency,
//    so the launch is as wide as the round (32 x 1080p = 261k workgroups).
//  * avc_intra_kernel / avc_deblock_kernel — the two inherently ordered passes. Intra
//    prediction reads reconstructed neighbours (left, top, top-right) and the loop filter reads
//    the left/top neighbours' filtered samples, so both run as a 2-MB-skewed wavefront over
//    MB rows. One 1024-lane workgroup (16 wave64s) per picture: wave w walks rows w, w+16, ...,
//    row r waits until row r-1 has finished MB x+1 via an LDS progress counter. Keeping a
//    picture's wavefront inside one workgroup (one CU) makes every hand-off a workgroup-scope
//    release/acquire: no cross-XCD L2 write-back / invalidate per macroblock (MI355X has one L2
//    per XCD), and no inter-workgroup spin that could deadlock. Pictures of different cameras
//    are different workgroups, spread over the XCDs by the dispatcher.
//    Per wave the MB under reconstruction lives in LDS; the left neighbour's edge columns are
//    carried in LDS (same-wave read-after-write never goes through global memory).
//
// All sample arithmetic comes from avc_recon.h, shared with the CPU reference decoder.
#include "avc_recon.h"
#include "gpu.h"

namespace vep::gpu {

using avc::MbRec;

namespace {

constexpr int kWaves = 16;
constexpr u32 kSpinLimit = 1u << 24;

__device__ inline const MbRec& rec(const AvcDesc& d, int mb) {
  return static_cast<const MbRec*>(d.mbs)[mb];
}

__device__ inline const i16* luma_block(const AvcDesc& d, const MbRec& m, int r) {
  return d.coefs + size_t(m.coef + u32(__popc(m.luma_coded & ((1u << r) - 1)))) * 16;
}
__device__ inline const i16* chroma_block(const AvcDesc& d, const MbRec& m, int k) {
  return d.coefs + size_t(m.coef + u32(__popc(m.luma_coded)) +
                          u32(__popc(m.chroma_coded & ((1u << k) - 1)))) * 16;
}

// --------------------------------------------------------------------------------- inter

__global__ __launch_bounds__(256) void avc_inter_kernel(const AvcDesc* __restrict__ descs, int n) {
  const int g = int(blockIdx.x);
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (descs[mid].mb_begin <= g) lo = mid;
    else hi = mid - 1;
  }
  const AvcDesc& d = descs[lo];
  const int mb = g - d.mb_begin;
  const MbRec m = rec(d, mb);
  if (m.kind != avc::kSkip && m.kind != avc::kInter && m.kind != avc::kIPcm) return;
  const int W = d.wmbs, wpx = W * 16, hpx = d.hmbs * 16, pitch = wpx;
  const int mx = mb % W, my = mb / W;
  u8* ty = d.y + d.slot_y * u64(d.target);
  u8* tuv = d.uv + d.slot_uv * u64(d.target);
  const int t = int(threadIdx.x), x = t & 15, y = t >> 4;
  const int cc = t >> 6, cq = t & 63, cx = cq & 7, cy = cq >> 3;  // chroma lane (t < 128)
  if (m.kind == avc::kIPcm) {
    const u8* s = reinterpret_cast<const u8*>(d.coefs + size_t(m.coef) * 16);
    ty[size_t(my * 16 + y) * pitch + mx * 16 + x] = s[t];
    if (t < 128) tuv[size_t(my * 8 + cy) * pitch + (mx * 8 + cx) * 2 + cc] = s[256 + t];
    return;
  }
  const i16* mv = d.mvs + size_t(m.mv) * 32;
  const int blk = (y >> 2) * 4 + (x >> 2);
  const int mvx = mv[2 * blk], mvy = mv[2 * blk + 1];
  const int ref = m.ref[((blk >> 3) << 1) | ((blk & 3) >> 1)];
  int v = avc::luma_qpel(d.y + d.slot_y * u64(ref), pitch, wpx, hpx, mx * 16 + x + (mvx >> 2),
                         my * 16 + y + (mvy >> 2), mvx & 3, mvy & 3);
  if ((m.luma_coded >> blk) & 1) v += avc::idct4x4_at(luma_block(d, m, blk), y & 3, x & 3);
  ty[size_t(my * 16 + y) * pitch + mx * 16 + x] = u8(avc::clip1(v));
  if (t < 128) {
    const int r = (cy >> 1) * 4 + (cx >> 1);
    const int c_mvx = mv[2 * r], c_mvy = mv[2 * r + 1];
    const int cref = m.ref[((r >> 3) << 1) | ((r & 3) >> 1)];
    int u = avc::chroma_epel(d.uv + d.slot_uv * u64(cref), pitch, wpx / 2, hpx / 2, cc,
                             mx * 8 + cx + (c_mvx >> 3), my * 8 + cy + (c_mvy >> 3), c_mvx & 7, c_mvy & 7);
    const int k = cc * 4 + (cy >> 2) * 2 + (cx >> 2);
    if ((m.chroma_coded >> k) & 1) u += avc::idct4x4_at(chroma_block(d, m, k), cy & 3, cx & 3);
    tuv[size_t(my * 8 + cy) * pitch + (mx * 8 + cx) * 2 + cc] = u8(avc::clip1(u));
  }
}

// ---------------------------------------------------------------------- wavefront helpers

struct Sync {
  u32 progress[kAvcMaxRows];  // MBs finished per row
  u32 abort;
};

__device__ inline void sync_init(Sync& s, int rows) {
  for (int i = int(threadIdx.x); i < rows; i += int(blockDim.x)) s.progress[i] = 0;
  if (threadIdx.x == 0) s.abort = 0;
  __syncthreads();
}

// Wait (whole wave, uniform) until row `r` has finished `need` MBs. A wave that spins too long
// flags the picture and aborts the whole workgroup's waits, so every wave always drains.
__device__ inline void wait_row(Sync& s, int r, u32 need, u32* err) {
  u32 spins = 0;
  while (__hip_atomic_load(&s.progress[r], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
    if (__hip_atomic_load(&s.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return;
    if (++spins > kSpinLimit) {
      __hip_atomic_store(&s.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if ((threadIdx.x & 63) == 0) atomicOr(err, 2u);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Publish (whole wave): this wave's global stores happen-before the new progress value.
__device__ inline void publish_row(Sync& s, int r, u32 v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_store(&s.progress[r], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ inline bool intra_avail(const AvcDesc& d, const MbRec& m, int nx, int ny) {
  if (nx < 0 || ny < 0 || nx >= d.wmbs) return false;
  const MbRec& n = rec(d, ny * d.wmbs + nx);
  if (n.slice != m.slice) return false;
  return !(d.constrained && !avc::is_intra(n.kind));
}

// wave-local barrier (one wave64 per "group" here: LDS ordering + compiler fence)
__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// --------------------------------------------------------------------------------- intra

struct alignas(16) IntraWave {
  u64 mask[kAvcMaxCols / 64];  // intra MBs (I4x4 / I16x16) of the current row
  i16 coef[24 * 16];  // the MB's dequantised residual blocks (coded blocks only, pool order)
  u8 mb[256];
  u8 mbc[2][64];
  u8 top[21];      // [0] top-left, [1..16] above, [17..20] above-right
  u8 left[16];
  u8 ctop[2][9];   // [0] top-left, [1..8] above
  u8 cleft[2][8];
  u8 carry[16];    // right luma column of the previous MB of this row (if this wave built it)
  u8 ccarry[2][8];
};

// One intra MB, whole wave. Every global load of the MB (coefficients, neighbour samples) is
// issued in one batch so the MB costs one memory round trip plus LDS work.
__device__ void intra_mb(const AvcDesc& d, IntraWave& L, const MbRec& m, int x, int row, bool carry,
                         int lane) {
  const int W = d.wmbs, pitch = W * 16;
  u8* Y = d.y + d.slot_y * u64(d.target);
  u8* UV = d.uv + d.slot_uv * u64(d.target);
  const bool A = intra_avail(d, m, x - 1, row), B = intra_avail(d, m, x, row - 1),
             C = intra_avail(d, m, x + 1, row - 1), D = intra_avail(d, m, x - 1, row - 1);
  const int x0 = x * 16, y0 = row * 16;
  // ---- batch: residual blocks (16 B per lane) + neighbour samples
  const int nblk = __popc(m.luma_coded) + __popc(m.chroma_coded);
  const uint4* src = reinterpret_cast<const uint4*>(d.coefs + size_t(m.coef) * 16);
  uint4* dst = reinterpret_cast<uint4*>(L.coef);
  if (lane < 2 * nblk) dst[lane] = src[lane];
  if (lane < 21) {
    u8 v = 128;
    if (lane == 0) { if (D) v = Y[size_t(y0 - 1) * pitch + x0 - 1]; }
    else if (lane <= 16) { if (B) v = Y[size_t(y0 - 1) * pitch + x0 + lane - 1]; }
    else if (C) v = Y[size_t(y0 - 1) * pitch + x0 + lane - 1];
    L.top[lane] = v;
  } else if (lane < 37) {
    const int k = lane - 21;
    L.left[k] = !A ? u8(128) : carry ? L.carry[k] : Y[size_t(y0 + k) * pitch + x0 - 1];
  } else if (lane < 55) {
    const int c = (lane - 37) / 9, k = (lane - 37) % 9;
    u8 v = 128;
    if (k == 0) { if (D) v = UV[size_t(row * 8 - 1) * pitch + (x * 8 - 1) * 2 + c]; }
    else if (B) v = UV[size_t(row * 8 - 1) * pitch + (x * 8 + k - 1) * 2 + c];
    L.ctop[c][k] = v;
  }
  if (lane >= 48) {
    const int c = (lane - 48) >> 3, k = (lane - 48) & 7;
    L.cleft[c][k] = !A ? u8(128) : carry ? L.ccarry[c][k] : UV[size_t(row * 8 + k) * pitch + (x * 8 - 1) * 2 + c];
  }
  wave_sync();
  auto lblk = [&](int r) { return L.coef + __popc(m.luma_coded & ((1u << r) - 1)) * 16; };
  // ---- luma (predictors read LDS through accessors: no private arrays, no scratch)
  if (m.kind == avc::kI16x16) {
    auto T = [&](int xx) { return int(L.top[xx + 1]); };
    auto Lf = [&](int yy) { return int(L.left[yy]); };
    const avc::PredConst pk = avc::intra16x16_const_g(T, Lf, B, A, m.i16_mode);
    for (int k = 0; k < 4; ++k) {
      const int p = lane + 64 * k, px = p & 15, py = p >> 4;
      int v = avc::intra16x16_pred_g(T, Lf, pk, m.i16_mode, px, py);
      const int blk = (py >> 2) * 4 + (px >> 2);
      if ((m.luma_coded >> blk) & 1) v += avc::idct4x4_at(lblk(blk), py & 3, px & 3);
      L.mb[p] = u8(avc::clip1(v));
    }
  } else {
    // Diagonal schedule: block (bx, by) only reads left / top / top-left / (when available in
    // coding order) top-right neighbours, all on earlier diagonals s = bx + 2 * by, so the 16
    // blocks run in 10 steps, up to 4 blocks (16 lanes each) at a time.
    const int g = lane >> 4, i = (lane >> 2) & 3, j = lane & 3;
    for (int st = 0; st < 10; ++st) {
      int bx = -1, by = -1, cnt = 0;
      for (int yy = 0; yy < 4; ++yy) {
        const int xx = st - 2 * yy;
        if (xx >= 0 && xx < 4) {
          if (cnt == g) bx = xx, by = yy;
          ++cnt;
        }
      }
      if (bx >= 0) {
        const int r = by * 4 + bx, idx = avc::raster_to_blk(r);
        const bool tr = by == 0 ? (bx < 3 ? B : C) : (bx < 3 && avc::raster_to_blk((by - 1) * 4 + bx + 1) < idx);
        auto P = [&](int ax, int ay) -> int {  // MB-relative, ax in -1..19, ay in -1..15
          if (ay < 0) return L.top[ax + 1];
          if (ax < 0) return L.left[ay];
          return L.mb[ay * 16 + ax];
        };
        auto T = [&](int xx) { return P(bx * 4 + (xx >= 4 && !tr ? 3 : xx), by * 4 - 1); };
        auto Lf = [&](int yy) { return P(bx * 4 - 1, by * 4 + yy); };
        int v = avc::intra4x4_pred_g(T, Lf, by > 0 || B, bx > 0 || A, avc::i4_mode(m, r), j, i);
        if ((m.luma_coded >> r) & 1) v += avc::idct4x4_at(lblk(r), i, j);
        L.mb[(by * 4 + i) * 16 + bx * 4 + j] = u8(avc::clip1(v));
      }
      wave_sync();
    }
  }
  // ---- chroma (2 samples per lane)
  const i16* cbase = L.coef + __popc(m.luma_coded) * 16;
  for (int k = 0; k < 2; ++k) {
    const int p = lane + 64 * k, c = p >> 6, q = p & 63, px = q & 7, py = q >> 3;
    auto T = [&](int xx) { return int(L.ctop[c][xx + 1]); };
    auto Lf = [&](int yy) { return int(L.cleft[c][yy]); };
    const avc::PredConst pk =
        m.chroma_mode == 3 ? avc::chroma_plane_const_g(T, Lf) : avc::PredConst{0, 0, 0, 0};
    int v = avc::chroma_pred_g(T, Lf, B, A, pk, m.chroma_mode, px, py);
    const int kk = c * 4 + (py >> 2) * 2 + (px >> 2);
    if ((m.chroma_coded >> kk) & 1)
      v += avc::idct4x4_at(cbase + __popc(m.chroma_coded & ((1u << kk) - 1)) * 16, py & 3, px & 3);
    L.mbc[c][q] = u8(avc::clip1(v));
  }
  wave_sync();
  // ---- write back + carry the right column for the next MB of this row
  {
    const int ry = lane >> 2, rx = (lane & 3) * 4;
    u32 w = 0;
    for (int b = 0; b < 4; ++b) w |= u32(L.mb[ry * 16 + rx + b]) << (8 * b);
    *reinterpret_cast<u32*>(Y + size_t(y0 + ry) * pitch + x0 + rx) = w;
    if (lane < 32) {  // NV12: 8 rows x 16 bytes
      const int cyr = lane >> 2, cxb = (lane & 3) * 2;
      u32 cw = 0;
      for (int b = 0; b < 2; ++b)
        cw |= (u32(L.mbc[0][cyr * 8 + cxb + b]) | u32(L.mbc[1][cyr * 8 + cxb + b]) << 8) << (16 * b);
      *reinterpret_cast<u32*>(UV + size_t(row * 8 + cyr) * pitch + (x * 8 + cxb) * 2) = cw;
    }
    if (lane < 16) L.carry[lane] = L.mb[lane * 16 + 15];
    if (lane < 16) L.ccarry[lane >> 3][lane & 7] = L.mbc[lane >> 3][(lane & 7) * 8 + 7];
  }
  wave_sync();
}

__global__ __launch_bounds__(1024) void avc_intra_kernel(const AvcDesc* __restrict__ descs) {
  __shared__ Sync sync;
  __shared__ IntraWave lds[kWaves];
  const AvcDesc& d = descs[blockIdx.x];
  const int W = d.wmbs, H = d.hmbs;
  sync_init(sync, H);
  const int wave = int(threadIdx.x) >> 6, lane = int(threadIdx.x) & 63;
  IntraWave& L = lds[wave];
  const int words = (W + 63) / 64;
  for (int row = wave; row < H; row += kWaves) {
    // ---- which MBs of this row need the wavefront (one parallel scan, ballot per 64 MBs)
    for (int wd = 0; wd < words; ++wd) {
      const int x = wd * 64 + lane;
      bool intra = false;
      if (x < W) {
        const u8 k = rec(d, row * W + x).kind;
        intra = k == avc::kI4x4 || k == avc::kI16x16;
      }
      const u64 b = __ballot(intra);
      if (lane == 0) L.mask[wd] = b;
    }
    wave_sync();
    int prev = -2;
    for (int wd = 0; wd < words; ++wd) {
      for (u64 b = L.mask[wd]; b; b &= b - 1) {
        const int x = wd * 64 + __ffsll(static_cast<unsigned long long>(b)) - 1;
        publish_row(sync, row, u32(x));  // every MB left of x is final
        if (row > 0) wait_row(sync, row - 1, u32(x + 2 < W ? x + 2 : W), d.err);
        const MbRec m = rec(d, row * W + x);
        intra_mb(d, L, m, x, row, prev == x - 1, lane);
        prev = x;
      }
    }
    publish_row(sync, row, u32(W));
  }
}

// ---------------------------------------------------------------------- boundary strengths

__global__ __launch_bounds__(256) void avc_bs_kernel(const AvcDesc* __restrict__ descs, int n,
                                                      int total) {
  const int g = int(blockIdx.x) * 256 + int(threadIdx.x);
  if (g >= total) return;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (descs[mid].mb_begin <= g) lo = mid;
    else hi = mid - 1;
  }
  const AvcDesc& d = descs[lo];
  const int mb = g - d.mb_begin, W = d.wmbs, x = mb % W, row = mb / W;
  const MbRec q = rec(d, mb);
  AvcDbkInfo info{};
  if (!(q.dbk & 1)) {
    const MbRec lm = x > 0 ? rec(d, mb - 1) : q;
    const MbRec tm = row > 0 ? rec(d, mb - W) : q;
    const bool left = x > 0 && !((q.dbk & 2) && lm.slice != q.slice);
    const bool top = row > 0 && !((q.dbk & 2) && tm.slice != q.slice);
    const i16* mq = avc::is_intra(q.kind) ? nullptr : d.mvs + size_t(q.mv) * 32;
    const i16* ml = avc::is_intra(lm.kind) ? nullptr : d.mvs + size_t(lm.mv) * 32;
    const i16* mt = avc::is_intra(tm.kind) ? nullptr : d.mvs + size_t(tm.mv) * 32;
    for (int dir = 0; dir < 2; ++dir)
      for (int e = 0; e < 4; ++e) {
        if (e == 0 && !(dir == 0 ? left : top)) continue;
        const MbRec& p = e > 0 ? q : (dir == 0 ? lm : tm);
        const i16* mp = e > 0 ? mq : (dir == 0 ? ml : mt);
        for (int sg = 0; sg < 4; ++sg) {
          const int bq = dir == 0 ? sg * 4 + e : e * 4 + sg;
          const int bp = e > 0 ? (dir == 0 ? bq - 1 : bq - 4) : (dir == 0 ? bq + 3 : bq + 12);
          const int bs = avc::boundary_strength(p, bp, mp ? mp + 2 * bp : nullptr, q, bq,
                                                mq ? mq + 2 * bq : nullptr, e == 0);
          const int i = dir * 16 + e * 4 + sg;
          info.bs[i >> 3] |= u32(bs) << (4 * (i & 7));
        }
      }
    info.any = (info.bs[0] | info.bs[1] | info.bs[2] | info.bs[3]) ? 1 : 0;
    const MbRec* ps[3] = {&lm, &tm, &q};
    for (int k = 0; k < 3; ++k) {
      const avc::EdgeParams el = avc::edge_params(ps[k]->qp, q.qp, q.alpha_off, q.beta_off);
      const avc::EdgeParams ec = avc::edge_params(ps[k]->qpc, q.qpc, q.alpha_off, q.beta_off);
      info.alpha[k] = u8(el.alpha);
      info.beta[k] = u8(el.beta);
      info.ia[k] = u8(el.index_a);
      info.alpha[3 + k] = u8(ec.alpha);
      info.beta[3 + k] = u8(ec.beta);
      info.ia[3 + k] = u8(ec.index_a);
    }
  }
  static_cast<AvcDbkInfo*>(d.dbk)[mb] = info;
}

// ------------------------------------------------------------------------------ deblocking

struct DbkWave {
  AvcDbkInfo info;
  u8 y[20 * 20];      // rows -4..15, cols -4..15 of the MB (top-left corner unused)
  u8 c[2][10 * 10];   // rows -2..7, cols -2..7 per chroma component
  u8 carry[16 * 4];   // previous MB's filtered luma columns 12..15
  u8 ccarry[2][8 * 2];
};

__device__ inline int bs_of(const AvcDbkInfo& in, int dir, int e, int sg) {
  const int i = dir * 16 + e * 4 + sg;
  return int((in.bs[i >> 3] >> (4 * (i & 7))) & 15u);
}

__global__ __launch_bounds__(1024) void avc_deblock_kernel(const AvcDesc* __restrict__ descs) {
  __shared__ Sync sync;
  __shared__ DbkWave lds[kWaves];
  const AvcDesc& d = descs[blockIdx.x];
  const int W = d.wmbs, H = d.hmbs, pitch = W * 16;
  sync_init(sync, H);
  const int wave = int(threadIdx.x) >> 6, lane = int(threadIdx.x) & 63;
  DbkWave& L = lds[wave];
  u8* Y = d.y + d.slot_y * u64(d.target);
  u8* UV = d.uv + d.slot_uv * u64(d.target);
  const AvcDbkInfo* infos = static_cast<const AvcDbkInfo*>(d.dbk);
  for (int row = wave; row < H; row += kWaves) {
    bool carry = false;
    for (int x = 0; x < W; ++x) {
      const int mb = row * W + x;
      if (row > 0) wait_row(sync, row - 1, u32(x + 2 < W ? x + 2 : W), d.err);
      const int x0 = x * 16, y0 = row * 16;
      // ---- batch: filter inputs, MB samples, left columns, top rows (luma + chroma)
      if (lane < 12) reinterpret_cast<u32*>(&L.info)[lane] = reinterpret_cast<const u32*>(&infos[mb])[lane];
      {
        const int ry = lane >> 2, rw = (lane & 3) * 4;
        const u32 w = *reinterpret_cast<const u32*>(Y + size_t(y0 + ry) * pitch + x0 + rw);
        for (int b = 0; b < 4; ++b) L.y[(ry + 4) * 20 + 4 + rw + b] = u8(w >> (8 * b));
      }
      if (lane < 16) {  // left columns -4..-1 of row `lane`
        if (x > 0) {
          u32 lw;
          if (carry) {
            lw = 0;
            for (int b = 0; b < 4; ++b) lw |= u32(L.carry[lane * 4 + b]) << (8 * b);
          } else {
            lw = *reinterpret_cast<const u32*>(Y + size_t(y0 + lane) * pitch + x0 - 4);
          }
          for (int b = 0; b < 4; ++b) L.y[(lane + 4) * 20 + b] = u8(lw >> (8 * b));
        }
      } else if (lane < 32) {  // top rows -4..-1
        if (row > 0) {
          const int k = lane - 16, tr = k >> 2, tw = (k & 3) * 4;
          const u32 tw32 = *reinterpret_cast<const u32*>(Y + size_t(y0 - 4 + tr) * pitch + x0 + tw);
          for (int b = 0; b < 4; ++b) L.y[tr * 20 + 4 + tw + b] = u8(tw32 >> (8 * b));
        }
      } else {  // chroma MB: 8 rows x 16 bytes NV12
        const int k = lane - 32, cyr = k >> 2, cb = (k & 3) * 2;
        const u32 cw = *reinterpret_cast<const u32*>(UV + size_t(row * 8 + cyr) * pitch + (x * 8 + cb) * 2);
        for (int b = 0; b < 2; ++b) {
          L.c[0][(cyr + 2) * 10 + 2 + cb + b] = u8(cw >> (16 * b));
          L.c[1][(cyr + 2) * 10 + 2 + cb + b] = u8(cw >> (16 * b + 8));
        }
      }
      if (lane >= 16 && lane < 24 && x > 0) {  // chroma left 2 columns of row `lane - 16`
        const int k = lane - 16;
        u8 v[4];
        if (carry) {
          v[0] = L.ccarry[0][k * 2];
          v[1] = L.ccarry[1][k * 2];
          v[2] = L.ccarry[0][k * 2 + 1];
          v[3] = L.ccarry[1][k * 2 + 1];
        } else {
          const u32 cw = *reinterpret_cast<const u32*>(UV + size_t(row * 8 + k) * pitch + (x * 8 - 2) * 2);
          for (int b = 0; b < 4; ++b) v[b] = u8(cw >> (8 * b));
        }
        L.c[0][(k + 2) * 10 + 0] = v[0];
        L.c[1][(k + 2) * 10 + 0] = v[1];
        L.c[0][(k + 2) * 10 + 1] = v[2];
        L.c[1][(k + 2) * 10 + 1] = v[3];
      } else if (lane >= 24 && lane < 32 && row > 0) {  // chroma top 2 rows
        const int k = lane - 24, tr = k >> 2, cb = (k & 3) * 2;
        const u32 cw = *reinterpret_cast<const u32*>(UV + size_t(row * 8 - 2 + tr) * pitch + (x * 8 + cb) * 2);
        for (int b = 0; b < 2; ++b) {
          L.c[0][tr * 10 + 2 + cb + b] = u8(cw >> (16 * b));
          L.c[1][tr * 10 + 2 + cb + b] = u8(cw >> (16 * b + 8));
        }
      }
      wave_sync();
      if (L.info.any) {
        // ---- filter: vertical edges then horizontal edges (luma lanes 0-15, chroma 16-31)
        for (int dir = 0; dir < 2; ++dir) {
          for (int e = 0; e < 4; ++e) {
            const int pk = e > 0 ? 2 : dir;  // edge params: left / top / internal
            if (lane < 16) {
              const int bs = bs_of(L.info, dir, e, lane >> 2);
              if (bs) {
                const avc::EdgeParams ep{L.info.alpha[pk], L.info.beta[pk], L.info.ia[pk]};
                if (dir == 0) avc::filter_line(&L.y[(4 + lane) * 20 + 4 + 4 * e], 1, bs, ep, false);
                else avc::filter_line(&L.y[(4 + 4 * e) * 20 + 4 + lane], 20, bs, ep, false);
              }
            } else if (lane < 32 && !(e & 1)) {
              const int c = (lane - 16) >> 3, k = (lane - 16) & 7;
              const int bs = bs_of(L.info, dir, e, k >> 1);
              if (bs) {
                const avc::EdgeParams ep{L.info.alpha[3 + pk], L.info.beta[3 + pk], L.info.ia[3 + pk]};
                if (dir == 0) avc::filter_line(&L.c[c][(2 + k) * 10 + 2 + 2 * e], 1, bs, ep, true);
                else avc::filter_line(&L.c[c][(2 + 2 * e) * 10 + 2 + k], 10, bs, ep, true);
              }
            }
            wave_sync();
          }
        }
        // ---- write back (MB, left columns, top rows)
        const bool left = (L.info.bs[0] & 0xFFFFu) != 0;   // dir 0, edge 0 nibbles
        const bool top = (L.info.bs[2] & 0xFFFFu) != 0;    // dir 1, edge 0 nibbles
        {
          const int ry = lane >> 2, rw = (lane & 3) * 4;
          u32 w = 0;
          for (int b = 0; b < 4; ++b) w |= u32(L.y[(ry + 4) * 20 + 4 + rw + b]) << (8 * b);
          *reinterpret_cast<u32*>(Y + size_t(y0 + ry) * pitch + x0 + rw) = w;
        }
        if (lane < 16) {
          if (left) {
            u32 lw = 0;
            for (int b = 0; b < 4; ++b) lw |= u32(L.y[(lane + 4) * 20 + b]) << (8 * b);
            *reinterpret_cast<u32*>(Y + size_t(y0 + lane) * pitch + x0 - 4) = lw;
          }
        } else if (lane < 32) {
          if (top) {
            const int k = lane - 16, tr = k >> 2, tw = (k & 3) * 4;
            u32 t32 = 0;
            for (int b = 0; b < 4; ++b) t32 |= u32(L.y[tr * 20 + 4 + tw + b]) << (8 * b);
            *reinterpret_cast<u32*>(Y + size_t(y0 - 4 + tr) * pitch + x0 + tw) = t32;
          }
        } else {
          const int k = lane - 32, cyr = k >> 2, cb = (k & 3) * 2;
          u32 cw = 0;
          for (int b = 0; b < 2; ++b)
            cw |= (u32(L.c[0][(cyr + 2) * 10 + 2 + cb + b]) | u32(L.c[1][(cyr + 2) * 10 + 2 + cb + b]) << 8)
                  << (16 * b);
          *reinterpret_cast<u32*>(UV + size_t(row * 8 + cyr) * pitch + (x * 8 + cb) * 2) = cw;
        }
        if (lane >= 16 && lane < 24 && left) {
          const int k = lane - 16;
          const u32 cw = u32(L.c[0][(k + 2) * 10]) | u32(L.c[1][(k + 2) * 10]) << 8 |
                         u32(L.c[0][(k + 2) * 10 + 1]) << 16 | u32(L.c[1][(k + 2) * 10 + 1]) << 24;
          *reinterpret_cast<u32*>(UV + size_t(row * 8 + k) * pitch + (x * 8 - 2) * 2) = cw;
        } else if (lane >= 24 && lane < 32 && top) {
          const int k = lane - 24, tr = k >> 2, cb = (k & 3) * 2;
          u32 cw = 0;
          for (int b = 0; b < 2; ++b)
            cw |= (u32(L.c[0][tr * 10 + 2 + cb + b]) | u32(L.c[1][tr * 10 + 2 + cb + b]) << 8) << (16 * b);
          *reinterpret_cast<u32*>(UV + size_t(row * 8 - 2 + tr) * pitch + (x * 8 + cb) * 2) = cw;
        }
      }
      // carry columns 12..15 (luma) / 6..7 (chroma) of this MB to the next one
      if (lane < 16)
        for (int b = 0; b < 4; ++b) L.carry[lane * 4 + b] = L.y[(lane + 4) * 20 + 16 + b];
      if (lane >= 16 && lane < 32) {
        const int c = (lane - 16) >> 3, k = (lane - 16) & 7;
        L.ccarry[c][k * 2] = L.c[c][(k + 2) * 10 + 8];
        L.ccarry[c][k * 2 + 1] = L.c[c][(k + 2) * 10 + 9];
      }
      wave_sync();
      carry = true;
      publish_row(sync, row, u32(x + 1));
    }
  }
}

}  // namespace

void launch_avc_inter(const AvcDesc* d_descs, int n, int total_mbs, hipStream_t s) {
  if (n <= 0 || total_mbs <= 0) return;
  hipLaunchKernelGGL(avc_inter_kernel, dim3(unsigned(total_mbs)), dim3(256), 0, s, d_descs, n);
  VEP_HIP(hipGetLastError());
}

void launch_avc_intra(const AvcDesc* d_descs, int n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(avc_intra_kernel, dim3(unsigned(n)), dim3(64 * kWaves), 0, s, d_descs);
  VEP_HIP(hipGetLastError());
}

void launch_avc_bs(const AvcDesc* d_descs, int n, int total_mbs, hipStream_t s) {
  if (n <= 0 || total_mbs <= 0) return;
  hipLaunchKernelGGL(avc_bs_kernel, dim3(unsigned((total_mbs + 255) / 256)), dim3(256), 0, s, d_descs,
                     n, total_mbs);
  VEP_HIP(hipGetLastError());
}

void launch_avc_deblock(const AvcDesc* d_descs, int n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(avc_deblock_kernel, dim3(unsigned(n)), dim3(64 * kWaves), 0, s, d_descs);
  VEP_HIP(hipGetLastError());
}

}  // namespace vep::gpu
