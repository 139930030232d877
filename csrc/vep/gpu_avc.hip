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

struct IntraWave {
  u8 mb[256];
  u8 mbc[2][64];
  u8 top[21];      // [0] top-left, [1..16] above, [17..20] above-right
  u8 left[16];
  u8 ctop[2][9];   // [0] top-left, [1..8] above
  u8 cleft[2][8];
  u8 carry[16];    // right luma column of the previous MB of this row (if this wave built it)
  u8 ccarry[2][8];
};

__global__ __launch_bounds__(1024) void avc_intra_kernel(const AvcDesc* __restrict__ descs) {
  __shared__ Sync sync;
  __shared__ IntraWave lds[kWaves];
  const AvcDesc& d = descs[blockIdx.x];
  const int W = d.wmbs, H = d.hmbs, pitch = W * 16;
  sync_init(sync, H);
  const int wave = int(threadIdx.x) >> 6, lane = int(threadIdx.x) & 63;
  IntraWave& L = lds[wave];
  u8* Y = d.y + d.slot_y * u64(d.target);
  u8* UV = d.uv + d.slot_uv * u64(d.target);
  for (int row = wave; row < H; row += kWaves) {
    bool carry = false;
    for (int x = 0; x < W; ++x) {
      const MbRec m = rec(d, row * W + x);
      const bool intra = m.kind == avc::kI4x4 || m.kind == avc::kI16x16;
      if (intra) {
        if (row > 0) wait_row(sync, row - 1, u32(x + 2 < W ? x + 2 : W), d.err);
        const bool A = intra_avail(d, m, x - 1, row), B = intra_avail(d, m, x, row - 1),
                   C = intra_avail(d, m, x + 1, row - 1), D = intra_avail(d, m, x - 1, row - 1);
        const int x0 = x * 16, y0 = row * 16;
        // ---- neighbour samples into LDS
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
        if (lane < 16) {
          const int c = lane >> 3, k = lane & 7;
          L.cleft[c][k] = !A ? u8(128) : carry ? L.ccarry[c][k] : UV[size_t(row * 8 + k) * pitch + (x * 8 - 1) * 2 + c];
        }
        wave_sync();
        // ---- luma
        if (m.kind == avc::kI16x16) {
          avc::Intra16Nb n;
          n.has_top = B;
          n.has_left = A;
          n.has_tl = D;
          n.top[0] = L.top[0];
          for (int k = 0; k < 16; ++k) {
            n.top[k + 1] = L.top[k + 1];
            n.left[k] = L.left[k];
          }
          const avc::PredConst pk = avc::intra16x16_const(n, m.i16_mode);
          for (int k = 0; k < 4; ++k) {
            const int p = lane + 64 * k, px = p & 15, py = p >> 4;
            int v = avc::intra16x16_pred(n, pk, m.i16_mode, px, py);
            const int blk = (py >> 2) * 4 + (px >> 2);
            if ((m.luma_coded >> blk) & 1) v += avc::idct4x4_at(luma_block(d, m, blk), py & 3, px & 3);
            L.mb[p] = u8(avc::clip1(v));
          }
        } else {
          for (int idx = 0; idx < 16; ++idx) {
            const int r = avc::blk_to_raster(idx), bx = r & 3, by = r >> 2;
            if (lane < 16) {
              auto P = [&](int xx, int yy) -> int {  // MB-relative, xx in -1..19, yy in -1..15
                if (yy < 0) return L.top[xx + 1];
                if (xx < 0) return L.left[yy];
                return L.mb[yy * 16 + xx];
              };
              avc::Intra4Nb n;
              n.has_top = by > 0 || B;
              n.has_left = bx > 0 || A;
              n.has_tl = (bx > 0 && by > 0) || (bx == 0 && by == 0 ? D : bx == 0 ? A : B);
              const bool tr = by == 0 ? (bx < 3 ? B : C)
                                      : (bx < 3 && avc::raster_to_blk((by - 1) * 4 + bx + 1) < idx);
              n.t[0] = n.has_tl ? P(bx * 4 - 1, by * 4 - 1) : 128;
              for (int k = 0; k < 4; ++k) {
                n.t[1 + k] = n.has_top ? P(bx * 4 + k, by * 4 - 1) : 128;
                n.l[k] = n.has_left ? P(bx * 4 - 1, by * 4 + k) : 128;
              }
              for (int k = 0; k < 4; ++k) n.t[5 + k] = tr ? P(bx * 4 + 4 + k, by * 4 - 1) : n.t[4];
              const int i = lane >> 2, j = lane & 3;
              int v = avc::intra4x4_pred(n, avc::i4_mode(m, r), j, i);
              if ((m.luma_coded >> r) & 1) v += avc::idct4x4_at(luma_block(d, m, r), i, j);
              L.mb[(by * 4 + i) * 16 + bx * 4 + j] = u8(avc::clip1(v));
            }
            wave_sync();
          }
        }
        // ---- chroma (2 samples per lane)
        for (int k = 0; k < 2; ++k) {
          const int p = lane + 64 * k, c = p >> 6, q = p & 63, px = q & 7, py = q >> 3;
          avc::IntraChromaNb n;
          n.has_top = B;
          n.has_left = A;
          n.has_tl = D;
          for (int i = 0; i < 9; ++i) n.top[i] = L.ctop[c][i];
          for (int i = 0; i < 8; ++i) n.left[i] = L.cleft[c][i];
          const avc::PredConst pk =
              m.chroma_mode == 3 ? avc::chroma_plane_const(n) : avc::PredConst{0, 0, 0, 0};
          int v = avc::chroma_pred(n, pk, m.chroma_mode, px, py);
          const int kk = c * 4 + (py >> 2) * 2 + (px >> 2);
          if ((m.chroma_coded >> kk) & 1) v += avc::idct4x4_at(chroma_block(d, m, kk), py & 3, px & 3);
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
        carry = true;
      } else {
        carry = false;
      }
      publish_row(sync, row, u32(x + 1));
    }
  }
}

// ------------------------------------------------------------------------------ deblocking

struct DbkWave {
  u8 y[20 * 20];      // rows -4..15, cols -4..15 of the MB (top-left corner unused)
  u8 c[2][10 * 10];   // rows -2..7, cols -2..7 per chroma component
  u8 carry[16 * 4];   // previous MB's filtered luma columns 12..15
  u8 ccarry[2][8 * 2];
};

__device__ inline int line_bs(const AvcDesc& d, const MbRec& q, const MbRec& lm, const MbRec& tm,
                              int dir, int e, int k) {
  const MbRec& p = e > 0 ? q : (dir == 0 ? lm : tm);
  const int bq = dir == 0 ? (k >> 2) * 4 + e : e * 4 + (k >> 2);
  const int bp = e > 0 ? (dir == 0 ? bq - 1 : bq - 4) : (dir == 0 ? bq + 3 : bq + 12);
  const i16* mp = avc::is_intra(p.kind) ? nullptr : d.mvs + size_t(p.mv) * 32 + 2 * bp;
  const i16* mq = avc::is_intra(q.kind) ? nullptr : d.mvs + size_t(q.mv) * 32 + 2 * bq;
  return avc::boundary_strength(p, bp, mp, q, bq, mq, e == 0);
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
  for (int row = wave; row < H; row += kWaves) {
    bool carry = false;
    for (int x = 0; x < W; ++x) {
      const int mb = row * W + x;
      const MbRec q = rec(d, mb);
      if (row > 0) wait_row(sync, row - 1, u32(x + 2 < W ? x + 2 : W), d.err);
      if (!(q.dbk & 1)) {
        const MbRec lm = x > 0 ? rec(d, mb - 1) : q;
        const MbRec tm = row > 0 ? rec(d, mb - W) : q;
        const bool left = x > 0 && !((q.dbk & 2) && lm.slice != q.slice);
        const bool top = row > 0 && !((q.dbk & 2) && tm.slice != q.slice);
        const int x0 = x * 16, y0 = row * 16;
        // ---- load: MB (16 rows x 4 words), left 4 columns, top 4 rows; chroma likewise
        {
          const int ry = lane >> 2, rw = (lane & 3) * 4;
          const u32 w = *reinterpret_cast<const u32*>(Y + size_t(y0 + ry) * pitch + x0 + rw);
          for (int b = 0; b < 4; ++b) L.y[(ry + 4) * 20 + 4 + rw + b] = u8(w >> (8 * b));
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
          } else if (lane < 32 && row > 0) {  // top rows -4..-1
            const int k = lane - 16, tr = k >> 2, tw = (k & 3) * 4;
            const u32 tw32 = *reinterpret_cast<const u32*>(Y + size_t(y0 - 4 + tr) * pitch + x0 + tw);
            for (int b = 0; b < 4; ++b) L.y[tr * 20 + 4 + tw + b] = u8(tw32 >> (8 * b));
          } else if (lane >= 32 && lane < 64) {  // chroma MB: 8 rows x 16 bytes NV12
            const int k = lane - 32, cyr = k >> 2, cb = (k & 3) * 2;
            const u32 cw = *reinterpret_cast<const u32*>(UV + size_t(row * 8 + cyr) * pitch + (x * 8 + cb) * 2);
            for (int b = 0; b < 2; ++b) {
              L.c[0][(cyr + 2) * 10 + 2 + cb + b] = u8(cw >> (16 * b));
              L.c[1][(cyr + 2) * 10 + 2 + cb + b] = u8(cw >> (16 * b + 8));
            }
          }
          if (lane < 8 && x > 0) {  // chroma left 2 columns of row `lane`
            u8 v[4];
            if (carry) {
              v[0] = L.ccarry[0][lane * 2];
              v[1] = L.ccarry[1][lane * 2];
              v[2] = L.ccarry[0][lane * 2 + 1];
              v[3] = L.ccarry[1][lane * 2 + 1];
            } else {
              const u32 cw = *reinterpret_cast<const u32*>(UV + size_t(row * 8 + lane) * pitch + (x * 8 - 2) * 2);
              for (int b = 0; b < 4; ++b) v[b] = u8(cw >> (8 * b));
            }
            L.c[0][(lane + 2) * 10 + 0] = v[0];
            L.c[1][(lane + 2) * 10 + 0] = v[1];
            L.c[0][(lane + 2) * 10 + 1] = v[2];
            L.c[1][(lane + 2) * 10 + 1] = v[3];
          } else if (lane >= 8 && lane < 16 && row > 0) {  // chroma top 2 rows
            const int k = lane - 8, tr = k >> 2, cb = (k & 3) * 2;
            const u32 cw = *reinterpret_cast<const u32*>(UV + size_t(row * 8 - 2 + tr) * pitch + (x * 8 + cb) * 2);
            for (int b = 0; b < 2; ++b) {
              L.c[0][tr * 10 + 2 + cb + b] = u8(cw >> (16 * b));
              L.c[1][tr * 10 + 2 + cb + b] = u8(cw >> (16 * b + 8));
            }
          }
        }
        wave_sync();
        // ---- filter: vertical edges then horizontal edges (luma lanes 0-15, chroma 16-31)
        for (int dir = 0; dir < 2; ++dir) {
          for (int e = 0; e < 4; ++e) {
            const bool on = e > 0 || (dir == 0 ? left : top);
            if (on) {
              const MbRec& p = e > 0 ? q : (dir == 0 ? lm : tm);
              if (lane < 16) {
                const int bs = line_bs(d, q, lm, tm, dir, e, lane);
                if (bs) {
                  const avc::EdgeParams ep = avc::edge_params(p.qp, q.qp, q.alpha_off, q.beta_off);
                  if (dir == 0) avc::filter_line(&L.y[(4 + lane) * 20 + 4 + 4 * e], 1, bs, ep, false);
                  else avc::filter_line(&L.y[(4 + 4 * e) * 20 + 4 + lane], 20, bs, ep, false);
                }
              } else if (lane < 32 && !(e & 1)) {
                const int c = (lane - 16) >> 3, k = (lane - 16) & 7;
                const int bs = line_bs(d, q, lm, tm, dir, e, 2 * k);
                if (bs) {
                  const avc::EdgeParams ep = avc::edge_params(p.qpc, q.qpc, q.alpha_off, q.beta_off);
                  if (dir == 0) avc::filter_line(&L.c[c][(2 + k) * 10 + 2 + 2 * e], 1, bs, ep, true);
                  else avc::filter_line(&L.c[c][(2 + 2 * e) * 10 + 2 + k], 10, bs, ep, true);
                }
              }
            }
            wave_sync();
          }
        }
        // ---- write back (MB, left columns, top rows) and carry columns 12..15 onwards
        {
          const int ry = lane >> 2, rw = (lane & 3) * 4;
          u32 w = 0;
          for (int b = 0; b < 4; ++b) w |= u32(L.y[(ry + 4) * 20 + 4 + rw + b]) << (8 * b);
          *reinterpret_cast<u32*>(Y + size_t(y0 + ry) * pitch + x0 + rw) = w;
          if (lane < 16) {
            if (left) {
              u32 lw = 0;
              for (int b = 0; b < 4; ++b) lw |= u32(L.y[(lane + 4) * 20 + b]) << (8 * b);
              *reinterpret_cast<u32*>(Y + size_t(y0 + lane) * pitch + x0 - 4) = lw;
            }
          } else if (lane < 32 && top) {
            const int k = lane - 16, tr = k >> 2, tw = (k & 3) * 4;
            u32 t32 = 0;
            for (int b = 0; b < 4; ++b) t32 |= u32(L.y[tr * 20 + 4 + tw + b]) << (8 * b);
            *reinterpret_cast<u32*>(Y + size_t(y0 - 4 + tr) * pitch + x0 + tw) = t32;
          } else if (lane >= 32) {
            const int k = lane - 32, cyr = k >> 2, cb = (k & 3) * 2;
            u32 cw = 0;
            for (int b = 0; b < 2; ++b)
              cw |= (u32(L.c[0][(cyr + 2) * 10 + 2 + cb + b]) | u32(L.c[1][(cyr + 2) * 10 + 2 + cb + b]) << 8)
                    << (16 * b);
            *reinterpret_cast<u32*>(UV + size_t(row * 8 + cyr) * pitch + (x * 8 + cb) * 2) = cw;
          }
          if (lane < 8 && left) {
            const u32 cw = u32(L.c[0][(lane + 2) * 10]) | u32(L.c[1][(lane + 2) * 10]) << 8 |
                           u32(L.c[0][(lane + 2) * 10 + 1]) << 16 | u32(L.c[1][(lane + 2) * 10 + 1]) << 24;
            *reinterpret_cast<u32*>(UV + size_t(row * 8 + lane) * pitch + (x * 8 - 2) * 2) = cw;
          } else if (lane >= 8 && lane < 16 && top) {
            const int k = lane - 8, tr = k >> 2, cb = (k & 3) * 2;
            u32 cw = 0;
            for (int b = 0; b < 2; ++b)
              cw |= (u32(L.c[0][tr * 10 + 2 + cb + b]) | u32(L.c[1][tr * 10 + 2 + cb + b]) << 8) << (16 * b);
            *reinterpret_cast<u32*>(UV + size_t(row * 8 - 2 + tr) * pitch + (x * 8 + cb) * 2) = cw;
          }
        }
        wave_sync();
        if (lane < 16)
          for (int b = 0; b < 4; ++b) L.carry[lane * 4 + b] = L.y[(lane + 4) * 20 + 16 + b];
        if (lane >= 16 && lane < 32) {
          const int c = (lane - 16) >> 3, k = (lane - 16) & 7;
          L.ccarry[c][k * 2] = L.c[c][(k + 2) * 10 + 8];
          L.ccarry[c][k * 2 + 1] = L.c[c][(k + 2) * 10 + 9];
        }
        wave_sync();
        carry = true;
      } else {
        carry = false;
      }
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

void launch_avc_deblock(const AvcDesc* d_descs, int n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(avc_deblock_kernel, dim3(unsigned(n)), dim3(64 * kWaves), 0, s, d_descs);
  VEP_HIP(hipGetLastError());
}

}  // namespace vep::gpu
