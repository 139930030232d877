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
//    MB rows. A picture runs avc_dbk_groups(H) workgroups of kAvcDbkWgRows rows each (one or
//    two rows per wave64): inside a workgroup row r waits until row r-1 has finished MB x+1 via
//    LDS progress counters (workgroup-scope release/acquire); a workgroup's first row polls the
//    previous workgroup's last row through tagged device-coherent exchange words (AvcDesc::xg).
//    That cross-workgroup spin relies on in-order dispatch: the grid order in launch_avc_*
//    puts a picture's workgroups on one XCD (one L2) in row order, so every workgroup a spin
//    waits on was dispatched earlier and is resident. Every spin is bounded (kSpinLimit): a
//    timeout sets AvcDesc::err bit 1, aborts the picture's waits so all waves drain, and the
//    worker drops the frame (logged as a wavefront timeout).
//    Per wave the MB under reconstruction lives in LDS; the left neighbour's edge columns are
//    carried in LDS (same-wave read-after-write never goes through global memory).
//
// All sample arithmetic comes from avc_recon.h, shared with the CPU reference decoder.
#define VEP_KERNEL_SOURCE 1  // descriptors' pointers are global-address-space here (gpu.h)
#include "avc_recon.h"
#include "gpu.h"

namespace vep::gpu {

using avc::MbRec;
using avc::kDenseCoefs;

namespace {

constexpr int kIntraWaves = kAvcDbkWgRows;  // intra wavefront: one row per wave, one workgroup
                                             // per kAvcDbkWgRows rows (shares AvcDesc::xg)
constexpr int kIntraXgWords = 8;  // intra exchange: 4 luma + 4 NV12 words of an MB's last line
constexpr int kIntraLine = 32;    // bytes of an MB's bottom line in LDS: 16 luma + 16 NV12
constexpr int kIntraLineCols = 240;  // LDS lines cover pictures up to 3840 samples wide
constexpr u32 kSpinLimit = 1u << 24;

__device__ inline const MbRec& rec(const AvcDesc& d, int mb) {
  return static_cast<const MbRec*>(d.mbs)[mb];
}


// wave-local barrier (one wave64 per "group" here: LDS ordering + compiler fence)
__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Global-memory accesses through address-space-1 pointers: global_load/global_store count only
// against vmcnt. Generic (flat) accesses also count against lgkmcnt, so every LDS wait would
// stall on them too — prefetches and fire-and-forget stores would serialise with the LDS work.
#define VEP_GLOBAL __attribute__((address_space(1)))
#define VEP_LDS __attribute__((address_space(3)))
__device__ inline u32 gld1(const void* p) { return *(const VEP_GLOBAL u8*)(p); }
__device__ inline u32 gld4(const void* p) { return *(const VEP_GLOBAL u32*)(p); }
// (uint2 / uint4 are classes: a copy goes through a generic reference, so the loads use the
// native vector types)
typedef u32 vu2 __attribute__((ext_vector_type(2)));
typedef u32 vu4 __attribute__((ext_vector_type(4)));
__device__ inline uint2 gld8(const void* p) {
  const vu2 v = *(const VEP_GLOBAL vu2*)(p);
  return make_uint2(v.x, v.y);
}
__device__ inline uint4 gld16(const void* p) {
  const vu4 v = *(const VEP_GLOBAL vu4*)(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ inline void gst4(void* p, u32 v) { *(VEP_GLOBAL u32*)(p) = v; }

// --------------------------------------------------------------------------------- inter

// The MB's sparse coefficient groups (avc_recon.h) expanded into the wave's dense LDS buffer D
// (kDenseCoefs entries, layout of avc::expand_coefs), whole wave: lanes 0..23 each take one mask
// word, a wave prefix sum of their popcounts places their values, and each scatters its own.
__device__ inline void expand_coefs_wave(const AvcDesc& d, const MbRec& m, int lane, i16* D) {
  if (lane < kDenseCoefs / 8) reinterpret_cast<uint4*>(D)[lane] = make_uint4(0, 0, 0, 0);
  const int nw = avc::coef_words(m);  // <= 24
  const VEP_DEV i16* pool = d.coefs + m.coef;
  u32 mask = 0;
  int base = 0;
  if (lane < nw) {
    mask = u32(u16(pool[lane]));
    base = avc::coef_word_base(m, lane);
  }
  const int cnt = __popc(mask);
  int incl = cnt;
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) {
    const int t = __shfl_up(incl, o);
    if (lane >= o) incl += t;
  }
  wave_sync();  // the zeros land before the scatter
  if (lane < nw) {
    const VEP_DEV i16* v = pool + nw + (incl - cnt);
    for (u32 b = mask; b; b &= b - 1) D[base + __ffs(int(b)) - 1] = *v++;
  }
  wave_sync();
}

// Luma residual of an 8x8-transform MB, whole wave: the four 8x8 inverse transforms as 32 row
// butterflies then 32 column butterflies (lanes 0-31, one 8-point transform each) through the
// wave's LDS buffer `T` (kT8Ints ints); afterwards T holds the MB's 16x16 residual (raster).
// The transpose runs at a row pitch of 9 (and a block pitch of 72): lane (q, i) writes row i of
// block q, so with pitch 8 the 32 lanes' stores fell on 4 banks (8-way conflicts); with 9 they
// fall on 32 distinct banks, and the column reads stay conflict-free.
constexpr int kT8Pitch = 9, kT8Block = 8 * kT8Pitch, kT8Ints = 4 * kT8Block;
static_assert(kT8Ints >= 256, "the transpose buffer also holds the 16x16 raster result");
__device__ inline void luma8_residual(const i16* D, const MbRec& m, int lane, int* T) {
  if (lane < 32) {
    const int q = lane >> 3, i = lane & 7;
    int v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if ((m.luma_coded >> ((q & 1) * 2 + (q >> 1) * 8)) & 1) {
      const uint4 w = *reinterpret_cast<const uint4*>(D + q * 64 + i * 8);
      const u32 ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[2 * k] = int(i16(ws[k] & 0xffff));
        v[2 * k + 1] = int(i16(ws[k] >> 16));
      }
      avc::idct8_1d(v);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) T[q * kT8Block + i * kT8Pitch + k] = v[k];
  }
  wave_sync();
  int c[8];
  const int q = (lane >> 3) & 3, j = lane & 7;
  if (lane < 32) {
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = T[q * kT8Block + k * kT8Pitch + j];
    avc::idct8_1d(c);
  }
  wave_sync();  // every lane has read the row pass before the buffer is overwritten
  if (lane < 32) {
#pragma unroll
    for (int k = 0; k < 8; ++k) T[((q >> 1) * 8 + k) * 16 + (q & 1) * 8 + j] = (c[k] + 32) >> 6;
  }
  wave_sync();
}

// Skip / inter / I_PCM MB of the inter kernel, whole wave, on u8 (8-bit) or u16 (High 10)
// surfaces, chroma format CF (1: 8x8 chroma per component, 2 lanes' worth of samples each;
// 2 = 4:2:2: 8x16, 4 per lane). D: the wave's dense coefficient buffer, T: its 8x8-transform
// buffer.
template <class P, int CF>
__device__ inline void inter_mb(const AvcDesc& d, const MbRec& m, int mb, int lane, int* T, i16* D, bool t8) {
  constexpr int CH = CF == 2 ? 16 : 8;  // chroma MB height
  constexpr int CS = 8 * CH;            // chroma samples per component
  constexpr int NCL = 2 * CS / 64;      // chroma samples per lane
  constexpr int NB = CF == 2 ? 8 : 4;   // chroma 4x4 blocks per component
  const int x = lane & 15, y0 = lane >> 4;  // luma sample (x, y0 + 4k), block row k
  const int W = d.wmbs, wpx = W * 16, hpx = d.hmbs * 16, pitch = wpx;
  const int mx = mb % W, my = mb / W;
  const int bd = sizeof(P) == 1 ? 8 : d.bd;
  VEP_DEV P* ty = reinterpret_cast<VEP_DEV P*>(d.y + d.slot_y * u64(d.target));
  VEP_DEV P* tuv = reinterpret_cast<VEP_DEV P*>(d.uv + d.slot_uv * u64(d.target));
  auto yref = [&](int s) { return reinterpret_cast<const VEP_DEV P*>(d.y + d.slot_y * u64(s)); };
  auto uvref = [&](int s) { return reinterpret_cast<const VEP_DEV P*>(d.uv + d.slot_uv * u64(s)); };
  // High 10 / 4:2:2 (not the 8-bit 4:2:0 hot path): bound checks of the pools, reported in *err
  constexpr bool kCheck = sizeof(P) == 2 || CF == 2;
  if (kCheck) {
    const u32 need = m.kind == avc::kIPcm ? u32((256 + 2 * CS) * sizeof(P) / 2) : 0u;
    if (u64(m.coef) + need > u64(d.ncoef)) {
      atomicOr(d.err, 0x4000u);
      return;
    }
  }
  if (m.kind == avc::kIPcm) {
    const VEP_DEV P* s = reinterpret_cast<const VEP_DEV P*>(d.coefs + m.coef);  // (u16: 384 samples)
#pragma unroll
    for (int k = 0; k < 4; ++k) ty[size_t(my * 16 + y0 + 4 * k) * pitch + mx * 16 + x] = s[(y0 + 4 * k) * 16 + x];
#pragma unroll
    for (int k = 0; k < NCL; ++k) {
      const int t = lane + 64 * k, cc = t / CS, cq = t % CS, cx = cq & 7, cy = cq >> 3;
      tuv[size_t(my * CH + cy) * pitch + (mx * 8 + cx) * 2 + cc] = s[256 + t];
    }
    return;
  }
  const i16* mvb = d.mvs + size_t(m.mv);  // the MB's vectors (granularity: m.flags)
  const bool l1 = (m.flags & avc::kMbL1) != 0;
  const avc::WpEntry* wpp =
      (m.flags & avc::kMbWp) ? static_cast<const avc::WpEntry*>(d.wps) + m.wp : nullptr;
  int v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int y = y0 + 4 * k, blk = k * 4 + (x >> 2), b8 = ((y >> 3) << 1) | (x >> 3);
    const int s0 = avc::byte_at(m.ref, b8), s1 = l1 ? avc::byte_at(m.ref1, b8) : 0xFF;
    int p0 = 0, p1 = 0;
    if (s0 != 0xFF) {
      const i16* v0 = mvb + avc::mv_sub(m.flags, 0, blk);
      p0 = avc::luma_qpel(yref(s0), pitch, wpx, hpx, mx * 16 + x + (v0[0] >> 2),
                          my * 16 + y + (v0[1] >> 2), v0[0] & 3, v0[1] & 3, bd);
    }
    if (s1 != 0xFF) {
      const i16* v1 = mvb + avc::mv_sub(m.flags, 1, blk);
      p1 = avc::luma_qpel(yref(s1), pitch, wpx, hpx, mx * 16 + x + (v1[0] >> 2),
                          my * 16 + y + (v1[1] >> 2), v1[0] & 3, v1[1] & 3, bd);
    }
    v[k] = avc::wp_sample(p0, p1, s0 != 0xFF, s1 != 0xFF, wpp ? wpp + b8 : nullptr, 0, bd);
  }
  if (m.luma_coded | m.chroma_coded) expand_coefs_wave(d, m, lane, D);  // (wave-uniform)
  if (t8) luma8_residual(D, m, lane, T);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int y = y0 + 4 * k, blk = k * 4 + (x >> 2);
    int o = v[k];
    if (t8) o += T[y * 16 + x];
    else if ((m.luma_coded >> blk) & 1) o += avc::idct4x4_at(D + 16 * blk, y & 3, x & 3);
    ty[size_t(my * 16 + y) * pitch + mx * 16 + x] = P(avc::clip1(o, bd));
  }
  int u[NCL];
  const int chp = CF == 2 ? hpx : hpx / 2;  // chroma plane height
#pragma unroll
  for (int k = 0; k < NCL; ++k) {
    const int t = lane + 64 * k, cc = t / CS, cq = t % CS, cx = cq & 7, cy = cq >> 3;
    const int ly = CF == 2 ? cy : 2 * cy;  // luma row of the sample
    const int r = (ly >> 2) * 4 + (cx >> 1), b8 = ((ly >> 3) << 1) | (cx >> 2);
    const int s0 = avc::byte_at(m.ref, b8), s1 = l1 ? avc::byte_at(m.ref1, b8) : 0xFF;
    int p0 = 0, p1 = 0, ix, fx, iy, fy;
    if (s0 != 0xFF) {
      const i16* v0 = mvb + avc::mv_sub(m.flags, 0, r);
      const int vy = v0[1] + (d.field ? 2 * ((d.field == 2) - (s0 & 1)) : 0);  // opposite-parity field
      avc::chroma_mv(v0[0], vy, CF, ix, fx, iy, fy);
      p0 = avc::chroma_epel(uvref(s0), pitch, wpx / 2, chp, cc, mx * 8 + cx + ix, my * CH + cy + iy, fx, fy);
    }
    if (s1 != 0xFF) {
      const i16* v1 = mvb + avc::mv_sub(m.flags, 1, r);
      const int vy = v1[1] + (d.field ? 2 * ((d.field == 2) - (s1 & 1)) : 0);
      avc::chroma_mv(v1[0], vy, CF, ix, fx, iy, fy);
      p1 = avc::chroma_epel(uvref(s1), pitch, wpx / 2, chp, cc, mx * 8 + cx + ix, my * CH + cy + iy, fx, fy);
    }
    u[k] = avc::wp_sample(p0, p1, s0 != 0xFF, s1 != 0xFF, wpp ? wpp + b8 : nullptr, 1 + cc, bd);
  }
#pragma unroll
  for (int k = 0; k < NCL; ++k) {
    const int t = lane + 64 * k, cc = t / CS, cq = t % CS, cx = cq & 7, cy = cq >> 3;
    const int kb = cc * NB + (cy >> 2) * 2 + (cx >> 2);
    int o = u[k];
    if ((m.chroma_coded >> kb) & 1) o += avc::idct4x4_at(D + 256 + 16 * kb, cy & 3, cx & 3);
    tuv[size_t(my * CH + cy) * pitch + (mx * 8 + cx) * 2 + cc] = P(avc::clip1(o, bd));
  }
}

// One wave64 per MB, four MBs per workgroup: each lane reconstructs 4 luma samples (one per
// 4x4-block row) and 2 chroma samples, so a lane has all of its reference loads in flight at
// once and the picture lookup / record / MV loads are paid once per wave instead of per
// 64 samples. List-0 / list-1 predictions are combined by avc::wp_sample (default average or
// the MB's weighted-prediction entries); 8x8-transform residuals go through LDS.
__global__ __launch_bounds__(256) void avc_inter_kernel(const AvcDesc* __restrict__ descs, int n,
                                                         int total) {
  __shared__ int lres[4][kT8Ints];
  __shared__ alignas(16) i16 lcoef[4][kDenseCoefs];  // the wave's MB coefficients, dense
  const int wv = int(threadIdx.x) >> 6;
  const int g = __builtin_amdgcn_readfirstlane(int(blockIdx.x) * 4 + wv);
  if (g >= total) return;  // (wave-uniform; the kernel has no workgroup barrier)
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (descs[mid].mb_begin <= g) lo = mid;
    else hi = mid - 1;
  }
  const AvcDesc d = descs[lo];
  const int mb = g - d.mb_begin;
  const MbRec m = rec(d, mb);
  const int lane = int(threadIdx.x) & 63;
  const int x = lane & 15, y0 = lane >> 4;  // luma sample (x, y0 + 4k), block row k
  int* T = lres[wv];
  const bool t8 = (m.flags & avc::kMbT8x8) && m.luma_coded;
  if (avc::is_wave_intra(m.kind)) {
    const int row = mb / d.wmbs;  // clear the intra wavefront's exchange tags of this MB
    if (lane < kIntraXgWords && row % kAvcDbkWgRows == kAvcDbkWgRows - 1 && row + 1 < d.hmbs)
      d.xg[(size_t(row / kAvcDbkWgRows) * d.wmbs + mb % d.wmbs) * kAvcXgWords + lane] = 0;
    // Intra MB: its residual samples do not depend on the prediction, so they are computed here
    // in parallel and the intra wavefront only adds them (same layout as IntraWave::res).
    if (m.res == avc::kNoRes) return;
    if ((d.bd > 8 || d.cf == 2) && m.res >= d.nres) {  // (High 10 / 4:2:2: bound check)
      atomicOr(d.err, 0x8000u);
      return;
    }
    i16* r = d.res + size_t(m.res) * kAvcResSamples;
    i16* D = lcoef[wv];
    expand_coefs_wave(d, m, lane, D);
    if (t8) luma8_residual(D, m, lane, T);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int y = y0 + 4 * k, blk = k * 4 + (x >> 2);
      int v;
      if (t8) v = T[y * 16 + x];
      else v = (m.luma_coded >> blk) & 1 ? avc::idct4x4_at(D + 16 * blk, y & 3, x & 3) : 0;
      r[y * 16 + x] = i16(v);
    }
    const int ncs = d.cf == 2 ? 128 : 64, nb = d.cf == 2 ? 8 : 4;  // (4:2:2: 8x16 chroma)
    for (int k = 0; k < 2 * ncs / 64; ++k) {
      const int t = lane + 64 * k, cc = t / ncs, cq = t % ncs, cx = cq & 7, cy = cq >> 3;
      const int kb = cc * nb + (cy >> 2) * 2 + (cx >> 2);
      r[256 + t] = i16((m.chroma_coded >> kb) & 1 ? avc::idct4x4_at(D + 256 + 16 * kb, cy & 3, cx & 3) : 0);
    }
    return;
  }
  if (m.kind != avc::kSkip && m.kind != avc::kInter && m.kind != avc::kIPcm) return;
  if (d.cf == 2) {
    if (d.bd > 8) inter_mb<u16, 2>(d, m, mb, lane, T, lcoef[wv], t8);
    else inter_mb<u8, 2>(d, m, mb, lane, T, lcoef[wv], t8);
  } else if (d.bd > 8) {
    inter_mb<u16, 1>(d, m, mb, lane, T, lcoef[wv], t8);
  } else {
    inter_mb<u8, 1>(d, m, mb, lane, T, lcoef[wv], t8);
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

// Tagged exchange words between the workgroups of one picture's wavefront (AvcDesc::xg): device-scope relaxed atomics (global_{load,store}_dwordx2 sc1, past
// the per-CU L1), single-copy atomic, so a reader sees a word's data and tag together.
__device__ inline void xg_put(u64* p, u32 v, u32 tag) {
  __hip_atomic_store((VEP_GLOBAL u64*)p, u64(tag) << 32 | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline u64 xg_get(u64* p) {
  return __hip_atomic_load((VEP_GLOBAL u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// --------------------------------------------------------------------------------- intra

constexpr int kTp = 28;  // luma tile pitch: row 0 = p[-1..23, -1] (Intra_8x8 top-right reaches
                         // p[23,-1]), rows 1..16 = p[-1..15, y]; 4 * kTp must fit the 7-bit
                         // Intra_4x4 tap offsets
constexpr int kCp = 12;  // chroma tile pitch: row 0 = p[-1..7, -1], rows 1..8 = p[-1..7, y]

struct alignas(16) IntraWave {
  MbRec rec[64];      // records of the current 64-MB chunk of the row
  i16 res[384];       // residual samples: 256 luma (raster) + 2 x 64 chroma (from the inter pass)
  u32 taps[256];      // Intra_4x4 tap words of the MB's samples
  u8 pf[32];          // Intra_8x8 filtered references of the current 8x8 block
  u8 tile[17 * kTp];  // luma neighbours + the MB being reconstructed (branch-free addressing)
  u8 ctile[2][9 * kCp];
  u8 carry[16];       // right luma column of the previous MB of this row (if this wave built it)
  u8 ccarry[2][8];
  u8 up[68];          // row above, MBs base-1 .. base+64 of the chunk: intra (published in xg)?
};

// h0 / h3: words 0 and 3 of the neighbour's MbRec (kind in byte 0, slice in bytes 14..15)
__device__ inline bool avail_hdr(const AvcDesc& d, u32 h0, u32 h3, bool in_pic, u16 slice) {
  if (!in_pic) return false;
  const u8 kind = u8(h0 & 0xff);
  if (u16(h3 >> 16) != slice) return false;
  return !(d.constrained && !avc::is_intra(kind));
}

// One intra MB, whole wave: one round trip of global loads (all issued before any is used),
// a parallel residual pass, then prediction out of LDS.
//
// The first row of a workgroup reads the row above's intra MBs (reconstructed by the previous
// workgroup in this same launch) from `xi_in` (tag 1 = final), polled per sample word;
// `up_intra[n]` says whether MB n of the row above is such an MB. The last row of a workgroup
// publishes its bottom lines to `xi_out`.
__device__ void intra_mb(const AvcDesc& d, IntraWave& L, const MbRec& m, int x, int row, bool carry,
                         int lane, const u32* tap_lut, const u32* tap8_lut, u64 t_start, u64* acc, Sync& sync,
                         int wave,
                         u32 wait_need, u64* xi_in, const u8* up_intra, const u8* line_in, u8* line_out,
                         u64* xi_out) {
  const int W = d.wmbs, pitch = W * 16;
  u8* Y = d.y + d.slot_y * u64(d.target);
  u8* UV = d.uv + d.slot_uv * u64(d.target);
  const int x0 = x * 16, y0 = row * 16;
  const bool up = row > 0, lf = x > 0;
  const MbRec* recs = static_cast<const MbRec*>(d.mbs);
  // ---- loads that do not depend on the row above, issued before waiting for it: residual
  // samples, the left column (a left MB that is not carried is inter / I_PCM, final since the
  // inter kernel), neighbour headers, and top samples of non-intra MBs above
  // residual samples (768 B = 48 lanes x 16 B), computed by the parallel inter pass.
  // Every load below is ONE full-wave instruction from an address valid in every lane (unused
  // lanes read a dummy, selected away after the wait): a load issued under a lane branch shares
  // its destination VGPR with the other lanes' default, so the default's write had to wait for
  // the load (vmcnt(0)) and every later load was serialised behind it.
  const bool has_res = m.res != avc::kNoRes;  // (wave-uniform)
  uint4 cv;  // (undefined without residual: never read)
  if (has_res)
    cv = gld16(reinterpret_cast<const uint4*>(d.res + size_t(m.res) * kAvcResSamples) + (lane < 48 ? lane : 47));
  // where sample `a` of a lane comes from: 0 = the early load below (ga_ok) or none, 1 = previous
  // workgroup's exchange word, 2 = this workgroup's LDS line of the row above, 3 = the picture
  // (the row above's intra MBs, no LDS line), read once the row above is ready
  int src = 0, xw = -1, xsh = 0, lo = 0;
  const u8* gp = Y;
  const u8* ga = Y;  // early source of `a` (ga_ok), else a dummy
  bool ga_ok = false;
  auto top = [&](int n, const u8* g, int word, int sh, int lo_off) {
    if (!up_intra || !up_intra[n]) {
      ga = g;
      ga_ok = true;
    } else if (xi_in) {
      src = 1;
      xw = n * kAvcXgWords + word;
      xsh = sh;
    } else if (line_in) {
      src = 2;
      lo = n * kIntraLine + lo_off;
    } else {
      src = 3;
      gp = g;
    }
  };
  if (lane < 25) {  // luma row above: x0-1 .. x0+23
    const int px = x0 - 1 + lane;
    if (up && px >= 0 && px < pitch)
      top(px >> 4, &Y[size_t(y0 - 1) * pitch + px], (px & 15) >> 2, (px & 3) * 8, px & 15);
  } else if (lane < 41) {  // luma left column
    if (lf && !carry) {
      ga = &Y[size_t(y0 + lane - 25) * pitch + x0 - 1];
      ga_ok = true;
    }
  } else if (lane < 59) {  // chroma row above: x*8-1 .. x*8+7 per component
    const int c = (lane - 41) / 9, k = (lane - 41) % 9, px = x * 8 - 1 + k;
    if (up && px >= 0) {
      const int bo = (px & 7) * 2 + c;  // byte of the MB's NV12 bottom line
      top(px >> 3, &UV[size_t(row * 8 - 1) * pitch + px * 2 + c], 4 + (bo >> 2), (bo & 3) * 8, 16 + bo);
    }
  }
  const u32 ra = gld1(ga);
  const u8* gb = UV;  // chroma left columns (lanes 48..63), else a dummy
  const bool gb_ok = lane >= 48 && lf && !carry;
  if (gb_ok) gb = &UV[size_t(row * 8 + ((lane - 48) & 7)) * pitch + (x * 8 - 1) * 2 + ((lane - 48) >> 3)];
  const u32 rb = gld1(gb);
  // neighbour record headers: B, C, D, A (lanes 56..59)
  bool in_pic = false;
  if (lane == 56) in_pic = up;
  else if (lane == 57) in_pic = up && x + 1 < W;
  else if (lane == 58) in_pic = up && lf;
  else if (lane == 59) in_pic = lf;
  const int hnx = lane == 56 ? x : lane == 57 ? x + 1 : x - 1, hny = lane == 59 ? row : row - 1;
  // (words 0 and 3 only: a dead component of a wider load is a register the compiler reuses,
  // which would wait for the load to land)
  const u32* hp = reinterpret_cast<const u32*>(&recs[in_pic ? hny * W + hnx : 0]);  // (read only where in_pic)
  const u32 h0 = gld4(hp), h3 = gld4(hp + 3);
  // ---- the row above: this workgroup's (LDS counter, then LDS line / picture) or the
  // previous workgroup's (exchange words, polled)
  const u64 t_wait = d.prof ? clock64() : 0;
  if (wait_need) wait_row(sync, wave - 1, wait_need, d.err);
  u32 xv = 0;
  if (xi_in) {  // (wave-uniform) poll the published words until every one is final
    u64 v = src == 1 ? xg_get(xi_in + xw) : 0;
    u32 spins = 0;
    while (__ballot(src == 1 && u32(v >> 32) != 1u)) {
      if (__hip_atomic_load(&sync.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
      if (++spins > (kSpinLimit >> 4)) {
        __hip_atomic_store(&sync.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (lane == 0) atomicOr(d.err, 2u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      if (src == 1) v = xg_get(xi_in + xw);
    }
    if (src == 1) xv = u32(v >> xsh) & 0xffu;
  }
  // the other sources, again one full-wave load each (line_in / xi_in are wave-uniform; lanes
  // that do not read one use a valid dummy address), then one select per lane
  u32 lv = 0, gv = 0;
  if (line_in) lv = *(const VEP_LDS u8*)(line_in + lo);
  else if (!xi_in) gv = gld1(gp);
  const u32 a = src == 1 ? xv : src == 2 ? lv : src == 3 ? gv : ga_ok ? ra : 128u;
  const u32 b = gb_ok ? rb : 128u;
  const u64 waited = d.prof ? clock64() - t_wait : 0;
  acc[0] += waited;
  // ---- availability (B, C, D, A) and the LDS neighbour tiles
  const bool av = avail_hdr(d, h0, h3, in_pic, m.slice);
  const bool B = __builtin_amdgcn_readlane(int(av), 56) != 0;
  const bool C = __builtin_amdgcn_readlane(int(av), 57) != 0;
  const bool D = __builtin_amdgcn_readlane(int(av), 58) != 0;
  const bool A = __builtin_amdgcn_readlane(int(av), 59) != 0;
  if (lane < 48) reinterpret_cast<uint4*>(L.res)[lane] = has_res ? cv : make_uint4(0, 0, 0, 0);
  if (lane < 25) {
    L.tile[lane] = u8((lane == 0 ? D : lane <= 16 ? B : C) ? a : 128u);
  } else if (lane < 41) {
    const int k = lane - 25;
    L.tile[(k + 1) * kTp] = !A ? u8(128) : carry ? L.carry[k] : u8(a);
  } else if (lane < 59) {
    const int c = (lane - 41) / 9, k = (lane - 41) % 9;
    L.ctile[c][k] = u8((k == 0 ? D : B) ? a : 128u);
  }
  if (lane >= 48) {
    const int c = (lane - 48) >> 3, k = (lane - 48) & 7;
    L.ctile[c][(k + 1) * kCp] = !A ? u8(128) : carry ? L.ccarry[c][k] : u8(b);
  }
  wave_sync();
  const u64 t_loaded = d.prof ? clock64() : 0;
  const u64 t_res = d.prof ? clock64() : 0;
  // ---- luma prediction
  auto P = [&](int ax, int ay) -> int { return L.tile[(ay + 1) * kTp + ax + 1]; };
  if (m.kind == avc::kI16x16) {
    // DC / plane constants: the neighbour sums by a wave reduction instead of 32 reads per lane
    int st = 0, sl = 0, H = 0, V = 0;
    if (lane < 16) st = P(lane, -1);
    else if (lane < 32) sl = P(-1, lane - 16);
    else if (lane < 40) H = (lane - 31) * (P(8 + lane - 32, -1) - P(6 - (lane - 32), -1));
    else if (lane < 48) {
      const int i = lane - 40;
      V = (i + 1) * (P(-1, 8 + i) - (6 - i >= 0 ? P(-1, 6 - i) : P(-1, -1)));
    }
    for (int off = 32; off > 0; off >>= 1) {
      st += __shfl_xor(st, off);
      sl += __shfl_xor(sl, off);
      H += __shfl_xor(H, off);
      V += __shfl_xor(V, off);
    }
    const avc::PredConst pk =
        avc::intra16x16_const_from_sums(m.i16_mode, B, A, st, sl, H, V, P(15, -1), P(-1, 15));
    auto T = [&](int xx) { return P(xx, -1); };
    auto Lf = [&](int yy) { return P(-1, yy); };
    u8 out[4];
    for (int k = 0; k < 4; ++k) {
      const int p = lane + 64 * k, px = p & 15, py = p >> 4;
      out[k] = u8(avc::clip1(avc::intra16x16_pred_g(T, Lf, pk, m.i16_mode, px, py) + L.res[p]));
    }
    wave_sync();  // every lane has read the neighbours before the MB is written over them
    for (int k = 0; k < 4; ++k) {
      const int p = lane + 64 * k;
      L.tile[((p >> 4) + 1) * kTp + (p & 15) + 1] = out[k];
    }
  } else if (m.kind == avc::kI8x8) {
    // Intra_8x8 in tap form (avc::intra8x8_filter_tap / intra8x8_pred_tap): four blocks in
    // order; per block lanes 0-24 filter the 25 reference samples (§8.3.2.2.1) into LDS, three
    // loads and one multiply-add each, then every lane predicts its sample from its tap word
    // (DC: a wave reduction) and adds its residual. No lane-divergent path per filter position
    // or prediction mode, so each step is one round of LDS loads.
    const int px = lane & 7, py = lane >> 3;
    for (int q = 0; q < 4; ++q) {
      const int bx = q & 1, by = q >> 1;
      const bool top = by > 0 || B, left = bx > 0 || A;
      const bool tl = (bx > 0 && by > 0) || (bx == 0 && by == 0 ? D : bx == 0 ? A : B);
      const bool tr = by == 0 ? (bx == 0 ? B : C) : (bx == 0);
      const u8* nb = &L.tile[(by * 8) * kTp + bx * 8];  // p[-1,-1] of the block
      const int mode = avc::i4_mode(m, q);
      const int rs = L.res[(by * 8 + py) * 16 + bx * 8 + px];
      const u32 pw = tap8_lut[mode * 64 + lane];
      if (lane < 25) {
        const u32 fw = avc::intra8x8_filter_tap(top, left, tl, lane);
        // sample u of the layout -> tile offset from p[-1,-1] (two selects: p[-1,-1] = 0,
        // p[x,-1] = 1 + x with the top-right substitution, p[-1,y] = (y + 1) * kTp)
        auto off = [&](u32 u) -> int { return u > 16 ? int(u - 16) * kTp : (u >= 9 && !tr) ? 8 : int(u); };
        const int s0 = nb[off(fw & 31)], s1 = nb[off((fw >> 5) & 31)], s2 = nb[off((fw >> 10) & 31)];
        const int fv = avc::eval_tap8(fw, s0, s1, s2);  // (kTap8Const: indices 0, value unused)
        L.pf[lane] = u8((fw & avc::kTap8Const) ? 128 : fv);
      }
      wave_sync();
      int v;
      if (mode == 2) {  // (wave-uniform)
        int sv = lane < 8 ? (top ? int(L.pf[1 + lane]) : 0) : lane < 16 ? (left ? int(L.pf[9 + lane]) : 0) : 0;
        for (int o = 8; o > 0; o >>= 1) sv += __shfl_xor(sv, o);
        sv = __shfl(sv, 0);
        v = top && left ? (sv + 8) >> 4 : (top || left) ? (sv + 4) >> 3 : 128;
      } else {
        v = avc::eval_tap8(pw, L.pf[pw & 31], L.pf[(pw >> 5) & 31], L.pf[(pw >> 10) & 31]);
      }
      L.tile[(by * 8 + py + 1) * kTp + bx * 8 + px + 1] = u8(avc::clip1(v + rs));
      wave_sync();
    }
  } else {
    // Tap words of all 256 samples: the (mode, y, x) table entry with its neighbour indices
    // resolved to tile offsets from the block's top-left neighbour (top-right substitution and
    // availability folded in), so the dependent steps below are plain loads + one multiply-add.
    //   non-DC: bits 0-6 / 7-13 / 14-20 offsets, 21-30 weights/add/shift; DC: bit 31, 21 top
    //   available, 22 left available
    for (int k = 0; k < 4; ++k) {
      const int p = lane + 64 * k, px = p & 15, py = p >> 4, bx = px >> 2, byy = py >> 2;
      const int r = byy * 4 + bx;
      const u32 tw = tap_lut[avc::i4_mode(m, r) * 16 + (py & 3) * 4 + (px & 3)];
      u32 word;
      if (tw & avc::kTapDc) {
        word = 1u << 31 | u32(byy > 0 || B) << 21 | u32(bx > 0 || A) << 22;
      } else {
        const bool tr = byy == 0 ? (bx < 3 ? B : C)
                                 : (bx < 3 && avc::raster_to_blk((byy - 1) * 4 + bx + 1) < avc::raster_to_blk(r));
        auto rel = [&](u32 n) -> u32 {
          return n == 0 ? 0u : n <= 8 ? 1u + ((n - 1 >= 4 && !tr) ? 3u : n - 1) : (n - 8) * u32(kTp);
        };
        word = rel(tw & 15) | rel((tw >> 4) & 15) << 7 | rel((tw >> 8) & 15) << 14 | ((tw >> 12) & 1023u) << 21;
      }
      L.taps[p] = word;
    }
    wave_sync();
    // Diagonal schedule: block (bx, by) only reads left / top / top-left / (when available in
    // coding order) top-right neighbours, all on earlier diagonals s = bx + 2 * by: 10 steps of
    // at most 2 blocks (lanes 0-15 and 16-31). Every step's tap word and residual sample are
    // loaded up front, so a step is only its neighbour reads, a multiply-add and one store.
    const int g = lane >> 4, i = (lane >> 2) & 3, j = lane & 3;
    auto slot = [&](int st) -> int {  // sample of this lane at step st, -1 if none
      // blocks of diagonal st: (st - 2*yy, yy) for yy = max(0, (st - 3 + 1) / 2) .. min(3, st / 2)
      const int y_lo = st > 3 ? (st - 2) / 2 : 0, y_hi = st / 2 < 3 ? st / 2 : 3;
      const int yy = y_lo + g;
      return g < 2 && yy <= y_hi ? (yy * 4 + i) * 16 + (st - 2 * yy) * 4 + j : -1;
    };
    u32 tws[10];
    int rss[10];
#pragma unroll
    for (int st = 0; st < 10; ++st) {
      const int p = slot(st);
      tws[st] = p >= 0 ? L.taps[p] : 0u;
      rss[st] = p >= 0 ? L.res[p] : 0;
    }
#pragma unroll
    for (int st = 0; st < 10; ++st) {
      const int p = slot(st);
      if (p >= 0) {
        const int yy = p >> 6, bx = (p & 15) >> 2;
        const u32 tw = tws[st];
        const u8* nb = &L.tile[(yy * 4) * kTp + bx * 4];  // neighbour N[0] (top-left) of the block
        int v;
        if (tw >> 31) {
          int st4 = 0, sl4 = 0;
          for (int q = 0; q < 4; ++q) {
            st4 += nb[1 + q];
            sl4 += nb[(q + 1) * kTp];
          }
          const bool ht = (tw >> 21) & 1, hl = (tw >> 22) & 1;
          v = ht && hl ? (st4 + sl4 + 4) >> 3 : hl ? (sl4 + 2) >> 2 : ht ? (st4 + 2) >> 2 : 128;
        } else {
          const int n0 = nb[tw & 127], n1 = nb[(tw >> 7) & 127], n2 = nb[(tw >> 14) & 127];
          v = (int((tw >> 21) & 3) * n0 + int((tw >> 23) & 3) * n1 + int((tw >> 25) & 3) * n2 +
               int((tw >> 27) & 3)) >> int((tw >> 29) & 3);
        }
        v += rss[st];
        L.tile[(yy * 4 + i + 1) * kTp + bx * 4 + j + 1] = u8(avc::clip1(v));
      }
      wave_sync();
    }
  }
  const u64 t_luma = d.prof ? clock64() : 0;
  // ---- chroma (2 samples per lane)
  {
    u8 out[2];
    for (int k = 0; k < 2; ++k) {
      const int p = lane + 64 * k, c = p >> 6, q = p & 63, px = q & 7, py = q >> 3;
      const u8* t = L.ctile[c];
      auto T = [&](int xx) { return int(t[xx + 1]); };
      auto Lf = [&](int yy) { return int(t[(yy + 1) * kCp]); };
      const avc::PredConst pk =
          m.chroma_mode == 3 ? avc::chroma_plane_const_g(T, Lf) : avc::PredConst{0, 0, 0, 0};
      out[k] = u8(avc::clip1(avc::chroma_pred_g(T, Lf, B, A, pk, m.chroma_mode, px, py) + L.res[256 + p]));
    }
    wave_sync();
    for (int k = 0; k < 2; ++k) {
      const int p = lane + 64 * k, c = p >> 6, q = p & 63;
      L.ctile[c][((q >> 3) + 1) * kCp + (q & 7) + 1] = out[k];
    }
  }
  wave_sync();
  const u64 t_chroma = d.prof ? clock64() : 0;
  // ---- write back + carry the right column for the next MB of this row
  {
    const int ry = lane >> 2, rx = (lane & 3) * 4;
    const u8* src = &L.tile[(ry + 1) * kTp + rx + 1];
    const u32 w = u32(src[0]) | u32(src[1]) << 8 | u32(src[2]) << 16 | u32(src[3]) << 24;
    gst4(Y + size_t(y0 + ry) * pitch + x0 + rx, w);
    if (xi_out && lane >= 60) xg_put(xi_out + size_t(x) * kAvcXgWords + (lane - 60), w, 1u);
    if (line_out && lane >= 60) *(VEP_LDS u32*)(line_out + x * kIntraLine + (lane - 60) * 4) = w;
    if (lane < 32) {  // NV12: 8 rows x 16 bytes
      const int cyr = lane >> 2, cxb = (lane & 3) * 2;
      const u8* c0 = &L.ctile[0][(cyr + 1) * kCp + cxb + 1];
      const u8* c1 = &L.ctile[1][(cyr + 1) * kCp + cxb + 1];
      const u32 cw = u32(c0[0]) | u32(c1[0]) << 8 | u32(c0[1]) << 16 | u32(c1[1]) << 24;
      gst4(UV + size_t(row * 8 + cyr) * pitch + (x * 8 + cxb) * 2, cw);
      if (xi_out && lane >= 28) xg_put(xi_out + size_t(x) * kAvcXgWords + 4 + (lane - 28), cw, 1u);
      if (line_out && lane >= 28) *(VEP_LDS u32*)(line_out + x * kIntraLine + 16 + (lane - 28) * 4) = cw;
    }
    if (lane < 16) L.carry[lane] = L.tile[(lane + 1) * kTp + 16];
    if (lane < 16) L.ccarry[lane >> 3][lane & 7] = L.ctile[lane >> 3][((lane & 7) + 1) * kCp + 8];
  }
  wave_sync();
  if (d.prof) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // count the store drain here
    const u64 t_end = clock64();
    acc[1] += t_loaded - t_start - waited;
    acc[2] += t_luma - t_res;
    acc[6] += t_res - t_loaded;
    acc[3] += t_chroma - t_luma;
    acc[4] += t_end - t_chroma;
    acc[5] += 1;
  }
}

// One row per wave, kIntraWaves rows per workgroup, avc_dbk_groups(H) workgroups per picture
// (same XCD-aware grid order as the deblocking wavefront): rows of a workgroup synchronise
// through LDS counters, a workgroup's first row polls the previous workgroup's published lines.
__global__ __launch_bounds__(64 * kIntraWaves) void avc_intra_kernel(const AvcDesc* __restrict__ descs,
                                                                      int n, int groups) {
  const int b = int(blockIdx.x), j = b >> 3;
  const int pic = (j / groups) * 8 + (b & 7), grp = j % groups;
  if (pic >= n) return;
  const AvcDesc d = descs[pic];  // by value: SGPRs, no reloads after stores
  const int W = d.wmbs, H = d.hmbs, g0 = grp * kIntraWaves;
  if (g0 >= H || d.bd > 8 || d.cf == 2) return;  // (uniform over the workgroup, before any barrier;
                                                  // High 10 / 4:2:2: avc_hbd_kernel)
  __shared__ Sync sync;
  __shared__ IntraWave lds[kIntraWaves];
  __shared__ u32 tap_lut[9 * 16];  // Intra_4x4 tap word per (mode, y, x) of a 4x4 block
  __shared__ u32 tap8_lut[9 * 64];  // Intra_8x8 tap word per (mode, y, x) of an 8x8 block
  // bottom lines of the intra MBs of rows 0..6 for the row below (pictures up to kIntraLineCols
  // MBs wide; wider ones read the picture)
  __shared__ u8 lines[kIntraWaves - 1][kIntraLineCols * kIntraLine];
  for (int t = int(threadIdx.x); t < 9 * 16; t += int(blockDim.x)) {
    const int mode = t >> 4, y = (t >> 2) & 3, x = t & 3;
    tap_lut[t] = mode == 2 ? avc::kTapDc : avc::pack_taps(avc::intra4x4_taps(mode, x, y));
  }
  for (int t = int(threadIdx.x); t < 9 * 64; t += int(blockDim.x))
    tap8_lut[t] = avc::intra8x8_pred_tap(t >> 6, t & 7, (t >> 3) & 7);
  sync_init(sync, kIntraWaves);  // (its barrier also publishes the table)
  const int wave = int(threadIdx.x) >> 6, lane = int(threadIdx.x) & 63;
  IntraWave& L = lds[wave];
  const MbRec* recs = static_cast<const MbRec*>(d.mbs);
  const int row = g0 + wave;
  const bool xin = grp > 0 && wave == 0;
  u64* xi_in = xin ? d.xg + size_t(grp - 1) * W * kAvcXgWords : nullptr;
  u64* xi_out = wave == kIntraWaves - 1 && row + 1 < H ? d.xg + size_t(grp) * W * kAvcXgWords : nullptr;
  const bool use_lines = W <= kIntraLineCols;
  const u8* line_in = use_lines && wave > 0 ? lines[wave - 1] : nullptr;
  u8* line_out = use_lines && wave + 1 < kIntraWaves ? lines[wave] : nullptr;
  u64 acc[7] = {0, 0, 0, 0, 0, 0, 0};  // phase clocks of this wave (flushed once at the end)
  if (row < H) {
    int prev = -2;
    for (int base = 0; base < W; base += 64) {
      // ---- the chunk's records into LDS (one round trip) and its intra MBs by ballot
      const int x = base + lane;
      bool intra = false;
      if (x < W) {
        constexpr int kWords = int(sizeof(MbRec) / sizeof(uint2));
        const uint2* src = reinterpret_cast<const uint2*>(&recs[row * W + x]);
        uint2* dst = reinterpret_cast<uint2*>(&L.rec[lane]);
        uint2 q[kWords];
        for (int k = 0; k < kWords; ++k) q[k] = gld8(src + k);
        for (int k = 0; k < kWords; ++k) dst[k] = q[k];
        intra = avc::is_wave_intra(u8(q[0].x & 0xff));
      }
      if (row > 0)  // which MBs base-1 .. base+64 of the row above are intra (this wavefront's)
        for (int q = lane; q < 66; q += 64) {
          const int ax = base - 1 + q;
          u8 v = 0;
          if (ax >= 0 && ax < W) {
            v = avc::is_wave_intra(u8(gld1(&recs[(row - 1) * W + ax].kind)));
          }
          L.up[q] = v;
        }
      const u64 mask = __ballot(intra);
      wave_sync();
      for (u64 bits = mask; bits; bits &= bits - 1) {
        const int xx = base + __ffsll(static_cast<unsigned long long>(bits)) - 1;
        const u64 t0 = d.prof ? clock64() : 0;
        publish_row(sync, wave, u32(xx));  // every MB left of xx is final
        // (intra_mb waits for the row above itself, after issuing the loads that do not need it)
        intra_mb(d, L, L.rec[xx - base], xx, row, prev == xx - 1, lane, tap_lut, tap8_lut, t0, acc, sync, wave,
                 wave > 0 ? u32(xx + 2 < W ? xx + 2 : W) : 0u, xi_in, row > 0 ? &L.up[1] - base : nullptr,
                 line_in, line_out, xi_out);
        prev = xx;
      }
    }
    publish_row(sync, wave, u32(W));
  }
  if (d.prof && lane == 0) {
    for (int k = 0; k < 6; ++k) atomicAdd(&d.prof[k], acc[k]);
    atomicAdd(&d.prof[11], acc[6]);
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
  const AvcDesc d = descs[lo];
  const int mb = g - d.mb_begin, W = d.wmbs, x = mb % W, row = mb / W;
  if (row % kAvcDbkWgRows == kAvcDbkWgRows - 1 && row + 1 < d.hmbs) {  // clear the deblock
    uint4* z = reinterpret_cast<uint4*>(                                  // exchange tags
        d.xg + (size_t(row / kAvcDbkWgRows) * W + x) * kAvcXgWords);
    for (int k = 0; k < kAvcXgWords / 2; ++k) z[k] = make_uint4(0, 0, 0, 0);
  }
  const MbRec q = rec(d, mb);
  AvcDbkInfo info{};
  if (!(q.dbk & 1)) {
    // (absent neighbours read as the MB itself, by index: a select between a loaded record and
    // the local q takes q's address and puts it in scratch)
    const MbRec lm = rec(d, x > 0 ? mb - 1 : mb);
    const MbRec tm = rec(d, row > 0 ? mb - W : mb);
    const bool left = x > 0 && !((q.dbk & 2) && lm.slice != q.slice);
    const bool top = row > 0 && !((q.dbk & 2) && tm.slice != q.slice);
    const i16* mq = avc::is_intra(q.kind) ? nullptr : d.mvs + size_t(q.mv);
    const i16* ml = avc::is_intra(lm.kind) ? nullptr : d.mvs + size_t(lm.mv);
    const i16* mt = avc::is_intra(tm.kind) ? nullptr : d.mvs + size_t(tm.mv);
    const bool t8 = (q.flags & avc::kMbT8x8) != 0;
    const avc::BsSide sq = avc::bs_side(q), sl = avc::bs_side(lm), st = avc::bs_side(tm);
    // (the 32 nibbles gathered in two 64-bit registers, one per direction: an index into
    // info.bs that varies with the loop counters put the whole struct in scratch memory)
    u64 bsw[2] = {0, 0};
    for (int dir = 0; dir < 2; ++dir)
      for (int e = 0; e < 4; ++e) {
        if (e == 0 && !(dir == 0 ? left : top)) continue;
        // no 4x4 edges inside 8x8 transform blocks — except, in 4:2:2, the horizontal ones the
        // chroma filters (avc_hbd_kernel skips them for luma)
        if ((e & 1) && t8 && !(d.cf == 2 && dir == 1)) continue;
        // (the sides as scalar words, selected by value: a record chosen at run time among
        // locals, or a pointer into one, needs their addresses and puts them in scratch)
        const avc::BsSide p = e > 0 ? sq : (dir == 0 ? sl : st);
        const i16* mp = e > 0 ? mq : (dir == 0 ? ml : mt);
        for (int sg = 0; sg < 4; ++sg) {
          const int bq = dir == 0 ? sg * 4 + e : e * 4 + sg;
          const int bp = e > 0 ? (dir == 0 ? bq - 1 : bq - 4) : (dir == 0 ? bq + 3 : bq + 12);
          const int bs = avc::boundary_strength(p, bp, mp, sq, bq, mq, e == 0, d.field != 0, dir == 0);
          const u64 v = u64(bs) << (4 * (e * 4 + sg));
          if (dir == 0) bsw[0] |= v;
          else bsw[1] |= v;
        }
      }
    info.bs[0] = u32(bsw[0]);
    info.bs[1] = u32(bsw[0] >> 32);
    info.bs[2] = u32(bsw[1]);
    info.bs[3] = u32(bsw[1] >> 32);
    info.any = (bsw[0] | bsw[1]) ? 1 : 0;
    // thresholds at 8-bit scale (QPs less the QpBdOffset bias; avc_hbd_kernel shifts them by
    // bd - 8)
    // (the P-side record by value select, not through an array of pointers to the locals, which
    // would put the records in scratch)
    const int qb = d.qp_bias, qcb = d.qpc_bias;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const MbRec& pk = k == 0 ? lm : (k == 1 ? tm : q);
      const avc::EdgeParams ep[3] = {avc::edge_params(pk.qp - qb, q.qp - qb, q.alpha_off, q.beta_off),
                                     avc::edge_params(pk.qpc - qcb, q.qpc - qcb, q.alpha_off, q.beta_off),
                                     avc::edge_params(pk.qpc2 - qcb, q.qpc2 - qcb, q.alpha_off, q.beta_off)};
      for (int c = 0; c < 3; ++c) {
        info.alpha[c * 3 + k] = u8(ep[c].alpha);
        info.beta[c * 3 + k] = u8(ep[c].beta);
        for (int j = 0; j < 3; ++j) info.tc0[c * 3 + k][j] = u8(ep[c].tc0[j]);
      }
    }
  }
  static_cast<AvcDbkInfo*>(d.dbk)[mb] = info;
}

// ------------------------------------------------------------------------------ deblocking

struct DbkWave {
  AvcDbkInfo info;
  u8 y[20 * 20];      // rows -4..15, cols -4..15 of the MB (top-left corner unused)
  // rows -2..7 per chroma component, kDbkCs bytes each: 2 pad bytes, then cols -2..7, so that a
  // row's words hold (pad, pad, -2, -1) (0..3) (4..7) like a luma row's edges' p / q words
  u8 c[2][10 * 12];
  u8 carry[16 * 4];   // previous MB's filtered luma columns 12..15
  u8 ccarry[2][8 * 2];
};

// Final bottom rows of one MB of a row, handed to the row below through LDS: luma rows 12..15
// and NV12 chroma rows 6..7 (the only samples of a row that the row below reads or filters).
struct alignas(16) DbkXch {
  u8 y[4 * 16];
  u8 c[2 * 16];
};

// A wave filters two adjacent MB rows at once: lanes 0-31 row 2p, lanes 32-63 row 2p+1, the
// second trailing by kDbkLag columns, all 64 lanes filtering. A workgroup of kDbkWaves waves
// owns kAvcDbkWgRows consecutive rows, and a picture runs avc_dbk_groups(H) workgroups at once
// (68 rows of 1080p: 9 workgroups, 34 waves, every row in flight), so each wave gets most of a
// SIMD to itself instead of sharing one CU with the whole picture.
//
// Rows hand their final bottom samples to the row below; the per-MB handshake never waits on
// the picture in global memory:
//  * inside a workgroup through an LDS exchange ring of kDbkDepth columns (the producer waits
//    when the consumer falls that far behind) guarded by LDS progress counters;
//  * from a workgroup's last row to the next workgroup's first row through `xg`, a whole-row
//    buffer of device-coherent (sc1) 64-bit words whose high half tags the word as final, so
//    the data is its own flag: no counter, no release fence, no L2 writeback; the consumer
//    prefetches the next MB's words one step ahead and re-polls only when they are not final;
//  * each sample is written to the picture by exactly one wave: a row stores rows 0..11 of its
//    MBs, the row below stores rows 12..15 (from the exchange, after its own top-edge filter),
//    so no global store ever needs to be ordered against another wave's;
//  * the MB's own samples are prefetched one column ahead (no wave writes them before the row
//    that owns the MB has filtered it).
// Workgroups wait only on the previous workgroup of their picture, which the XCD-aware grid
// order (launch_avc_deblock) dispatches first, so every wait is on a resident workgroup.
constexpr int kDbkLag = 1;  // the second row filters MB x's top edge after the first row's
                            // vertical edges of MB x + 1, in the same step
constexpr int kDbkDepth = 8;
// (rows per deblocking workgroup: VEP_DBK_WG_ROWS at build time, default kAvcDbkWgRows; the
// exchange slots between its workgroups are a subset of the kAvcDbkWgRows-row slots that
// avc_bs_kernel clears for every launch)
#ifndef VEP_DBK_WG_ROWS
#define VEP_DBK_WG_ROWS kAvcDbkWgRows
#endif
constexpr int kDbkRows = VEP_DBK_WG_ROWS;
constexpr int kDbkWaves = kDbkRows / 2;
constexpr u32 kXgFinal = 2u, kXgPartial = 1u;
static_assert(kDbkRows % 2 == 0 && kDbkDepth > kDbkLag && kDbkRows % kAvcDbkWgRows == 0 && kDbkRows <= 32,
              "deblock wavefront geometry");

struct DbkSync {
  u32 progress[kDbkRows];  // MBs finished per row of the workgroup
  u32 abort;
};

__device__ inline void st4(u8* p, u32 v) { *reinterpret_cast<u32*>(p) = v; }
__device__ inline u32 ld4(const u8* p) { return *reinterpret_cast<const u32*>(p); }

// LDS-only handshake: progress counters and the data they guard both live in LDS.
__device__ inline void wait_row_lds(DbkSync& s, int r, u32 need, u32* err) {
  u32 spins = 0;
  while (__hip_atomic_load(&s.progress[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
    if (__hip_atomic_load(&s.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
    if (++spins > kSpinLimit) {
      __hip_atomic_store(&s.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if ((threadIdx.x & 63) == 0) atomicOr(err, 2u);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ inline int bs_of(const AvcDbkInfo& in, int dir, int e, int sg) {
  const int i = dir * 16 + e * 4 + sg;
  return int((in.bs[i >> 3] >> (4 * (i & 7))) & 15u);
}

// filter_samples (avc_recon.h) for a luma or a chroma line in one instruction stream, so the
// luma lanes (0-15) and chroma lanes (16-31) of a half-wave run one filter body together instead
// of the two type-specialised copies back to back. p2/p3/q2/q3 are read for chroma lines too
// (in-bounds LDS of the DbkWave tile, values unused) and only p0/q0 are stored for them.
// The filter on values (p0..p3, q0..q3 across the edge): false when the line is left as it is,
// else the new p0..p2 / q0..q2 (chroma: p0 / q0 only).
__device__ inline bool filter_vals(int p0, int p1, int p2, int p3, int q0, int q1, int q2, int q3, int bs, int alpha,
                                   int beta, int tc0, bool chroma, int& np0, int& np1, int& np2, int& nq0, int& nq1,
                                   int& nq2) {
  if (!(avc::iabs(p0 - q0) < alpha && avc::iabs(p1 - p0) < beta && avc::iabs(q1 - q0) < beta)) return false;
  const int ap = avc::iabs(p2 - p0), aq = avc::iabs(q2 - q0);
  const bool lp = !chroma && ap < beta, lq = !chroma && aq < beta;
  np1 = p1;
  nq1 = q1;
  np2 = p2;
  nq2 = q2;
  if (bs < 4) {
    const int tc = chroma ? tc0 + 1 : tc0 + int(lp) + int(lq);
    const int dl = avc::clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3);
    np0 = avc::clip1(p0 + dl);
    nq0 = avc::clip1(q0 - dl);
    if (lp) np1 = p1 + avc::clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1);
    if (lq) nq1 = q1 + avc::clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1);
  } else {
    const bool strong = !chroma && avc::iabs(p0 - q0) < ((alpha >> 2) + 2);
    if (lp && strong) {
      np0 = (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3;
      np1 = (p2 + p1 + p0 + q0 + 2) >> 2;
      np2 = (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3;
    } else {
      np0 = (2 * p1 + p0 + q1 + 2) >> 2;
    }
    if (lq && strong) {
      nq0 = (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3;
      nq1 = (p0 + q0 + q1 + q2 + 2) >> 2;
      nq2 = (2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3;
    } else {
      nq0 = (2 * q1 + q0 + p1 + 2) >> 2;
    }
  }
  return true;
}

// A vertical edge's line is contiguous in the LDS tile: luma p3..p0 / q0..q3 are two aligned
// words (rows of 20 bytes, the edge 4 bytes from a word boundary), chroma p1 p0 / q0 q1 two
// half-words; one load and one store each instead of a byte per sample. The loads and stores
// differ between luma and chroma lanes, the filter body between them is one (filter_vals) for
// the whole half-wave, as in filter_line_any.
__device__ inline void filter_vert_any(u8* q0p, int bs, int alpha, int beta, int tc0, bool chroma) {
  int p0, p1, p2, p3, q0, q1, q2, q3;
  u32 P = 0, Q = 0;
  if (!chroma) {
    const u32* w = reinterpret_cast<const u32*>(q0p - 4);
    P = w[0];
    Q = w[1];
    p3 = int(P & 255);
    p2 = int((P >> 8) & 255);
    p1 = int((P >> 16) & 255);
    p0 = int(P >> 24);
    q0 = int(Q & 255);
    q1 = int((Q >> 8) & 255);
    q2 = int((Q >> 16) & 255);
    q3 = int(Q >> 24);
  } else {
    const u16* h = reinterpret_cast<const u16*>(q0p - 2);
    P = h[0];
    Q = h[1];
    p1 = p2 = p3 = int(P & 255);
    p0 = int(P >> 8);
    q0 = int(Q & 255);
    q1 = q2 = q3 = int(Q >> 8);
  }
  int np0, np1, np2, nq0, nq1, nq2;
  if (!filter_vals(p0, p1, p2, p3, q0, q1, q2, q3, bs, alpha, beta, tc0, chroma, np0, np1, np2, nq0, nq1, nq2)) return;
  if (!chroma) {
    u32* w = reinterpret_cast<u32*>(q0p - 4);
    w[0] = (P & 255u) | u32(np2) << 8 | u32(np1) << 16 | u32(np0) << 24;
    w[1] = u32(nq0) | u32(nq1) << 8 | u32(nq2) << 16 | (Q & 0xFF000000u);
  } else {
    u16* h = reinterpret_cast<u16*>(q0p - 2);
    h[0] = u16((P & 255u) | u32(np0) << 8);
    h[1] = u16(u32(nq0) | (Q & 0xFF00u));
  }
}

__device__ inline void filter_line_any(u8* s, int step, int bs, int alpha, int beta, int tc0, bool chroma) {
  const int p0 = s[-step], p1 = s[-2 * step], q0 = s[0], q1 = s[step];
  const int p2 = s[-3 * step], p3 = s[-4 * step], q2 = s[2 * step], q3 = s[3 * step];
  if (!(avc::iabs(p0 - q0) < alpha && avc::iabs(p1 - p0) < beta && avc::iabs(q1 - q0) < beta)) return;
  const int ap = avc::iabs(p2 - p0), aq = avc::iabs(q2 - q0);
  const bool lp = !chroma && ap < beta, lq = !chroma && aq < beta;
  int np0, nq0, np1 = p1, nq1 = q1, np2 = p2, nq2 = q2;
  if (bs < 4) {
    const int tc = chroma ? tc0 + 1 : tc0 + int(lp) + int(lq);
    const int dl = avc::clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3);
    np0 = avc::clip1(p0 + dl);
    nq0 = avc::clip1(q0 - dl);
    if (lp) np1 = p1 + avc::clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1);
    if (lq) nq1 = q1 + avc::clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1);
  } else {
    const bool strong = !chroma && avc::iabs(p0 - q0) < ((alpha >> 2) + 2);
    if (lp && strong) {
      np0 = (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3;
      np1 = (p2 + p1 + p0 + q0 + 2) >> 2;
      np2 = (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3;
    } else {
      np0 = (2 * p1 + p0 + q1 + 2) >> 2;
    }
    if (lq && strong) {
      nq0 = (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3;
      nq1 = (p0 + q0 + q1 + q2 + 2) >> 2;
      nq2 = (2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3;
    } else {
      nq0 = (2 * q1 + q0 + p1 + 2) >> 2;
    }
  }
  s[-step] = u8(np0);
  s[0] = u8(nq0);
  if (!chroma) {
    s[-2 * step] = u8(np1);
    s[step] = u8(nq1);
    s[-3 * step] = u8(np2);
    s[2 * step] = u8(nq2);
  }
}

// One direction of an MB's edges, whole wave (lanes of a half-wave: luma lines 0-15, chroma
// lines 16-31, `any` = this half's MB has an edge to filter): 4 edges in order, each line by
// filter_line_any on the LDS tile (chroma lines on the even edges only). The four edges' bS and
// thresholds are read up front (one round of LDS loads), so each edge step is only its samples'
// round trip.
__device__ inline void dbk_dir(DbkWave& L, bool any, int l, int dir, bool packed, bool sync_each) {
  const bool ch = l >= 16;
  const int c = (l - 16) >> 3, k = (l - 16) & 7;
  int bs[4], al[4], be[4], tc[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    bs[e] = any && (!ch || !(e & 1)) ? bs_of(L.info, dir, e, ch ? k >> 1 : l >> 2) : 0;
    const int pi = (e > 0 ? 2 : dir) + (ch ? 3 + 3 * c : 0);  // component, then left / top / internal
    al[e] = L.info.alpha[pi];
    be[e] = L.info.beta[pi];
    tc[e] = L.info.tc0[pi][bs[e] > 0 && bs[e] < 4 ? bs[e] - 1 : 0];
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (bs[e] && dir == 0 && packed) {  // vertical edge: packed LDS accesses
      u8* q0p = !ch ? &L.y[(4 + l) * 20 + 4 + 4 * e] : &L.c[c][(2 + k) * 12 + 4 + 2 * e];
      filter_vert_any(q0p, bs[e], al[e], be[e], bs[e] < 4 ? tc[e] : 0, ch);
    } else if (bs[e]) {
      u8* sp;
      int step;
      if (!ch) {
        sp = dir == 0 ? &L.y[(4 + l) * 20 + 4 + 4 * e] : &L.y[(4 + 4 * e) * 20 + 4 + l];
        step = dir == 0 ? 1 : 20;
      } else {
        sp = dir == 0 ? &L.c[c][(2 + k) * 12 + 4 + 2 * e] : &L.c[c][(2 + 2 * e) * 12 + 4 + k];
        step = dir == 0 ? 1 : 12;
      }
      filter_line_any(sp, step, bs[e], al[e], be[e], bs[e] < 4 ? tc[e] : 0, ch);
    }
    // Within one direction every lane filters its own line (a row for vertical edges, a column
    // for horizontal ones) through all four edges: edge e + 1 reads only what this lane wrote at
    // edge e, which a wave's in-order LDS accesses already order. Other lanes read it only in
    // the other direction, so one sync per direction, after its last edge (VEP_DBK_SYNC=0 keeps
    // one per edge, for A/B).
    if (sync_each) wave_sync();
  }
  if (!sync_each) wave_sync();
}

// One direction of an MB's edges with each lane's line in VGPRs (VEP_DBK_REGS, the default): a
// luma lane (0-15) holds its row (vertical edges) / column (horizontal edges) as 20 samples, 4 of
// the neighbour then the MB's 16, in five words; a chroma lane (16-31) holds 10 samples of its
// component (2 + 8) in the same five-word shape (pad, pad, -2, -1 | 0..3 | 4..7), so chroma edges
// 0 / 2 fall on the word boundaries 0 / 1 exactly like luma edges 0 / 1 and one filter body serves
// every lane. The line comes in with one LDS round trip (words for rows, bytes for columns), the
// four (chroma: two) dependent edge filters run in registers, and it goes back in one: round 4's
// form did an LDS round trip per edge (the wavefront's per-MB critical path).
__device__ inline void dbk_dir_regs(DbkWave& L, bool any, int l, int dir) {
  const bool ch = l >= 16;
  const int c = (l - 16) >> 3, k = (l - 16) & 7;
  int bs[4], al[4], be[4], tc[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int ee = ch ? 2 * e : e;  // the MB edge register edge e stands for
    bs[e] = any && (!ch || e < 2) ? bs_of(L.info, dir, ee, ch ? k >> 1 : l >> 2) : 0;
    const int pi = (ee > 0 ? 2 : dir) + (ch ? 3 + 3 * c : 0);
    al[e] = L.info.alpha[pi];
    be[e] = L.info.beta[pi];
    tc[e] = L.info.tc0[pi][bs[e] > 0 && bs[e] < 4 ? bs[e] - 1 : 0];
  }
  u32 w[5] = {0, 0, 0, 0, 0};
  // rows: the line's words are the tile row's words; columns: sample i of the line is tile row
  // i - 4 (luma rows -4..15, chroma rows -2..7 at line positions 2..11)
  u8* row = !ch ? &L.y[(4 + l) * 20] : &L.c[c][(2 + k) * 12];
  u8* col = !ch ? &L.y[4 * 20 + 4 + l] : &L.c[c][2 * 12 + 4 + k];  // (row 0 of the column)
  const int stride = ch ? 12 : 20, lo = ch ? 2 : 0, hi = ch ? 12 : 20, nw = ch ? 3 : 5;
  if (dir == 0) {
#pragma unroll
    for (int i = 0; i < 5; ++i)
      if (i < nw) w[i] = ld4(row + 4 * i);
  } else {
#pragma unroll
    for (int i = 0; i < 20; ++i)
      if (i >= lo && i < hi) w[i >> 2] |= u32(col[(i - 4) * stride]) << (8 * (i & 3));
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (!bs[e]) continue;
    const u32 P = w[e], Q = w[e + 1];
    int np0, np1, np2, nq0, nq1, nq2;
    if (!filter_vals(int(P >> 24), int((P >> 16) & 255), int((P >> 8) & 255), int(P & 255), int(Q & 255),
                     int((Q >> 8) & 255), int((Q >> 16) & 255), int(Q >> 24), bs[e], al[e], be[e],
                     bs[e] < 4 ? tc[e] : 0, ch, np0, np1, np2, nq0, nq1, nq2))
      continue;
    w[e] = (P & 255u) | u32(np2) << 8 | u32(np1) << 16 | u32(np0) << 24;
    w[e + 1] = u32(nq0) | u32(nq1) << 8 | u32(nq2) << 16 | (Q & 0xFF000000u);
  }
  // (chroma: filter_vals leaves p1 / q1 / p2 / q2 as they were, so the repacked words are exact)
  if (dir == 0) {
#pragma unroll
    for (int i = 0; i < 5; ++i)
      if (i < nw) st4(row + 4 * i, w[i]);
  } else {
#pragma unroll
    for (int i = 1; i < 20; ++i)  // (sample 0, luma row -4, is never written by a filter)
      if (i >= lo && i < hi) col[(i - 4) * stride] = u8(w[i >> 2] >> (8 * (i & 3)));
  }
  wave_sync();
}

struct DbkRegs {  // one MB's inputs as loaded from global memory (per lane of a half-wave)
  u32 info, m0, m1, c;
};

__global__ __launch_bounds__(64 * kDbkWaves) void avc_deblock_kernel(const AvcDesc* __restrict__ descs,
                                                                      int n, int groups, int packed) {
  // grid order: workgroup b runs on XCD b % 8; picture p's group k is b = ((p / 8) * groups +
  // k) * 8 + p % 8, so a picture stays on one XCD and its groups dispatch in order
  const int b = int(blockIdx.x), j = b >> 3;
  const int pic = (j / groups) * 8 + (b & 7), grp = j % groups;
  if (pic >= n) return;
  const AvcDesc d = descs[pic];  // by value: SGPRs, no reloads after stores
  const int W = d.wmbs, H = d.hmbs, pitch = W * 16;
  const int g0 = grp * kDbkRows;  // first row of this workgroup
  if (g0 >= H || d.bd > 8 || d.cf == 2) return;  // (uniform over the workgroup, before any barrier;
                                                  // High 10 / 4:2:2: avc_hbd_kernel)
  __shared__ DbkSync sync;
  __shared__ DbkWave lds[kDbkWaves][2];
  __shared__ DbkXch xring[kDbkRows - 1][kDbkDepth];
  if (threadIdx.x < kDbkRows) sync.progress[threadIdx.x] = 0;
  if (threadIdx.x == 0) sync.abort = 0;
  __syncthreads();
  const int wave = int(threadIdx.x) >> 6, lane = int(threadIdx.x) & 63;
  const int h = lane >> 5, l = lane & 31;  // row of the pair / lane within the half-wave
  DbkWave& L = lds[wave][h];
  u8* Y = d.y + d.slot_y * u64(d.target);
  u8* UV = d.uv + d.slot_uv * u64(d.target);
  const AvcDbkInfo* infos = static_cast<const AvcDbkInfo*>(d.dbk);
  auto xch = [&](int r, int x) -> DbkXch& { return xring[r - g0][x % kDbkDepth]; };
  // Branch-free (row / column clamped, the result unused when out of range): a conditional
  // load would merge with a default at the join and force an immediate vmcnt wait.
  auto load_mb = [&](int row, int x) {
    row = row < H ? row : H - 1;
    x = x < 0 ? 0 : (x < W ? x : W - 1);
    DbkRegs v;
    v.info = gld4(reinterpret_cast<const u32*>(&infos[size_t(row) * W + x]) + (l < 16 ? l : 0));
    const u8* ym = Y + size_t(row * 16 + (l >> 2)) * pitch + x * 16 + (l & 3) * 4;
    v.m0 = gld4(ym);                      // MB rows 0..7
    v.m1 = gld4(ym + size_t(8) * pitch);  // MB rows 8..15
    v.c = gld4(UV + size_t(row * 8 + (l >> 2)) * pitch + x * 16 + (l & 3) * 4);  // 8 x 16 B
    return v;
  };
  const int r0 = g0 + 2 * wave, row = r0 + h, lrow = row - g0;
  const bool last = row == H - 1;
  const bool prod = row + 1 < H;                          // hands its bottom rows down
  const bool xout = prod && lrow == kDbkRows - 1;          // ... to the next workgroup
  const bool xin = grp > 0 && wave == 0;                   // row r0 reads the previous group's
  // exchange word this lane of row r0 reads: luma lanes 16..31 -> words 0..15, chroma lanes
  // 8..15 -> words 16..23
  const int xw = l >= 16 ? l - 16 : (l >= 8 ? 16 + (l - 8) : -1);
  const bool xneed = xin && h == 0 && xw >= 0;
  u64* xg_in = xin ? d.xg + size_t(grp - 1) * W * kAvcXgWords : nullptr;
  u64* xg_out = d.xg + size_t(grp) * W * kAvcXgWords;
  u64 gx = 0;  // row r0's exchange word of the current MB (prefetched one step ahead)
  if (xneed) gx = xg_get(xg_in + xw);
  u64 acc[5] = {0, 0, 0, 0, 0};  // phase clocks of this wave (flushed once at the end)
  DbkRegs cur = load_mb(row, -kDbkLag * h);
  for (int i = 0; r0 < H && i < W + kDbkLag; ++i) {
    const int x = i - h * kDbkLag;
    const bool act = row < H && x >= 0 && x < W;
    const u64 t0 = d.prof ? clock64() : 0;
    const DbkRegs nxt = load_mb(row, x + 1);  // prefetch: in flight across this MB's work
    {  // back-pressure: the pair's second row feeds the next wave through a kDbkDepth ring
      // (the consumer has read column c once its progress reaches c + 2)
      const int x1 = i - kDbkLag;
      if (r0 + 2 < H && wave + 1 < kDbkWaves && x1 < W && x1 - kDbkDepth + 2 > 0)
        wait_row_lds(sync, 2 * wave + 2, u32(x1 - kDbkDepth + 2), d.err);
    }
    const u64 t1 = d.prof ? clock64() : 0;
    const int x0 = x * 16, y0 = row * 16;
    // ---- LDS: MB samples and left columns (carried)
    if (act) {
      // (the carried columns read first, in range for every lane: one wait for all the reads)
      const u32 carry = ld4(&L.carry[(l & 15) * 4]);
      const int l7 = l & 7;
      const u8 cc0 = L.ccarry[0][l7 * 2], cc1 = L.ccarry[1][l7 * 2], cc2 = L.ccarry[0][l7 * 2 + 1],
               cc3 = L.ccarry[1][l7 * 2 + 1];
      if (l < 16) reinterpret_cast<u32*>(&L.info)[l] = cur.info;
      st4(&L.y[((l >> 2) + 4) * 20 + 4 + (l & 3) * 4], cur.m0);
      st4(&L.y[((l >> 2) + 12) * 20 + 4 + (l & 3) * 4], cur.m1);
      if (l < 16 && x > 0) st4(&L.y[(l + 4) * 20], carry);
      {
        const int cyr = l >> 2, cb = (l & 3) * 2;
        for (int q = 0; q < 2; ++q) {
          L.c[0][(cyr + 2) * 12 + 4 + cb + q] = u8(cur.c >> (16 * q));
          L.c[1][(cyr + 2) * 12 + 4 + cb + q] = u8(cur.c >> (16 * q + 8));
        }
      }
      if (l < 8 && x > 0) {
        L.c[0][(l + 2) * 12 + 2] = cc0;
        L.c[1][(l + 2) * 12 + 2] = cc1;
        L.c[0][(l + 2) * 12 + 3] = cc2;
        L.c[1][(l + 2) * 12 + 3] = cc3;
      }
    }
    wave_sync();
    const u64 t2 = d.prof ? clock64() : 0;
    const bool any = act && L.info.any;
    const bool wany = __ballot(any) != 0;
    // ---- vertical edges (per half: luma lanes 0-15, chroma 16-31): they touch only this MB's
    // rows, so they need nothing from the row above
    if (wany) {
      if (packed & 4) dbk_dir_regs(L, any, l, 0);
      else dbk_dir(L, any, l, 0, (packed & 1) != 0, (packed & 2) != 0);
    }
    // ---- the previous MB's right columns are final now (this MB's left edge was the last
    // filter to touch them): complete its exchange entry for the row below, then publish
    // "vertical edges of MB x done" (the row below may filter MB x - 1's top edge)
    if (act && prod && x > 0) {
      u32 fw = 0;
      int fi = -1;  // exchange word: luma rows 12..15 columns 12..15 / NV12 rows 6..7 bytes 12..15
      if (l >= 24 && l < 28) {
        const int k = l - 24;
        fw = ld4(&L.y[(16 + k) * 20]);
        fi = k * 4 + 3;
      } else if (l >= 28 && l < 30) {
        const int k = l - 28, cr = 8 + k;
        fw = u32(L.c[0][cr * 12 + 2]) | u32(L.c[1][cr * 12 + 2]) << 8 | u32(L.c[0][cr * 12 + 3]) << 16 |
             u32(L.c[1][cr * 12 + 3]) << 24;
        fi = 16 + k * 4 + 3;
      }
      if (fi >= 0) {
        if (xout) xg_put(xg_out + size_t(x - 1) * kAvcXgWords + fi, fw, kXgFinal);
        else st4(fi < 16 ? &xch(row, x - 1).y[fi * 4] : &xch(row, x - 1).c[(fi - 16) * 4], fw);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    if (l == 0 && act)
      __hip_atomic_store(&sync.progress[lrow], u32(x + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const u64 t3 = d.prof ? clock64() : 0;
    // ---- wait for the row above: its exchange entry of MB x is complete once it has done the
    // vertical edges of MB x + 1 (progress x + 2; W + 1 after its last MB)
    if (xin && i < W) {  // previous workgroup's bottom samples of MB i: poll until final
      u32 spins = 0;
      while (__ballot(xneed && u32(gx >> 32) != kXgFinal)) {
        if (__hip_atomic_load(&sync.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
        if (++spins > (kSpinLimit >> 4)) {
          __hip_atomic_store(&sync.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (lane == 0) atomicOr(d.err, 2u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        if (xneed) gx = xg_get(xg_in + size_t(i) * kAvcXgWords + xw);
      }
    }
    const u32 gv = u32(gx);
    if (xneed && i + 1 < W) gx = xg_get(xg_in + size_t(i + 1) * kAvcXgWords + xw);  // prefetch
    if (wave > 0 && i < W) wait_row_lds(sync, 2 * wave - 1, u32(i + 2), d.err);
    wave_sync();  // (the pair's second row reads what the first row completed just above)
    const u64 t4 = d.prof ? clock64() : 0;
    // ---- LDS: top rows (the row above's exchange)
    const bool top_g = xin && h == 0;  // this row's top samples come from xg
    if (act && row > 0) {
      if (l >= 16) {
        const int k = l - 16;
        st4(&L.y[(k >> 2) * 20 + 4 + (k & 3) * 4], top_g ? gv : ld4(&xch(row - 1, x).y[k * 4]));
      } else if (l >= 8) {
        const int k = l - 8, tr = k >> 2, cb = (k & 3) * 2;
        const u32 v = top_g ? gv : ld4(&xch(row - 1, x).c[k * 4]);
        for (int q = 0; q < 2; ++q) {
          L.c[0][tr * 12 + 4 + cb + q] = u8(v >> (16 * q));
          L.c[1][tr * 12 + 4 + cb + q] = u8(v >> (16 * q + 8));
        }
      }
    }
    wave_sync();
    const u64 t5 = d.prof ? clock64() : 0;
    // ---- horizontal edges
    if (wany) {
      if (packed & 4) dbk_dir_regs(L, any, l, 1);
      else dbk_dir(L, any, l, 1, false, (packed & 2) != 0);
    }
    const u64 t6 = d.prof ? clock64() : 0;
    if (act) {
      // ---- write back: MB rows 0..11 (0..15 for the last row) if filtered, the left
      // neighbour's columns 12..15 if the left edge was filtered, and always the MB above's
      // final rows 12..15 (this wave is their only writer)
      const bool left = any && (L.info.bs[0] & 0xFFFFu) != 0;  // dir 0, edge 0 nibbles
      // Every LDS read of the write-back first (in-range addresses for every lane, the values
      // unused where a store below does not happen), so they are in flight together and the
      // wave waits once, not once per store.
      auto cbyte = [&](int c, int i) { return u32(L.c[c][i]); };
      auto cword = [&](int base) {  // 2 columns x 2 components from chroma tile entry base
        return cbyte(0, base) | cbyte(1, base) << 8 | cbyte(0, base + 1) << 16 | cbyte(1, base + 1) << 24;
      };
      const int q4 = l >> 2, r4 = (l & 3) * 4, cb = (l & 3) * 2, k16 = (l - 16) & 15;
      const u32 w_top = ld4(&L.y[(q4 + 4) * 20 + 4 + r4]);                 // MB rows 0..7
      const u32 w_bot = ld4(&L.y[(q4 + 12) * 20 + 4 + r4]);                // MB rows 8..15
      const u32 w_c = cword((q4 + 2) * 12 + 4 + cb);                        // chroma rows 0..7
      const u32 w_side = ld4(l < 16 ? &L.y[(l + 4) * 20]                    // left columns 12..15
                                    : &L.y[(k16 >> 2) * 20 + 4 + (k16 & 3) * 4]);  // MB above, rows 12..15
      const int l8 = l & 7, k8 = (l - 8) & 7;
      const u32 w_cside = l < 8 ? cword((l8 + 2) * 12 + 2)                 // left chroma columns 6..7
                                : cword((k8 >> 2) * 12 + 4 + (k8 & 3) * 2);  // above: chroma rows 6..7
      const int kx = (l - 16) & 7;
      const u32 w_x = l < 16 ? ld4(&L.y[(16 + q4) * 20 + 4 + r4])          // exchange: rows 12..15
                             : cword((8 + (kx >> 2)) * 12 + 4 + (kx & 3) * 2);  // chroma rows 6..7
      const u32 w_carry = ld4(&L.y[((l & 15) + 4) * 20 + 16]);
      const int cc = ((l - 16) >> 3) & 1, ck = (l - 16) & 7;
      const u8 cr0 = L.c[cc][(ck + 2) * 12 + 10], cr1 = L.c[cc][(ck + 2) * 12 + 11];
      if (any) {
        u8* ym = Y + size_t(y0 + q4) * pitch + x0 + r4;
        gst4(ym, w_top);
        if (q4 < 4 || last) gst4(ym + size_t(8) * pitch, w_bot);
        if (q4 < 6 || last) gst4(UV + size_t(row * 8 + q4) * pitch + x0 + cb * 2, w_c);
      }
      if (l < 16) {
        if (left && (l < 12 || last)) gst4(Y + size_t(y0 + l) * pitch + x0 - 4, w_side);
      } else if (row > 0) {
        gst4(Y + size_t(y0 - 4 + (k16 >> 2)) * pitch + x0 + (k16 & 3) * 4, w_side);
      }
      if (l < 8) {
        if (left && (l < 6 || last)) gst4(UV + size_t(row * 8 + l) * pitch + x0 - 4, w_cside);
      } else if (l < 16 && row > 0) {
        gst4(UV + size_t(row * 8 - 2 + (k8 >> 2)) * pitch + x0 + (k8 & 3) * 4, w_cside);
      }
      // ---- exchange for the row below: this MB's rows 12..15 / chroma rows 6..7 (the last
      // word of each 4-word row, columns 12..15 / 6..7, is completed by the next MB's vertical
      // edges above)
      if (prod && l < 24) {
        if (xout)
          xg_put(xg_out + size_t(x) * kAvcXgWords + l, w_x, (l & 3) == 3 && x + 1 < W ? kXgPartial : kXgFinal);
        else
          st4(l < 16 ? &xch(row, x).y[l * 4] : &xch(row, x).c[(l - 16) * 4], w_x);
      }
      // ---- carry columns 12..15 (luma) / 6..7 (chroma) of this MB to the next one of the row
      if (l < 16) {
        st4(&L.carry[l * 4], w_carry);
      } else {
        L.ccarry[cc][ck * 2] = cr0;
        L.ccarry[cc][ck * 2 + 1] = cr1;
      }
    }
    if (x == W - 1) {  // the row's exchange is complete (no MB to its right)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
      if (l == 0 && act)
        __hip_atomic_store(&sync.progress[lrow], u32(W + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    wave_sync();
    cur = nxt;
    if (d.prof) {
      const u64 t7 = clock64();
      acc[0] += (t1 - t0) + (t4 - t3);
      acc[1] += (t2 - t1) + (t5 - t4);
      acc[2] += (t3 - t2) + (t6 - t5);
      acc[3] += t7 - t6;
      acc[4] += u64(__popcll(__ballot(act) & 0x100000001ull));
    }
  }
  if (d.prof && lane == 0)
    for (int k = 0; k < 5; ++k) atomicAdd(&d.prof[6 + k], acc[k]);
}

// Field pair -> frame: the frame slot holds the top field's rows, then the bottom field's (luma
// h / 2 rows each, chroma h / 4); frame row r is row r >> 1 of field r & 1. 16 bytes per lane.
__global__ __launch_bounds__(256) void weave_kernel(const WeaveDesc* __restrict__ descs) {
  const WeaveDesc d = descs[blockIdx.y];
  const u8* __restrict__ y = d.y;
  const u8* __restrict__ uv = d.uv;
  u8* __restrict__ y8 = d.y8;
  u8* __restrict__ uv8 = d.uv8;
  const int pitch = d.pitch, h = d.height;
  const int per_row = pitch / 16;
  const size_t g = size_t(blockIdx.x) * 256 + threadIdx.x, total = size_t(per_row) * size_t(h + h / 2);
  if (g >= total) return;
  const int row = int(g / size_t(per_row)), col = int(g % size_t(per_row)) * 16;
  const bool luma = row < h;
  const int r = luma ? row : row - h, fh = luma ? h / 2 : h / 4;  // rows per field
  const u8* src = (luma ? y : uv) + (size_t(r & 1) * size_t(fh) + size_t(r >> 1)) * size_t(pitch) + size_t(col);
  u8* dst = (luma ? y8 : uv8) + size_t(r) * size_t(pitch) + size_t(col);
  *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
}

}  // namespace

void launch_weave(const WeaveDesc* d_descs, int n, int max_pitch, int max_height, hipStream_t s) {
  if (n <= 0 || max_pitch <= 0 || max_height <= 0) return;
  const size_t lanes = size_t(max_pitch / 16) * size_t(max_height + max_height / 2);
  hipLaunchKernelGGL(weave_kernel, dim3(unsigned((lanes + 255) / 256), unsigned(n)), dim3(256), 0, s, d_descs);
  VEP_HIP(hipGetLastError());
}

void launch_avc_inter(const AvcDesc* d_descs, int n, int total_mbs, hipStream_t s) {
  if (n <= 0 || total_mbs <= 0) return;
  hipLaunchKernelGGL(avc_inter_kernel, dim3(unsigned((total_mbs + 3) / 4)), dim3(256), 0, s, d_descs, n,
                     total_mbs);
  VEP_HIP(hipGetLastError());
}

void launch_avc_intra(const AvcDesc* d_descs, int n, int max_hmbs, hipStream_t s) {
  if (n <= 0 || max_hmbs <= 0) return;
  const int groups = avc_dbk_groups(max_hmbs);
  const unsigned blocks = unsigned((n + 7) / 8) * unsigned(groups) * 8u;
  hipLaunchKernelGGL(avc_intra_kernel, dim3(blocks), dim3(64 * kIntraWaves), 0, s, d_descs, n, groups);
  VEP_HIP(hipGetLastError());
}

void launch_avc_bs(const AvcDesc* d_descs, int n, int total_mbs, hipStream_t s) {
  if (n <= 0 || total_mbs <= 0) return;
  hipLaunchKernelGGL(avc_bs_kernel, dim3(unsigned((total_mbs + 255) / 256)), dim3(256), 0, s, d_descs,
                     n, total_mbs);
  VEP_HIP(hipGetLastError());
}

void launch_avc_deblock(const AvcDesc* d_descs, int n, int max_hmbs, hipStream_t s, int packed) {
  if (n <= 0 || max_hmbs <= 0) return;
  const int groups = (max_hmbs + kDbkRows - 1) / kDbkRows;
  const unsigned blocks = unsigned((n + 7) / 8) * unsigned(groups) * 8u;
  hipLaunchKernelGGL(avc_deblock_kernel, dim3(blocks), dim3(64 * kDbkWaves), 0, s, d_descs, n, groups, packed);
  VEP_HIP(hipGetLastError());
}

}  // namespace vep::gpu
