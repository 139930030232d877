// gfx950 reconstruction kernels of the general H.265 path (records from hevc::Decoder in
// records mode, hevc_kern.h). Per reconstruction round (round r = the r-th picture of each
// camera's job):
//
//  * hevc_mc_kernel — every prediction block of the round, one 256-lane workgroup per block:
//    8-tap luma / 4-tap chroma motion compensation from the camera's DPB surfaces with uni- or
//    bi-prediction. No neighbour dependency: the launch is as wide as the round.
//  * hevc_tu_kernel — level 0: the inter residuals and PCM blocks (independent), one wave per
//    block, four per workgroup.
//  * hevc_tu_queue_kernel — every intra transform block of the round in ONE launch. The CPU
//    parser gives each block a dependency level (1 + the highest level among the intra blocks
//    its references read); persistent waves take blocks in level order from a ticket counter and
//    wait on a done counter only when they cross into a new level. Per block the wave prepares
//    the substituted / filtered references in its LDS, runs the 4..32-point inverse transform as
//    two LDS passes and writes prediction + residual. An I picture's ~190 dependency levels no
//    longer cost ~190 launches.
//  * hevc_deblock_kernel — HEVC filters every vertical edge of the picture before any
//    horizontal one, and edges 8 samples apart never touch the same samples: one launch per
//    direction, one lane per 4-line edge segment, no wavefront.
//  * hevc_sao_copy_kernel + hevc_sao_kernel — SAO reads the deblocked picture: a copy, then one
//    lane per 4x4 block (16 luma + 2 x 4 chroma samples).
//
// All sample arithmetic comes from hevc_kern.h, shared with the CPU mirror (hevc_gpu.cpp) that
// is tested bit-exact against the reference decoder.
#define VEP_KERNEL_SOURCE 1  // descriptors' pointers are global-address-space here (gpu.h)
#include <algorithm>
#include <cstdlib>

#include "gpu.h"
#include "hevc_kern.h"

namespace vep::gpu {

using hevc::GpuPu;
using hevc::GpuSao;
using hevc::GpuSlice;
using hevc::GpuTu;

namespace {

__device__ inline int pick_pu(const HevcDesc* d, int n, int b) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].pu_begin <= b) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ inline int pick_blk(const HevcDesc* d, int n, int b) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].blk_begin <= b) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ inline int pick_range(const HevcTuRange* r, int n, int b) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (r[mid].begin <= b) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Sample type of a picture: u8 planes (8-bit streams: the bit depth is the constant 8, so the
// shifts of the shared math fold away) or u16 planes (Main10, HevcDesc::bd_y / bd_c).
template <class P>
__device__ inline int bd_of(int bd) {
  return sizeof(P) == 1 ? 8 : bd;
}

// ------------------------------------------------------------------------------ MC
// Each output sample's taps are read from the picture (edge-clamped) by its own thread. A
// separable form staged through LDS (reference window, horizontal pass, vertical taps) was
// measured 2.5-3x slower on the camera streams (profiles/r3/mcab/): most blocks are small and
// their loads hit L1/L2, so the staging syncs and idle lanes cost more than the taps saved.
template <class P>
__device__ __attribute__((always_inline)) inline void mc_block(const HevcDesc& d, const GpuPu& u) {
  const int stride = d.stride, W = d.width, H = d.height, bdy = bd_of<P>(d.bd_y), bdc = bd_of<P>(d.bd_c);
  P* y = reinterpret_cast<P*>(d.y + size_t(d.target) * d.slot_y);
  P* uv = reinterpret_cast<P*>(d.uv + size_t(d.target) * d.slot_uv);
  const P* ry[2] = {nullptr, nullptr};
  const P* ruv[2] = {nullptr, nullptr};
  for (int l = 0; l < 2; ++l)
    if ((u.pred >> l) & 1) {
      ry[l] = reinterpret_cast<const P*>(d.y + size_t(u.slot[l]) * d.slot_y);
      ruv[l] = reinterpret_cast<const P*>(d.uv + size_t(u.slot[l]) * d.slot_uv);
    }
  const bool bi = u.pred == 3;
  // explicit weighted prediction: the PU's weights / offsets (uniform per workgroup)
  const hevc::GpuWp* wp = u.wp ? static_cast<const hevc::GpuWp*>(d.wp) + (u.wp - 1) : nullptr;
  const int ul = (u.pred & 1) ? 0 : 1;
  const int nl = u.w * u.h;
  for (int s = int(threadIdx.x); s < nl; s += 256) {
    const int i = s % u.w, j = s / u.w;
    int v[2] = {0, 0}, k = 0;
    for (int l = 0; l < 2; ++l)
      if (ry[l])
        v[k++] = hevc::hk_luma_mc(ry[l], stride, W, H, u.x + i + (u.mv[l][0] >> 2), u.y + j + (u.mv[l][1] >> 2),
                                  u.mv[l][0] & 3, u.mv[l][1] & 3, bdy);
    y[(u.y + j) * stride + u.x + i] =
        P(wp ? hevc::hk_weight_explicit(*wp, 0, v[0], v[1], bi, ul, bdy) : hevc::hk_weight(v[0], v[1], bi, bdy));
  }
  const int wc = u.w >> 1, hc = u.h >> 1, nc = wc * hc;
  for (int s = int(threadIdx.x); s < 2 * nc; s += 256) {
    const int c = s / nc, r = s - c * nc, i = r % wc, j = r / wc;
    int v[2] = {0, 0}, k = 0;
    for (int l = 0; l < 2; ++l)
      if (ruv[l])
        v[k++] = hevc::hk_chroma_mc(ruv[l], stride, W >> 1, H >> 1, c, (u.x >> 1) + i + (u.mv[l][0] >> 3),
                                    (u.y >> 1) + j + (u.mv[l][1] >> 3), u.mv[l][0] & 7, u.mv[l][1] & 7, bdc);
    uv[((u.y >> 1) + j) * stride + u.x + 2 * i + c] =
        P(wp ? hevc::hk_weight_explicit(*wp, 1 + c, v[0], v[1], bi, ul, bdc) : hevc::hk_weight(v[0], v[1], bi, bdc));
  }
}

__global__ __launch_bounds__(256) void hevc_mc_kernel(const HevcDesc* __restrict__ descs, int n) {
  const int b = int(blockIdx.x);
  const HevcDesc& d = descs[pick_pu(descs, n, b)];
  const GpuPu u = static_cast<const GpuPu*>(d.pus)[b - d.pu_begin];
  // (8-bit pictures: bd = 8 folds into the same code as before; Main10 pictures: u16 samples)
  if (d.flags & kHevcWide) mc_block<u16>(d, u);
  else mc_block<u8>(d, u);
}


// ------------------------------------------------------------------------------ TUs
// One wave per transform block: LDS of the wave (the block's column pass, references and their
// substitution scratch). Blocks are at most 32x32 = 16 samples per lane.
struct alignas(16) TuWave {
  int g[32 * 32];
  i16 dq[32 * 32];  // the block's coefficients, dense (expanded from the sparse records)
  int top[129];
  int left[128];
  int sbuf[129], sref[129];
  u8 sav[132];
};

__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Intra edge exchange of the queue kernel: 64-bit words (epoch << 32 | sample) accessed with
// device-scope relaxed atomics, coherent across the XCDs' L2s without fences. Word of component
// c's sample (x, y) in a column x % 4 == 3 / a row y % 4 == 3 (see gpu::hevc_xg_words).
__device__ inline u64* xg_col(const HevcDesc& d, int c, int x, int y) {
  const size_t W = size_t(d.stride), H = size_t(d.xg_h);
  if (c == 0) return d.xg + size_t(y) * (W >> 2) + size_t(x >> 2);
  const size_t Wc = W >> 1, Hc = H >> 1, comp = Hc * (Wc >> 2) + (Hc >> 2) * Wc;
  return d.xg + (W * H >> 1) + size_t(c - 1) * comp + size_t(y) * (Wc >> 2) + size_t(x >> 2);
}
__device__ inline u64* xg_row(const HevcDesc& d, int c, int x, int y) {
  const size_t W = size_t(d.stride), H = size_t(d.xg_h);
  if (c == 0) return d.xg + H * (W >> 2) + size_t(y >> 2) * W + size_t(x);
  const size_t Wc = W >> 1, Hc = H >> 1, comp = Hc * (Wc >> 2) + (Hc >> 2) * Wc;
  return d.xg + (W * H >> 1) + size_t(c - 1) * comp + Hc * (Wc >> 2) + size_t(y >> 2) * Wc + size_t(x);
}
__device__ inline void xg_put(u64* p, u32 epoch, u32 v) {
  __hip_atomic_store(p, u64(epoch) << 32 | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline u64 xg_get(const u64* p) {
  return __hip_atomic_load(const_cast<u64*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr u32 kXgSpinLimit = 1u << 18;  // polls (x at most nap_max x 256 cycles): a few seconds at most
constexpr int kTuQueueWgs = 128;

// Reference samples of an intra block with the 64 lanes of a wave (the parallel form of
// hk_prepare_refs, same result): gather by availability, substitution as "nearest available
// sample before, else the first available one", then the [1 2 1] / strong filters. Units in
// `pend` (queue kernel only) come from the epoch-tagged edge words, polled until current.
template <class P>
__device__ void prepare_refs_wave(const HevcDesc& d, const GpuTu& t, const P* plane, int stride, int step, int lane,
                                  TuWave& L, int bd) {
  const int x0 = t.x, y0 = t.y, log2 = t.log2;
  const bool luma = t.c == 0;
  const u64 avail = t.avail, pend = d.xg ? t.pend : 0;
  const int n = 1 << log2, g = luma ? 4 : 2, last = 4 * n;
  for (int k = lane; k <= last; k += 64) {  // scan order: p[-1][2n-1] .. p[-1][-1] .. p[2n-1][-1]
    int bit, px, py;
    if (k < 2 * n) {
      const int y = 2 * n - 1 - k;
      bit = 1 + y / g;
      px = x0 - 1;
      py = y0 + y;
    } else if (k == 2 * n) {
      bit = 0;
      px = x0 - 1;
      py = y0 - 1;
    } else {
      const int x = k - 2 * n - 1;
      bit = 17 + x / g;
      px = x0 + x;
      py = y0 - 1;
    }
    const bool a = (avail >> bit) & 1;
    const bool xq = a && ((pend >> bit) & 1);  // produced in this launch: poll its edge word
    int v = 0;
    if (a && !xq) v = plane[py * stride + px * step];
    // the corner is on the right column or on the bottom row of the block covering it (a block
    // reaching right of it / below it): only that block writes either word, so poll both
    const u64* wp = nullptr;
    const u64* wp2 = nullptr;
    u64 w = 0;
    if (xq) {
      wp = k <= 2 * n ? xg_col(d, t.c, px, py) : xg_row(d, t.c, px, py);
      if (k == 2 * n) wp2 = xg_row(d, t.c, px, py);
      w = xg_get(wp);
      if (wp2 && u32(w >> 32) != d.epoch) w = xg_get(wp2);
    }
    u32 spins = 0, nap = 1;
    while (__ballot(xq && u32(w >> 32) != d.epoch)) {
      if (++spins > kXgSpinLimit) {
        if (xq && u32(w >> 32) != d.epoch) atomicOr(d.err, 2u);  // (the frame is dropped)
        break;
      }
      for (u32 z = 0; z < nap; ++z) __builtin_amdgcn_s_sleep(4);
      nap = nap < d.nap_max ? 2 * nap : nap;  // (HevcDesc::nap_max: exponential backoff)
      if (xq && u32(w >> 32) != d.epoch) {
        w = xg_get(wp);
        if (wp2 && u32(w >> 32) != d.epoch) w = xg_get(wp2);
      }
    }
    if (xq) v = int(u32(w) & 0xffffu);
    L.sbuf[k] = v;
    L.sav[k] = a ? 1 : 0;
  }
  wave_sync();
  for (int k = lane; k <= last; k += 64) {
    int src = -1;
    for (int j = k; j >= 0 && src < 0; --j)
      if (L.sav[j]) src = j;
    for (int j = k + 1; j <= last && src < 0; ++j)
      if (L.sav[j]) src = j;
    L.sref[k] = src >= 0 ? L.sbuf[src] : 1 << (bd - 1);
  }
  wave_sync();
  // filtering decision (luma): same rule as hk_prepare_refs
  const int mode = t.mode;
  const bool strong = (t.flags & hevc::kTuStrong) != 0;
  bool filt = false, strong_f = false;
  if (luma && mode != 1 && n != 4) {
    const int dm = mode - 26 < 0 ? 26 - mode : mode - 26, dh = mode - 10 < 0 ? 10 - mode : mode - 10;
    const int dist = dm < dh ? dm : dh;
    const int thres = n == 8 ? 7 : (n == 16 ? 1 : 0);
    filt = dist > thres;
    if (filt && strong && n == 32) {
      // tl = ref[2n], top[2n] = ref[4n], top[n] = ref[3n], left[2n-1] = ref[0], left[n-1] = ref[n]
      const int tl = L.sref[2 * n];
      const int a1 = tl + L.sref[4 * n] - 2 * L.sref[3 * n], a2 = tl + L.sref[0] - 2 * L.sref[n];
      strong_f = (a1 < 0 ? -a1 : a1) < (1 << (bd - 5)) && (a2 < 0 ? -a2 : a2) < (1 << (bd - 5));
    }
  }
  for (int k = lane; k <= last; k += 64) {
    int v = L.sref[k];
    if (filt) {
      if (strong_f) {  // bilinear between the corner and the far ends
        const int tl = L.sref[2 * n];
        if (k < 2 * n) {
          const int y = 2 * n - 1 - k;
          if (y < 63) v = ((63 - y) * tl + (y + 1) * L.sref[0] + 32) >> 6;
        } else if (k > 2 * n) {
          const int x = k - 2 * n - 1;
          if (x < 63) v = ((63 - x) * tl + (x + 1) * L.sref[last] + 32) >> 6;
        }
      } else if (k > 0 && k < last) {
        v = (L.sref[k - 1] + 2 * L.sref[k] + L.sref[k + 1] + 2) >> 2;
      }
    }
    if (k < 2 * n) L.left[2 * n - 1 - k] = v;
    else L.top[k - 2 * n] = v;
  }
  wave_sync();
}

// One transform block with one wave: PCM copy, or (intra prediction +) inverse transform +
// reconstruction into the picture.
// (inlined into both launch kernels: as a call its pointer arguments would be generic, i.e. flat
// accesses)
template <class P>
__device__ __attribute__((always_inline)) inline void tu_wave_t(const HevcDesc& d, const GpuTu& t, int lane, TuWave& L,
                                                                bool publish) {
  const int stride = d.stride;
  P* y = reinterpret_cast<P*>(d.y + size_t(d.target) * d.slot_y);
  P* uv = reinterpret_cast<P*>(d.uv + size_t(d.target) * d.slot_uv);
  wave_sync();  // the wave's previous block has finished reading its LDS
  if (t.flags & hevc::kTuPcm) {  // (the records hold the samples at the picture's sample type)
    const int n = 1 << t.log2, nc = n >> 1;
    const P* src = reinterpret_cast<const P*>(d.pcm + t.data);
    for (int s = lane; s < n * n; s += 64) y[(t.y + s / n) * stride + t.x + s % n] = src[s];
    for (int s = lane; s < 2 * nc * nc; s += 64) {
      const int c = s / (nc * nc), r = s - c * nc * nc;
      uv[((t.y >> 1) + r / nc) * stride + t.x + 2 * (r % nc) + c] = src[n * n + s];
    }
    return;
  }
  const int log2 = t.log2, n = 1 << log2;
  P* plane = t.c == 0 ? y : uv + (t.c - 1);
  const int step = t.c == 0 ? 1 : 2;
  const int bd = bd_of<P>(t.c == 0 ? d.bd_y : d.bd_c);
  const bool intra = t.flags & hevc::kTuIntra;
  const bool coef = t.flags & hevc::kTuCoef;
  const bool tskip = t.flags & hevc::kTuSkip;
  const bool bypass = t.flags & hevc::kTuBypass;  // lossless CU: the coefficients are the residual
  const bool dst = t.flags & hevc::kTuDst;
  if (coef) {  // (uniform per wave) sparse -> dense: lane w takes mask word w, a wave prefix sum
               // of the popcounts places its values (hevc::hk_sparse_store's layout)
    const int nn = n * n, nw = nn >> 4;
    for (int k = lane * 8; k < nn; k += 64 * 8) *reinterpret_cast<uint4*>(&L.dq[k]) = make_uint4(0, 0, 0, 0);
    const VEP_DEV i16* src = d.coefs + t.data;
    const u32 mask = lane < nw ? u32(u16(src[lane])) : 0u;
    const int cnt = __popc(mask);
    int incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(incl, o);
      if (lane >= o) incl += u;
    }
    wave_sync();  // the zeros land before the scatter
    const VEP_DEV i16* v = src + nw + (incl - cnt);
    for (u32 b = mask; b; b &= b - 1) L.dq[16 * lane + __ffs(int(b)) - 1] = *v++;
    wave_sync();
  }
  const i16* dq = L.dq;
  if (intra)  // (uniform per wave)
    prepare_refs_wave(d, t, plane, stride, step, lane, L, bd);
  const int mx = t.ext_x, my = t.ext_y;
  if (coef && !tskip && !bypass) {
    for (int s = lane; s < n * (mx + 1); s += 64) {
      const int yy = s / (mx + 1), xx = s - yy * (mx + 1);
      L.g[yy * n + xx] = hevc::hk_itx_col(dq, log2, dst, yy, xx, my);
    }
    wave_sync();
  }
  for (int s = lane; s < n * n; s += 64) {
    const int yy = s >> log2, xx = s & (n - 1);
    P& q = plane[(t.y + yy) * stride + (t.x + xx) * step];
    int v = intra ? hevc::hk_intra_sample(L.top, L.left, log2, t.mode, t.c == 0, xx, yy, bd) : int(q);
    if (coef)
      v += bypass ? int(dq[s]) : (tskip ? hevc::hk_tskip(dq[s], bd) : hevc::hk_itx_row(&L.g[yy * n], log2, dst, xx, mx, bd));
    const P o = P(hevc::hk_clip(v, bd));
    q = o;
    if (publish) {  // the right column / bottom row other intra blocks of the launch may read
      if (xx == n - 1) xg_put(xg_col(d, t.c, t.x + xx, t.y + yy), d.epoch, o);
      if (yy == n - 1) xg_put(xg_row(d, t.c, t.x + xx, t.y + yy), d.epoch, o);
    }
  }
}

__device__ __attribute__((always_inline)) inline void tu_wave(const HevcDesc& d, const GpuTu& t, int lane, TuWave& L,
                                                              bool publish) {
  if (d.flags & kHevcWide) tu_wave_t<u16>(d, t, lane, L, publish);
  else tu_wave_t<u8>(d, t, lane, L, publish);
}

// Independent blocks (level 0, or one intra level when levels are launched one by one):
// tickets base .. end, four blocks per workgroup, one per wave.
__global__ __launch_bounds__(256) void hevc_tu_kernel(const HevcDesc* __restrict__ descs,
                                                     const HevcTuRange* __restrict__ ranges, int nranges, int base,
                                                     int end) {
  __shared__ TuWave lds[4];
  const int wave = int(threadIdx.x) >> 6, lane = int(threadIdx.x) & 63;
  const int b = base + int(blockIdx.x) * 4 + wave;
  if (b >= end) return;  // (uniform per wave; no workgroup barrier below)
  const HevcTuRange& rg = ranges[pick_range(ranges, nranges, b)];
  const HevcDesc& d = descs[rg.desc];
  tu_wave(d, static_cast<const GpuTu*>(d.tus)[rg.first + (b - rg.begin)], lane, lds[wave], false);
}

// Intra levels: every intra block of the round in ONE launch. Waves take tickets in level order
// until the queue is empty, so a block's producers (lower levels) were taken earlier by running
// waves and the lowest unfinished ticket can always proceed (no co-residency assumption). A block
// reads its references from the picture, except the units written in this launch (GpuTu::pend),
// which it polls from the producers' epoch-tagged edge words: the data is its own flag, so there
// is no completion counter, no release fence and no L2 writeback. A wait that exceeds the spin
// limit marks the picture's error word (the frame is dropped) and goes on, so the grid drains.
// Tickets base .. end of the round's queue (a window of consecutive levels, or all of them);
// producers in an earlier window of the round finished before this launch started (stream order)
// and their edge words already carry this round's epoch.
// Windows (persistent = 0): one wave per block, but the block is still taken from the ticket
// counter, not from blockIdx: a wave only ever waits on blocks with lower tickets, which were
// claimed by waves that are already running, so progress never depends on the order in which
// the hardware dispatches workgroups (round 3's grid-order windows stalled when rocprofv3's
// counter collection changed it).
__global__ __launch_bounds__(256) void hevc_tu_queue_kernel(const HevcDesc* __restrict__ descs,
                                                           const HevcTuRange* __restrict__ ranges, int nranges,
                                                           int base, int end, u32* __restrict__ ctr,
                                                           int persistent) {
  __shared__ TuWave lds[4];
  const int wave = int(threadIdx.x) >> 6, lane = int(threadIdx.x) & 63;
  TuWave& L = lds[wave];
  for (int it = 0; persistent || it == 0; ++it) {
    int t = 0;
    if (lane == 0) t = base + int(__hip_atomic_fetch_add(&ctr[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    t = __shfl(t, 0);
    if (t >= end) break;
    const HevcTuRange& rg = ranges[pick_range(ranges, nranges, t)];
    const HevcDesc& d = descs[rg.desc];
    tu_wave(d, static_cast<const GpuTu*>(d.tus)[rg.first + (t - rg.begin)], lane, L, true);
  }
}

// One picture's intra blocks per workgroup (VEP_HEVC_TU_WINDOW=-1): pics[blockIdx.x] names the
// picture and its intra blocks tus[first .. first + count), level-major. The workgroup's 16 waves
// take them in that order from an LDS counter, so every block a wave waits on (a lower level of
// the same picture) was claimed by a wave of the SAME workgroup: co-resident by construction, so
// no wait depends on how or when the hardware dispatches other workgroups. The edge-word exchange
// is the queue kernel's.
constexpr int kTuPicWaves = 16;
__global__ __launch_bounds__(64 * kTuPicWaves) void hevc_tu_pic_kernel(const HevcDesc* __restrict__ descs,
                                                                       const HevcTuRange* __restrict__ pics) {
  __shared__ TuWave lds[kTuPicWaves];
  __shared__ u32 next;
  const int wave = int(threadIdx.x) >> 6, lane = int(threadIdx.x) & 63;
  if (threadIdx.x == 0) next = 0;
  __syncthreads();
  const HevcTuRange pr = pics[blockIdx.x];
  const HevcDesc& d = descs[pr.desc];
  const GpuTu* tus = static_cast<const GpuTu*>(d.tus) + pr.first;
  for (;;) {
    int t = 0;
    if (lane == 0) t = int(__hip_atomic_fetch_add(&next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    t = __shfl(t, 0);
    if (t >= pr.count) break;
    tu_wave(d, tus[t], lane, lds[wave], true);
  }
}

// ------------------------------------------------------------------------------ deblocking
template <class P>
__device__ __attribute__((always_inline)) inline void deblock_edge(const HevcDesc& d, int k, int x, int yy, int bs,
                                                                   int dir) {
  const int w4 = d.width >> 2;
  const int stride = d.stride, bdy = bd_of<P>(d.bd_y), bdc = bd_of<P>(d.bd_c);
  P* y = reinterpret_cast<P*>(d.y + size_t(d.target) * d.slot_y);
  P* uv = reinterpret_cast<P*>(d.uv + size_t(d.target) * d.slot_uv);
  const int xp = dir == 0 ? x - 1 : x, yp = dir == 0 ? yy : yy - 1;
  const int kp = (yp >> 2) * w4 + (xp >> 2);
  const GpuSlice& sl =
      static_cast<const GpuSlice*>(d.slices)[d.ctb_slice[(yy >> d.log2ctb) * d.wctb + (x >> d.log2ctb)]];
  const bool nof = d.flags & 4;
  const bool nfp = nof && d.pcm_map[kp], nfq = nof && d.pcm_map[k];
  // (bS is non-zero only on the 8x8 grid)
  hevc::HkLumaEdgeT<P> e{y + yy * stride + x, dir == 0 ? stride : 1, dir == 0 ? 1 : stride};
  hevc::hk_deblock_luma(e, bs, (d.qp[kp] + d.qp[k] + 1) >> 1, sl.beta_offset, sl.tc_offset, nfp, nfq, bdy);
  if (bs == 2 && ((dir == 0 ? x : yy) & 15) == 0)
    for (int c = 0; c < 2; ++c)
      hevc::hk_deblock_chroma(uv + (yy >> 1) * stride + x + c, dir == 0 ? stride : 2, dir == 0 ? 2 : stride,
                              d.qp[kp], d.qp[k], c == 0 ? d.cb_qp_offset : d.cr_qp_offset, sl.tc_offset, nfp,
                              nfq, bdc);
}

__global__ __launch_bounds__(256) void hevc_deblock_kernel(const HevcDesc* __restrict__ descs, int n, int total,
                                                          int dir) {
  const int b = int(blockIdx.x * blockDim.x + threadIdx.x);
  if (b >= total) return;
  const HevcDesc& d = descs[pick_blk(descs, n, b)];
  if (!(d.flags & 1)) return;
  const int w4 = d.width >> 2, k = b - d.blk_begin;
  const int x = (k % w4) << 2, yy = (k / w4) << 2;
  const u8* bsm = dir == 0 ? d.bs_v : d.bs_h;
  const int bs = bsm[k];
  if (!bs) return;
  if (d.flags & kHevcWide) deblock_edge<u16>(d, k, x, yy, bs, dir);
  else deblock_edge<u8>(d, k, x, yy, bs, dir);
}

// ------------------------------------------------------------------------------ SAO
// The deblocked picture into the SAO scratch surface: 4 samples per row of the lane's 4x4 block
// (one u32, or one u64 for u16 samples).
__global__ __launch_bounds__(256) void hevc_sao_copy_kernel(const HevcDesc* __restrict__ descs, int n, int total) {
  const int b = int(blockIdx.x * blockDim.x + threadIdx.x);
  if (b >= total) return;
  const HevcDesc& d = descs[pick_blk(descs, n, b)];
  if (!(d.flags & 2)) return;
  const int w4 = d.width >> 2, k = b - d.blk_begin;
  const int x = (k % w4) << 2, yy = (k / w4) << 2;
  const int stride = d.stride;
  const u8* y = d.y + size_t(d.target) * d.slot_y;
  const u8* uv = d.uv + size_t(d.target) * d.slot_uv;
  if (d.flags & kHevcWide) {  // byte offsets of u16 samples: 8-byte aligned rows of 4
    for (int j = 0; j < 4; ++j)
      *reinterpret_cast<u64*>(d.sao_y + 2 * ((yy + j) * stride + x)) =
          *reinterpret_cast<const u64*>(y + 2 * ((yy + j) * stride + x));
    for (int j = 0; j < 2; ++j)
      *reinterpret_cast<u64*>(d.sao_uv + 2 * (((yy >> 1) + j) * stride + x)) =
          *reinterpret_cast<const u64*>(uv + 2 * (((yy >> 1) + j) * stride + x));
    return;
  }
  for (int j = 0; j < 4; ++j)
    *reinterpret_cast<u32*>(d.sao_y + (yy + j) * stride + x) = *reinterpret_cast<const u32*>(y + (yy + j) * stride + x);
  for (int j = 0; j < 2; ++j)
    *reinterpret_cast<u32*>(d.sao_uv + ((yy >> 1) + j) * stride + x) =
        *reinterpret_cast<const u32*>(uv + ((yy >> 1) + j) * stride + x);
}

template <class P>
__device__ __attribute__((always_inline)) inline void sao_block(const HevcDesc& d, int x4, int y4) {
  const int ci = (y4 >> d.log2ctb) * d.wctb + (x4 >> d.log2ctb);
  const GpuSao sp = static_cast<const GpuSao*>(d.sao)[ci];
  const int si = d.ctb_slice[ci];
  const GpuSlice* slices = static_cast<const GpuSlice*>(d.slices);
  const GpuSlice sl = slices[si];
  const int stride = d.stride;
  P* y = reinterpret_cast<P*>(d.y + size_t(d.target) * d.slot_y);
  P* uv = reinterpret_cast<P*>(d.uv + size_t(d.target) * d.slot_uv);
  for (int c = 0; c < 3; ++c) {
    if (!sp.type[c] || (c == 0 ? !sl.sao_luma : !sl.sao_chroma)) continue;
    const int sub = c ? 1 : 0, step = c ? 2 : 1;
    const int bd = bd_of<P>(c ? d.bd_c : d.bd_y);
    const P* src = c == 0 ? reinterpret_cast<const P*>(d.sao_y) : reinterpret_cast<const P*>(d.sao_uv) + (c - 1);
    P* dst = c == 0 ? y : uv + (c - 1);
    const int pw = d.width >> sub, ph = d.height >> sub;
    auto nb_ok = [&](int nx, int ny) {
      if (nx < 0 || ny < 0 || nx >= pw || ny >= ph) return false;
      const int nci = ((ny << sub) >> d.log2ctb) * d.wctb + ((nx << sub) >> d.log2ctb);
      if ((d.flags & 8) && d.ctb_tile[nci] != d.ctb_tile[ci]) return false;
      const int nsi = d.ctb_slice[nci];
      if (nsi == si) return true;
      return nsi > si ? slices[nsi].across != 0 : sl.across != 0;
    };
    const int sz = 4 >> sub, x0 = x4 >> sub, y0 = y4 >> sub;
    for (int j = 0; j < sz; ++j)
      for (int i = 0; i < sz; ++i)
        dst[(y0 + j) * stride + (x0 + i) * step] =
            P(hevc::hk_sao_sample(src, stride, step, sp, c, x0 + i, y0 + j, nb_ok, bd));
  }
}

__global__ __launch_bounds__(256) void hevc_sao_kernel(const HevcDesc* __restrict__ descs, int n, int total) {
  const int b = int(blockIdx.x * blockDim.x + threadIdx.x);
  if (b >= total) return;
  const HevcDesc& d = descs[pick_blk(descs, n, b)];
  if (!(d.flags & 2)) return;
  const int w4 = d.width >> 2, k = b - d.blk_begin;
  const int x4 = (k % w4) << 2, y4 = (k / w4) << 2;
  if ((d.flags & 4) && d.pcm_map[k]) return;
  if (d.flags & kHevcWide) sao_block<u16>(d, x4, y4);
  else sao_block<u8>(d, x4, y4);
}

// 8 samples per lane: one 16-byte load, one 8-byte store.
// 8-bit NV12 copy of a published slot: one thread per 8 output bytes (w is a multiple of 16, so
// a group never straddles a row). Luma: rounded to 8 bits; chroma: NV12 row r from row r of the
// source (4:2:0) or the average of rows 2r and 2r + 1 (4:2:2, NV16), then rounded.
template <class P>
__global__ __launch_bounds__(256) void narrow_kernel(const P* __restrict__ y, const P* __restrict__ uv,
                                                    u8* __restrict__ y8, u8* __restrict__ uv8, int w, int h, int bd,
                                                    int cf) {
  const size_t ny = size_t(w) * size_t(h);
  const size_t g = size_t(blockIdx.x) * 256 + threadIdx.x, groups = (ny + ny / 2) / 8;
  if (g >= groups) return;
  const bool luma = g < ny / 8;
  const size_t o = luma ? g * 8 : (g - ny / 8) * 8;
  int v[8];
  if (luma) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = int(y[o + size_t(k)]);
  } else {
    const size_t r = o / size_t(w), x = o % size_t(w);
    if (cf == 2) {
      const P* a = uv + 2 * r * size_t(w) + x;
      const P* b = a + w;
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = (int(a[k]) + int(b[k]) + 1) >> 1;
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = int(uv[o + size_t(k)]);
    }
  }
  const int sh = bd - 8, rnd = (1 << sh) >> 1;
  u32 out[2] = {0, 0};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int n = (v[k] + rnd) >> sh;
    out[k >> 2] |= u32(n > 255 ? 255 : n) << (8 * (k & 3));
  }
  *reinterpret_cast<uint2*>((luma ? y8 : uv8) + o) = make_uint2(out[0], out[1]);
}

}  // namespace

void launch_narrow(const void* y, const void* uv, u8* y8, u8* uv8, int w, int h, int bd, int cf, hipStream_t s) {
  const size_t n = size_t(w) * size_t(h);
  if (!n) return;
  const size_t groups = (n + n / 2) / 8;
  const dim3 grid(unsigned((groups + 255) / 256));
  if (bd > 8)
    hipLaunchKernelGGL(narrow_kernel<u16>, grid, dim3(256), 0, s, static_cast<const u16*>(y),
                       static_cast<const u16*>(uv), y8, uv8, w, h, bd, cf);
  else
    hipLaunchKernelGGL(narrow_kernel<u8>, grid, dim3(256), 0, s, static_cast<const u8*>(y),
                       static_cast<const u8*>(uv), y8, uv8, w, h, 8, cf);
}

void launch_hevc_mc(const HevcDesc* d_descs, int n, int total_pus, hipStream_t s) {
  if (n <= 0 || total_pus <= 0) return;
  hipLaunchKernelGGL(hevc_mc_kernel, dim3(total_pus), dim3(256), 0, s, d_descs, n);
}

void launch_hevc_tu(const HevcDesc* d_descs, const HevcTuRange* d_ranges, int nranges, int base, int count,
                    hipStream_t s) {
  if (nranges <= 0 || count <= 0) return;
  hipLaunchKernelGGL(hevc_tu_kernel, dim3((count + 3) / 4), dim3(256), 0, s, d_descs, d_ranges, nranges, base,
                     base + count);
}

void launch_hevc_tu_queue(const HevcDesc* d_descs, const HevcTuRange* d_ranges, int nranges, int base, int count,
                          u32* ctr, bool persistent, hipStream_t s) {
  if (nranges <= 0 || count <= 0 || !ctr) return;
  // persistent waves: a fraction of the chip (4 per workgroup) — the other lanes' kernels run
  // beside it, and waves that run far ahead of the wavefront only poll. Windows: a wave per block.
  static const int queue_wgs = [] {
    const char* e = std::getenv("VEP_HEVC_TU_QUEUE_WGS");
    return e ? std::clamp(std::atoi(e), 1, 65536) : kTuQueueWgs;
  }();
  const int wgs = persistent ? std::min((count + 3) / 4, queue_wgs) : (count + 3) / 4;
  hipLaunchKernelGGL(hevc_tu_queue_kernel, dim3(wgs), dim3(256), 0, s, d_descs, d_ranges, nranges, base, base + count,
                     ctr, persistent ? 1 : 0);
}

void launch_hevc_tu_pics(const HevcDesc* d_descs, const HevcTuRange* d_pics, int npics, hipStream_t s) {
  if (npics <= 0) return;
  hipLaunchKernelGGL(hevc_tu_pic_kernel, dim3(npics), dim3(64 * kTuPicWaves), 0, s, d_descs, d_pics);
}

void launch_hevc_deblock(const HevcDesc* d_descs, int n, int total_blocks, int dir, hipStream_t s) {
  if (n <= 0 || total_blocks <= 0) return;
  hipLaunchKernelGGL(hevc_deblock_kernel, dim3((total_blocks + 255) / 256), dim3(256), 0, s, d_descs, n,
                     total_blocks, dir);
}

void launch_hevc_sao(const HevcDesc* d_descs, int n, int total_blocks, hipStream_t s) {
  if (n <= 0 || total_blocks <= 0) return;
  const dim3 grid((total_blocks + 255) / 256);
  hipLaunchKernelGGL(hevc_sao_copy_kernel, grid, dim3(256), 0, s, d_descs, n, total_blocks);
  hipLaunchKernelGGL(hevc_sao_kernel, grid, dim3(256), 0, s, d_descs, n, total_blocks);
}

}  // namespace vep::gpu
