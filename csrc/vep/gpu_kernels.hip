// gfx950 (CDNA4) kernels of the vep data plane. See gpu.h for the contracts.
//
// Design notes (MI355X):
//  * Both kernels are HBM-bound streaming kernels (≈9.3 MB moved per 1080p frame for
//    decode_convert), so the levers are 16-B vector accesses, full 64-lane waves with
//    contiguous per-wave output, and >>256 workgroups per launch: one launch covers every
//    camera on the GPU (32 x 1080p = 16,320 workgroups).
//  * decode_convert maps a 256-thread workgroup onto an 8x2-macroblock tile, lane = one
//    16-pixel row segment: 8 consecutive lanes write 8 x 48 B = 384 contiguous bytes of one
//    BGR row, a wave covers 8 rows (no LDS needed — there is no intra-tile reuse).
//  * PCM slots are 384 = 24 x 16 B, so every payload read is an aligned dwordx4 / dwordx2.
//  * letterbox reads the NV12 surface (1.5 B/px) instead of the BGR slot (3 B/px).
#define VEP_KERNEL_SOURCE 1  // descriptors' pointers are global-address-space here (gpu.h)
#include <algorithm>
#include <cmath>

#include "color.h"
#include "gpu.h"

namespace vep::gpu {

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

__device__ __forceinline__ uint32_t pack4(uint8_t a, uint8_t b, uint8_t c, uint8_t d) {
  return uint32_t(a) | (uint32_t(b) << 8) | (uint32_t(c) << 16) | (uint32_t(d) << 24);
}

// 16 luma bytes + 8 interleaved (Cb,Cr) pairs -> 48 BGR bytes as 12 dwords.
__device__ __forceinline__ void convert16(const uint4 yv, const uint4 uvv, uint32_t out[12]) {
  const uint32_t yw[4] = {yv.x, yv.y, yv.z, yv.w};
  const uint32_t cw[4] = {uvv.x, uvv.y, uvv.z, uvv.w};
  uint8_t px[48];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    int y = (yw[i >> 2] >> (8 * (i & 3))) & 0xff;
    int pair = i >> 1;  // chroma sample index 0..7: word pair>>1, byte (pair&1)*2
    uint32_t w = cw[pair >> 1];
    int u = (w >> (16 * (pair & 1))) & 0xff;
    int v = (w >> (16 * (pair & 1) + 8)) & 0xff;
    int c = (y - 16) * kCy + 32768;
    int d = u - 128, e = v - 128;
    px[3 * i + 0] = clip_u8((c + kCbu * d) >> 16);
    px[3 * i + 1] = clip_u8((c - kCgu * d - kCgv * e) >> 16);
    px[3 * i + 2] = clip_u8((c + kCrv * e) >> 16);
  }
#pragma unroll
  for (int k = 0; k < 12; ++k)
    out[k] = pack4(px[4 * k], px[4 * k + 1], px[4 * k + 2], px[4 * k + 3]);
}

// One 8x2-MB tile per 256-thread workgroup. Phase 1 stages the tile's coded PCM blocks into LDS
// with coalesced loads: 24 lanes x 16 B cover one block's 384 contiguous bytes, so a block is a
// few full PCIe read requests when the bytes live in pinned host memory (direct mode) and full
// cache lines otherwise. Phase 2: each lane owns one 16-pixel row of one MB — reconstructs it
// into the NV12 reference surfaces and converts it to 48 bytes of BGR24.
__device__ __forceinline__ void decode_convert_tile(const DecodeDesc& d, const int tile,
                                                   uint8_t (*blk)[kPcmMbBytes]) {
  const int tx = tile % d.tiles_x, ty = tile / d.tiles_x;
  const int t = threadIdx.x;
  auto slot_of = [&](int mbx, int mby) {
    if (!d.mask || mbx >= d.wmbs || mby >= d.hmbs) return -1;
    const int mb = mby * d.wmbs + mbx;
    const uint32_t w = d.mask[mb >> 5];
    const uint32_t bit = 1u << (mb & 31);
    return (w & bit) ? int(d.prefix[mb >> 5] + __builtin_popcount(w & (bit - 1u))) : -1;
  };
  auto src_of = [&](int slot) {
    return d.ptrs ? reinterpret_cast<const uint8_t*>(d.ptrs[slot]) : d.payload + d.offsets[slot];
  };
  // phase 1: LDS staging (MB i of the tile = column i & 7, MB row i >> 3)
  constexpr int kParts = kPcmMbBytes / 16;  // 24
  for (int idx = t; idx < kTileMbW * kTileMbH * kParts; idx += 256) {
    const int i = idx / kParts, part = idx - i * kParts;
    const int slot = slot_of(tx * kTileMbW + (i & 7), ty * kTileMbH + (i >> 3));
    if (slot < 0) continue;
    const uint8_t* src = src_of(slot);
    uint4 v;
    __builtin_memcpy(&v, src + part * 16, 16);
    *reinterpret_cast<uint4*>(&blk[i][part * 16]) = v;
    if (part == 0 && slot >= d.chk_lo && slot < d.chk_hi &&
        (uint32_t(src[-2]) | (uint32_t(src[-1]) << 8)) != d.chk_pat)
      __hip_atomic_store(d.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  // phase 2
  const int r = t >> 3, c = t & 7;
  const int mbx = tx * kTileMbW + c;
  const int mby = ty * kTileMbH + (r >> 4);
  const int row = r & 15;
  if (mbx >= d.wmbs || mby >= d.hmbs) return;
  const int pitch = d.wmbs * 16;
  const int slot = slot_of(mbx, mby);
  uint8_t* yp = d.y + size_t(mby * 16 + row) * pitch + mbx * 16;
  uint8_t* uvp = d.uv + size_t(mby * 8 + (row >> 1)) * pitch + mbx * 16;
  uint4 yv, uvv;
  if (slot >= 0) {
    const uint8_t* b = blk[(r >> 4) * kTileMbW + c];
    yv = *reinterpret_cast<const uint4*>(b + row * 16);
    const uint2 cb = *reinterpret_cast<const uint2*>(b + 256 + (row >> 1) * 8);
    const uint2 cr = *reinterpret_cast<const uint2*>(b + 320 + (row >> 1) * 8);
    // interleave Cb/Cr bytes: (cb0 cr0 cb1 cr1) ...
    uvv.x = __builtin_amdgcn_perm(cr.x, cb.x, 0x05010400u);
    uvv.y = __builtin_amdgcn_perm(cr.x, cb.x, 0x07030602u);
    uvv.z = __builtin_amdgcn_perm(cr.y, cb.y, 0x05010400u);
    uvv.w = __builtin_amdgcn_perm(cr.y, cb.y, 0x07030602u);
    *reinterpret_cast<uint4*>(yp) = yv;
    if ((row & 1) == 0) *reinterpret_cast<uint4*>(uvp) = uvv;
  } else {
    yv = *reinterpret_cast<const uint4*>(yp);
    uvv = *reinterpret_cast<const uint4*>(uvp);
  }
  if (!d.bgr) return;
  const int oy = mby * 16 + row - d.crop_top;
  const int ox = mbx * 16 - d.crop_left;
  if (oy < 0 || oy >= d.out_h || ox + 16 <= 0 || ox >= d.out_w) return;
  uint32_t o[12];
  convert16(yv, uvv, o);
  uint8_t* dst = d.bgr + (size_t(oy) * d.out_w + ox) * 3;
  if (ox >= 0 && ox + 16 <= d.out_w) {
    // 48 contiguous bytes; 16-B aligned whenever out_w % 16 == 0 and crop_left % 16 == 0
    uint4 a = make_uint4(o[0], o[1], o[2], o[3]), bq = make_uint4(o[4], o[5], o[6], o[7]),
          cq = make_uint4(o[8], o[9], o[10], o[11]);
    __builtin_memcpy(dst, &a, 16);
    __builtin_memcpy(dst + 16, &bq, 16);
    __builtin_memcpy(dst + 32, &cq, 16);
  } else {  // ragged left/right crop edge
    for (int i = 0; i < 16; ++i) {
      int x = ox + i;
      if (x < 0 || x >= d.out_w) continue;
      for (int k = 0; k < 3; ++k) {
        int bi = 3 * i + k;
        d.bgr[(size_t(oy) * d.out_w + x) * 3 + k] = uint8_t(o[bi >> 2] >> (8 * (bi & 3)));
      }
    }
  }
}

__global__ __launch_bounds__(256) void decode_convert_kernel(const DecodeDesc* __restrict__ descs,
                                                             int n) {
  // block -> job: binary search over the tile prefix (wave-uniform, scalar loads)
  const int b = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (descs[mid].tile_begin <= b) lo = mid; else hi = mid - 1;
  }
  const DecodeDesc d = descs[lo];
  __shared__ __attribute__((aligned(16))) uint8_t blk[kTileMbW * kTileMbH][kPcmMbBytes];
  decode_convert_tile(d, b - d.tile_begin, blk);
}

__global__ __launch_bounds__(256) void decode_convert_one_kernel(const DecodeDesc d) {
  __shared__ __attribute__((aligned(16))) uint8_t blk[kTileMbW * kTileMbH][kPcmMbBytes];
  decode_convert_tile(d, blockIdx.x, blk);
}

void launch_decode_convert_one(const DecodeDesc& d, hipStream_t s) {
  hipLaunchKernelGGL(decode_convert_one_kernel, dim3(tiles_for(d.wmbs, d.hmbs)), dim3(256), 0, s,
                     d);
  VEP_HIP(hipGetLastError());
}

void launch_decode_convert(const DecodeDesc* d_descs, int n, int total_tiles, hipStream_t s) {
  if (n <= 0 || total_tiles <= 0) return;
  hipLaunchKernelGGL(decode_convert_kernel, dim3(total_tiles), dim3(256), 0, s, d_descs, n);
  VEP_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------------------------
// Gather (pinned host -> device). The source is read once over PCIe: 256 lanes x 16 B per
// iteration keeps 4 KiB in flight per workgroup; dst offsets are 16-byte aligned.

__global__ __launch_bounds__(256) void gather_kernel(const GatherChunk* __restrict__ chunks) {
  const GatherChunk c = chunks[blockIdx.x];
  const u32 full = c.len & ~15u;
  for (u32 o = threadIdx.x * 16u; o < full; o += 256u * 16u) {
    uint4 v;
    __builtin_memcpy(&v, c.src + o, 16);
    *reinterpret_cast<uint4*>(c.dst + o) = v;
  }
  const u32 tail = c.len - full;
  if (threadIdx.x < tail) c.dst[full + threadIdx.x] = c.src[full + threadIdx.x];
}

void launch_gather(const GatherChunk* d_chunks, int n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gather_kernel, dim3(n), dim3(256), 0, s, d_chunks);
  VEP_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------------------------
// Letterbox: bilinear (align_corners=False, as torch F.interpolate / cv2 INTER_LINEAR) resize of
// the BT.601-converted picture into an S x S canvas, centred, padded with pad_value.

__device__ __forceinline__ void bgr_at(const uint8_t* __restrict__ y,
                                       const uint8_t* __restrict__ uv, int pitch, int x, int yy,
                                       float& b, float& g, float& r) {
  int Y = y[size_t(yy) * pitch + x];
  const uint8_t* c = uv + size_t(yy >> 1) * pitch + (x & ~1);
  uint8_t bb, gg, rr;
  yuv_to_bgr(Y, c[0], c[1], &bb, &gg, &rr);
  b = bb;
  g = gg;
  r = rr;
}

__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return uint16_t(u >> 16);
}

__device__ __forceinline__ void letterbox_quad(const LetterboxDesc& d, const LetterboxParams& p) {
  const int S = p.size;
  const int q = blockIdx.x * 256 + threadIdx.x;  // quad index (4 px)
  const int pix0 = q * 4;
  if (pix0 >= S * S) return;
  const int oy = pix0 / S, ox0 = pix0 % S;
  float vb[4], vg[4], vr[4];
  bool inside_row = (oy >= d.pad_y && oy < d.pad_y + d.nh);
  float sy = 0.f, ly = 0.f;
  int y0 = 0, y1 = 0;
  if (inside_row) {
    sy = fmaxf((float(oy - d.pad_y) + 0.5f) * d.ry - 0.5f, 0.f);
    y0 = int(sy);
    y1 = y0 + (y0 < d.src_h - 1 ? 1 : 0);
    ly = sy - float(y0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ox = ox0 + i;
    if (!inside_row || ox < d.pad_x || ox >= d.pad_x + d.nw) {
      vb[i] = vg[i] = vr[i] = float(p.pad_value);
      continue;
    }
    float sx = fmaxf((float(ox - d.pad_x) + 0.5f) * d.rx - 0.5f, 0.f);
    int x0 = int(sx);
    int x1 = x0 + (x0 < d.src_w - 1 ? 1 : 0);
    float lx = sx - float(x0);
    float b00, g00, r00, b01, g01, r01, b10, g10, r10, b11, g11, r11;
    const int X0 = x0 + d.crop_left, X1 = x1 + d.crop_left;
    const int Y0 = y0 + d.crop_top, Y1 = y1 + d.crop_top;
    bgr_at(d.y, d.uv, d.pitch, X0, Y0, b00, g00, r00);
    bgr_at(d.y, d.uv, d.pitch, X1, Y0, b01, g01, r01);
    bgr_at(d.y, d.uv, d.pitch, X0, Y1, b10, g10, r10);
    bgr_at(d.y, d.uv, d.pitch, X1, Y1, b11, g11, r11);
    const float w00 = (1.f - ly) * (1.f - lx), w01 = (1.f - ly) * lx, w10 = ly * (1.f - lx),
                w11 = ly * lx;
    vb[i] = w00 * b00 + w01 * b01 + w10 * b10 + w11 * b11;
    vg[i] = w00 * g00 + w01 * g01 + w10 * g10 + w11 * g11;
    vr[i] = w00 * r00 + w01 * r01 + w10 * r10 + w11 * r11;
  }
  if (d.out_hwc) {
    uint8_t o[12];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[3 * i + 0] = uint8_t(fminf(fmaxf(vb[i] + 0.5f, 0.f), 255.f));
      o[3 * i + 1] = uint8_t(fminf(fmaxf(vg[i] + 0.5f, 0.f), 255.f));
      o[3 * i + 2] = uint8_t(fminf(fmaxf(vr[i] + 0.5f, 0.f), 255.f));
    }
    __builtin_memcpy(d.out_hwc + size_t(pix0) * 3, o, 12);
  }
  if (p.chw_dtype != kChwNone && d.out_chw) {
    const size_t plane = size_t(S) * S;
    float ch[3][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // RGB planes
      ch[0][i] = (vr[i] * (1.f / 255.f) - p.mean[0]) * p.inv_std[0];
      ch[1][i] = (vg[i] * (1.f / 255.f) - p.mean[1]) * p.inv_std[1];
      ch[2][i] = (vb[i] * (1.f / 255.f) - p.mean[2]) * p.inv_std[2];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (p.chw_dtype == kChwF32) {
        float4 v = make_float4(ch[k][0], ch[k][1], ch[k][2], ch[k][3]);
        *reinterpret_cast<float4*>(static_cast<float*>(d.out_chw) + k * plane + pix0) = v;
      } else if (p.chw_dtype == kChwF16) {
        _Float16 h[4] = {(_Float16)ch[k][0], (_Float16)ch[k][1], (_Float16)ch[k][2],
                         (_Float16)ch[k][3]};
        __builtin_memcpy(static_cast<_Float16*>(d.out_chw) + k * plane + pix0, h, 8);
      } else {
        uint16_t h[4] = {f32_to_bf16(ch[k][0]), f32_to_bf16(ch[k][1]), f32_to_bf16(ch[k][2]),
                         f32_to_bf16(ch[k][3])};
        __builtin_memcpy(static_cast<uint16_t*>(d.out_chw) + k * plane + pix0, h, 8);
      }
    }
  }
}

__global__ __launch_bounds__(256) void letterbox_kernel(const LetterboxDesc* __restrict__ descs,
                                                        LetterboxParams p) {
  const LetterboxDesc d = descs[blockIdx.y];
  letterbox_quad(d, p);
}

__global__ __launch_bounds__(256) void letterbox_one_kernel(const LetterboxDesc d,
                                                            LetterboxParams p) {
  letterbox_quad(d, p);
}

static inline u8 pad_luma(u8 pad);
__global__ void letterbox_nv12_one_kernel(const LetterboxDesc d, int size, uint8_t pad_y);

void launch_letterbox_one(const LetterboxDesc& d, const LetterboxParams& p, hipStream_t s) {
  VEP_CHECK(p.size % 8 == 0, "letterbox size must be a multiple of 8");
  if (p.format == kLbNV12) {
    const int work = p.size * p.size / 4 + p.size * p.size / 8;
    hipLaunchKernelGGL(letterbox_nv12_one_kernel, dim3((work + 255) / 256), dim3(256), 0, s, d,
                       p.size, pad_luma(p.pad_value));
  } else {
    int quads = p.size * p.size / 4;
    hipLaunchKernelGGL(letterbox_one_kernel, dim3((quads + 255) / 256), dim3(256), 0, s, d, p);
  }
  VEP_HIP(hipGetLastError());
}

void fill_letterbox_geometry(LetterboxDesc& d, int size, bool even) {
  float scale = std::min(float(size) / float(d.src_w), float(size) / float(d.src_h));
  d.nw = std::max(1, std::min(size, int(std::lround(d.src_w * scale))));
  d.nh = std::max(1, std::min(size, int(std::lround(d.src_h * scale))));
  d.pad_x = (size - d.nw) / 2;
  d.pad_y = (size - d.nh) / 2;
  if (even) {
    d.nw = std::max(2, d.nw & ~1);
    d.nh = std::max(2, d.nh & ~1);
    d.pad_x = ((size - d.nw) / 2) & ~1;
    d.pad_y = ((size - d.nh) / 2) & ~1;
  }
  d.rx = float(d.src_w) / float(d.nw);
  d.ry = float(d.src_h) / float(d.nh);
}

// ---------------------------------------------------------------------------------------------
// NV12 letterbox: the Y and the interleaved UV planes are resized independently (bilinear,
// align_corners=False) into an S x S NV12 canvas. Threads [0, S*S/4) produce 4 luma bytes each,
// threads [S*S/4, S*S/4 + S*S/8) produce 2 chroma pairs (4 bytes) each; one dword store per
// thread, consecutive lanes on consecutive dwords.

__device__ __forceinline__ float bilerp(const uint8_t* __restrict__ p, int pitch, int step,
                                        int x0, int x1, int y0, int y1, float lx, float ly) {
  const float a = p[size_t(y0) * pitch + x0 * step], b = p[size_t(y0) * pitch + x1 * step];
  const float c = p[size_t(y1) * pitch + x0 * step], e = p[size_t(y1) * pitch + x1 * step];
  return (1.f - ly) * ((1.f - lx) * a + lx * b) + ly * ((1.f - lx) * c + lx * e);
}

__device__ __forceinline__ void axis(int o, int pad, int n, float r, int src, int& i0, int& i1,
                                     float& l) {
  const float s = fmaxf((float(o - pad) + 0.5f) * r - 0.5f, 0.f);
  i0 = int(s);
  i1 = i0 + (i0 < src - 1 ? 1 : 0);
  l = s - float(i0);
}

__device__ __forceinline__ void letterbox_nv12_body(const LetterboxDesc& d, const int size,
                                                    const uint8_t pad_y) {
  const int S = size;
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int ny = S * S / 4, nuv = S * S / 8;
  if (t >= ny + nuv) return;
  uint8_t o[4];
  uint8_t* dst;
  if (t < ny) {  // luma
    const int pix0 = t * 4, oy = pix0 / S, ox0 = pix0 % S;
    const bool row_in = oy >= d.pad_y && oy < d.pad_y + d.nh;
    int y0 = 0, y1 = 0;
    float ly = 0.f;
    if (row_in) axis(oy, d.pad_y, d.nh, d.ry, d.src_h, y0, y1, ly);
    const uint8_t* Y = d.y + size_t(d.crop_top) * d.pitch + d.crop_left;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ox = ox0 + i;
      if (!row_in || ox < d.pad_x || ox >= d.pad_x + d.nw) {
        o[i] = pad_y;
        continue;
      }
      int x0, x1;
      float lx;
      axis(ox, d.pad_x, d.nw, d.rx, d.src_w, x0, x1, lx);
      o[i] = uint8_t(fminf(bilerp(Y, d.pitch, 1, x0, x1, y0, y1, lx, ly) + 0.5f, 255.f));
    }
    dst = d.out_hwc + size_t(pix0);
  } else {  // chroma: 2 (U,V) pairs
    const int q = t - ny;
    const int c0 = q * 2, Sc = S / 2, cy = c0 / Sc, cx0 = c0 % Sc;
    const int px = d.pad_x / 2, py = d.pad_y / 2, nwc = d.nw / 2, nhc = d.nh / 2;
    const int sw = (d.src_w + 1) / 2, sh = (d.src_h + 1) / 2;
    const bool row_in = cy >= py && cy < py + nhc;
    int y0 = 0, y1 = 0;
    float ly = 0.f;
    if (row_in) axis(cy, py, nhc, d.ry, sh, y0, y1, ly);
    const uint8_t* UV = d.uv + size_t(d.crop_top / 2) * d.pitch + (d.crop_left & ~1);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int cx = cx0 + i;
      if (!row_in || cx < px || cx >= px + nwc) {
        o[2 * i] = o[2 * i + 1] = 128;
        continue;
      }
      int x0, x1;
      float lx;
      axis(cx, px, nwc, d.rx, sw, x0, x1, lx);
      o[2 * i] = uint8_t(fminf(bilerp(UV, d.pitch, 2, x0, x1, y0, y1, lx, ly) + 0.5f, 255.f));
      o[2 * i + 1] = uint8_t(fminf(bilerp(UV + 1, d.pitch, 2, x0, x1, y0, y1, lx, ly) + 0.5f, 255.f));
    }
    dst = d.out_hwc + size_t(S) * S + size_t(c0) * 2;
  }
  __builtin_memcpy(dst, o, 4);
}

__global__ __launch_bounds__(256) void letterbox_nv12_kernel(const LetterboxDesc* __restrict__ descs,
                                                             int size, uint8_t pad_y) {
  const LetterboxDesc d = descs[blockIdx.y];
  letterbox_nv12_body(d, size, pad_y);
}

__global__ __launch_bounds__(256) void letterbox_nv12_one_kernel(const LetterboxDesc d, int size,
                                                                 uint8_t pad_y) {
  letterbox_nv12_body(d, size, pad_y);
}

// Consumer: NV12 [n][S*S*3/2] -> RGB CHW normalised, 4 pixels of a row per thread.
template <int DT>
__global__ __launch_bounds__(256) void nv12_to_chw_kernel(const uint8_t* __restrict__ in,
                                                          void* __restrict__ out, int size,
                                                          LetterboxParams p) {
  const int S = size;
  const int cam = blockIdx.y;
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q * 4 >= S * S) return;
  const int pix0 = q * 4, oy = pix0 / S, ox0 = pix0 % S;
  const uint8_t* base = in + size_t(cam) * (size_t(S) * S * 3 / 2);
  uint32_t yw, cw;
  __builtin_memcpy(&yw, base + pix0, 4);
  __builtin_memcpy(&cw, base + size_t(S) * S + size_t(oy >> 1) * S + ox0, 4);  // 2 UV pairs
  float ch[3][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int pair = i >> 1;
    uint8_t b, g, r;
    yuv_to_bgr(int((yw >> (8 * i)) & 0xff), int((cw >> (16 * pair)) & 0xff),
               int((cw >> (16 * pair + 8)) & 0xff), &b, &g, &r);
    ch[0][i] = (float(r) * (1.f / 255.f) - p.mean[0]) * p.inv_std[0];
    ch[1][i] = (float(g) * (1.f / 255.f) - p.mean[1]) * p.inv_std[1];
    ch[2][i] = (float(b) * (1.f / 255.f) - p.mean[2]) * p.inv_std[2];
  }
  const size_t plane = size_t(S) * S;
  const size_t obase = size_t(cam) * 3 * plane + size_t(pix0);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if constexpr (DT == kChwF32) {
      float4 v = make_float4(ch[k][0], ch[k][1], ch[k][2], ch[k][3]);
      *reinterpret_cast<float4*>(static_cast<float*>(out) + obase + k * plane) = v;
    } else if constexpr (DT == kChwF16) {
      _Float16 h[4] = {(_Float16)ch[k][0], (_Float16)ch[k][1], (_Float16)ch[k][2], (_Float16)ch[k][3]};
      __builtin_memcpy(static_cast<_Float16*>(out) + obase + k * plane, h, 8);
    } else {
      uint16_t h[4] = {f32_to_bf16(ch[k][0]), f32_to_bf16(ch[k][1]), f32_to_bf16(ch[k][2]),
                       f32_to_bf16(ch[k][3])};
      __builtin_memcpy(static_cast<uint16_t*>(out) + obase + k * plane, h, 8);
    }
  }
}

void launch_nv12_to_chw(const u8* in, void* out, int n, int size, int chw_dtype,
                        const float mean[3], const float inv_std[3], hipStream_t s) {
  if (n <= 0) return;
  VEP_CHECK(size % 4 == 0, "size must be a multiple of 4");
  LetterboxParams p{};
  p.size = size;
  for (int k = 0; k < 3; ++k) {
    p.mean[k] = mean[k];
    p.inv_std[k] = inv_std[k];
  }
  dim3 grid((size * size / 4 + 255) / 256, n);
  if (chw_dtype == kChwF32)
    hipLaunchKernelGGL(nv12_to_chw_kernel<kChwF32>, grid, dim3(256), 0, s, in, out, size, p);
  else if (chw_dtype == kChwF16)
    hipLaunchKernelGGL(nv12_to_chw_kernel<kChwF16>, grid, dim3(256), 0, s, in, out, size, p);
  else if (chw_dtype == kChwBF16)
    hipLaunchKernelGGL(nv12_to_chw_kernel<kChwBF16>, grid, dim3(256), 0, s, in, out, size, p);
  else
    throw Error("nv12_to_chw: unsupported dtype");
  VEP_HIP(hipGetLastError());
}

static inline u8 pad_luma(u8 pad) { return u8(std::lround(16.0 + pad * 219.0 / 255.0)); }

void launch_letterbox(const LetterboxDesc* d_descs, int n, const LetterboxParams& p,
                      hipStream_t s) {
  if (n <= 0) return;
  VEP_CHECK(p.size % 8 == 0, "letterbox size must be a multiple of 8");
  if (p.format == kLbNV12) {
    const int work = p.size * p.size / 4 + p.size * p.size / 8;
    hipLaunchKernelGGL(letterbox_nv12_kernel, dim3((work + 255) / 256, n), dim3(256), 0, s,
                       d_descs, p.size, pad_luma(p.pad_value));
  } else {
    int quads = p.size * p.size / 4;
    hipLaunchKernelGGL(letterbox_kernel, dim3((quads + 255) / 256, n), dim3(256), 0, s, d_descs,
                       p);
  }
  VEP_HIP(hipGetLastError());
}

}  // namespace vep::gpu
