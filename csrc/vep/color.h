// BT.601 limited-range YCbCr -> BGR24 fixed-point conversion shared by the CPU reference
// path and the gfx950 HIP kernels, so both produce bit-identical pixels.
//
// Reference parity: python/read_image.py:94 `frame.to_ndarray(format='bgr24')` (libswscale
// unscaled yuv420p->bgr24 path: BT.601 matrix, limited range, nearest-neighbour chroma).
// Coefficients are 16.16 fixed point of the BT.601 inverse matrix (255/219 luma gain).
// Parity with swscale itself is unpinned (no FFmpeg in the image); the CPU reference below is
// the oracle for the GPU kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vep {

constexpr int kCy = 76309;    // 1.164383 * 65536
constexpr int kCrv = 104597;  // 1.596027 * 65536
constexpr int kCgu = 25675;   // 0.391762 * 65536
constexpr int kCgv = 53279;   // 0.812968 * 65536
constexpr int kCbu = 132201;  // 2.017232 * 65536

__host__ __device__ inline uint8_t clip_u8(int v) {
  return uint8_t(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// One pixel: writes b,g,r.
__host__ __device__ inline void yuv_to_bgr(int y, int u, int v, uint8_t* b, uint8_t* g,
                                           uint8_t* r) {
  int c = (y - 16) * kCy + 32768;
  int d = u - 128, e = v - 128;
  *r = clip_u8((c + kCrv * e) >> 16);
  *g = clip_u8((c - kCgu * d - kCgv * e) >> 16);
  *b = clip_u8((c + kCbu * d) >> 16);
}

}  // namespace vep
