// Internals shared by the H.264 slice layer (avc.cpp) and the generic macroblock layer
// (avc_mb.cpp). Not part of the decoder's interface.
#pragma once

#include "avc.h"

namespace vep::avc {

// Everything the macroblock layer of one slice needs from the slice / picture level.
struct SliceEnv {
  const SliceHdr* sh = nullptr;
  const h264::Sps* sps = nullptr;
  const h264::Pps* pps = nullptr;
  int slice = 0;                             // slice index within the picture
  const std::vector<ListEntry>* list[2] = {nullptr, nullptr};
  int cur_poc = 0;
  h264::ScalingLists scaling;                // in force for this slice (resolved)
};

// The macroblock layer of one slice (both entropy modes, I/P/B, 8x8 transform, direct and
// weighted prediction). `data`/`n` = slice RBSP after the NAL header byte, `bitpos` = first bit
// of slice_data(). Fills pic.mbs[] for the slice's MBs and nb's state.
void decode_slice_generic(MbNeighbours& nb, Picture& pic, const SliceEnv& env, const u8* data, size_t n,
                          size_t bitpos);

inline i16 sat16(int v) { return i16(v < -32768 ? -32768 : v > 32767 ? 32767 : v); }

// 4x4 Hadamard, in place: f = H c H (Intra16x16 DC, §8.5.10).
inline void hadamard4x4(int c[16]) {
  int t[16];
  for (int i = 0; i < 4; ++i) {
    const int a = c[i * 4], b = c[i * 4 + 1], d = c[i * 4 + 2], e = c[i * 4 + 3];
    t[i * 4] = a + b + d + e;
    t[i * 4 + 1] = a + b - d - e;
    t[i * 4 + 2] = a - b - d + e;
    t[i * 4 + 3] = a - b + d - e;
  }
  for (int j = 0; j < 4; ++j) {
    const int a = t[j], b = t[4 + j], d = t[8 + j], e = t[12 + j];
    c[j] = a + b + d + e;
    c[4 + j] = a + b - d - e;
    c[8 + j] = a - b - d + e;
    c[12 + j] = a - b + d - e;
  }
}

}  // namespace vep::avc
