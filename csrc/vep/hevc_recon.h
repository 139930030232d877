// HEVC reconstruction primitives (hevc_recon.cpp), exposed for the CTU layer, the encoder and
// the spec oracle tests.
#pragma once

#include "codec.h"

namespace vep::hevc {

// Inverse transform of one n x n block (n = 1 << log2) of scaled coefficients d (raster) into
// residual samples r (§8.6.4): DCT, 4x4 DST (intra luma) or transform skip.
// bd: the component's bit depth (bdShift of the second stage = 20 - bd).
void inverse_transform(const i32* d, int log2, bool dst, bool tskip, i32* r, int bd = 8);
// Scaling of one coefficient level (§8.6.3, flat scaling: m = 16); qp = Qp' (QpBdOffset added).
int dequant_level(int level, int qp, int log2, int m = 16, int bd = 8);  // m: ScalingFactor (16 = flat)
// Intra sample prediction (§8.4.4.2.4-6) of an n x n block from the (substituted, filtered)
// references: top[x + 1] = p[x][-1] for x = -1 .. 2n-1, left[y] = p[-1][y] for y = 0 .. 2n-1.
void intra_predict(const int* top, const int* left, int log2, int mode, bool luma, u16* out, int stride,
                   bool filter_edges = true, int bd = 8);
// Reference sample filtering (§8.4.4.2.3) of the luma references, in place.
void filter_intra_refs(int* top, int* left, int log2, int mode, bool strong_enabled, int bd = 8);
// 14-bit intermediate inter prediction samples (§8.5.3.3.3) from a reference surface.
int luma_inter_sample(const HostSurface& r, int xi, int yi, int fx, int fy);
int chroma_inter_sample(const HostSurface& r, int c, int xi, int yi, int fx, int fy);

}  // namespace vep::hevc
