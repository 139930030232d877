// Internals shared by the H.264 slice layer (avc.cpp) and the generic macroblock layer
// (avc_mb.cpp). Not part of the decoder's interface.
#pragma once

#include <array>

#include "avc.h"
#include "bits.h"

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
  bool field = false;                        // field picture: field scan of the 4x4 levels
};

// The macroblock layer of one slice (both entropy modes, I/P/B, 8x8 transform, direct and
// weighted prediction). `data`/`n` = slice RBSP after the NAL header byte, `bitpos` = first bit
// of slice_data(). Fills pic.mbs[] for the slice's MBs and nb's state.
void decode_slice_generic(MbNeighbours& nb, Picture& pic, const SliceEnv& env, const u8* data, size_t n,
                          size_t bitpos);

// Weighted-prediction entry of an 8x8 partition with reference indices (r0, r1) (-1 = unused):
// explicit (slice header tables) or implicit (POC distances) per the slice's PPS.
WpEntry wp_entry(const SliceEnv& env, int r0, int r1);

// Motion of a decoded reference picture kept for direct prediction (per 4x4: list-0 motion if
// used, else list-1; `slice_uids[slice][list][refIdx]` = the referenced picture's uid).
// `corners`: direct_8x8_inference is on, keep only each 8x8's outer corner block.
std::shared_ptr<ColMotion> build_col_motion(const MbNeighbours& nb, int wmbs, int hmbs,
                                            const std::vector<std::array<std::vector<u32>, 2>>& slice_uids,
                                            bool corners, Recycler<ColMotion>* pool = nullptr);

// Inter prediction of one MB (list-0 / list-1 + weights), exactly the reconstruction's: py 16x16
// luma, pc 2 x 8x8 chroma. mv0 / mv1: 16 (x, y) per list (mv1 may be null).
// structure: Picture::structure (field pictures: slots are fields, slot parity = field parity).
void predict_inter(const std::vector<HostSurface>& slots, const MbRec& m, const i16* mv0, const i16* mv1,
                   const WpEntry* wp, int mx, int my, int* py, int (*pc)[128], int structure = 0);

// Encoder side of the generic macroblock layer: the decisions of one macroblock. The layer turns
// them into syntax (predicted intra modes -> prev/rem flags, motion -> mvd against the same
// predictors the decoder uses, levels -> residual blocks, context selection from the same
// neighbour state) and records the MB exactly as the decoder will (MbState, MbRec, coefficient
// pool), so the encoder's closed loop is the decoder's own reconstruction.
struct MbDesc {
  bool skip = false;     // P_Skip / B_Skip
  int mb_type = 0;       // raw: I 0..25; P 0..3 (P_8x8 = 3) or 5 + I type; B 0..22 or 23 + I type
  int sub[4] = {0, 0, 0, 0};
  bool t8x8 = false;
  u8 ipred[16] = {};     // Intra4x4PredMode per raster 4x4 block / Intra8x8PredMode per 8x8 ([0..3])
  int chroma_mode = 0;
  int ref[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};  // refIdx per partition (16x16: [0]; 16x8 / 8x16:
                                                  // [0..1]; 8x8: per 8x8)
  i16 mv[2][16][2] = {};  // motion per raster 4x4 block (each partition uniform)
  int cbp = 0;            // luma | chroma << 4 (I_16x16: implied by mb_type)
  int qp_delta = 0;
  // levels in scan order
  int dc[16] = {};          // Intra16x16 DC
  int ac[16][16] = {};      // per raster 4x4 block; Intra16x16 AC in [0..14] (scan 1..15)
  int l8[4][64] = {};       // 8x8 transform blocks
  int cdc[2][8] = {};       // chroma DC (4:2:2: 8 per component, parsing order)
  int cac[2][8][15] = {};   // chroma AC per raster block (4:2:2: 8 per component), scan 1..15
  const u8* pcm = nullptr;  // I_PCM samples (384 bytes; 4:2:2 512; above 8 bits u16 samples)
};

// Writes the macroblocks of one slice (slice header already in `bw`).
class SliceWriter {
 public:
  SliceWriter(MbNeighbours& nb, Picture& pic, const SliceEnv& env, BitWriter& bw);
  ~SliceWriter();
  void write_mb(int mb, const MbDesc& d);
  // end_of_slice / pending mb_skip_run, then the RBSP trailing bits
  void finish();
  // Motion a P_Skip / B_Skip macroblock at `mb` would get (call before write_mb of that MB):
  // fills refIdx / mv of both lists in `out` as the decoder derives them.
  void skip_motion(int mb, MbState& out);
  int qp() const;

 private:
  struct Impl;
  std::unique_ptr<Impl> p_;
};

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
