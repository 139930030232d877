// H.264 reconstruction primitives shared by the CPU reference decoder, the synthetic encoder's
// closed loop and the gfx950 reconstruction kernels (gpu_avc.hip): dequantisation tables, the
// 4x4 inverse transform, intra prediction, quarter-sample motion compensation and the in-loop
// deblocking filter (ITU-T H.264 §8.3, §8.4.2.2, §8.5, §8.7).
//
// Everything here is plain integer arithmetic with no state, compiled for both host and device,
// so the GPU path is bit-exact with the CPU path by construction; the numerics tests still
// compare the two on real bitstreams.
//
// Reference parity: replaces libavcodec's h264 reconstruction behind PyAV `packet.decode()`
// (python/read_image.py:87; SURVEY.md §2.2 N2, §2.3 K1 idct4x4_dequant / intra_pred /
// inter_mc_qpel / deblock_edge).
#pragma once

#include "common.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define VEP_HD __host__ __device__ inline
#else
#define VEP_HD inline
#endif
// Lookup tables live in constant memory in the device pass and in ordinary host memory in the
// host pass (a __constant__ object's host shadow is not initialised).
#if defined(__HIP_DEVICE_COMPILE__)
#define VEP_CONST __constant__
#else
#define VEP_CONST
#endif

namespace vep::avc {

using i16 = int16_t;
using i8 = int8_t;

// ------------------------------------------------------------------------------ MB records
// One macroblock of a parsed picture, as shipped to the GPU (56 bytes).
enum MbKind : u8 { kSkip = 0, kInter = 1, kI4x4 = 2, kI16x16 = 3, kIPcm = 4, kI8x8 = 5 };
VEP_HD bool is_intra(u8 k) { return k >= kI4x4; }
// intra MBs reconstructed by the wavefront (prediction from reconstructed neighbours)
VEP_HD bool is_wave_intra(u8 k) { return k == kI4x4 || k == kI16x16 || k == kI8x8; }

// MbRec::flags
constexpr u8 kMbT8x8 = 1;  // luma residual in 8x8 transform blocks (4 pool blocks each: 64
                           // coefficients, raster 8x8); deblocking skips internal 4x4 edges
constexpr u8 kMbL1 = 2;    // list-1 motion present: its vectors follow the list-0 ones
constexpr u8 kMbWp = 4;    // weighted prediction: MbRec::wp names 4 WpEntry (one per 8x8)
// Motion granularity in the mv pool (neither: 16 vectors per list, raster 4x4). Skip / direct /
// 16x16 macroblocks are uniform per 8x8 or per MB, so a B picture's pool shrinks ~8x (host
// memory traffic and the per-tick upload).
constexpr u8 kMbMv8x8 = 8;   // 4 vectors per list (raster 8x8)
constexpr u8 kMbMv16 = 16;   // 1 vector per list

struct MbRec {
  u8 kind;          // MbKind
  u8 qp;            // QP_Y (0 for I_PCM)
  u8 qpc;           // QP_C of Cb (chroma_qp_index_offset applied)
  u8 qpc2;          // QP_C of Cr (second_chroma_qp_index_offset applied)
  u8 i16_mode;      // Intra16x16PredMode
  u8 chroma_mode;   // intra_chroma_pred_mode
  u8 dbk;           // deblocking: bit0 filter disabled (idc 1), bit1 slice-edge mode (idc 2)
  u8 flags;         // kMbT8x8 | kMbL1 | kMbWp | kMbMv8x8 | kMbMv16
  u16 nz;           // luma 4x4 blocks (raster) with non-zero coefficients (deblocking bS 2; for
                    // 8x8-transform MBs all four blocks of a coded 8x8)
  u16 luma_coded;   // luma 4x4 blocks (raster) with residual samples to add (8x8 transform: all
                    // four blocks of a coded 8x8 set)
  i8 alpha_off;     // FilterOffsetA
  i8 beta_off;      // FilterOffsetB
  u16 slice;        // slice index within the picture (neighbour availability); bytes 14..15
  u16 chroma_coded;  // chroma 4x4 blocks (raster per component) with residual: 4:2:0 bits 0-3 Cb,
                     // 4-7 Cr; 4:2:2 (8 blocks per component, 2 wide x 4 tall) bits 0-7 Cb, 8-15 Cr
  u16 pad1;
  u8 ref[4];        // per 8x8 (raster): DPB slot of the list-0 reference picture (0xFF = none)
  u8 ref1[4];       // per 8x8: DPB slot of the list-1 reference picture (0xFF = none)
  u32 coef;         // first 16-coefficient block in the picture's coefficient pool (I_PCM:
                    // 384 raw sample bytes = 12 blocks)
  u32 mv;           // i16 offset of the MB's motion vectors in the mv pool: (x, y) per vector,
                    // list 0 then (kMbL1) list 1; see mv_sub()
  u8 i4[8];         // Intra4x4PredMode per raster 4x4 block / Intra8x8PredMode per raster 8x8
                    // block (nibbles 0..3), 4 bits each (low nibble first)
  u32 res;          // intra MBs with residual: slot of their 384 residual samples (GPU scratch,
                    // filled by the parallel pass); kNoRes otherwise
  u32 wp;           // kMbWp: first of 4 WpEntry in the picture's weight pool
  u32 pad2;
};
static_assert(sizeof(MbRec) == 56, "MbRec layout");
constexpr u32 kNoRes = 0xFFFFFFFFu;

// i16 entries per list of an MB's motion (2, 8 or 32).
VEP_HD int mv_per_list(u8 flags) { return (flags & kMbMv16) ? 2 : ((flags & kMbMv8x8) ? 8 : 32); }
// Offset (i16 units, from the MB's pool base) of the (x, y) vector of raster 4x4 block `blk` in
// list `list`.
// Byte i of a 4-byte array (MbRec::ref / ref1) as one word and a shift: an index into the
// array itself, when it varies per GPU lane, puts the whole record in scratch memory.
VEP_HD int byte_at(const u8* a, int i) {
  u32 w;
  __builtin_memcpy(&w, a, 4);
  return int((w >> (8 * i)) & 0xFFu);
}

VEP_HD int mv_sub(u8 flags, int list, int blk) {
  const int k = (flags & kMbMv16) ? 0 : ((flags & kMbMv8x8) ? 2 * (((blk >> 3) << 1) | ((blk & 3) >> 1)) : 2 * blk);
  return list * mv_per_list(flags) + k;
}

// Weighted sample prediction of one 8x8 partition (§8.4.2.3), per component (Y, Cb, Cr):
// explicit (pred_weight_table) or implicit (POC distances) weights resolved on the host.
struct WpEntry {
  i16 w0[3], w1[3];  // list-0 / list-1 weights
  i16 o[3];          // single-list: that list's offset; bi-prediction: (o0 + o1 + 1) >> 1
  u8 lwd[3];         // logWD
  u8 pad[11];
};
static_assert(sizeof(WpEntry) == 32, "WpEntry layout");

// Final prediction sample from the list-0 / list-1 predictions (§8.4.2.3.1 default, §8.4.2.3.2
// weighted); c = component.
// bd: sample bit depth (High 10: the offsets in WpEntry are already scaled by 1 << (bd - 8)).
VEP_HD int wp_sample(int p0, int p1, bool has0, bool has1, const WpEntry* w, int c, int bd = 8) {
  if (!w) return has0 && has1 ? (p0 + p1 + 1) >> 1 : (has0 ? p0 : p1);
  const int lwd = w->lwd[c], mx = (1 << bd) - 1;
  if (has0 && has1) {
    const int v = ((p0 * w->w0[c] + p1 * w->w1[c] + (1 << lwd)) >> (lwd + 1)) + w->o[c];
    return v < 0 ? 0 : (v > mx ? mx : v);
  }
  const int p = has0 ? p0 : p1, ww = has0 ? w->w0[c] : w->w1[c];
  const int v = lwd >= 1 ? ((p * ww + (1 << (lwd - 1))) >> lwd) + w->o[c] : p * ww + w->o[c];
  return v < 0 ? 0 : (v > mx ? mx : v);
}

// ---- sparse coefficient records
// An MB's dequantised coefficients in the picture's pool, from i16 offset MbRec::coef:
//   * one mask word (u16) per coded 16-coefficient group: bit i set = coefficient i of the group
//     (raster order) is non-zero. Groups, in order: the coded luma 4x4 blocks (raster order of
//     luma_coded's bits) or, for 8x8-transform MBs, the coded 8x8 blocks in raster order with
//     four words each (raster positions 16w .. 16w + 15 of the 8x8); then the coded chroma 4x4
//     blocks (order of chroma_coded's bits, Cb then Cr). Either way the word count is
//     popcount(luma_coded) + popcount(chroma_coded).
//   * then the non-zero values, group by group, ascending bit order.
// 93% of the dense blocks' entries are zero on the camera streams (89% on IDR pictures): this is
// 5-7x fewer bytes for the parse to write and the GPU to pull over PCIe.
// Dense layout (kDenseCoefs entries): luma 4x4 block r at 16 r, or 8x8 block q at 64 q (raster
// 8x8); chroma block k (bit k of chroma_coded: 4:2:0 0-3 Cb, 4-7 Cr; 4:2:2 0-7 Cb, 8-15 Cr) at
// 256 + 16 k.
// I_PCM: the 384 (4:2:2: 512) samples from i16 offset MbRec::coef (bytes, or u16 above 8 bits).
constexpr int kDenseCoefs = 512;
VEP_HD int coef_words(const MbRec& m) {
  return __builtin_popcount(u32(m.luma_coded)) + __builtin_popcount(u32(m.chroma_coded));
}
// Dense offset of mask word j (j < coef_words(m)).
VEP_HD int coef_word_base(const MbRec& m, int j) {
  const u32 lc = m.luma_coded;
  const int nl = __builtin_popcount(lc);
  if (j >= nl) {  // chroma: the (j - nl)-th coded block
    u32 cc = m.chroma_coded;
    for (int k = j - nl; k > 0; --k) cc &= cc - 1;
    return 256 + 16 * __builtin_ctz(cc);
  }
  if (m.flags & kMbT8x8) {  // the (j / 4)-th coded 8x8 block, word j % 4
    const u32 qm = (lc & 1u) | ((lc >> 1) & 2u) | ((lc >> 6) & 4u) | ((lc >> 7) & 8u);
    u32 q = qm;
    for (int k = j >> 2; k > 0; --k) q &= q - 1;
    return 64 * __builtin_ctz(q) + 16 * (j & 3);
  }
  u32 w = lc;
  for (int k = j; k > 0; --k) w &= w - 1;
  return 16 * __builtin_ctz(w);
}
// The MB's coefficients into dense[kDenseCoefs] (CPU reconstruction; the GPU expands in parallel).
inline void expand_coefs(const i16* pool, const MbRec& m, i16* dense) {
  for (int i = 0; i < kDenseCoefs; ++i) dense[i] = 0;
  const int nw = coef_words(m);
  const i16* v = pool + m.coef + nw;
  for (int j = 0; j < nw; ++j) {
    const u32 mask = u16(pool[m.coef + j]);
    i16* d = dense + coef_word_base(m, j);
    for (u32 b = mask; b; b &= b - 1) d[__builtin_ctz(b)] = *v++;
  }
}
// Number of values the MB's mask words announce (validation).
inline u32 coef_values(const i16* pool, const MbRec& m) {
  u32 n = 0;
  for (int j = 0, nw = coef_words(m); j < nw; ++j) n += u32(__builtin_popcount(u32(u16(pool[m.coef + j]))));
  return n;
}

VEP_HD int i4_mode(const MbRec& m, int blk) { return (m.i4[blk >> 1] >> ((blk & 1) * 4)) & 15; }

// Coding order of the 4x4 luma blocks (luma4x4BlkIdx) <-> raster position within the MB.
VEP_HD int blk_to_raster(int idx) {
  return ((idx >> 3) << 3) | (((idx >> 1) & 1) << 2) | (((idx >> 2) & 1) << 1) | (idx & 1);
}
VEP_HD int raster_to_blk(int r) {  // r = by*4 + bx
  const int bx = r & 3, by = r >> 2;
  return ((by >> 1) << 3) | ((bx >> 1) << 2) | ((by & 1) << 1) | (bx & 1);
}

// ------------------------------------------------------------------------------ tables
// normAdjust4x4 (§8.5.9): v[m][0] even/even positions, [1] odd/odd, [2] mixed.
VEP_CONST static const u8 kNormAdjust[6][3] = {
    {10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};

VEP_HD int norm_adjust(int m, int i, int j) {
  const int cls = ((i & 1) == 0 && (j & 1) == 0) ? 0 : ((i & 1) && (j & 1)) ? 1 : 2;
  return kNormAdjust[m][cls];
}

// QP_C as a function of qPI (Table 8-15), qPI in [0, 51].
VEP_CONST static const u8 kChromaQp[52] = {
    0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
    18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 32, 33,
    34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};

VEP_HD int chroma_qp(int qpy, int offset) {
  int q = qpy + offset;
  q = q < 0 ? 0 : q > 51 ? 51 : q;
  return kChromaQp[q];
}
// High bit depth (§8.5.8): qPI = Clip3(-QpBdOffsetC, 51, QPY + offset); QPC = qPI below 30 (so
// it may be negative), the table above it. (QP'C = QPC + QpBdOffsetC is the dequantisation QP.)
VEP_HD int chroma_qp_bd(int qpy, int offset, int qpbd_c) {
  int q = qpy + offset;
  q = q < -qpbd_c ? -qpbd_c : q > 51 ? 51 : q;
  return q < 0 ? q : kChromaQp[q];
}

// Zig-zag scan (frame macroblocks): scan index -> raster position in the 4x4 block.
VEP_CONST static const u8 kZigzag4x4[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
// Field scan (field pictures, Table 8-13): mostly vertical, the field's rows being twice as far
// apart as the frame's. (Scaling lists keep the zig-zag order in either case.)
VEP_CONST static const u8 kFieldScan4x4[16] = {0, 4, 1, 8, 12, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15};

// Deblocking thresholds (Table 8-16 / 8-17), indexed by indexA / indexB.
VEP_CONST static const u8 kAlpha[52] = {
    0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,   0,   0,   0,   0,   4,   4,
    5,  6,  7,  8,  9,  10, 12, 13, 15, 17, 20, 22,  25,  28,  32,  36,  40,  45,
    50, 56, 63, 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
VEP_CONST static const u8 kBeta[52] = {
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  2,  2,  2,  3,  3,  3,  3,  4,  4,  4,
    6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18};
VEP_CONST static const u8 kTc0[52][3] = {
    {0, 0, 0},   {0, 0, 0},   {0, 0, 0},   {0, 0, 0},   {0, 0, 0},    {0, 0, 0},    {0, 0, 0},
    {0, 0, 0},   {0, 0, 0},   {0, 0, 0},   {0, 0, 0},   {0, 0, 0},    {0, 0, 0},    {0, 0, 0},
    {0, 0, 0},   {0, 0, 0},   {0, 0, 0},   {0, 0, 1},   {0, 0, 1},    {0, 0, 1},    {0, 0, 1},
    {0, 1, 1},   {0, 1, 1},   {1, 1, 1},   {1, 1, 1},   {1, 1, 1},    {1, 1, 1},    {1, 1, 2},
    {1, 1, 2},   {1, 1, 2},   {1, 1, 2},   {1, 2, 3},   {1, 2, 3},    {2, 2, 3},    {2, 2, 4},
    {2, 3, 4},   {2, 3, 4},   {3, 3, 5},   {3, 4, 6},   {3, 4, 6},    {4, 5, 7},    {4, 5, 8},
    {4, 6, 9},   {5, 7, 10},  {6, 8, 11},  {6, 8, 13},  {7, 10, 14},  {8, 11, 16},  {9, 12, 18},
    {10, 13, 20}, {11, 15, 23}, {13, 17, 25}};

// ------------------------------------------------------------------------------ helpers
VEP_HD int clip1(int x, int bd = 8) { return x < 0 ? 0 : (x > (1 << bd) - 1 ? (1 << bd) - 1 : x); }
VEP_HD int clip3(int lo, int hi, int x) { return x < lo ? lo : (x > hi ? hi : x); }
VEP_HD int iabs(int x) { return x < 0 ? -x : x; }
VEP_HD int imin(int a, int b) { return a < b ? a : b; }
VEP_HD int imax(int a, int b) { return a > b ? a : b; }

// ------------------------------------------------------------------------------ transform
// Scale one parsed 4x4 coefficient level at raster position (i = row, j = column) (§8.5.12.1,
// flat weight matrices: LevelScale4x4 = 16 * normAdjust4x4).
VEP_HD int dequant4x4(int c, int qp, int i, int j) {
  const int ls = 16 * norm_adjust(qp % 6, i, j);
  if (qp >= 24) return c * ls * (1 << (qp / 6 - 4));
  return (c * ls + (1 << (3 - qp / 6))) >> (4 - qp / 6);
}

// Inverse 4x4 transform (§8.5.12.2) of one block, d row-major (d[i*4+j]); r receives the
// residual samples (h + 32) >> 6.
VEP_HD void idct4x4(const i16* d, int* r) {
  int f[16];
  for (int i = 0; i < 4; ++i) {
    const int d0 = d[i * 4], d1 = d[i * 4 + 1], d2 = d[i * 4 + 2], d3 = d[i * 4 + 3];
    const int e0 = d0 + d2, e1 = d0 - d2, e2 = (d1 >> 1) - d3, e3 = d1 + (d3 >> 1);
    f[i * 4] = e0 + e3;
    f[i * 4 + 1] = e1 + e2;
    f[i * 4 + 2] = e1 - e2;
    f[i * 4 + 3] = e0 - e3;
  }
  for (int j = 0; j < 4; ++j) {
    const int f0 = f[j], f1 = f[4 + j], f2 = f[8 + j], f3 = f[12 + j];
    const int g0 = f0 + f2, g1 = f0 - f2, g2 = (f1 >> 1) - f3, g3 = f1 + (f3 >> 1);
    r[j] = (g0 + g3 + 32) >> 6;
    r[4 + j] = (g1 + g2 + 32) >> 6;
    r[8 + j] = (g1 - g2 + 32) >> 6;
    r[12 + j] = (g0 - g3 + 32) >> 6;
  }
}

// One residual sample (row i, column j) of the same transform: identical integer operations,
// one output per GPU lane.
VEP_HD int idct4x4_at(const i16* d, int i, int j) {
  int f[4];
  for (int k = 0; k < 4; ++k) {
    const int d0 = d[k * 4], d1 = d[k * 4 + 1], d2 = d[k * 4 + 2], d3 = d[k * 4 + 3];
    const int e0 = d0 + d2, e1 = d0 - d2, e2 = (d1 >> 1) - d3, e3 = d1 + (d3 >> 1);
    f[k] = j == 0 ? e0 + e3 : j == 1 ? e1 + e2 : j == 2 ? e1 - e2 : e0 - e3;
  }
  const int g0 = f[0] + f[2], g1 = f[0] - f[2], g2 = (f[1] >> 1) - f[3], g3 = f[1] + (f[3] >> 1);
  const int h = i == 0 ? g0 + g3 : i == 1 ? g1 + g2 : i == 2 ? g1 - g2 : g0 - g3;
  return (h + 32) >> 6;
}

// 8x8 zig-zag scan (frame macroblocks): scan index -> raster position (row * 8 + column).
VEP_CONST static const u8 kZigzag8x8[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// 8x8 field scan (field pictures, Table 8-13): down the first columns first. Written from the
// standard's table; no source in this image holds it to check against (the closed loop pins
// encoder / decoder agreement only): parity unpinned.
VEP_CONST static const u8 kFieldScan8x8[64] = {
    0,  8,  16, 1,  9,  24, 32, 17, 2,  25, 40, 48, 56, 33, 10, 3,  18, 41, 49, 57, 26, 11,
    4,  19, 34, 42, 50, 58, 27, 12, 5,  20, 35, 43, 51, 59, 28, 13, 6,  21, 36, 44, 52, 60,
    29, 14, 22, 37, 45, 53, 61, 30, 7,  15, 38, 46, 54, 62, 23, 31, 39, 47, 55, 63};

// normAdjust8x8 (§8.5.13.1): v[m][class] with the six position classes below.
VEP_CONST static const u8 kNormAdjust8[6][6] = {{20, 18, 32, 19, 25, 24}, {22, 19, 35, 21, 28, 26},
                                                {26, 23, 42, 24, 33, 31}, {28, 25, 45, 26, 35, 33},
                                                {32, 28, 51, 30, 40, 38}, {36, 32, 58, 34, 46, 43}};
VEP_HD int norm_adjust8(int m, int i, int j) {
  int cls;
  if ((i & 3) == 0 && (j & 3) == 0) cls = 0;
  else if ((i & 1) && (j & 1)) cls = 1;
  else if ((i & 3) == 2 && (j & 3) == 2) cls = 2;
  else if (((i & 3) == 0 && (j & 1)) || ((i & 1) && (j & 3) == 0)) cls = 3;
  else if (((i & 3) == 0 && (j & 3) == 2) || ((i & 3) == 2 && (j & 3) == 0)) cls = 4;
  else cls = 5;
  return kNormAdjust8[m][cls];
}

// One 8-point inverse transform butterfly (§8.5.13.2), in place on x[0..7].
VEP_HD void idct8_1d(int* x) {
  const int a0 = x[0] + x[4], a4 = x[0] - x[4];
  const int a2 = (x[2] >> 1) - x[6], a6 = x[2] + (x[6] >> 1);
  const int b0 = a0 + a6, b2 = a4 + a2, b4 = a4 - a2, b6 = a0 - a6;
  const int a1 = -x[3] + x[5] - x[7] - (x[7] >> 1);
  const int a3 = x[1] + x[7] - x[3] - (x[3] >> 1);
  const int a5 = -x[1] + x[7] + x[5] + (x[5] >> 1);
  const int a7 = x[3] + x[5] + x[1] + (x[1] >> 1);
  const int b1 = a1 + (a7 >> 2), b7 = a7 - (a1 >> 2), b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5;
  x[0] = b0 + b7;
  x[1] = b2 + b5;
  x[2] = b4 + b3;
  x[3] = b6 + b1;
  x[4] = b6 - b1;
  x[5] = b4 - b3;
  x[6] = b2 - b5;
  x[7] = b0 - b7;
}

// Inverse 8x8 transform of one block (d raster 8x8); r receives (h + 32) >> 6.
VEP_HD void idct8x8(const i16* d, int* r) {
  int t[64];
  for (int i = 0; i < 8; ++i) {
    int x[8];
    for (int k = 0; k < 8; ++k) x[k] = d[i * 8 + k];
    idct8_1d(x);
    for (int k = 0; k < 8; ++k) t[i * 8 + k] = x[k];
  }
  for (int j = 0; j < 8; ++j) {
    int x[8];
    for (int k = 0; k < 8; ++k) x[k] = t[k * 8 + j];
    idct8_1d(x);
    for (int k = 0; k < 8; ++k) r[k * 8 + j] = (x[k] + 32) >> 6;
  }
}

// ------------------------------------------------------------------------------ intra 8x8
// Reference sample filtering (§8.3.2.2.1). Inputs (after the top-right substitution of
// §8.3.2.2): T(x) = p[x, -1] for x in -1..15, L(y) = p[-1, y] for y in 0..7. Output
// f[0] = p'[-1,-1], f[1 + x] = p'[x,-1] (x 0..15), f[17 + y] = p'[-1,y] (y 0..7).
// One filtered reference sample: k = 0 -> p'[-1,-1], 1..16 -> p'[k-1,-1], 17..24 -> p'[-1,k-17]
// (128 where the side is unavailable; such samples are never used by a prediction mode).
template <class TF, class LF>
VEP_HD int intra8x8_filter_at(TF T, LF L, bool has_top, bool has_left, bool has_tl, int k) {
  if (k == 0) {
    if (!has_tl) return 128;
    if (has_top && has_left) return (T(0) + 2 * T(-1) + L(0) + 2) >> 2;
    if (has_top) return (3 * T(-1) + T(0) + 2) >> 2;
    if (has_left) return (3 * T(-1) + L(0) + 2) >> 2;
    return T(-1);
  }
  if (k <= 16) {
    if (!has_top) return 128;
    const int x = k - 1;
    if (x == 0) return has_tl ? (T(-1) + 2 * T(0) + T(1) + 2) >> 2 : (3 * T(0) + T(1) + 2) >> 2;
    if (x == 15) return (T(14) + 3 * T(15) + 2) >> 2;
    return (T(x - 1) + 2 * T(x) + T(x + 1) + 2) >> 2;
  }
  if (!has_left) return 128;
  const int y = k - 17;
  if (y == 0) return has_tl ? (T(-1) + 2 * L(0) + L(1) + 2) >> 2 : (3 * L(0) + L(1) + 2) >> 2;
  if (y == 7) return (L(6) + 3 * L(7) + 2) >> 2;
  return (L(y - 1) + 2 * L(y) + L(y + 1) + 2) >> 2;
}

// Reference sample filtering (§8.3.2.2.1). Inputs (after the top-right substitution of
// §8.3.2.2): T(x) = p[x, -1] for x in -1..15, L(y) = p[-1, y] for y in 0..7. Output
// f[0] = p'[-1,-1], f[1 + x] = p'[x,-1] (x 0..15), f[17 + y] = p'[-1,y] (y 0..7).
template <class TF, class LF>
VEP_HD void intra8x8_filter(TF T, LF L, bool has_top, bool has_left, bool has_tl, int* f) {
  for (int k = 0; k < 25; ++k) f[k] = intra8x8_filter_at(T, L, has_top, has_left, has_tl, k);
}

// Intra_8x8 sample prediction (§8.3.2.2.2 - 8.3.2.2.10) from the filtered references.
// Generic: T(x) = p'[x,-1] for x in -1..15, L(y) = p'[-1,y] for y in -1..7 (L(-1) = T(-1)).
template <class TF, class LF>
VEP_HD int intra8x8_pred_g(TF T, LF L, bool has_top, bool has_left, int mode, int x, int y, int bd = 8) {
  switch (mode) {
    case 0: return T(x);
    case 1: return L(y);
    case 2: {
      int s = 0;
      if (has_top && has_left) {
        for (int k = 0; k < 8; ++k) s += T(k) + L(k);
        return (s + 8) >> 4;
      }
      if (has_left) {
        for (int k = 0; k < 8; ++k) s += L(k);
        return (s + 4) >> 3;
      }
      if (has_top) {
        for (int k = 0; k < 8; ++k) s += T(k);
        return (s + 4) >> 3;
      }
      return 1 << (bd - 1);
    }
    case 3:
      if (x == 7 && y == 7) return (T(14) + 3 * T(15) + 2) >> 2;
      return (T(x + y) + 2 * T(x + y + 1) + T(x + y + 2) + 2) >> 2;
    case 4:
      if (x > y) return (T(x - y - 2) + 2 * T(x - y - 1) + T(x - y) + 2) >> 2;
      if (x < y) return (L(y - x - 2) + 2 * L(y - x - 1) + L(y - x) + 2) >> 2;
      return (T(0) + 2 * T(-1) + L(0) + 2) >> 2;
    case 5: {
      const int z = 2 * x - y;
      if (z >= 0 && (z & 1) == 0) return (T(x - (y >> 1) - 1) + T(x - (y >> 1)) + 1) >> 1;
      if (z >= 0) return (T(x - (y >> 1) - 2) + 2 * T(x - (y >> 1) - 1) + T(x - (y >> 1)) + 2) >> 2;
      if (z == -1) return (L(0) + 2 * L(-1) + T(0) + 2) >> 2;
      return (L(y - 2 * x - 1) + 2 * L(y - 2 * x - 2) + L(y - 2 * x - 3) + 2) >> 2;
    }
    case 6: {
      const int z = 2 * y - x;
      if (z >= 0 && (z & 1) == 0) return (L(y - (x >> 1) - 1) + L(y - (x >> 1)) + 1) >> 1;
      if (z >= 0) return (L(y - (x >> 1) - 2) + 2 * L(y - (x >> 1) - 1) + L(y - (x >> 1)) + 2) >> 2;
      if (z == -1) return (L(0) + 2 * L(-1) + T(0) + 2) >> 2;
      return (T(x - 2 * y - 1) + 2 * T(x - 2 * y - 2) + T(x - 2 * y - 3) + 2) >> 2;
    }
    case 7:
      if ((y & 1) == 0) return (T(x + (y >> 1)) + T(x + (y >> 1) + 1) + 1) >> 1;
      return (T(x + (y >> 1)) + 2 * T(x + (y >> 1) + 1) + T(x + (y >> 1) + 2) + 2) >> 2;
    default: {  // 8: Horizontal_Up
      const int z = x + 2 * y;
      if (z > 13) return L(7);
      if (z == 13) return (L(6) + 3 * L(7) + 2) >> 2;
      if ((z & 1) == 0) return (L(y + (x >> 1)) + L(y + (x >> 1) + 1) + 1) >> 1;
      return (L(y + (x >> 1)) + 2 * L(y + (x >> 1) + 1) + L(y + (x >> 1) + 2) + 2) >> 2;
    }
  }
}

// Intra_8x8 as taps, for the GPU's branch-free form (each lane: three loads + one multiply-add,
// no lane-divergent path per mode): a sample is (w0 * s[i0] + w1 * s[i1] + w2 * s[i2] + add) >>
// shift over 25 samples in the intra8x8_filter layout (0 = p[-1,-1], 1 + x = p[x,-1],
// 17 + y = p[-1,y]). Packed: bits 0-4 i0, 5-9 i1, 10-14 i2, 15-16 w0, 17-18 w1, 19-20 w2,
// 21-22 add, 23-24 shift; kTap8Const: the sample is 128 (side unavailable); kTap8Dc: DC mode.
constexpr u32 kTap8Const = 1u << 30, kTap8Dc = 1u << 31;
VEP_HD u32 pack_tap8(int i0, int i1, int i2, int w0, int w1, int w2, int add, int shift) {
  return u32(i0) | u32(i1) << 5 | u32(i2) << 10 | u32(w0) << 15 | u32(w1) << 17 | u32(w2) << 19 |
         u32(add) << 21 | u32(shift) << 23;
}
VEP_HD int eval_tap8(u32 t, int s0, int s1, int s2) {
  return (int((t >> 15) & 3) * s0 + int((t >> 17) & 3) * s1 + int((t >> 19) & 3) * s2 + int((t >> 21) & 3)) >>
         int((t >> 23) & 3);
}
// Prediction sample (x, y) of `mode` (intra8x8_pred_g) over the filtered references.
VEP_HD u32 intra8x8_pred_tap(int mode, int x, int y) {
  auto T = [](int i) { return 1 + i; };            // p'[i,-1], i = -1..15
  auto L = [](int j) { return j < 0 ? 0 : 17 + j; };  // p'[-1,j], j = -1..7
  auto t3 = [](int a, int b, int c) { return pack_tap8(a, b, c, 1, 2, 1, 2, 2); };
  auto t2 = [](int a, int b) { return pack_tap8(a, b, 0, 1, 1, 0, 1, 1); };
  auto cp = [](int a) { return pack_tap8(a, a, a, 1, 2, 1, 2, 2); };  // (4a + 2) >> 2 = a
  switch (mode) {
    case 0: return cp(T(x));
    case 1: return cp(L(y));
    case 2: return kTap8Dc;
    case 3:
      if (x == 7 && y == 7) return pack_tap8(T(14), T(15), 0, 1, 3, 0, 2, 2);
      return t3(T(x + y), T(x + y + 1), T(x + y + 2));
    case 4:
      if (x > y) return t3(T(x - y - 2), T(x - y - 1), T(x - y));
      if (x < y) return t3(L(y - x - 2), L(y - x - 1), L(y - x));
      return t3(T(0), T(-1), L(0));
    case 5: {
      const int z = 2 * x - y;
      if (z >= 0 && (z & 1) == 0) return t2(T(x - (y >> 1) - 1), T(x - (y >> 1)));
      if (z >= 0) return t3(T(x - (y >> 1) - 2), T(x - (y >> 1) - 1), T(x - (y >> 1)));
      if (z == -1) return t3(L(0), L(-1), T(0));
      return t3(L(y - 2 * x - 1), L(y - 2 * x - 2), L(y - 2 * x - 3));
    }
    case 6: {
      const int z = 2 * y - x;
      if (z >= 0 && (z & 1) == 0) return t2(L(y - (x >> 1) - 1), L(y - (x >> 1)));
      if (z >= 0) return t3(L(y - (x >> 1) - 2), L(y - (x >> 1) - 1), L(y - (x >> 1)));
      if (z == -1) return t3(L(0), L(-1), T(0));
      return t3(T(x - 2 * y - 1), T(x - 2 * y - 2), T(x - 2 * y - 3));
    }
    case 7:
      if ((y & 1) == 0) return t2(T(x + (y >> 1)), T(x + (y >> 1) + 1));
      return t3(T(x + (y >> 1)), T(x + (y >> 1) + 1), T(x + (y >> 1) + 2));
    default: {  // 8
      const int z = x + 2 * y;
      if (z > 13) return cp(L(7));
      if (z == 13) return pack_tap8(L(6), L(7), 0, 1, 3, 0, 2, 2);
      if ((z & 1) == 0) return t2(L(y + (x >> 1)), L(y + (x >> 1) + 1));
      return t3(L(y + (x >> 1)), L(y + (x >> 1) + 1), L(y + (x >> 1) + 2));
    }
  }
}
// Filtered reference k (intra8x8_filter_at) over the unfiltered samples in the same layout.
VEP_HD u32 intra8x8_filter_tap(bool has_top, bool has_left, bool has_tl, int k) {
  auto T = [](int i) { return 1 + i; };
  auto L = [](int j) { return 17 + j; };
  auto t3 = [](int a, int b, int c) { return pack_tap8(a, b, c, 1, 2, 1, 2, 2); };
  auto w31 = [](int a, int b) { return pack_tap8(a, b, 0, 3, 1, 0, 2, 2); };  // (3a + b + 2) >> 2
  auto w13 = [](int a, int b) { return pack_tap8(a, b, 0, 1, 3, 0, 2, 2); };  // (a + 3b + 2) >> 2
  if (k == 0) {
    if (!has_tl) return kTap8Const;
    if (has_top && has_left) return t3(T(0), T(-1), L(0));
    if (has_top) return w31(T(-1), T(0));
    if (has_left) return w31(T(-1), L(0));
    return t3(T(-1), T(-1), T(-1));
  }
  if (k <= 16) {
    if (!has_top) return kTap8Const;
    const int x = k - 1;
    if (x == 0) return has_tl ? t3(T(-1), T(0), T(1)) : w31(T(0), T(1));
    if (x == 15) return w13(T(14), T(15));
    return t3(T(x - 1), T(x), T(x + 1));
  }
  if (!has_left) return kTap8Const;
  const int y = k - 17;
  if (y == 0) return has_tl ? t3(T(-1), L(0), L(1)) : w31(L(0), L(1));
  if (y == 7) return w13(L(6), L(7));
  return t3(L(y - 1), L(y), L(y + 1));
}

VEP_HD int intra8x8_pred(const int* f, bool has_top, bool has_left, int mode, int x, int y, int bd = 8) {
  return intra8x8_pred_g([&](int xx) { return f[1 + xx]; }, [&](int yy) { return yy < 0 ? f[0] : f[17 + yy]; },
                         has_top, has_left, mode, x, y, bd);
}

// ------------------------------------------------------------------------------ intra 4x4
// Neighbour samples of a 4x4 block: t[0] = p[-1,-1], t[1..8] = p[0..7,-1], l[0..3] = p[-1,0..3].
// Unavailable top-right samples must already be substituted by p[3,-1] (§8.3.1.2).
struct Intra4Nb {
  int t[9];
  int l[4];
  bool has_top, has_left, has_tl;
};

// Generic form: T(xx) = p[xx, -1] for xx in -1..7 (top-right already substituted), L(yy) =
// p[-1, yy] for yy in -1..3. The GPU passes LDS accessors, the CPU the Intra4Nb arrays; the
// arithmetic is shared.
template <class TF, class LF>
VEP_HD int intra4x4_pred_g(TF T, LF L, bool has_top, bool has_left, int mode, int x, int y, int bd = 8) {
  switch (mode) {
    case 0: return T(x);
    case 1: return L(y);
    case 2: {
      int s = 0;
      if (has_top && has_left) {
        for (int k = 0; k < 4; ++k) s += T(k) + L(k);
        return (s + 4) >> 3;
      }
      if (has_left) {
        for (int k = 0; k < 4; ++k) s += L(k);
        return (s + 2) >> 2;
      }
      if (has_top) {
        for (int k = 0; k < 4; ++k) s += T(k);
        return (s + 2) >> 2;
      }
      return 1 << (bd - 1);
    }
    case 3:
      if (x == 3 && y == 3) return (T(6) + 3 * T(7) + 2) >> 2;
      return (T(x + y) + 2 * T(x + y + 1) + T(x + y + 2) + 2) >> 2;
    case 4:
      if (x > y) return (T(x - y - 2) + 2 * T(x - y - 1) + T(x - y) + 2) >> 2;
      if (x < y) return (L(y - x - 2) + 2 * L(y - x - 1) + L(y - x) + 2) >> 2;
      return (T(0) + 2 * T(-1) + L(0) + 2) >> 2;
    case 5: {
      const int z = 2 * x - y;
      if (z >= 0 && (z & 1) == 0) return (T(x - (y >> 1) - 1) + T(x - (y >> 1)) + 1) >> 1;
      if (z >= 0) return (T(x - (y >> 1) - 2) + 2 * T(x - (y >> 1) - 1) + T(x - (y >> 1)) + 2) >> 2;
      if (z == -1) return (L(0) + 2 * L(-1) + T(0) + 2) >> 2;
      return (L(y - 1) + 2 * L(y - 2) + L(y - 3) + 2) >> 2;
    }
    case 6: {
      const int z = 2 * y - x;
      if (z >= 0 && (z & 1) == 0) return (L(y - (x >> 1) - 1) + L(y - (x >> 1)) + 1) >> 1;
      if (z >= 0) return (L(y - (x >> 1) - 2) + 2 * L(y - (x >> 1) - 1) + L(y - (x >> 1)) + 2) >> 2;
      if (z == -1) return (L(0) + 2 * L(-1) + T(0) + 2) >> 2;
      return (T(x - 1) + 2 * T(x - 2) + T(x - 3) + 2) >> 2;
    }
    case 7:
      if ((y & 1) == 0) return (T(x + (y >> 1)) + T(x + (y >> 1) + 1) + 1) >> 1;
      return (T(x + (y >> 1)) + 2 * T(x + (y >> 1) + 1) + T(x + (y >> 1) + 2) + 2) >> 2;
    default: {  // 8: Horizontal_Up
      const int z = x + 2 * y;
      if (z > 5) return L(3);
      if (z == 5) return (L(2) + 3 * L(3) + 2) >> 2;
      if ((z & 1) == 0) return (L(y + (x >> 1)) + L(y + (x >> 1) + 1) + 1) >> 1;
      return (L(y + (x >> 1)) + 2 * L(y + (x >> 1) + 1) + L(y + (x >> 1) + 2) + 2) >> 2;
    }
  }
}

// Tap form of the non-DC Intra_4x4 predictors (same formulas as intra4x4_pred_g): the sample
// is (sum_k w[k] * N[idx[k]] + add) >> shift over the 13 neighbours
// N = {p[-1,-1], p[0..7,-1], p[-1,0..3]}. The GPU evaluates it with all LDS reads issued at
// once; tests pin it to intra4x4_pred_g for every mode and position.
struct Taps4 {
  u8 idx[3], w[3];
  u8 n, add, shift;
};
VEP_HD Taps4 intra4x4_taps(int mode, int x, int y) {
  auto T = [](int xx) { return u8(xx + 1); };
  auto L = [](int yy) { return u8(yy < 0 ? 0 : 9 + yy); };
  Taps4 t{{0, 0, 0}, {1, 2, 1}, 3, 2, 2};
  auto set3 = [&](u8 a, u8 b, u8 c) {
    t.idx[0] = a;
    t.idx[1] = b;
    t.idx[2] = c;
  };
  auto set2 = [&](u8 a, u8 b) {  // (a + b + 1) >> 1
    t.idx[0] = a;
    t.idx[1] = b;
    t.idx[2] = a;
    t.w[0] = 1;
    t.w[1] = 1;
    t.w[2] = 0;
    t.n = 2;
    t.add = 1;
    t.shift = 1;
  };
  auto set1 = [&](u8 a) {
    t.idx[0] = t.idx[1] = t.idx[2] = a;
    t.w[0] = 1;
    t.w[1] = 0;
    t.w[2] = 0;
    t.n = 1;
    t.add = 0;
    t.shift = 0;
  };
  switch (mode) {
    case 0: set1(T(x)); break;
    case 1: set1(L(y)); break;
    case 3:
      if (x == 3 && y == 3) {
        set3(T(6), T(7), T(7));
        t.w[0] = 1, t.w[1] = 3, t.w[2] = 0;
      } else {
        set3(T(x + y), T(x + y + 1), T(x + y + 2));
      }
      break;
    case 4:
      if (x > y) set3(T(x - y - 2), T(x - y - 1), T(x - y));
      else if (x < y) set3(L(y - x - 2), L(y - x - 1), L(y - x));
      else set3(T(0), T(-1), L(0));
      break;
    case 5: {
      const int z = 2 * x - y, b = x - (y >> 1);
      if (z >= 0 && (z & 1) == 0) set2(T(b - 1), T(b));
      else if (z >= 0) set3(T(b - 2), T(b - 1), T(b));
      else if (z == -1) set3(L(0), L(-1), T(0));
      else set3(L(y - 1), L(y - 2), L(y - 3));
      break;
    }
    case 6: {
      const int z = 2 * y - x, b = y - (x >> 1);
      if (z >= 0 && (z & 1) == 0) set2(L(b - 1), L(b));
      else if (z >= 0) set3(L(b - 2), L(b - 1), L(b));
      else if (z == -1) set3(L(0), L(-1), T(0));
      else set3(T(x - 1), T(x - 2), T(x - 3));
      break;
    }
    case 7: {
      const int b = x + (y >> 1);
      if ((y & 1) == 0) set2(T(b), T(b + 1));
      else set3(T(b), T(b + 1), T(b + 2));
      break;
    }
    default: {  // 8
      const int z = x + 2 * y, b = y + (x >> 1);
      if (z > 5) set1(L(3));
      else if (z == 5) {
        set3(L(2), L(3), L(3));
        t.w[0] = 1, t.w[1] = 3, t.w[2] = 0;
      } else if ((z & 1) == 0) set2(L(b), L(b + 1));
      else set3(L(b), L(b + 1), L(b + 2));
      break;
    }
  }
  return t;
}

// Packed tap word (GPU LDS): idx0..2 (4 bits each), w0..2 (2 bits), add (2), shift (2), dc (1).
constexpr u32 kTapDc = 1u << 24;
VEP_HD u32 pack_taps(const Taps4& t) {
  return u32(t.idx[0]) | u32(t.idx[1]) << 4 | u32(t.idx[2]) << 8 | u32(t.w[0]) << 12 |
         u32(t.w[1]) << 14 | u32(t.w[2]) << 16 | u32(t.add) << 18 | u32(t.shift) << 20;
}

VEP_HD int intra4x4_pred(const Intra4Nb& n, int mode, int x, int y, int bd = 8) {
  return intra4x4_pred_g([&](int xx) { return n.t[xx + 1]; },
                         [&](int yy) { return yy < 0 ? n.t[0] : n.l[yy]; }, n.has_top, n.has_left,
                         mode, x, y, bd);
}

// ------------------------------------------------------------------------------ intra 16x16
// top[0] = p[-1,-1], top[1..16] = p[0..15,-1]; left[0..15] = p[-1,0..15].
struct Intra16Nb {
  int top[17];
  int left[16];
  bool has_top, has_left, has_tl;
};

// Per-MB constants of a 16x16 / chroma prediction (DC value or plane a, b, c).
struct PredConst {
  int dc, a, b, c;
};

// Generic forms: T(x) = p[x, -1] for x in -1..15, L(y) = p[-1, y] for y in 0..15.
// Final step of the 16x16 constants from the neighbour sums (the GPU computes the sums with a
// wave reduction): st / sl = sum of the 16 top / left samples, H / V the plane gradients.
VEP_HD PredConst intra16x16_const_from_sums(int mode, bool has_top, bool has_left, int st, int sl,
                                            int H, int V, int top15, int left15, int bd = 8) {
  PredConst k{1 << (bd - 1), 0, 0, 0};
  if (mode == 2) {
    if (has_top && has_left) k.dc = (st + sl + 16) >> 5;
    else if (has_left) k.dc = (sl + 8) >> 4;
    else if (has_top) k.dc = (st + 8) >> 4;
  } else if (mode == 3) {
    k.a = 16 * (left15 + top15);
    k.b = (5 * H + 32) >> 6;
    k.c = (5 * V + 32) >> 6;
  }
  return k;
}

// Generic forms: T(x) = p[x, -1] for x in -1..15, L(y) = p[-1, y] for y in 0..15.
template <class TF, class LF>
VEP_HD PredConst intra16x16_const_g(TF T, LF L, bool has_top, bool has_left, int mode, int bd = 8) {
  int st = 0, sl = 0, H = 0, V = 0;
  for (int i = 0; i < 16; ++i) {
    st += T(i);
    sl += L(i);
  }
  for (int i = 0; i < 8; ++i) {
    H += (i + 1) * (T(8 + i) - T(6 - i));
    V += (i + 1) * (L(8 + i) - (6 - i >= 0 ? L(6 - i) : T(-1)));
  }
  return intra16x16_const_from_sums(mode, has_top, has_left, st, sl, H, V, T(15), L(15), bd);
}

template <class TF, class LF>
VEP_HD int intra16x16_pred_g(TF T, LF L, const PredConst& k, int mode, int x, int y, int bd = 8) {
  switch (mode) {
    case 0: return T(x);
    case 1: return L(y);
    case 2: return k.dc;
    default: return clip1((k.a + k.b * (x - 7) + k.c * (y - 7) + 16) >> 5, bd);
  }
}

VEP_HD PredConst intra16x16_const(const Intra16Nb& n, int mode, int bd = 8) {
  return intra16x16_const_g([&](int x) { return n.top[x + 1]; }, [&](int y) { return n.left[y]; },
                            n.has_top, n.has_left, mode, bd);
}

VEP_HD int intra16x16_pred(const Intra16Nb& n, const PredConst& k, int mode, int x, int y, int bd = 8) {
  return intra16x16_pred_g([&](int xx) { return n.top[xx + 1]; }, [&](int yy) { return n.left[yy]; },
                           k, mode, x, y, bd);
}

// Chroma (8x8 per component in 4:2:0, 8x16 in 4:2:2): top[0] = p[-1,-1], top[1..8]; left[0..7]
// (4:2:2: left[0..15]).
struct IntraChromaNb {
  int top[9];
  int left[16];
  bool has_top, has_left, has_tl;
};

// DC of chroma 4x4 block (bx, by) (§8.3.4.1-3). Generic: T(x) = p[x, -1] (x in -1..7),
// L(y) = p[-1, y] (y in 0..7).
template <class TF, class LF>
VEP_HD int chroma_dc_g(TF T, LF L, bool has_top, bool has_left, int bx, int by, int bd = 8) {
  int st = 0, sl = 0;
  for (int i = 0; i < 4; ++i) {
    st += T(bx * 4 + i);
    sl += L(by * 4 + i);
  }
  const bool corner_rule = (bx == 0 && by == 0) || (bx > 0 && by > 0);
  if (corner_rule) {
    if (has_top && has_left) return (st + sl + 4) >> 3;
    if (has_left) return (sl + 2) >> 2;
    if (has_top) return (st + 2) >> 2;
    return 1 << (bd - 1);
  }
  if (bx > 0) {  // top-right block: top first
    if (has_top) return (st + 2) >> 2;
    if (has_left) return (sl + 2) >> 2;
    return 1 << (bd - 1);
  }
  if (has_left) return (sl + 2) >> 2;  // bottom-left block: left first
  if (has_top) return (st + 2) >> 2;
  return 1 << (bd - 1);
}

// Plane prediction constants (§8.3.4.4) with xCF = 0 and yCF = 4 * (chroma_format_idc == 2): the
// 8x16 4:2:2 block sums 8 vertical gradient terms and weighs them by 5 instead of 34.
template <class TF, class LF>
VEP_HD PredConst chroma_plane_const_g(TF T, LF L, int cf = 1) {
  int H = 0, V = 0;
  for (int i = 0; i < 4; ++i) H += (i + 1) * (T(4 + i) - T(2 - i));
  if (cf == 2) {
    for (int i = 0; i < 8; ++i) V += (i + 1) * (L(8 + i) - (6 - i >= 0 ? L(6 - i) : T(-1)));
    return PredConst{0, 16 * (L(15) + T(7)), (34 * H + 32) >> 6, (5 * V + 32) >> 6};
  }
  for (int i = 0; i < 4; ++i) V += (i + 1) * (L(4 + i) - (2 - i >= 0 ? L(2 - i) : T(-1)));
  return PredConst{0, 16 * (L(7) + T(7)), (34 * H + 32) >> 6, (34 * V + 32) >> 6};
}

// mode: 0 DC, 1 horizontal, 2 vertical, 3 plane. (x, y) in the 8x8 (4:2:2: 8x16) block; the DC
// rule of 4x4 block (x >> 2, y >> 2) covers the 4:2:2 blocks below the first row as well.
template <class TF, class LF>
VEP_HD int chroma_pred_g(TF T, LF L, bool has_top, bool has_left, const PredConst& k, int mode, int x,
                         int y, int bd = 8, int cf = 1) {
  switch (mode) {
    case 0: return chroma_dc_g(T, L, has_top, has_left, x >> 2, y >> 2, bd);
    case 1: return L(y);
    case 2: return T(x);
    default: return clip1((k.a + k.b * (x - 3) + k.c * (y - (cf == 2 ? 7 : 3)) + 16) >> 5, bd);
  }
}

VEP_HD PredConst chroma_plane_const(const IntraChromaNb& n, int cf = 1) {
  return chroma_plane_const_g([&](int x) { return n.top[x + 1]; }, [&](int y) { return n.left[y]; }, cf);
}

VEP_HD int chroma_pred(const IntraChromaNb& n, const PredConst& k, int mode, int x, int y, int bd = 8, int cf = 1) {
  return chroma_pred_g([&](int xx) { return n.top[xx + 1]; }, [&](int yy) { return n.left[yy]; },
                       n.has_top, n.has_left, k, mode, x, y, bd, cf);
}

// ---- 4:2:2 chroma DC (§8.5.11): 8 levels in parsing order -> c[4][2] (chroma DC scan of 4:2:2),
// the 4x4 x 2x2 Hadamard-type transform f = A c B, then the scaling at qP,DC = QP'C + 3.
// dcv[blk] for chroma block blk (raster, 2 wide x 4 tall). ls = LevelScale4x4(qP,DC % 6, 0, 0).
// c[4][2] = [[c0, c2], [c1, c5], [c3, c6], [c4, c7]] (8-330): raster (x + 2 y) -> parsing index,
// and its inverse
VEP_CONST static const u8 kChroma422DcRasterToScan[8] = {0, 2, 1, 5, 3, 6, 4, 7};
VEP_CONST static const u8 kChroma422DcScanToRaster[8] = {0, 2, 1, 4, 6, 3, 5, 7};
VEP_HD void chroma422_dc(const int* lv_scan, int qpdc, int ls, int* dcv) {
  int c[8];
  for (int r = 0; r < 8; ++r) c[r] = lv_scan[kChroma422DcRasterToScan[r]];
  int f[8];
  for (int x = 0; x < 2; ++x) {  // A (4 x 4) on the columns
    const int c0 = c[x], c1 = c[2 + x], c2 = c[4 + x], c3 = c[6 + x];
    f[x] = c0 + c1 + c2 + c3;
    f[2 + x] = c0 + c1 - c2 - c3;
    f[4 + x] = c0 - c1 - c2 + c3;
    f[6 + x] = c0 - c1 + c2 - c3;
  }
  for (int y = 0; y < 4; ++y) {  // B (2 x 2) on the rows
    const int a = f[2 * y], b = f[2 * y + 1];
    f[2 * y] = a + b;
    f[2 * y + 1] = a - b;
  }
  for (int k = 0; k < 8; ++k)
    dcv[k] = qpdc >= 36 ? (f[k] * ls) * (1 << (qpdc / 6 - 6))
                        : (f[k] * ls + (1 << (5 - qpdc / 6))) >> (6 - qpdc / 6);
}

// Chroma vector of a luma vector (§8.4.1.4 / §8.4.2.2.2) as integer + eighth-sample fraction per
// axis: horizontally 1/8 chroma sample in both formats; vertically 1/8 in 4:2:0 and, in 4:2:2
// (full-height chroma), the quarter-sample luma position scaled to eighths.
VEP_HD void chroma_mv(int mvx, int mvy, int cf, int& ix, int& fx, int& iy, int& fy) {
  ix = mvx >> 3;
  fx = mvx & 7;
  if (cf == 2) {
    iy = mvy >> 2;
    fy = (mvy & 3) << 1;
  } else {
    iy = mvy >> 3;
    fy = mvy & 7;
  }
}

// ------------------------------------------------------------------------------ inter
// Reference sample fetch with edge clamping (§8.4.2.2.1 Clip3 on xInt/yInt).
template <class P>
VEP_HD int ref_px(const P* p, int pitch, int w, int h, int x, int y) {
  x = clip3(0, w - 1, x);
  y = clip3(0, h - 1, y);
  return p[size_t(y) * pitch + x];
}

VEP_HD int tap6(int a, int b, int c, int d, int e, int f) {
  return a - 5 * b + 20 * c + 20 * d - 5 * e + f;
}

// Luma sample prediction at integer (xi, yi) with fractional offset (fx, fy) in quarter samples
// (Table 8-12).
// (P: u8 planes, or u16 at bit depth bd: High 10)
template <class P>
VEP_HD int luma_qpel(const P* p, int pitch, int w, int h, int xi, int yi, int fx, int fy, int bd = 8) {
  auto G = [&](int dx, int dy) { return ref_px(p, pitch, w, h, xi + dx, yi + dy); };
  // unrounded half-sample intermediates
  auto b1 = [&](int dy) {  // horizontal half sample between (0,dy) and (1,dy)
    return tap6(G(-2, dy), G(-1, dy), G(0, dy), G(1, dy), G(2, dy), G(3, dy));
  };
  auto h1 = [&](int dx) {  // vertical half sample between (dx,0) and (dx,1)
    return tap6(G(dx, -2), G(dx, -1), G(dx, 0), G(dx, 1), G(dx, 2), G(dx, 3));
  };
  auto rb = [&](int v) { return clip1((v + 16) >> 5, bd); };
  if (fx == 0 && fy == 0) return G(0, 0);
  if (fy == 0) {
    const int b = rb(b1(0));
    if (fx == 2) return b;
    return (b + G(fx == 1 ? 0 : 1, 0) + 1) >> 1;  // a / c
  }
  if (fx == 0) {
    const int hh = rb(h1(0));
    if (fy == 2) return hh;
    return (hh + G(0, fy == 1 ? 0 : 1) + 1) >> 1;  // d / n
  }
  if (fx == 2 || fy == 2) {
    // j from the vertical 6-tap over horizontal intermediates
    const int j1 = tap6(b1(-2), b1(-1), b1(0), b1(1), b1(2), b1(3));
    const int j = clip1((j1 + 512) >> 10, bd);
    if (fx == 2 && fy == 2) return j;
    if (fx == 2) {  // f (fy 1) / q (fy 3): with b (row 0) or s (row 1)
      const int o = rb(b1(fy == 1 ? 0 : 1));
      return (o + j + 1) >> 1;
    }
    // i (fx 1) / k (fx 3): with h (column 0) or m (column 1)
    const int o = rb(h1(fx == 1 ? 0 : 1));
    return (o + j + 1) >> 1;
  }
  // diagonal quarter positions e, g, p, r: average of a horizontal and a vertical half sample
  const int hb = rb(b1(fy == 1 ? 0 : 1));  // b (row 0) or s (row 1)
  const int hv = rb(h1(fx == 1 ? 0 : 1));  // h (column 0) or m (column 1)
  return (hb + hv + 1) >> 1;
}

// Chroma sample prediction (§8.4.2.2.2) at integer (xi, yi) with eighth-sample (fx, fy) in one
// component of an interleaved NV12 plane (component c in {0, 1}); w, h in chroma samples.
template <class P>
VEP_HD int chroma_epel(const P* uv, int pitch, int w, int h, int c, int xi, int yi, int fx,
                       int fy) {
  auto S = [&](int x, int y) {
    x = clip3(0, w - 1, x);
    y = clip3(0, h - 1, y);
    return int(uv[size_t(y) * pitch + 2 * x + c]);
  };
  const int A = S(xi, yi), B = S(xi + 1, yi), C = S(xi, yi + 1), D = S(xi + 1, yi + 1);
  return ((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C + fx * fy * D + 32) >> 6;
}

// ------------------------------------------------------------------------------ deblocking
// Boundary strength of the edge between 4x4 luma blocks P (in MB mp, raster block bp) and Q (in
// MB mq, block bq) (§8.7.2.1, frame macroblocks). mv_p / mv_q point at the MBs' vectors in the
// mv pool (granularity by the MbRec flags, see mv_sub()); unused for intra MBs. Reference
// pictures are compared by DPB slot (= picture identity within one picture's decode), so a
// picture reached through list 0 and list 1 counts as the same picture.
// Field pictures (`field`): an intra horizontal MB edge gets bS 3, not 4, and vertical vectors
// (quarter field samples) differ "by 4 quarter frame samples" at 2.
VEP_HD bool mv_far(const i16* a, const i16* b, int ylim = 4) {
  return iabs(a[0] - b[0]) >= 4 || iabs(a[1] - b[1]) >= ylim;
}
// The fields of one MB record the bS decision reads, as scalars: the reference-slot arrays
// become words (their bytes read by a shift), so a GPU lane keeps the side in registers
// rather than taking the address of a local record.
struct BsSide {
  u32 ref, ref1;
  u16 nz;
  u8 kind, flags;
};
VEP_HD BsSide bs_side(const MbRec& m) {
  BsSide s;
  __builtin_memcpy(&s.ref, m.ref, 4);
  __builtin_memcpy(&s.ref1, m.ref1, 4);
  s.nz = m.nz;
  s.kind = m.kind;
  s.flags = m.flags;
  return s;
}
VEP_HD int word_byte(u32 w, int i) { return int((w >> (8 * i)) & 0xFFu); }

// (the non-intra part: coefficients, reference pictures, vectors)
VEP_HD int boundary_strength_mv(BsSide mp, int bp, const i16* mv_p, BsSide mq, int bq,
                                const i16* mv_q, int ylim) {
  if (((mp.nz >> bp) & 1) || ((mq.nz >> bq) & 1)) return 2;
  const int p8 = ((bp >> 3) << 1) | ((bp & 3) >> 1), q8 = ((bq >> 3) << 1) | ((bq & 3) >> 1);
  const int p0 = word_byte(mp.ref, p8), p1 = (mp.flags & kMbL1) ? word_byte(mp.ref1, p8) : 0xFF;
  const int q0 = word_byte(mq.ref, q8), q1 = (mq.flags & kMbL1) ? word_byte(mq.ref1, q8) : 0xFF;
  const int np = (p0 != 0xFF) + (p1 != 0xFF), nq = (q0 != 0xFF) + (q1 != 0xFF);
  if (np != nq) return 1;
  const i16* pa = mv_p + mv_sub(mp.flags, 0, bp);  // list 0 of P
  const i16* pb = mv_p + mv_sub(mp.flags, 1, bp);  // list 1 of P (valid when p1 used)
  const i16* qa = mv_q + mv_sub(mq.flags, 0, bq);
  const i16* qb = mv_q + mv_sub(mq.flags, 1, bq);
  if (np == 1) {
    const int rp = p0 != 0xFF ? p0 : p1, rq = q0 != 0xFF ? q0 : q1;
    if (rp != rq) return 1;
    return mv_far(p0 != 0xFF ? pa : pb, q0 != 0xFF ? qa : qb, ylim) ? 1 : 0;
  }
  if (!((p0 == q0 && p1 == q1) || (p0 == q1 && p1 == q0))) return 1;
  if (p0 != p1) {  // two different reference pictures: compare the vectors of the same picture
    if (p0 == q0) return (mv_far(pa, qa, ylim) || mv_far(pb, qb, ylim)) ? 1 : 0;
    return (mv_far(pa, qb, ylim) || mv_far(pb, qa, ylim)) ? 1 : 0;
  }
  // both vectors of both blocks reference the same picture
  return ((mv_far(pa, qa, ylim) || mv_far(pb, qb, ylim)) && (mv_far(pa, qb, ylim) || mv_far(pb, qa, ylim))) ? 1 : 0;
}

VEP_HD int boundary_strength(BsSide mp, int bp, const i16* mv_p, BsSide mq, int bq,
                             const i16* mv_q, bool mb_edge, bool field = false, bool vertical = true) {
  if (is_intra(mp.kind) || is_intra(mq.kind)) return (mb_edge && (vertical || !field)) ? 4 : 3;
  if (field) return boundary_strength_mv(mp, bp, mv_p, mq, bq, mv_q, 2);
  return boundary_strength_mv(mp, bp, mv_p, mq, bq, mv_q, 4);
}

VEP_HD int boundary_strength(const MbRec& mp, int bp, const i16* mv_p, const MbRec& mq, int bq,
                             const i16* mv_q, bool mb_edge, bool field = false, bool vertical = true) {
  return boundary_strength(bs_side(mp), bp, mv_p, bs_side(mq), bq, mv_q, mb_edge, field, vertical);
}

struct EdgeParams {
  int alpha, beta;
  int tc0[3];  // tC0 for bS 1..3 (Table 8-17), resolved once per edge, not per sample line
};

// (qp_p / qp_q: QPY of the two MBs, or their QPC for chroma edges; negative at high bit depth.
// bd > 8: alpha / beta / tC0 scaled by 1 << (bd - 8), §8.7.2.2)
VEP_HD EdgeParams edge_params(int qp_p, int qp_q, int off_a, int off_b, int bd = 8) {
  const int qav = (qp_p + qp_q + 1) >> 1;
  const int ia = clip3(0, 51, qav + off_a), ib = clip3(0, 51, qav + off_b);
  const int s = bd - 8;
  return EdgeParams{kAlpha[ia] << s, kBeta[ib] << s, {kTc0[ia][0] << s, kTc0[ia][1] << s, kTc0[ia][2] << s}};
}

// Filter one line of samples across an edge: s points at q0, `step` is the distance between
// successive samples across the edge (1 for a vertical edge, pitch for a horizontal one).
// chroma lines use the two-sample filters (§8.7.2.3 / §8.7.2.4).
// Filter one sample line in registers: p[k] = p_k, q[k] = q_k (k = 0..3; chroma uses k < 2).
// Returns false (nothing changed) when the edge is not filtered at this line. tc0 = tC0 of
// the line's bS (ignored for bS 4).
VEP_HD bool filter_samples(int* p, int* q, int bs, int alpha, int beta, int tc0, bool chroma, int bd = 8) {
  const int p0 = p[0], p1 = p[1], q0 = q[0], q1 = q[1];
  if (!(iabs(p0 - q0) < alpha && iabs(p1 - p0) < beta && iabs(q1 - q0) < beta)) return false;
  if (chroma) {
    if (bs < 4) {
      const int tc = tc0 + 1;
      const int d = clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3);
      p[0] = clip1(p0 + d, bd);
      q[0] = clip1(q0 - d, bd);
    } else {
      p[0] = (2 * p1 + p0 + q1 + 2) >> 2;
      q[0] = (2 * q1 + q0 + p1 + 2) >> 2;
    }
    return true;
  }
  const int p2 = p[2], q2 = q[2];
  const int ap = iabs(p2 - p0), aq = iabs(q2 - q0);
  if (bs < 4) {
    const int tc = tc0 + (ap < beta) + (aq < beta);
    const int d = clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3);
    p[0] = clip1(p0 + d, bd);
    q[0] = clip1(q0 - d, bd);
    if (ap < beta) p[1] = p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1);
    if (aq < beta) q[1] = q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1);
    return true;
  }
  const int p3 = p[3], q3 = q[3];
  const bool strong = iabs(p0 - q0) < ((alpha >> 2) + 2);
  if (ap < beta && strong) {
    p[0] = (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3;
    p[1] = (p2 + p1 + p0 + q0 + 2) >> 2;
    p[2] = (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3;
  } else {
    p[0] = (2 * p1 + p0 + q1 + 2) >> 2;
  }
  if (aq < beta && strong) {
    q[0] = (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3;
    q[1] = (p0 + q0 + q1 + q2 + 2) >> 2;
    q[2] = (2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3;
  } else {
    q[0] = (2 * q1 + q0 + p1 + 2) >> 2;
  }
  return true;
}

// filter_samples on samples in memory (stride `step` across the edge; s = q0).
// filter_samples with one instruction stream for luma and chroma lines (GPU lanes of both kinds in
// one wave): a chroma line is a luma line whose ap / aq tests fail (no p1 / q1 / strong update)
// and whose tC is tC0 + 1. Same results as filter_samples for every input (hbd_emu checks it).
VEP_HD bool filter_samples_u(int* p, int* q, int bs, int alpha, int beta, int tc0, bool chroma, int bd = 8) {
  const int p0 = p[0], p1 = p[1], p2 = p[2], p3 = p[3], q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
  if (!(iabs(p0 - q0) < alpha && iabs(p1 - p0) < beta && iabs(q1 - q0) < beta)) return false;
  const bool lp = !chroma && iabs(p2 - p0) < beta, lq = !chroma && iabs(q2 - q0) < beta;
  if (bs < 4) {
    const int tc = chroma ? tc0 + 1 : tc0 + int(lp) + int(lq);
    const int dl = clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3);
    p[0] = clip1(p0 + dl, bd);
    q[0] = clip1(q0 - dl, bd);
    if (lp) p[1] = p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1);
    if (lq) q[1] = q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1);
    return true;
  }
  const bool strong = iabs(p0 - q0) < ((alpha >> 2) + 2);
  if (lp && strong) {
    p[0] = (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3;
    p[1] = (p2 + p1 + p0 + q0 + 2) >> 2;
    p[2] = (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3;
  } else {
    p[0] = (2 * p1 + p0 + q1 + 2) >> 2;
  }
  if (lq && strong) {
    q[0] = (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3;
    q[1] = (p0 + q0 + q1 + q2 + 2) >> 2;
    q[2] = (2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3;
  } else {
    q[0] = (2 * q1 + q0 + p1 + 2) >> 2;
  }
  return true;
}

template <typename Px>
VEP_HD void filter_line_t(Px* s, long step, int bs, int alpha, int beta, int tc0, bool chroma, int bd = 8) {
  const int n = chroma ? 2 : 4;
  int p[4] = {0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
  for (int k = 0; k < n; ++k) {
    p[k] = s[-(k + 1) * step];
    q[k] = s[k * step];
  }
  if (!filter_samples(p, q, bs, alpha, beta, tc0, chroma, bd)) return;
  const int m = chroma ? 1 : 3;
  for (int k = 0; k < m; ++k) {
    s[-(k + 1) * step] = Px(p[k]);
    s[k * step] = Px(q[k]);
  }
}

template <typename Px>
VEP_HD void filter_line(Px* s, long step, int bs, const EdgeParams& e, bool chroma, int bd = 8) {
  filter_line_t(s, step, bs, e.alpha, e.beta, bs < 4 ? e.tc0[bs - 1] : 0, chroma, bd);
}

}  // namespace vep::avc
