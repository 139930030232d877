// Constant tables of the general H.265/HEVC decoder (ITU-T H.265 v3 (04/2015) clause numbers):
// CABAC context initialisation values (§9.3.2.2, Tables 9-5 .. 9-37) for the three
// initialisation types, scan orders (§6.5.3-5), intra angles (§8.4.4.2.6), the inverse
// transform matrix (§8.6.4.2), the interpolation filters (§8.5.3.3.3) and the deblocking
// thresholds (§8.7.2.5.3, Table 8-12).
//
// Parity note: no third-party HEVC bitstream exists in this image, so these values are
// exercised by the closed-loop encoder (which shares them) and the spec oracle tests; parity
// with another decoder is unpinned.
#pragma once

#include <cstdint>

#include "common.h"

namespace vep::hevc {

using i8 = std::int8_t;

// Tables the gfx950 kernels read live in constant memory in the device pass.
#if defined(__HIP_DEVICE_COMPILE__)
#define HK_TABLE __constant__ constexpr
#else
#define HK_TABLE inline constexpr
#endif

// ---------------------------------------------------------------------------- CABAC contexts
// Context index layout (one array per slice): every syntax element's contexts for the slice's
// initialisation type are copied to these offsets.
enum CtxOff : int {
  kCtxSaoMerge = 0,          // 1
  kCtxSaoType = 1,           // 1
  kCtxSplitCu = 2,           // 3
  kCtxTransquantBypass = 5,  // 1
  kCtxSkip = 6,              // 3
  kCtxPredMode = 9,          // 1
  kCtxPartMode = 10,         // 4
  kCtxPrevIntra = 14,        // 1
  kCtxChromaMode = 15,       // 1
  kCtxRqtRootCbf = 16,       // 1
  kCtxMergeFlag = 17,        // 1
  kCtxMergeIdx = 18,         // 1
  kCtxInterPred = 19,        // 5
  kCtxRefIdx = 24,           // 2
  kCtxMvpFlag = 26,          // 1
  kCtxSplitTransform = 27,   // 3
  kCtxCbfLuma = 30,          // 2
  kCtxCbfChroma = 32,        // 4
  kCtxMvdGt0 = 36,           // 1
  kCtxMvdGt1 = 37,           // 1
  kCtxQpDelta = 38,          // 2
  kCtxTransformSkip = 40,    // 2 (luma, chroma)
  kCtxLastX = 42,            // 18
  kCtxLastY = 60,            // 18
  kCtxCsbf = 78,             // 4
  kCtxSig = 82,              // 42 (27 luma + 15 chroma)
  kCtxGt1 = 124,             // 24 (16 luma + 8 chroma)
  kCtxGt2 = 148,             // 6 (4 luma + 2 chroma)
  kCtxCount = 154,
};

// initValue per context for initType 0 (I), 1 and 2 (P / B, swapped by cabac_init_flag).
// Elements that do not exist in I slices carry 154 (unused).
inline constexpr u8 kCtxInit[3][kCtxCount] = {
    {// initType 0
     153,                                        // sao_merge
     200,                                        // sao_type_idx
     139, 141, 157,                              // split_cu_flag
     154,                                        // cu_transquant_bypass_flag
     154, 154, 154,                              // cu_skip_flag (unused)
     154,                                        // pred_mode_flag (unused)
     184, 154, 154, 154,                         // part_mode
     184,                                        // prev_intra_luma_pred_flag
     63,                                         // intra_chroma_pred_mode
     154,                                        // rqt_root_cbf (unused)
     154,                                        // merge_flag (unused)
     154,                                        // merge_idx (unused)
     154, 154, 154, 154, 154,                    // inter_pred_idc (unused)
     154, 154,                                   // ref_idx (unused)
     154,                                        // mvp_flag (unused)
     153, 138, 138,                              // split_transform_flag
     111, 141,                                   // cbf_luma
     94, 138, 182, 154,                          // cbf_cb / cbf_cr
     154,                                        // abs_mvd_greater0 (unused)
     154,                                        // abs_mvd_greater1 (unused)
     154, 154,                                   // cu_qp_delta_abs
     139, 139,                                   // transform_skip_flag luma / chroma
     110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,  // last x
     110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,  // last y
     91, 171, 134, 141,                          // coded_sub_block_flag
     111, 111, 125, 110, 110, 94, 124, 108, 124, 107, 125, 141, 179, 153, 125, 107, 125, 141, 179, 153,
     125, 107, 125, 141, 179, 153, 125, 140, 139, 182, 182, 152, 136, 152, 136, 153, 136, 139, 111, 136,
     139, 111,                                   // sig_coeff_flag
     140, 92, 137, 138, 140, 152, 138, 139, 153, 74, 149, 92, 139, 107, 122, 152, 140, 179, 166, 182,
     140, 227, 122, 197,                         // coeff_abs_level_greater1_flag
     138, 153, 136, 167, 152, 152},              // coeff_abs_level_greater2_flag
    {// initType 1
     153, 185, 107, 139, 126, 154, 197, 185, 201, 149, 154, 139, 154, 154, 154, 152, 79, 110, 122, 95, 79, 63,
     31, 31, 153, 153, 168, 124, 138, 94, 153, 111, 149, 107, 167, 154, 140, 198, 154, 154, 139, 139,
     125, 110, 94, 110, 95, 79, 125, 111, 110, 78, 110, 111, 111, 95, 94, 108, 123, 108,
     125, 110, 94, 110, 95, 79, 125, 111, 110, 78, 110, 111, 111, 95, 94, 108, 123, 108,
     121, 140, 61, 154,
     155, 154, 139, 153, 139, 123, 123, 63, 153, 166, 183, 140, 136, 153, 154, 166, 183, 140, 136, 153,
     154, 166, 183, 140, 136, 153, 154, 170, 153, 123, 123, 107, 121, 107, 121, 167, 151, 183, 140, 151,
     183, 140,
     154, 196, 196, 167, 154, 152, 167, 182, 182, 134, 149, 136, 153, 121, 136, 137, 169, 194, 166, 167,
     154, 167, 137, 182,
     107, 167, 91, 122, 107, 167},
    {// initType 2
     153, 160, 107, 139, 126, 154, 197, 185, 201, 134, 154, 139, 154, 154, 183, 152, 79, 154, 137, 95, 79, 63,
     31, 31, 153, 153, 168, 224, 167, 122, 153, 111, 149, 92, 167, 154, 169, 198, 154, 154, 139, 139,
     125, 110, 124, 110, 95, 94, 125, 111, 111, 79, 125, 126, 111, 111, 79, 108, 123, 93,
     125, 110, 124, 110, 95, 94, 125, 111, 111, 79, 125, 126, 111, 111, 79, 108, 123, 93,
     121, 140, 61, 154,
     170, 154, 139, 153, 139, 123, 123, 63, 124, 166, 183, 140, 136, 153, 154, 166, 183, 140, 136, 153,
     154, 166, 183, 140, 136, 153, 154, 170, 153, 138, 138, 122, 121, 122, 121, 167, 151, 183, 140, 151,
     183, 140,
     154, 196, 167, 167, 154, 152, 167, 182, 182, 134, 149, 136, 153, 121, 136, 122, 169, 208, 166, 167,
     154, 152, 167, 182,
     107, 167, 91, 107, 107, 167},
};

// ---------------------------------------------------------------------------- scans (§6.5.3-5)
// Scan position -> (x, y) for a 4x4 block / the sub-block grid: diagonal (up-right), horizontal,
// vertical. kScan4[scanIdx][k] = x | y << 2.
struct Scan4 {
  u8 s[3][16];
  constexpr Scan4() : s{} {
    int k = 0;  // up-right diagonal
    for (int d = 0; d < 7; ++d)
      for (int y = d; y >= 0; --y) {
        const int x = d - y;
        if (x < 4 && y < 4) s[0][k++] = u8(x | y << 2);
      }
    for (int i = 0; i < 16; ++i) {
      s[1][i] = u8((i & 3) | (i >> 2) << 2);  // horizontal: row by row
      s[2][i] = u8((i >> 2) | (i & 3) << 2);  // vertical: column by column
    }
  }
};
inline constexpr Scan4 kScan4{};

// Diagonal scan of an n x n sub-block grid (n = 2, 4, 8): positions x | y << 3.
struct ScanDiag8 {
  u8 s[4][64];  // [log2 n - 0] n = 1, 2, 4, 8
  constexpr ScanDiag8() : s{} {
    for (int l = 0; l < 4; ++l) {
      const int n = 1 << l;
      int k = 0;
      for (int d = 0; d < 2 * n - 1; ++d)
        for (int y = d; y >= 0; --y) {
          const int x = d - y;
          if (x < n && y < n) s[l][k++] = u8(x | y << 3);
        }
    }
  }
};
inline constexpr ScanDiag8 kScanDiag{};

// Inverse scans: kScan4Inv[scanIdx][x | y << 2] = k, kScanDiagInv[log2 n][x | y << 3] = k.
struct Scan4Inv {
  u8 s[3][16];
  constexpr Scan4Inv() : s{} {
    for (int t = 0; t < 3; ++t)
      for (int k = 0; k < 16; ++k) s[t][kScan4.s[t][k]] = u8(k);
  }
};
inline constexpr Scan4Inv kScan4Inv{};
struct ScanDiag8Inv {
  u8 s[4][64];
  constexpr ScanDiag8Inv() : s{} {
    for (int l = 0; l < 4; ++l)
      for (int k = 0; k < (1 << (2 * l)); ++k) s[l][kScanDiag.s[l][k]] = u8(k);
  }
};
inline constexpr ScanDiag8Inv kScanDiagInv{};

// ---------------------------------------------------------------------------- intra
// intraPredAngle for modes 2..34 (index mode - 2) and invAngle for modes 11..25.
HK_TABLE i8 kIntraAngle[33] = {32,  26,  21,  17,  13,  9,  5,  2,  0,  -2, -5, -9, -13, -17, -21, -26, -32,
                                       -26, -21, -17, -13, -9, -5, -2, 0,   2,  5,  9,  13,  17,  21,  26,  32};
HK_TABLE i16 kInvAngle[15] = {-4096, -1638, -910, -630, -482, -390, -315, -256,
                                      -315,  -390,  -482, -630, -910, -1638, -4096};

// ---------------------------------------------------------------------------- transform
// transMatrix coefficient of the 32-point inverse transform at (row k, column j): the unique
// magnitudes by angle a (units of pi/64) and the sign pattern of cos(pi * k * (2j + 1) / 64).
inline constexpr u8 kDctMag[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
                                   61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9,  4,  0};
struct DctMatrix {
  i8 m[32][32];
  constexpr DctMatrix() : m{} {
    for (int k = 0; k < 32; ++k)
      for (int j = 0; j < 32; ++j) {
        const int p = (k * (2 * j + 1)) % 128;
        int v = 0;
        if (p <= 32) v = kDctMag[p];
        else if (p <= 64) v = -int(kDctMag[64 - p]);
        else if (p <= 96) v = -int(kDctMag[p - 64]);
        else v = kDctMag[128 - p];
        m[k][j] = i8(v);
      }
  }
};
HK_TABLE DctMatrix kDct{};
// 4x4 DST-VII (intra luma 4x4).
HK_TABLE i8 kDst4[4][4] = {{29, 55, 74, 84}, {74, 74, 0, -74}, {84, -29, -74, 55}, {55, -84, 74, -29}};

// ---------------------------------------------------------------------------- interpolation
HK_TABLE i8 kLumaFilter[4][8] = {
    {0, 0, 0, 64, 0, 0, 0, 0}, {-1, 4, -10, 58, 17, -5, 1, 0}, {-1, 4, -11, 40, 40, -11, 4, -1},
    {0, 1, -5, 17, 58, -10, 4, -1}};
HK_TABLE i8 kChromaFilter[8][4] = {{0, 64, 0, 0},     {-2, 58, 10, -2}, {-4, 54, 16, -2}, {-6, 46, 28, -4},
                                           {-4, 36, 36, -4},  {-4, 28, 46, -6}, {-2, 16, 54, -4}, {-2, 10, 58, -2}};

// ---------------------------------------------------------------------------- deblocking
HK_TABLE u8 kBetaTable[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  6,  7,
                                      8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 28, 30, 32,
                                      34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64};
HK_TABLE u8 kTcTable[54] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                    2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24};
// QpC as a function of qPi for 4:2:0 (Table 8-10).
inline int hevc_chroma_qp(int qpi) {
  static constexpr u8 k[14] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37};  // qPi 30..43
  if (qpi < 30) return qpi;
  if (qpi > 43) return qpi - 6;
  return k[qpi - 30];
}

}  // namespace vep::hevc
