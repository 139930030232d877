// Internals of the general HEVC decoder shared by the decoder (hevc_dec.cpp) and the
// closed-loop encoder (hevc_enc.cpp): the picture-level state and the CTU layer interface.
#pragma once

#include <array>

#include "cabac.h"
#include "hevc_dec.h"
#include "hevc_kern.h"
#include "hevc_tables.h"

namespace vep::hevc {

struct SaoParams {
  u8 type[3] = {0, 0, 0};   // 0 off, 1 band, 2 edge
  u8 band[3] = {0, 0, 0};   // sao_band_position
  u8 eo[3] = {0, 0, 0};     // sao_eo_class
  i8 off[3][4] = {};        // SaoOffsetVal[1..4]
};

// Per-slice state needed after parsing (loop filters, TMVP).
struct SliceInfo {
  SliceHeader sh;
  int qp = 26;
  std::vector<FramePtr> list[2];
  std::vector<int> list_poc[2];
};

struct PicCtx {
  const Sps* sps = nullptr;
  const Pps* pps = nullptr;
  int W = 0, H = 0;           // coded luma size (multiple of MinCb)
  int w4 = 0, h4 = 0;         // 4x4 grid
  int log2ctb = 4, wctb = 0, hctb = 0;
  int poc = 0;
  HostSurface* s = nullptr;   // target surface (reconstruction, then loop filters)
  // per 4x4 block
  std::vector<u8> depth, skip, intra, ipm, done, rec, pcm, cbf, edge;
  std::vector<i8> qp;
  std::vector<MvField> mf;
  std::vector<u16> slice;     // slice index per CTB (not per 4x4)
  std::vector<SaoParams> sao; // per CTB
  std::vector<SliceInfo> slices;
  Decoder::Stats stats;
  // records mode (GPU reconstruction): the CTU layer emits work instead of samples
  GpuPicture* gpu = nullptr;
  std::vector<u16> lvl_y, lvl_c;  // intra dependency level of each 4x4 block's samples

  void init(const Sps& sp, const Pps& pp, HostSurface* surf) {
    sps = &sp;
    pps = &pp;
    W = sp.width;
    H = sp.height;
    w4 = W >> 2;
    h4 = H >> 2;
    log2ctb = sp.log2_ctb;
    wctb = sp.width_ctbs();
    hctb = sp.height_ctbs();
    s = surf;
    const size_t n = size_t(w4) * h4;
    if (depth.size() != n) {  // (every other per-4x4 array is written by the CU covering it
      depth.assign(n, 0);     // before anything reads it: only the decoded flags are reset)
      skip.assign(n, 0);
      intra.assign(n, 0);
      ipm.assign(n, 1);
      pcm.assign(n, 0);
      cbf.assign(n, 0);
      edge.assign(n, 0);
      qp.assign(n, 0);
      mf.assign(n, MvField{});
    }
    done.assign(n, 0);
    rec.assign(n, 0);
    slice.assign(size_t(wctb) * hctb, 0xFFFF);
    sao.assign(size_t(wctb) * hctb, SaoParams{});
    slices.clear();
    stats = {};
    gpu = nullptr;
  }
  void init_gpu(GpuPicture* g) {
    gpu = g;
    lvl_y.assign(size_t(w4) * h4, 0);
    lvl_c.assign(size_t(w4) * h4, 0);
  }
  size_t i4(int x, int y) const { return size_t(y >> 2) * w4 + size_t(x >> 2); }
  int ctb_of(int x, int y) const { return (y >> log2ctb) * wctb + (x >> log2ctb); }
  // z-scan availability of luma location (xn, yn) for the block at (x, y) (§6.4.1): inside the
  // picture, same slice, already decoded.
  bool avail(int x, int y, int xn, int yn, const std::vector<u8>& flag) const {
    if (xn < 0 || yn < 0 || xn >= W || yn >= H) return false;
    if (!flag[i4(xn, yn)]) return false;
    // a decoded block of a single-slice picture is in the current block's slice
    return slices.size() == 1 || slice[size_t(ctb_of(xn, yn))] == slice[size_t(ctb_of(x, y))];
  }
};

// edge flags per 4x4 (deblocking): the left / top side of the block is a transform / prediction
// block boundary
enum : u8 { kEdgeTuV = 1, kEdgeTuH = 2, kEdgePuV = 4, kEdgePuH = 8 };

// Decisions of the encoder for one CTU (write mode of the CTU layer).
struct CtuDecider {
  virtual ~CtuDecider() = default;
  virtual bool split(int x0, int y0, int log2) = 0;
  virtual void cu(int x0, int y0, int log2, CuDesc& d) = 0;
  virtual void sao(int rx, int ry, SaoParams& p, bool& merge_left, bool& merge_up) = 0;
  ResidualFn residual;
};

// Walk (decode or encode + reconstruct) the CTUs of one slice segment. `data` / `n`: the slice
// NAL RBSP (read mode); `out`: the RBSP being written (write mode, slice header already in it,
// byte aligned).
void decode_slice_data(PicCtx& pc, int slice_idx, const u8* data, size_t n, size_t bytepos);
void encode_slice_data(PicCtx& pc, int slice_idx, std::vector<u8>& out, CtuDecider& dec, int first_ctb,
                       int end_ctb);

// Loop filters over the finished picture.
void deblock_picture(PicCtx& pc);
// Boundary strength of the left / top edge of every 4x4 block (0 where the edge is not filtered).
void deblock_strengths(const PicCtx& pc, std::vector<u8>& bsv, std::vector<u8>& bsh);
// Records mode: the loop-filter inputs of the finished picture into pc.gpu.
void finish_gpu_picture(PicCtx& pc);

void sao_picture(PicCtx& pc);

// TMVP store of a decoded picture.
std::shared_ptr<std::vector<ColMv>> build_col(const PicCtx& pc, int& col_w);

// Merge / AMVP candidate derivation (exposed for the encoder's decisions).
struct MergeCand {
  i16 mv[2][2];
  i8 ref[2];
  u8 pred;
};
int merge_candidates(const PicCtx& pc, int si, int xCb, int yCb, int nCbS, int xPb, int yPb, int nPbW, int nPbH,
                     int partIdx, int part_mode, MergeCand* out);
void amvp_candidates(const PicCtx& pc, int si, int xCb, int yCb, int nCbS, int xPb, int yPb, int nPbW, int nPbH,
                     int partIdx, int X, int refIdx, i16 out[2][2]);

// Sample prediction of one PU into 16-bit intermediate arrays (before weighting) and final
// samples (tests / encoder).
void predict_pu(const PicCtx& pc, int si, int xPb, int yPb, int w, int h, const MvField& m, u8* y, int ys, u8* cb,
                u8* cr, int cs);

}  // namespace vep::hevc
