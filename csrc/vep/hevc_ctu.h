// Internals of the general HEVC decoder shared by the decoder (hevc_dec.cpp) and the
// closed-loop encoder (hevc_enc.cpp): the picture-level state and the CTU layer interface.
#pragma once

#include <array>
#include <atomic>
#include <memory>

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

// Per-slice-segment state needed after parsing (loop filters, TMVP). The segments of one slice
// (an independent segment and its dependent ones) share `ord` and the slice-level fields.
struct SliceInfo {
  SliceHeader sh;
  int qp = 26;
  int ord = 0;       // ordinal of the slice in the picture (decoding order)
  int addr_rs = 0;   // SliceAddrRs: raster address of the slice's first CTB
  std::vector<FramePtr> list[2];
  std::vector<int> list_poc[2];
  std::vector<u8> list_lt[2];  // the entry is a long-term reference picture
};

// Wavefront rows of one picture parsed in parallel (Decoder, WPP): per CTB a done flag
// (release / acquire), per CTB row the contexts stored after its 2nd CTB, and an abort flag (a
// row that fails releases the rows waiting on it).
struct WppSync {
  std::unique_ptr<std::atomic<u8>[]> done;
  std::vector<cabac::Ctx> rows;  // hctb x kCtxCount
  std::atomic<bool> abort{false};
  int wctb = 0;
  void reset(int w, int h) {
    if (w * h != wctb * int(rows.size() / kCtxCount) || !done) done.reset(new std::atomic<u8>[size_t(w) * h]);
    for (int k = 0; k < w * h; ++k) done[size_t(k)].store(0, std::memory_order_relaxed);
    rows.resize(size_t(h) * kCtxCount);
    wctb = w;
    abort.store(false);
  }
  // until CTB rs is parsed (spin, then yield); throws when another row failed
  void wait(int rs) const;
};

struct PicCtx {
  const Sps* sps = nullptr;
  const Pps* pps = nullptr;
  int W = 0, H = 0;           // coded luma size (multiple of MinCb)
  int w4 = 0, h4 = 0;         // 4x4 grid
  int log2ctb = 4, wctb = 0, hctb = 0;
  int poc = 0;
  HostSurface* s = nullptr;   // target surface (reconstruction, then loop filters)
  // sample bit depths and QpBdOffsetY / C (Main10: 10 / 12)
  int bd_y = 8, bd_c = 8, qp_off_y = 0, qp_off_c = 0;
  // per 4x4 block
  std::vector<u8> depth, skip, intra, ipm, done, rec, pcm, cbf, edge;
  std::vector<i8> qp;
  std::vector<MvField> mf;
  std::vector<u16> slice;     // slice segment index per CTB (not per 4x4)
  std::vector<u16> sord;      // slice ordinal per CTB
  std::vector<SaoParams> sao; // per CTB
  std::vector<SliceInfo> slices;
  // tiles (§6.5.1): column / row boundaries in CTBs, CTB address conversions, tile id per CTB
  std::vector<int> col_bd, row_bd, rs2ts, ts2rs;
  std::vector<u16> tile;
  bool multi = false;         // several slices or tiles: availability consults sord / tile
  // per 4x4: CU coded with cu_transquant_bypass_flag (loop filters leave its samples alone)
  std::vector<u8> bypass;
  bool any_bypass = false;
  // scaling factors m[x][y] per sizeId / matrixId (raster, n x n) when scaling lists are on
  bool scaling = false;
  std::vector<u8> sf[4][6];
  // CABAC state carried across CTUs / segments: WPP storage (after the 2nd CTB of a row) and
  // the end of the previous slice segment (dependent slice segments)
  cabac::Ctx wpp_ctx[kCtxCount];
  WppSync* wpp_sync = nullptr;  // rows in parallel: per-row storage + CTB done flags
  cabac::Ctx ds_ctx[kCtxCount];
  int ds_qp = 26;
  Decoder::Stats stats;
  // records mode (GPU reconstruction): the CTU layer emits work instead of samples
  GpuPicture* gpu = nullptr;
  // Independent slices parsed in parallel (Decoder): `slice` / `sord` are filled for the whole
  // picture before the slices run, so no CTU writes them and every availability test reads a
  // value that does not change while other slices are being decoded.
  bool prefilled = false;
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
    bd_y = sp.bit_depth_luma;
    bd_c = sp.bit_depth_chroma;
    qp_off_y = 6 * (bd_y - 8);
    qp_off_c = 6 * (bd_c - 8);
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
    sord.assign(size_t(wctb) * hctb, 0xFFFF);
    sao.assign(size_t(wctb) * hctb, SaoParams{});
    slices.clear();
    stats = {};
    gpu = nullptr;
    init_tiles();
    multi = col_bd.size() > 2 || row_bd.size() > 2;
    any_bypass = false;
    if (pp.transquant_bypass) bypass.assign(n, 0);
    init_scaling();
  }
  void init_tiles();
  void init_scaling();
  int tile_col_start(int rx) const {  // first CTB column of the tile column containing rx
    int s = 0;
    for (size_t i = 0; i + 1 < col_bd.size() && col_bd[i] <= rx; ++i) s = col_bd[i];
    return s;
  }
  bool first_ctb_in_tile(int rs) const {
    const int ts = rs2ts[size_t(rs)];
    return ts == 0 || tile[size_t(ts2rs[size_t(ts) - 1])] != tile[size_t(rs)];
  }
  bool ctb_row_start(int rs) const { return rs % wctb == tile_col_start(rs % wctb); }
  bool nofilter(size_t k) const {  // loop filters must not modify the 4x4 block's samples
    return (sps->pcm_loop_filter_disabled && pcm[k]) || (any_bypass && bypass[k]);
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
    // a decoded block of a single-slice, single-tile picture is in the current block's slice;
    // otherwise the slice / tile test comes first, so the decoded flag is only read for blocks of
    // the current slice (another slice's may be written concurrently: parallel slices)
    if (multi) {
      const size_t a = size_t(ctb_of(xn, yn)), b = size_t(ctb_of(x, y));
      if (sord[a] != sord[b] || tile[a] != tile[b]) return false;
    }
    return flag[i4(xn, yn)] != 0;
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

// Outputs of one slice decoded in parallel with the picture's other slices (Decoder): merged
// into the picture in slice order afterwards, so the records equal a sequential parse's.
struct SliceShard {
  GpuPicture g;               // records mode: the slice's tus / pus / coefs / pcm / wp
  Decoder::Stats stats;
  bool any_bypass = false;
  int ctus = 0;               // CTUs the slice decoded
};

// Walk (decode or encode + reconstruct) the CTUs of one slice segment. `data` / `n`: the slice
// NAL RBSP (read mode); `out`: the RBSP being written (write mode, slice header already in it,
// byte aligned). `shard`: the slice's own outputs (parallel slices, see SliceShard). Returns the
// number of CTUs decoded.
int decode_slice_data(PicCtx& pc, int slice_idx, const u8* data, size_t n, size_t bytepos,
                      SliceShard* shard = nullptr);
// One substream of a slice segment (a tile): CTUs [first_ts, end_ts) in tile scan, from RBSP
// byte `bytepos` (its entry point); `last`: the segment's final substream (ends with
// end_of_slice_segment_flag, the others with end_of_subset_one_bit). Returns the CTUs decoded.
int decode_substream(PicCtx& pc, int slice_idx, const u8* data, size_t n, size_t bytepos, int first_ts, int end_ts,
                     bool last, SliceShard* shard);
// Write mode: CTUs [first_ts, end_ts) in tile scan. `out` receives the slice segment data only;
// `substreams` (when given) the byte offsets in `out` where each further WPP row / tile
// substream starts (entry points, before emulation prevention).
void encode_slice_data(PicCtx& pc, int slice_idx, std::vector<u8>& out, CtuDecider& dec, int first_ts, int end_ts,
                       std::vector<size_t>* substreams = nullptr);

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
void predict_pu(const PicCtx& pc, int si, int xPb, int yPb, int w, int h, const MvField& m, u16* y, int ys, u16* cb,
                u16* cr, int cs);
// Explicit weighting record of one PU for the components' bit depths (log2WD and scaled offsets).
GpuWp explicit_weights(const SliceHeader& sh, const MvField& m, int bd_y, int bd_c);

}  // namespace vep::hevc
