// General H.265/HEVC Main / Main10 decoder (8..10-bit 4:2:0, progressive): I, P and B slices with
// CABAC coding quadtrees (CTB 16..64, CU 8..64, all partition modes incl. AMP), intra prediction
// (35 modes, reference substitution / smoothing, strong intra smoothing), PCM, transform trees
// (4..32 DCT, 4x4 DST, transform skip, sign data hiding, cu_qp_delta), merge / AMVP with
// temporal motion-vector prediction, 8-tap / 4-tap motion compensation with bi-prediction,
// the deblocking filter and SAO; short-term reference picture sets and output in POC order.
//
// Split of work: one `CtuLayer` walks the CTU syntax and reconstructs as it goes (intra
// prediction needs the reconstructed neighbours), in read mode for the decoder and in write
// mode for the closed-loop synthetic encoder (hevc_enc.cpp), so both share the binarizations,
// the context selection, the candidate derivations and the reconstruction; the loop filters run
// over the finished picture. This is the CPU reference of the H.265 path (bit-exact oracle for
// GPU reconstruction kernels). Also: tiles, wavefront (WPP) substreams, dependent slice
// segments, long-term reference pictures, explicit weighted prediction, scaling lists and
// transquant-bypass (lossless) CUs. Main10: 9..10-bit samples are kept in 16-bit surfaces
// (HostSurface::y16 / uv16; QpBdOffset, bit-depth shifts of MC / transforms / loop filters,
// 10-bit SAO offsets, PCM at any PCM bit depth). Range extensions (non-4:2:0, > 10 bit,
// different luma / chroma bit depths) are reported as UnsupportedStream.
//
// Reference parity: libavcodec's hevc decoder behind PyAV (python/read_image.py:87
// `p.decode()`), BASELINE config 5 (H.265 cameras). No third-party HEVC stream exists in this
// image: conformance beyond the closed loop and the spec oracle tests is unpinned.
#pragma once

#include <functional>
#include <array>
#include <map>
#include <memory>

#include "recycle.h"
#include "avc.h"
#include "codec.h"
#include "hevc.h"
#include "hevc_tables.h"

namespace vep::hevc {

struct WppSync;

// Motion of one 4x4 block (also the TMVP store of a reference picture, at 16x16 granularity).
struct MvField {
  i16 mv[2][2] = {{0, 0}, {0, 0}};
  i8 ref[2] = {-1, -1};  // refIdx per list (-1: list unused)
  u8 pred = 0;           // bit 0 list 0, bit 1 list 1; 0 = intra / not available
};

struct ColMv {  // a reference picture's motion as seen by TMVP
  i16 mv[2][2];
  i32 poc[2];    // POC of the picture each list's vector points at
  u8 pred;       // 0 = intra
  u8 lt;         // bit l: that reference was a long-term picture when this picture was decoded
};

// A decoded picture.
struct HevcFrame {
  HostSurface s;
  int poc = 0;
  bool is_ref = false, needed_for_output = false;
  bool long_term = false;  // marked "used for long-term reference"
  u32 uid = 0;
  i64 pts = 0, dts = 0, tag = 0;
  bool keyframe = false;
  char type = 'I';
  std::shared_ptr<std::vector<ColMv>> col;  // 16x16 grid
  int col_w = 0;
  int width = 0, height = 0, crop_left = 0, crop_top = 0;  // conformance window (output size)
  int slot = 0;                                             // DPB surface slot (GPU mode)
  int latency = 0;                                          // (output bumping, C.5.2.3)
  i64 rasl_of = -1;  // RASL picture: decode tag of its associated CRA (-1: not a RASL picture)
};
using FramePtr = std::shared_ptr<HevcFrame>;

// Encoder side of the CTU layer: the decisions of one coding unit. Residual levels are asked
// for once the prediction of each transform block is known (`residual`).
struct CuDesc {
  bool skip = false;
  bool intra = false;
  bool bypass = false;        // cu_transquant_bypass_flag (lossless CU)
  int part = 0;               // PartMode: 0 2Nx2N 1 2NxN 2 Nx2N 3 NxN 4 2NxnU 5 2NxnD 6 nLx2N 7 nRx2N
  bool pcm = false;
  const u16* pcm_samples = nullptr;  // (2N)^2 luma then 2 * N^2 chroma (at the PCM bit depths)
  int luma_mode[4] = {1, 1, 1, 1};  // IntraPredModeY per partition
  int chroma_mode = 4;              // intra_chroma_pred_mode (4 = DM)
  struct Pu {
    bool merge = false;
    int merge_idx = 0;
    int dir = 1;              // 1 L0, 2 L1, 3 bi
    int ref[2] = {0, 0};
    int mvp[2] = {0, 0};      // mvp_lX_flag
    i16 mv[2][2] = {{0, 0}, {0, 0}};  // wanted vectors (mvd = mv - predictor)
  } pu[4];
  int tu_log2 = 5;            // split the transform tree down to this size (clamped to limits)
  int qp_delta = 0;
  bool tskip = false;         // transform_skip_flag for 4x4 TUs
};

// Supplies levels for one transform block in write mode: `pred` is the prediction (stride
// `pstride`), `src` the source samples, the levels go to `lv` (raster n x n). Returns whether the
// block is coded with transform skip (4x4 only).
using ResidualFn = std::function<void(int c, int x0, int y0, int log2, const u16* pred, int pstride, int qp,
                                      bool tskip_allowed, bool intra, int* lv, bool& tskip)>;

struct PicCtx;

class Decoder {
 public:
  Decoder();
  ~Decoder();
  // Parse + reconstruct one access unit. Returns the frames that leave the output queue (POC
  // order), possibly none; throws UnsupportedStream / Error.
  std::vector<FramePtr> decode(const AccessUnit& au, i64 tag = 0);
  std::vector<FramePtr> flush();  // end of stream
  bool has_sps() const { return !sps_.empty(); }
  // Records mode (GPU reconstruction): pictures are parsed into GpuPicture work lists instead of
  // being reconstructed; frames carry their DPB surface slot. take_gpu_pictures() hands over the
  // pictures parsed since the last call, in decoding order.
  void set_gpu_mode(bool on) { gpu_mode_ = on; }
  bool gpu_mode() const { return gpu_mode_; }
  std::vector<std::shared_ptr<struct GpuPicture>> take_gpu_pictures();
  int gpu_slots() const { return gpu_slots_; }  // surfaces a camera needs (max DPB + 2)
  FramePtr last_decoded() const { return last_; }
  // slices / tile substreams parsed as parallel units so far (tests)
  u64 parallel_units() const { return parallel_units_; }
  // statistics of the last picture (tests): CU counts by kind
  struct Stats {
    int intra = 0, inter = 0, skip = 0, pcm = 0, merge = 0, bi = 0, tskip = 0, amp = 0;
  } stats;

 private:
  void start_picture(const SliceHeader& sh, int tid, const Sps& sps, const Pps& pps, const AccessUnit& au, i64 tag,
                     std::vector<FramePtr>& out);
  void finish_picture(std::vector<FramePtr>& out);
  void bump(std::vector<FramePtr>& out);
  // (ebsp / en: the NAL as received, for the RBSP positions of the entry points)
  void decode_slice(const SliceHeader& sh, const u8* rbsp, size_t n, const u8* ebsp, size_t en);
  // the picture's deferred slices: in parallel when the picture is complete, else in order
  void run_deferred(bool parallel);
  std::map<int, Vps> vps_;
  std::map<int, Sps> sps_;
  std::map<int, Pps> pps_;
  std::vector<FramePtr> dpb_;
  FramePtr cur_, last_;
  std::vector<FramePtr> st_before_, st_after_;  // RefPicSetStCurrBefore / After of the picture
  std::vector<FramePtr> lt_curr_;               // RefPicSetLtCurr
  SliceHeader prev_sh_;                         // the picture's previous slice segment header
  bool have_prev_sh_ = false;
  std::unique_ptr<PicCtx> pc_;
  const Sps* sps_act_ = nullptr;
  const Pps* pps_act_ = nullptr;
  std::vector<u8> rbsp_;
  int prev_tid0_poc_ = 0;
  int act_w_ = 0, act_h_ = 0;  // picture size of the active coded video sequence
  int act_bd_ = 8;             // and its bit depth
  bool first_ = true, no_rasl_output_ = true, skip_pic_ = false;
  i64 irap_tag_ = -1;  // decode tag of the last IRAP picture (RASL pictures' association)
  u32 next_uid_ = 1;
  bool gpu_mode_ = false;
  int gpu_slots_ = 0, last_out_slot_ = -1;
  std::shared_ptr<struct GpuPicture> cur_gpu_;
  // records-mode pictures recycled per decoder (recycle.h: resident buffers, no page faults)
  std::shared_ptr<Recycler<struct GpuPicture>> gpu_pool_;
  std::vector<std::shared_ptr<struct GpuPicture>> gpu_out_;
  // Independent slices (and the tiles inside them) of one picture are parsed in parallel on the
  // shared fan-out pool
  // (fanout.h): their slice data is kept (deferred_: slice index, RBSP bytes, data offset) until
  // the picture's last slice arrived. Pictures with WPP or dependent slice segments (contexts
  // carried between segments) are parsed slice by slice as before. VEP_HEVC_SLICE_THREADS=0: off.
  bool parallel_slices_ = true;
  bool defer_ = false;
  std::vector<std::vector<u8>> slice_rbsp_;
  std::vector<std::array<size_t, 3>> deferred_;
  // Tiles: the RBSP offsets of a deferred slice's 2nd.. substreams (its entry points), so each
  // tile of the slice is parsed as a unit of its own (tiles share no CABAC state or prediction)
  std::vector<std::vector<size_t>> slice_subs_;
  u64 parallel_units_ = 0;
  std::unique_ptr<WppSync> wpp_sync_;  // wavefront rows in parallel (hevc_ctu.h)
  std::vector<std::unique_ptr<struct SliceShard>> shards_;
};

// CPU mirror of the GPU reconstruction of one picture (hevc_gpu.cpp): executes the records of a
// records-mode picture on the DPB surfaces `slots` with the kernels' per-sample math (CPU
// backend of the records path; the oracle of gpu_hevc.hip).
void cpu_execute(const struct GpuPicture& p, std::vector<HostSurface>& slots);
// The queue kernel's edge exchange, checked on the records: every reference sample an intra
// block polls (GpuTu::pend) must be on the right column / bottom row of an intra block of a
// lower level. Returns the number of samples that are not (0 for a consistent picture).
u64 exchange_violations(const struct GpuPicture& p);


// Closed-loop synthetic HEVC Main encoder (tests, camera farm): I / P / B pictures over the
// shared CTU layer; `coverage` randomises every decision (all CU sizes, partition modes incl.
// AMP, intra modes, merge candidates, AMVP, bi-prediction, transform trees, transform skip, PCM,
// QP deltas, SAO types), otherwise decisions come from a simple SAD search on the synthetic
// scene.
struct HevcEncConfig {
  int width = 416, height = 240;
  int fps = 30, gop = 16;
  int idr_phase = 0;         // IDR when display index d == 0 or (d + idr_phase) % gop == 0
  int bframes = 0;           // B pictures between anchors (0 = IPPP)
  int qp = 30;
  int log2_ctb = 5, log2_min_cb = 3;
  bool amp = true, sao = true, deblock = true, tskip = true, sign_hiding = true, cu_qp_delta = true;
  bool pcm = true, tmvp = true;
  int slices = 1;
  // stream structure / coding tools beyond the basic Main stream
  int tile_cols = 1, tile_rows = 1;  // tiles (coverage: explicit, non-uniform spacing at random)
  bool wpp = false;                  // entropy_coding_sync (one substream per CTB row)
  int segments = 1;                  // slice segments per slice: the 2nd.. are dependent
  bool scaling_lists = false;        // scaling lists (coverage: custom SPS / PPS lists)
  bool weighted = false;             // explicit weighted prediction in P and B slices
  bool long_term = false;            // each GOP's IDR stays referenced as a long-term picture
  // open GOPs: every IRAP after the first is a CRA, coded before the B pictures that precede it in
  // display order (RASL pictures: they predict from the previous GOP's anchor and the CRA)
  bool open_gop = false;
  bool lossless = false;             // transquant bypass enabled (coverage: lossless CUs)
  int bit_depth = 8;                 // 8 (Main) or 10 (Main10: 10-bit samples, 16-bit surfaces)
  bool coverage = false;
  int objects = 3;
  double noise = 3.0, temporal_noise = 0.0;
  u64 seed = 1;
};

class HevcEncoder : public avc::StreamEncoder {
 public:
  explicit HevcEncoder(const HevcEncConfig& cfg);
  ~HevcEncoder() override;
  std::shared_ptr<AccessUnit> next() override;
  const HostSurface& reconstruction() const override;
  const HostSurface& source() const override;
  i64 last_pts() const override;
  char last_type() const;
  const std::vector<u8>& vps_nal() const;
  const std::vector<u8>& sps_nal() const override;
  const std::vector<u8>& pps_nal() const override;

 private:
  struct Impl;
  std::unique_ptr<Impl> p_;
};

}  // namespace vep::hevc
