// General H.264 decoding path: the macroblock layer of I, P and B slices in both entropy modes
// (CAVLC and CABAC; Baseline / Main / High profile, progressive 8-bit 4:2:0), 4x4 and 8x8
// transforms, scaling matrices, explicit and implicit weighted prediction, spatial and temporal
// direct prediction, reference picture management with picture-order-count output reordering,
// the CPU reference reconstruction and a closed-loop synthetic encoder that emits the same
// syntax.
//
// Split of work (MI355X-first):
//  * CPU (`Decoder::parse`): the inherently serial entropy layer — slice headers, mb_type,
//    prediction modes, motion-vector prediction (incl. direct modes), residual levels and
//    dequantisation — into a compact per-picture record array (`Picture`: 56-byte MbRec per MB
//    + a pool of dequantised coefficient blocks + a motion-vector pool + a weight pool), and the
//    DPB / reference-list / output-order bookkeeping (which GPU surface holds which picture).
//  * GPU (gpu_avc.hip): everything that touches samples — motion compensation (bi-predictive and
//    weighted) + residual for all inter MBs of all cameras in one launch, intra prediction
//    (4x4 / 8x8 / 16x16) in a row-ticketed wavefront, the deblocking filter in a second
//    wavefront, then the NV12->BGR24 conversion of each camera's newest output picture.
//  * `cpu_reconstruct` is the bit-exact CPU reference (and the CPU backend) built from the same
//    primitives (avc_recon.h).
//
// Reference parity: this is the libavcodec h264 decoder the reference calls through PyAV
// (python/read_image.py:87 `p.decode()`, :94 `to_ndarray('bgr24')`; SURVEY.md §2.2 N2 and
// §2.3 K1), including its output order (frames leave in picture-order-count order). Interlaced
// streams that code frame pictures decode like progressive ones; CAVLC I / P field pairs (PAFF)
// decode as half-height pictures in field slots (Picture::structure). MBAFF frames, CABAC / B /
// 8x8-transform field pictures, 4:2:2 / 4:4:4, high bit depth, lossless, data partitioning,
// FMO/ASO, SP/SI slices and CABAC streams with cabac_init_idc 1 or 2 are reported as
// UnsupportedStream (the VCN backend's job).
#pragma once

#include <array>
#include <map>
#include <memory>

#include "hostmem.h"
#include "recycle.h"
#include "avc_recon.h"
#include "codec.h"

namespace vep::avc {

constexpr int kMaxDpbSlots = 34;  // 16 references + 16 pictures waiting for output + current + pin

// Access-unit metadata a picture carries to its output (VideoFrame fields).
struct AuMeta {
  i64 pts = 0, dts = 0, arrival_ms = 0;
  i64 tag = 0;  // caller's tag (the camera passes the packet's index in its GOP)
  bool keyframe = false, corrupt = false;
};

// A decoded picture leaving the reorder buffer (output order).
struct OutFrame {
  int slot = -1;     // DPB slot holding its samples
  PictureInfo info;  // size, crop, picture type
  AuMeta au;
  int poc = 0;
  // A field pair: the frame slot holds the top field's rows then the bottom field's (field slots
  // 2 * slot and 2 * slot + 1, each half a frame); the output weaves them.
  bool fields = false;
};

struct ColBuild;

// One parsed picture, ready for reconstruction into DPB slot `target`.
struct Picture {
  int wmbs = 0, hmbs = 0;
  // Records in pinned pool memory once a GPU worker exists (hostmem::PinnedAllocator): the
  // worker's gather kernel pulls them over PCIe, no host copy into its staging buffer.
  hostmem::pinned_vector<MbRec> mbs;     // raster order
  hostmem::pinned_vector<i16> coefs;     // sparse dequantised coefficient groups per MB (avc_recon.h); I_PCM raw samples
  hostmem::pinned_vector<i16> mvs;       // 32 entries (16 x (mvx, mvy), quarter samples) per list per MB
  hostmem::pinned_vector<WpEntry> wps;   // weighted-prediction entries (4 per weighted MB)
  int target = 0;             // DPB slot this picture is reconstructed into
  int dpb_slots = 1;          // surfaces the camera needs for this stream
  // 0 frame; 1 / 2 top / bottom field picture. Field pictures address field slots (half a frame
  // each, parity = slot & 1: frame slot s = field slots 2s, 2s + 1), wmbs x hmbs is the field.
  int structure = 0;
  // Sample bit depth (High 10: 9 / 10; the surfaces then hold u16 samples) and the QP bias of the
  // records: MbRec::qp = QPY + QpBdOffsetY, MbRec::qpc / qpc2 = QPC + QpBdOffsetC (QPY / QPC may
  // be negative above 8 bits); the loop filter subtracts them.
  int bd = 8, qp_bias = 0, qpc_bias = 0;
  int cf = 1;  // chroma_format_idc: 0 / 1 NV12 surfaces, 2 (4:2:2) NV16 (full-height chroma plane)
  bool second_field = false;  // completes a field pair (frame counters count these, not first fields)
  bool constrained_intra = false;
  int intra_mbs = 0;          // I4x4 / I8x8 / I16x16 MBs (need the wavefront pass)
  int intra_res = 0;          // intra MBs with residual samples (MbRec::res slots)
  int inter_mbs = 0;          // skip / inter / I_PCM MBs (the parallel pass)
  bool deblock = false;       // any MB with the loop filter enabled
  bool idr = false;
  int poc = 0;
  PictureInfo info;
  AuMeta au;
  // Pictures that left the reorder buffer when this one was decoded, in output order (the last
  // one is the newest frame a client can be shown after this picture).
  std::vector<OutFrame> outputs;
  // While the decoder parses a reference picture whose motion later B pictures may use: the
  // colocated-motion table, filled as each MB is stored (no pass over the picture afterwards).
  ColBuild* colb = nullptr;

  int nmbs() const { return wmbs * hmbs; }
};
using PicturePtr = std::shared_ptr<const Picture>;

// Structural invariants the reconstruction kernels rely on: every record's coefficient-pool,
// motion-vector and weight indices lie inside the picture's pools, reference / target slots
// inside the DPB, modes in range. Throws Error otherwise (defence in depth against a parser bug
// on hostile input: the GPU kernels index with these values unchecked).
void validate(const Picture& p);

// Full slice header (the fields reconstruction needs).
struct SliceHdr {
  int nal_type = 0, nal_ref_idc = 0;
  int first_mb = 0, slice_type = 0, pps_id = 0, frame_num = 0, idr_pic_id = 0;
  bool field_pic = false, bottom_field = false;
  int redundant_pic_cnt = 0;  // > 0: a slice of a redundant coded picture (skipped)
  int poc_lsb = 0, delta_poc_bottom = 0, delta_poc[2] = {0, 0};
  bool direct_spatial = true;
  int num_ref_idx[2] = {1, 1};
  struct RefMod {
    int idc, val;
  };
  std::vector<RefMod> ref_mods[2];  // ref_pic_list_modification per list
  // pred_weight_table (explicit weighted prediction); weights default to 1 << log2_denom
  bool explicit_wp = false;
  int luma_lwd = 0, chroma_lwd = 0;
  struct Weight {
    i16 w[3], o[3];  // Y, Cb, Cr
  };
  std::vector<Weight> wt[2];
  bool no_output_of_prior_pics = false, long_term_reference = false;
  bool adaptive_marking = false;
  struct Mmco {
    int op, a, b;
  };
  std::vector<Mmco> mmcos;
  int cabac_init_idc = 0;
  int qp = 26;                   // SliceQP_Y
  int disable_deblocking = 0, alpha_off = 0, beta_off = 0;  // offsets already doubled
  bool idr() const { return nal_type == h264::kNalIdr; }
  int type() const { return slice_type % 5; }
  bool has_mmco5() const {
    for (const auto& m : mmcos)
      if (m.op == 5) return true;
    return false;
  }
};

// Parse-time state of one MB of the current picture (neighbour derivations of both entropy
// modes, direct prediction of later B pictures).
struct MbState {
  u8 kind = 0xFF;    // MbKind; 0xFF = not decoded in this picture
  u8 skip = 0;       // P_Skip / B_Skip (mb_skip_flag context)
  u8 direct16 = 0;   // B_Skip / B_Direct_16x16 (B mb_type context)
  u8 direct8 = 0;    // bit per 8x8: predicted by direct mode (ref_idx context)
  u8 t8x8 = 0;       // transform_size_8x8_flag
  u8 cbp = 0;        // CodedBlockPatternLuma | CodedBlockPatternChroma << 4 (I_PCM: 0x2F)
  u8 chroma_mode = 0;
  u8 qp = 0;
  u16 slice = 0;
  u16 cbf = 0;       // coded_block_flag of the luma 4x4 blocks (raster)
  u8 cbf_dc = 0;     // bit 0 luma DC (Intra16x16), bits 1-2 Cb / Cr DC
  u8 cbf_cac[2] = {0, 0};  // chroma AC blocks (raster, 2 wide: 2x2 in 4:2:0, 2x4 in 4:2:2) per component
  i8 ref[2][4] = {{-1, -1, -1, -1}, {-1, -1, -1, -1}};  // refIdx per list per 8x8 (-1: unused)
  i16 mv[2][16][2] = {};
  u8 mvd[2][16][2] = {};  // min(|mvd|, 127) per 4x4 (CABAC mvd context)
  u8 tc[16] = {};     // CAVLC luma total_coeff (raster)
  u8 tcc[2][8] = {};  // CAVLC chroma AC total_coeff per component (raster, 2 wide)
  u8 i4[16] = {};     // Intra4x4PredMode (raster; Intra8x8PredMode replicated over its 4 blocks)
};

// Neighbour derivations shared by the decoder and the encoder (§6.4.11, §8.3.1.1, §8.4.1.3,
// §9.2.1): availability is "same slice and already decoded".
class MbNeighbours {
 public:
  // ring: keep only the state of the most recent MBs (a power-of-two ring of at least two MB
  // rows + 2) instead of the whole picture's — every derivation of the decoder reads the current
  // MB and its A / B / C / D neighbours (at most one row + 1 back), and the colocated motion of
  // later B pictures is copied out as each MB is stored (ColBuild). The ring (~64 KB at 1080p)
  // stays cache resident, where the whole picture's state (2 MB) was written and read back through
  // the cache hierarchy for every picture. The encoders keep the whole picture (build_col_motion).
  void reset(int wmbs, int hmbs, bool ring = false);
  // Announce the MB being decoded (after its kind and slice are set): caches the A/B/C/D
  // neighbour availability so the per-block derivations below need no division or lookup.
  void begin(int mb);
  MbState& at(int mb) { return st_[size_t(mb) & mask_]; }
  const MbState& at(int mb) const { return st_[size_t(mb) & mask_]; }
  int wmbs() const { return w_; }
  int hmbs() const { return h_; }
  // MB containing luma location (x, y) relative to MB `mb` (x, y may be -1 or >= 16); -1 if not
  // available. For locations inside `mb` itself returns mb.
  int mb_at(int mb, int x, int y) const;
  bool mb_available(int mb, int nb) const {
    const size_t i = size_t(nb) & mask_;
    return nb >= 0 && stamp_[size_t(nb)] == epoch_ && tag_[i] == u32(nb) && st_[i].kind != 0xFF &&
           st_[i].slice == st_[size_t(mb) & mask_].slice;
  }
  // decoded in the current picture (announced by begin() since the last reset())
  bool decoded(int mb) const {
    return stamp_[size_t(mb)] == epoch_ && tag_[size_t(mb) & mask_] == u32(mb) && st_[size_t(mb) & mask_].kind != 0xFF;
  }
  bool announced(int mb) const { return stamp_[size_t(mb)] == epoch_; }
  int announced_count() const { return announced_; }  // distinct MBs announced this picture
  // nC for luma block (raster) `blk` / chroma component c block `blk` (§9.2.1).
  int nc_luma(int mb, int blk) const;
  int nc_chroma(int mb, int c, int blk, int nbc = 4) const;  // nbc: chroma 4x4 blocks per component
  // predIntra4x4PredMode for raster block `blk` (also predIntra8x8PredMode with blk = the
  // 8x8's top-left 4x4 block and n8 = true: §8.3.2.1's neighbour block choice).
  int pred_intra4x4(int mb, int blk, bool constrained_intra) const;
  int pred_intra8x8(int mb, int b8, bool constrained_intra) const;
  // Motion-vector predictor of list `list` for partition (x, y, w, h) in 4x4 units with reference
  // `ref`; `done` = 4x4 blocks of the current MB whose motion is already set; shape: 0 generic,
  // 1 16x8, 2 8x16.
  void pred_mv(int mb, int x4, int y4, int w4, int h4, int list, int ref, u16 done, int shape,
               int out[2]) const;
  void pred_mv(int mb, int x4, int y4, int w4, int h4, int ref, u16 done, int shape, int out[2]) const {
    pred_mv(mb, x4, y4, w4, h4, 0, ref, done, shape, out);
  }
  void pskip_mv(int mb, int out[2]) const;
  // Neighbour A/B/C(D) motion of the whole MB for list `list` (direct spatial prediction):
  // ref[k] = refIdx (-1 unavailable / intra / list unused).
  void mb_neighbour_refs(int mb, int list, int ref[3]) const;
  // Spatial direct (§8.4.1.2.2) for list `list`: refIdx = MinPositive over A, B, C and the
  // 16x16 motion-vector predictor for it (mv = 0 when ref < 0), from one neighbour fetch.
  void direct_spatial_pred(int mb, int list, int& ref, int mv[2]) const;
  // The same for both lists at once, for the MB announced by begin() (B_Skip / B_Direct_16x16:
  // one fetch of the A / B / C(D) neighbours' motion instead of four motion_at() per list).
  void direct_spatial_both(int ref[2], int mv[2][2]) const;

 private:
  struct Nb {
    bool avail;
    int ref;
    int mv[2];
  };
  Nb motion_at(int mb, int x, int y, u16 done, int list) const;  // x, y in luma samples rel. to mb
  // A, B and C (D when C is unavailable) of the whole announced MB for one list: the
  // motion_at() results of (-1, 0), (0, -1), (16, -1) / (-1, -1) without the coordinate walk
  void nb16(int list, Nb n[3]) const;
  void pred_mv16(int list, int ref, int out[2]) const;  // pred_mv() of the 16x16 partition
  int w_ = 0, h_ = 0;
  int cur_ = -1, cx_ = 0, cy_ = 0, a_ = -1, b_ = -1, c_ = -1, d_ = -1;
  u32 run_slice_ = ~0u;  // begin(): the slice of the run of consecutively announced MBs
  int run_start_ = 0;    // ... and its first MB
  // "decoded in this picture": begin() stamped the MB with the picture's epoch (and its kind is
  // set). A new picture bumps the epoch instead of touching every MB's 256-byte state (a 1080p
  // state array is 2 MB; the stamps are 32 KB).
  u32 epoch_ = 0;
  int announced_ = 0;
  size_t mask_ = ~size_t(0);  // state index = mb & mask_ (all ones: the whole picture)
  std::vector<u32> stamp_;    // per MB of the picture
  std::vector<u32> tag_;      // per state entry: the MB whose state it holds (ring)
  std::vector<MbState> st_;
};

// Hot neighbour derivations, inline (called several times per macroblock).
inline void MbNeighbours::begin(int mb) {
  int mx, my;
  const int prev = cur_;
  const bool next = mb == prev + 1 && prev >= 0;
  if (mb == prev) {
    mx = cx_;
    my = cy_;
  } else if (next) {  // raster order: no division
    mx = cx_ + 1;
    my = cy_;
    if (mx == w_) {
      mx = 0;
      ++my;
    }
  } else {
    mx = mb % w_;
    my = mb / w_;
  }
  cur_ = mb;
  cx_ = mx;
  cy_ = my;
  if (stamp_[size_t(mb)] != epoch_) {
    stamp_[size_t(mb)] = epoch_;
    ++announced_;
  }
  tag_[size_t(mb) & mask_] = u32(mb);
  const u32 sl = st_[size_t(mb) & mask_].slice;
  if (next && sl == run_slice_) {
    // the next MB of a run announced consecutively in one slice since run_start_ (this
    // picture): a neighbour is available exactly when it lies in the picture at or after the
    // run's first MB — every MB from there to mb - 1 is of this slice and decoded, every earlier
    // one of another slice. The generic test below gives the same answer with four state lookups.
    const int f = run_start_;
    a_ = mx > 0 && mb - 1 >= f ? mb - 1 : -1;
    b_ = my > 0 && mb - w_ >= f ? mb - w_ : -1;
    c_ = my > 0 && mx + 1 < w_ && mb - w_ + 1 >= f ? mb - w_ + 1 : -1;
    d_ = my > 0 && mx > 0 && mb - w_ - 1 >= f ? mb - w_ - 1 : -1;
    return;
  }
  if (!(mb == prev && sl == run_slice_)) {  // (the same MB announced again keeps its run)
    run_slice_ = sl;
    run_start_ = mb;
  }
  auto nb = [&](int nx, int ny) {
    if (nx < 0 || nx >= w_ || ny < 0) return -1;
    const int n = ny * w_ + nx;
    return mb_available(mb, n) ? n : -1;
  };
  a_ = nb(mx - 1, my);
  b_ = nb(mx, my - 1);
  c_ = nb(mx + 1, my - 1);
  d_ = nb(mx - 1, my - 1);
}

inline int MbNeighbours::mb_at(int mb, int x, int y) const {
  if (y >= 16) return -1;
  if (mb != cur_) {  // slow path (not the MB announced by begin())
    const int dx = x < 0 ? -1 : (x >= 16 ? 1 : 0);
    const int dy = y < 0 ? -1 : 0;
    if (dx == 0 && dy == 0) return mb;
    if (dx > 0 && dy == 0) return -1;
    const int nx = mb % w_ + dx, ny = mb / w_ + dy;
    if (nx < 0 || nx >= w_ || ny < 0) return -1;
    const int n = ny * w_ + nx;
    return mb_available(mb, n) ? n : -1;
  }
  if (y < 0) return x < 0 ? d_ : (x < 16 ? b_ : c_);
  if (x < 0) return a_;
  return x < 16 ? mb : -1;  // right neighbour: later in decoding order
}

inline MbNeighbours::Nb MbNeighbours::motion_at(int mb, int x, int y, u16 done, int list) const {
  Nb r{false, -1, {0, 0}};
  const int m = mb_at(mb, x, y);
  if (m < 0) return r;
  const int blk = ((y & 15) >> 2) * 4 + ((x & 15) >> 2);
  if (m == mb && !((done >> blk) & 1)) return r;  // partition not yet decoded
  r.avail = true;
  const MbState& s = st_[size_t(m) & mask_];
  if (is_intra(s.kind)) return r;
  r.ref = s.ref[list][((blk >> 3) << 1) | ((blk & 3) >> 1)];
  if (r.ref < 0) return r;  // list unused: refIdx -1, mv 0
  r.mv[0] = s.mv[list][blk][0];
  r.mv[1] = s.mv[list][blk][1];
  return r;
}

inline void MbNeighbours::nb16(int list, Nb n[3]) const {
  const int nm[3] = {a_, b_, c_ >= 0 ? c_ : d_};
  const int nblk[3] = {3, 12, c_ >= 0 ? 12 : 15};
  for (int k = 0; k < 3; ++k) {
    n[k] = Nb{nm[k] >= 0, -1, {0, 0}};
    if (nm[k] < 0) continue;
    const MbState& s = st_[size_t(nm[k]) & mask_];
    if (is_intra(s.kind)) continue;
    const int b8 = ((nblk[k] >> 3) << 1) | ((nblk[k] & 3) >> 1);
    n[k].ref = s.ref[list][b8];
    if (n[k].ref < 0) continue;
    n[k].mv[0] = s.mv[list][nblk[k]][0];
    n[k].mv[1] = s.mv[list][nblk[k]][1];
  }
}

inline void MbNeighbours::pred_mv16(int list, int ref, int out[2]) const {
  Nb n[3];
  nb16(list, n);
  if (!n[1].avail && !n[2].avail && n[0].avail) n[1] = n[2] = n[0];
  const int match = (n[0].ref == ref) + (n[1].ref == ref) + (n[2].ref == ref);
  if (match == 1) {
    const Nb& t = n[0].ref == ref ? n[0] : (n[1].ref == ref ? n[1] : n[2]);
    out[0] = t.mv[0];
    out[1] = t.mv[1];
    return;
  }
  for (int c = 0; c < 2; ++c) {
    const int a = n[0].mv[c], b = n[1].mv[c], d = n[2].mv[c];
    const int lo = a < b ? a : b, hi = a < b ? b : a;
    out[c] = d < lo ? lo : (d > hi ? hi : d);  // median
  }
}

inline void MbNeighbours::direct_spatial_both(int ref[2], int mv[2][2]) const {
  // A: the left MB's block 3, B: the above MB's block 12, C: the above-right MB's block 12, or
  // D (the above-left MB's block 15) when C is unavailable (§8.4.1.3.2 for the whole MB)
  const int nm[3] = {a_, b_, c_ >= 0 ? c_ : d_};
  const int nblk[3] = {3, 12, c_ >= 0 ? 12 : 15};
  bool avail[3];
  int r[2][3];
  int v[2][3][2];
  for (int k = 0; k < 3; ++k) {
    avail[k] = nm[k] >= 0;
    for (int l = 0; l < 2; ++l) {
      r[l][k] = -1;
      v[l][k][0] = v[l][k][1] = 0;
    }
    if (!avail[k]) continue;
    const MbState& s = st_[size_t(nm[k]) & mask_];
    if (is_intra(s.kind)) continue;
    const int b8 = ((nblk[k] >> 3) << 1) | ((nblk[k] & 3) >> 1);
    for (int l = 0; l < 2; ++l) {
      r[l][k] = s.ref[l][b8];
      if (r[l][k] < 0) continue;
      v[l][k][0] = s.mv[l][nblk[k]][0];
      v[l][k][1] = s.mv[l][nblk[k]][1];
    }
  }
  auto minpos = [](int a, int b) { return (a >= 0 && b >= 0) ? (a < b ? a : b) : (a > b ? a : b); };
  // B and C unavailable, A available: B = C = A for the predictor (after refIdx is chosen)
  const bool only_a = !avail[1] && !avail[2] && avail[0];
  for (int l = 0; l < 2; ++l) {
    const int rf = minpos(r[l][0], minpos(r[l][1], r[l][2]));
    ref[l] = rf;
    mv[l][0] = mv[l][1] = 0;
    if (rf < 0) continue;
    if (only_a) {
      mv[l][0] = v[l][0][0];
      mv[l][1] = v[l][0][1];
      continue;
    }
    const int match = (r[l][0] == rf) + (r[l][1] == rf) + (r[l][2] == rf);
    if (match == 1) {
      const int k = r[l][0] == rf ? 0 : (r[l][1] == rf ? 1 : 2);
      mv[l][0] = v[l][k][0];
      mv[l][1] = v[l][k][1];
      continue;
    }
    for (int c = 0; c < 2; ++c) {
      const int a = v[l][0][c], b = v[l][1][c], d = v[l][2][c];
      const int lo = a < b ? a : b, hi = a < b ? b : a;
      mv[l][c] = d < lo ? lo : (d > hi ? hi : d);  // median
    }
  }
}

// Motion of a reference picture as the colocated picture of direct prediction (§8.4.1.2.1):
// per 4x4 block the vector and reference index of list 0 if the block used it, else of list 1,
// and the identity of the referenced picture. With direct_8x8_inference (every stream this
// decoder accepts that has B slices sets it in practice) only the outer corner block of each 8x8
// is ever read, so only those four blocks per MB are kept.
struct ColMotion {
  struct Blk {
    i16 mv[2];
    u32 pid;  // uid of the picture the block references
    i8 ref;   // refIdxCol (-1: intra / not available)
  };
  int wmbs = 0, hmbs = 0;
  bool corners = false;  // 4 entries per MB (8x8 outer corners), else 16 (raster 4x4 blocks)
  std::vector<Blk> b;
  // entry of raster 4x4 block `blk` of MB `mb` (corners: the block's 8x8)
  size_t index(int mb, int blk) const {
    return corners ? size_t(mb) * 4 + size_t(((blk >> 3) << 1) | ((blk & 3) >> 1)) : size_t(mb) * 16 + size_t(blk);
  }
};

// Colocated motion built as the MBs of a picture are stored (store_mb): the entries of one MB
// from its final state, with the picture uids of the current slice's reference lists.
struct ColBuild {
  ColMotion* col = nullptr;
  const std::array<std::vector<u32>, 2>* uids = nullptr;  // the current slice's list uids
  u32 uid_tab[2][32] = {};  // uids by refIdx (0 past the list), filled by set_uids
  void set_uids(const std::array<std::vector<u32>, 2>* u) {
    uids = u;
    for (int l = 0; l < 2; ++l)
      for (size_t k = 0; k < 32; ++k) uid_tab[l][k] = u && k < (*u)[size_t(l)].size() ? (*u)[size_t(l)][k] : 0u;
  }
  void store(int mb, const MbState& st);
  void none(int mb);  // intra / concealed: no motion
};

// Reference picture (DPB entry).
struct RefPic {
  int slot = -1;
  int frame_num = 0;
  int frame_num_wrap = 0;
  bool long_term = false;
  int lt_idx = 0;
  int poc = 0;
  u32 uid = 0;
  std::shared_ptr<const ColMotion> col;
  // field decoding: short-term / long-term reference fields of the frame (bit 0 top, bit 1
  // bottom; frame decoding uses `long_term` instead), their POCs and uids
  u8 fields = 3;
  u8 lt_fields = 0;
  int poc_f[2] = {0, 0};
  u32 uid_f[2] = {0, 0};
  std::shared_ptr<const ColMotion> col_f[2];  // each field's motion (B fields' direct prediction)
};

// Per-slice list entry (a RefPic snapshot).
struct ListEntry {
  int slot = -1;
  int poc = 0;
  bool long_term = false;
  u32 uid = 0;
  const ColMotion* col = nullptr;
};

// Stateful decoder of one H.264 stream (parameter sets, DPB marking, output order, neighbour
// state).
class Decoder {
 public:
  // Parse one access unit into a Picture (decode order). Throws UnsupportedStream for syntax
  // outside the supported subset and Error for corrupt data. `tag` is carried to the output.
  // `next_nal` (optional): parse from that NAL on and stop before a second picture of the access
  // unit (both fields of a pair in one access unit, as some packetizers deliver them), returning
  // where it starts (au.nals.size(): none left). Without it a second picture is an error.
  PicturePtr parse(const AccessUnit& au, i64 tag = 0, size_t* next_nal = nullptr);
  void absorb_parameter_sets(const AccessUnit& au);
  bool has_sps() const { return !sps_.empty(); }
  // Forget the DPB and the reorder buffer (e.g. after a failed picture): the next picture must
  // be an IDR.
  void reset_references();
  int dpb_slots() const { return dpb_slots_; }
  // Frames still waiting in the reorder buffer (flushed by the next IDR / end of stream).
  int pending_output() const { return int(pending_.size()); }
  // Output every pending frame now (end of stream); returns them in output order.
  std::vector<OutFrame> flush_output();

 private:
  struct Pending {
    OutFrame f;
    u32 epoch;  // IDR / MMCO5 period the picture belongs to (output order: epoch, then POC)
  };
  void build_lists(const SliceHdr& sh, const h264::Sps& sps, int cur_poc);
  void build_field_lists(const SliceHdr& sh, const h264::Sps& sps, int cur_poc);
  void mark_field(const SliceHdr& sh, const h264::Sps& sps, int slot, int poc, u32 uid, bool second,
                  std::shared_ptr<const ColMotion> col);
  void mark_references(const SliceHdr& sh, const h264::Sps& sps, int slot, int poc, u32 uid,
                       std::shared_ptr<const ColMotion> col);
  int pick_slot() const;
  int compute_poc(const SliceHdr& sh, const h264::Sps& sps);
  void bump(Picture& pic, const OutFrame& f, bool new_epoch, bool hard);
  OutFrame out_of(const Picture& pic) const;
  int reorder_depth(const h264::Sps& sps) const;
  void parse_slice_data(MbNeighbours& nb, Picture& pic, const SliceHdr& sh, const h264::Sps& sps,
                        const h264::Pps& pps, const u8* data, size_t n, size_t bitpos, int slice_idx,
                        const std::vector<ListEntry> (&lists)[2]);

  std::map<int, h264::Sps> sps_;
  std::map<int, h264::Pps> pps_;
  std::vector<u8> rbsp_;
  std::vector<u32> epb_;
  MbNeighbours nb_;
  std::vector<RefPic> dpb_;
  // buffer recycling (recycle.h): pictures in flight per camera (parse window + GPU stages)
  std::shared_ptr<Recycler<Picture>> pic_pool_ = Recycler<Picture>::make(12);
  std::shared_ptr<Recycler<ColMotion>> col_pool_ = Recycler<ColMotion>::make(8);
  std::vector<Pending> pending_;  // decoded, not yet output (POC order decides)
  std::vector<ListEntry> list_[2];  // refIdx -> entry of the current slice
  int max_lt_idx_ = -1;     // MaxLongTermFrameIdx ("no long-term frame indices" = -1)
  int dpb_slots_ = 2;
  int wmbs_ = 0, hmbs_ = 0;  // active picture size (changes only at an IDR)
  int bd_ = 8;               // active sample bit depth (changes only at an IDR)
  int cf_ = 1;               // active chroma format (2: 4:2:2; changes only at an IDR)
  bool have_idr_ = false;
  int pinned_slot_ = -1;    // newest output: kept until a newer one leaves the reorder buffer
  int last_out_poc_ = 0;
  i64 last_out_epoch_ = -1;
  u32 epoch_ = 0;
  int adaptive_reorder_ = 0;  // reorder depth learnt from the stream when the SPS gives none
  int reorder_cur_ = 0;       // reorder depth in force for the active SPS
  u32 next_uid_ = 1;
  // picture order count state (§8.2.1)
  int prev_poc_msb_ = 0, prev_poc_lsb_ = 0;
  int prev_frame_num_ = 0, prev_frame_num_offset_ = 0;
  bool prev_ref_mmco5_ = false;
  std::vector<std::vector<MbState>> spare_;  // recycled MbState arrays
  // Slices of one picture are parsed in parallel on the shared fan-out pool (fanout.h) when the
  // access unit holds several: each slice into its own neighbour state (other slices' MBs are
  // unavailable to it by definition, §6.4.11) and its own records shard, merged into the
  // picture in slice order (the records then equal a sequential parse's). VEP_AVC_SLICE_THREADS=0:
  // off.
  struct SliceUnit;
  bool parallel_slices_ = true;
  std::vector<std::unique_ptr<SliceUnit>> units_;
  u64 parallel_slices_run_ = 0;
  // Field pictures (PAFF): decided per IDR period (a stream mixing frame and field pictures in
  // one period is UnsupportedStream). A field pair shares frame slot `slot`; the frame is output
  // once its second field is decoded (or, unpaired, when the next frame starts).
  bool field_mode_ = false;
  struct OpenPair {
    bool open = false;
    int slot = -1, frame_num = 0, bottom = 0;
    int poc[2] = {0, 0};
    bool ref = false, boundary = false, hard = false;
    u8 have = 0;       // fields decoded (bit 0 top, bit 1 bottom)
    OutFrame f;        // the frame as output (info / au of the first field)
  } pair_;
  void close_pair(Picture& pic);  // output the open pair's frame through pic's outputs

 public:
  Decoder();
  ~Decoder();
  u64 parallel_slices_run() const { return parallel_slices_run_; }  // (tests)
  // reference-marking coverage (tests): MMCOs executed by operation, list modification commands
  // applied, pictures marked long-term
  u64 mmco_ops[7] = {0, 0, 0, 0, 0, 0, 0};
  u64 list_mods = 0, long_term_marked = 0;
  u64 redundant_slices_skipped = 0;
};

// CPU reference reconstruction of `pic` into DPB surfaces `slots` (coded size; references are
// read from the slots named by the MbRecs). Bit-exact with the GPU kernels.
void cpu_reconstruct(const Picture& pic, std::vector<HostSurface>& slots);
// Field pair -> frame (frame row r = row r >> 1 of field r & 1), 8-bit NV12.
void weave_fields(const HostSurface& top, const HostSurface& bottom, HostSurface& frame);

// ---- internals shared by the decoder and the encoder -------------------------------------
// Levels of one MB in scan order (luma per raster block; I16x16 AC at index 1..15 with the DC
// levels in `dc`; chroma AC at index 1..15).
// Only the blocks named by the masks are read (the decoder zeroes a block just before parsing
// into it, so nothing else needs initialising); update_masks() derives them from the arrays.
struct MbLevels {
  int luma[16][16];
  int dc[16];
  int cdc[2][4];
  int cac[2][4][16];
  u16 lmask = 0;   // luma blocks (raster) with levels in `luma`
  u8 cmask = 0;    // chroma AC blocks (c * 4 + b) with levels in `cac`
  u8 dcmask = 0;   // bit 0: Intra16x16 DC levels; bits 1-2: chroma DC of Cb / Cr
  void update_masks() {
    lmask = cmask = dcmask = 0;
    for (int r = 0; r < 16; ++r)
      for (int k = 0; k < 16; ++k)
        if (luma[r][k]) lmask |= u16(1u << r);
    for (int k = 0; k < 16; ++k)
      if (dc[k]) dcmask |= 1;
    for (int c = 0; c < 2; ++c)
      for (int b = 0; b < 4; ++b) {
        if (cdc[c][b]) dcmask |= u8(2 << c);
        for (int k = 0; k < 16; ++k)
          if (cac[c][b][k]) cmask |= u8(1u << (c * 4 + b));
      }
  }
};
// Dequantised residual blocks of one MB (16 luma raster, 4 Cb, 4 Cr) and their coded masks.
struct MbResidual {
  i16 blk[32][16];  // 16 luma 4x4 (raster), then chroma block k at 16 + k (MbRec::chroma_coded order)
  i16 b8[4][64];    // 8x8-transform luma blocks (raster 8x8 in each; t8 MBs)
  u16 luma = 0;     // coded luma 4x4 blocks (t8: all four blocks of each coded 8x8)
  u16 chroma = 0;
  bool t8 = false;
};
void dequantize_mb(const MbLevels& lv, bool i16x16, int qp, int qpc, MbResidual& out);
// Append MB `mb` to `pic`: coefficient blocks (or I_PCM samples), motion vectors and the
// bookkeeping fields of `m` (coef, mv, coded masks, nz from s.tc); stores pic.mbs[mb] = m.
// (m.nz is the caller's; wp = 4 WpEntry when m.flags has kMbWp)
void store_mb(Picture& pic, int mb, MbRec m, const MbState& s, const MbResidual* res, const u8* pcm,
              const WpEntry* wp = nullptr);
// store_mb() of a skipped MB without weights (P_Skip, B_Skip): `m` holds the header fields
// (kind, QPs, deblocking, slice, reference slots, kMbL1); no residual.
void store_skip_mb(Picture& pic, int mb, MbRec& m, const MbState& s);
void cpu_reconstruct_mb(const Picture& pic, int mb, std::vector<HostSurface>& slots);
void cpu_deblock(const Picture& pic, HostSurface& target);
// Neighbour samples for intra prediction from the surface being reconstructed.
void intra4x4_neighbours(const Picture& pic, int mb, int idx, const HostSurface& T, Intra4Nb& n);
void intra16_neighbours(const Picture& pic, int mb, const HostSurface& T, Intra16Nb& n);
void chroma_neighbours(const Picture& pic, int mb, int c, const HostSurface& T, IntraChromaNb& n);
// Filtered Intra_8x8 references of 8x8 block q: f[0] = p'[-1,-1], f[1..16] = p'[0..15,-1],
// f[17..24] = p'[-1,0..7].
void intra8x8_neighbours(const Picture& pic, int mb, int q, const HostSurface& T, int* f, bool& has_top,
                         bool& has_left);

// ------------------------------------------------------------------------------ encoders
// What the synthetic camera (synth.h) needs from an encoder.
class StreamEncoder {
 public:
  virtual ~StreamEncoder() = default;
  virtual std::shared_ptr<AccessUnit> next() = 0;
  // Encoder's own reconstruction of the last coded picture (what a conformant decoder must
  // output for it) and the source picture that was encoded (for PSNR).
  virtual const HostSurface& reconstruction() const = 0;
  virtual const HostSurface& source() const = 0;
  virtual i64 last_pts() const = 0;  // pts of the last access unit (B pictures: display time)
  // Escaped parameter-set NALs (what the muxers put in avcC / the FLV sequence header).
  virtual const std::vector<u8>& sps_nal() const = 0;
  virtual const std::vector<u8>& pps_nal() const = 0;
};

// Closed-loop synthetic H.264 encoder (CAVLC I/P): intra 16x16 / 4x4 and chroma prediction,
// motion-compensated P macroblocks (16x16, 16x8, 8x16, 8x8 with sub-partitions, P_Skip),
// multiple reference frames, residual coding and the deblocking filter — a real compressed
// stream for the camera farm and for decoder coverage. The scene is a static textured
// background with moving textured objects (known motion seeds the motion search).
struct AvcEncConfig {
  int width = 640, height = 480;
  int fps = 30, gop = 30;
  int idr_phase = 0;         // IDR when frame 0 or (frame + idr_phase) % gop == 0
  int qp = 28;
  int slices = 1;            // per picture (MB-row aligned)
  int refs = 1;              // max_num_ref_frames
  int objects = 3;
  u64 seed = 1;
  int deblock_idc = 0;       // disable_deblocking_filter_idc for every slice
  int alpha_off = 0, beta_off = 0;  // slice_alpha_c0_offset_div2 / slice_beta_offset_div2
  bool constrained_intra = false;
  int chroma_qp_offset = 0;
  bool coverage = false;     // randomised mode decisions: every MB type / partition / mode
  int pcm_rate = 0;          // percent of I_PCM macroblocks in coverage mode
  int nonref_rate = 0;       // percent of non-reference P pictures in coverage mode
  double noise = 3.0;        // background texture amplitude
  double temporal_noise = 0; // per-frame sensor noise amplitude (drives P-picture residual bits)
};

class AvcEncoder : public StreamEncoder {
 public:
  explicit AvcEncoder(const AvcEncConfig& cfg);
  ~AvcEncoder() override;
  std::shared_ptr<AccessUnit> next() override;
  const HostSurface& reconstruction() const override;
  const HostSurface& source() const override;
  i64 last_pts() const override;
  const AvcEncConfig& config() const { return cfg_; }
  const std::vector<u8>& sps_nal() const override;
  const std::vector<u8>& pps_nal() const override;

 private:
  struct Impl;
  AvcEncConfig cfg_;
  std::unique_ptr<Impl> p_;
};

// Closed-loop synthetic H.264 Main / High-profile encoder (avc_enc_high.cpp): CABAC or CAVLC;
// I, P and B pictures in mini-GOPs (anchor P, then the B pictures, the middle one a reference
// when `pyramid`); 8x8 transform with Intra_8x8; spatial / temporal direct; explicit (P and B)
// or implicit (B) weighted prediction; explicit scaling matrices. Every macroblock is written
// by the decoder's own macroblock layer and reconstructed by its reconstruction, so the
// encoder's pictures are what a conforming decoder outputs.
struct AvcHighConfig {
  int width = 640, height = 480;
  int fps = 30, gop = 30;
  int idr_phase = 0;          // IDR when display index 0 or (index + idr_phase) % gop == 0
  int bframes = 2;            // B pictures between anchors (0..4)
  bool pyramid = true;        // middle B of each mini-GOP is a reference (bframes >= 2)
  int refs = 2;               // P reference pictures searched / listed (1..8)
  int qp = 28;                // I / P; B pictures +1 (reference) / +2
  bool cabac = true;
  bool t8x8 = true;           // High profile: transform_8x8_mode + Intra_8x8
  bool weighted_p = false;    // explicit weighted prediction in P slices
  int weighted_b = 0;         // weighted_bipred_idc: 0 default, 1 explicit, 2 implicit
  bool direct_spatial = true; // B direct mode (false: temporal)
  bool scaling = false;       // explicit (non-flat) sequence scaling matrices
  int slices = 1;             // per picture (MB-row aligned)
  int deblock_idc = 0;
  int chroma_qp_offset = 0, second_chroma_qp_offset = 0;
  bool coverage = false;      // randomised decisions: every MB / sub-MB type, mode, transform
  bool interlaced = false;    // interlaced SPS (frame_mbs_only 0) coding frame pictures, with
                              // delta_pic_order_cnt_bottom (top field first)
  // Reference marking coverage (frame pictures): random ref_pic_list_modification commands
  // (short- and long-term), MMCO 1 / 2 / 3 / 4 / 6 and IDR long_term_reference_flag.
  bool marking = false;
  bool fields = false;        // (interlaced) code every frame as a field pair (PAFF): top field
                              // first; I / P, P / P anchors and non-reference B / B pairs; CAVLC,
                              // 4x4 transforms
  bool mono = false;          // 4:0:0 (monochrome, High profile): luma only, chroma decodes grey
  int bit_depth = 8;          // 9 / 10: High 10 profile (u16 samples; frame pictures only); qp may
                              // then go down to -6 * (bit_depth - 8)
  int chroma_format = 1;      // 2: 4:2:2 (High 4:2:2 profile; frame pictures, 8..10 bits)
  int objects = 3;
  double noise = 3.0, temporal_noise = 0.0;
  u64 seed = 1;
};

class AvcHighEncoder : public StreamEncoder {
 public:
  explicit AvcHighEncoder(const AvcHighConfig& cfg);
  ~AvcHighEncoder() override;
  std::shared_ptr<AccessUnit> next() override;  // coding order
  const HostSurface& reconstruction() const override;
  const HostSurface& source() const override;
  i64 last_pts() const override;
  i64 last_display_index() const;
  char last_type() const;  // 'I' / 'P' / 'B'
  const AvcHighConfig& config() const { return cfg_; }
  const std::vector<u8>& sps_nal() const override;
  const std::vector<u8>& pps_nal() const override;

 private:
  struct Impl;
  AvcHighConfig cfg_;
  std::unique_ptr<Impl> p_;
};

}  // namespace vep::avc
