// Synthetic camera: a conformant H.264 Baseline encoder emitting IDR pictures of I_PCM
// macroblocks and P pictures of P_Skip + I_PCM macroblocks (a moving object over a static
// random background) — or, with `codec = kH265`, a conformant HEVC Main encoder (CABAC) emitting
// the same pictures as 16x16 CTBs of PCM CUs (IDR_W_RADL) and skip + PCM CUs (TRAIL_R).
// Lets every BASELINE.json config run without cameras or network.
//
// The reference had no synthetic source at all — its tests used real cameras
// (README.md:117-239).
#pragma once

#include "avc.h"
#include "codec.h"

namespace vep {

struct SynthConfig {
  int width = 640, height = 480;
  int fps = 30;
  int gop = 30;            // IDR period in frames
  double motion = 0.05;    // fraction of the picture covered by the moving object
  u64 seed = 1;
  int slices = 1;          // slices per picture (MB-row aligned)
  bool zero_samples = false;  // allow 0x00 PCM samples (forces emulation-prevention bytes)
  int idr_phase = 0;       // GOP phase offset (IDR when (frame + phase) % gop == 0, and frame 0)
  Codec codec = Codec::kH264;
  int merge_cands = 1;     // HEVC MaxNumMergeCand (merge_idx coded when > 1)
  // Emit a real compressed stream instead of the I_PCM / P_Skip fast-path subset: H.264 per
  // `profile` below, H.265 Main (CABAC CTU trees, intra / merge / AMVP / B, deblocking, SAO:
  // hevc::HevcEncoder).
  bool compressed = false;
  int qp = 28;
  int refs = 1;            // max_num_ref_frames
  int objects = 3;         // moving textured objects in the compressed scene
  int deblock_idc = 0;     // disable_deblocking_filter_idc
  bool coverage = false;   // randomised mode decisions (decoder coverage streams)
  double noise = 3.0;      // static texture amplitude of the compressed scene
  double temporal_noise = 0.0;  // per-frame sensor noise (P-picture residual, bitrate)
  // Compressed H.264 profile: "baseline" (CAVLC I/P, avc::AvcEncoder), "main" (CABAC, B
  // pictures) or "high" (main + 8x8 transform / Intra_8x8) — avc::AvcHighEncoder.
  std::string profile = "baseline";
  int bframes = 2;           // main / high: B pictures between anchors (pyramid when >= 2)
  bool cabac = true;         // main / high entropy coder (false: CAVLC)
  bool weighted_p = false;   // main / high: explicit weighted prediction in P slices
  int weighted_b = 0;        // main / high: weighted_bipred_idc
  bool direct_spatial = true;
  // H.265 stream structure / tools (hevc::HevcEncConfig; weighted_p turns on HEVC weighted
  // prediction in P and B slices)
  int tile_cols = 1, tile_rows = 1;
  bool wpp = false;
  int segments = 1;
  bool scaling_lists = false;
  bool long_term = false;
  bool open_gop = false;  // H.265: CRA + RASL pictures at every IRAP after the first
  bool lossless = false;
  int bit_depth = 8;         // 10: H.265 Main10 / H.264 High 10 (main / high profiles; 10-bit samples)
  int chroma_format = 1;     // 2: H.264 4:2:2 (High 4:2:2; main / high profiles, progressive)
  // main / high H.264: 1 = interlaced SPS coding frame pictures, 2 = every frame a field pair
  // (PAFF: CAVLC, 4x4 transforms, B pairs non-reference; overrides cabac / the 8x8 transform)
  int interlaced = 0;
  bool mono = false;  // High profile: 4:0:0 (monochrome) stream
};

class SynthH264 {  // (both codecs; the name predates H.265 support)
 public:
  explicit SynthH264(const SynthConfig& cfg);
  std::shared_ptr<AccessUnit> next();
  // ground truth of the last AU (compressed streams: the encoder's reconstruction, i.e. what a
  // conforming decoder outputs)
  const HostSurface& picture() const { return avc_ ? avc_->reconstruction() : pic_; }
  // the scene that was encoded (compressed streams: the encoder's source picture)
  const HostSurface& source() const { return avc_ ? avc_->source() : pic_; }
  // pts of the last AU (compressed streams with B pictures: the display time of `picture()`)
  i64 last_pts() const { return avc_ ? avc_->last_pts() : frame_ * 90000 / cfg_.fps; }
  const std::vector<u8>& sps_nal() const { return sps_nal_; }
  const std::vector<u8>& pps_nal() const { return pps_nal_; }
  const std::vector<u8>& vps_nal() const { return vps_nal_; }  // H.265 only
  const SynthConfig& config() const { return cfg_; }
  i64 frame_index() const { return frame_; }

 private:
  struct Rect { int x0, y0, x1, y1; };
  u64 rnd();
  void paint_background();
  void paint_box(const Rect& r);
  Rect box_at(i64 f) const;
  void pcm_payload(int mb, u8* out) const;
  std::vector<u8> encode_slice(bool idr, int mb0, int mb1, const std::vector<u8>& coded);
  std::vector<u8> encode_slice_hevc(bool idr, int ctb0, int ctb1, const std::vector<u8>& coded);

  SynthConfig cfg_;
  h264::Sps sps_;
  h264::Pps pps_;
  hevc::Vps hvps_;
  hevc::Sps hsps_;
  hevc::Pps hpps_;
  std::vector<u8> sps_nal_, pps_nal_, vps_nal_;
  std::vector<u8> skip_;  // HEVC per-CTB cu_skip_flag of the picture being encoded
  int poc_ = 0;
  HostSurface pic_, bg_;
  int wmbs_, hmbs_, bw_, bh_;
  i64 frame_ = -1;
  int idr_id_ = 0, frame_num_ = 0;
  u64 state_;
  Rect prev_box_{0, 0, 0, 0};
  std::unique_ptr<avc::StreamEncoder> avc_;  // compressed H.264 streams
};

}  // namespace vep
