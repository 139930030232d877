// Access units, the native H.264 macroblock-layer parser and the CPU reference reconstructor.
//
// Split of work (MI355X-first): the CPU does what is inherently serial — NAL parsing and the
// CAVLC macroblock-layer walk — and emits a compact, 16-byte-aligned *MB update list*
// (dense per-MB slot map + 384-byte sample slots). Reconstruction + colour conversion run as
// one batched HIP kernel over all cameras of a GPU (gpu_kernels.hip).
//
// Native subset decoder: I_PCM macroblocks in I/P slices and P_Skip (zero-MV, single
// reference, every picture a reference picture). This is the decodable subset emitted by the
// synthetic camera farm (synth.h). Anything else is reported as unsupported so a
// RocDecode/VCN backend can take the stream (SURVEY.md §7.4 hard part 1).
//
// Reference parity: python/read_image.py:47-133 (decode loop), :70-85 (GOP catch-up).
#pragma once

#include <map>
#include <memory>

#include "common.h"
#include "h264.h"
#include "hevc.h"
#include "hostmem.h"

namespace vep {

enum class Codec : int { kH264 = 0, kH265 = 1 };

// One demuxed packet ≈ PyAV Packet (python/rtsp_to_rtmp.py:92).
struct AccessUnit {
  Codec codec = Codec::kH264;
  std::vector<u8> data;                         // escaped NAL payloads, back to back
  std::vector<std::pair<u32, u32>> nals;        // (offset, size) into data, no start codes
  i64 pts = 0, dts = 0, duration = 0;           // 90 kHz
  bool keyframe = false;
  bool corrupt = false;
  i64 arrival_ms = 0;
  u64 seq = 0;                                  // per-camera packet counter

  void add_nal(const u8* p, size_t n) {
    VEP_CHECK(!pinned_, "access unit is finalised");
    nals.emplace_back(u32(data.size()), u32(n));
    data.insert(data.end(), p, p + n);
  }
  const u8* base() const { return pinned_ ? pinned_.get() : data.data(); }
  const u8* nal(size_t i) const { return base() + nals[i].first; }
  size_t nal_size(size_t i) const { return nals[i].second; }
  size_t bytes() const { return pinned_ ? pinned_len_ : data.size(); }
  // Finalise into device-accessible pinned memory (hostmem.h) so the GPU can read the slice
  // bytes in place; the emulation-prevention scan is fused into the copy (each chunk is scanned
  // while hot in cache), so the parser never makes its own pass over the bytes. Call before the
  // AU is shared with other threads. Without a pool only the scan is done.
  bool pin();
  bool pinned() const { return bool(pinned_); }
  // EPB positions (indices of the 0x03 bytes, relative to the NAL) recorded by pin(); false if
  // the AU was never scanned.
  bool epb_of(size_t i, const u32** begin, const u32** end) const {
    if (epb_idx_.empty()) return false;
    *begin = epb_.data() + epb_idx_[i];
    *end = epb_.data() + epb_idx_[i + 1];
    return true;
  }

 private:
  std::shared_ptr<u8> pinned_;
  size_t pinned_len_ = 0;
  std::vector<u32> epb_, epb_idx_;
};
using AuPtr = std::shared_ptr<const AccessUnit>;

// Latest escaped parameter-set NALs of a stream (VPS only for H.265): what the muxers need for
// avcC / hvcC and the FLV / enhanced-RTMP sequence header.
struct ParamSets {
  Codec codec = Codec::kH264;
  std::vector<u8> vps, sps, pps;
  void absorb(const u8* nal, size_t n);  // no-op for non-parameter-set NALs
  void absorb(const AccessUnit& au) {
    codec = au.codec;
    for (size_t i = 0; i < au.nals.size(); ++i) absorb(au.nal(i), au.nal_size(i));
  }
  bool complete() const {
    return !sps.empty() && !pps.empty() && (codec == Codec::kH264 || !vps.empty());
  }
  // Cropped output size from the SPS ({0, 0} if absent or unparsable).
  std::pair<int, int> size() const;
};

// Accumulated macroblock updates for one camera surface; several AUs of a GOP can be
// collapsed into one update (latest writer wins), which is how GOP catch-up
// (read_image.py:80-85) becomes a single batched GPU launch.
struct MbUpdate {
  int width_mbs = 0, height_mbs = 0;
  std::vector<i32> slot;          // per MB: payload slot or -1 (keep reference sample)
  std::vector<const u8*> src;     // per slot: the MB's 384 sample bytes, *in place* in the AU
                                  // bitstream (no parse-time copy) or in an unescaped RBSP
  std::vector<AuPtr> keep;        // AUs that `src` points into
  std::vector<std::shared_ptr<const std::vector<u8>>> own;  // unescaped RBSPs `src` points into
  std::vector<i32> coded;         // MBs with a slot, in first-coded order (raster per AU)
  // Contiguous byte ranges (slice RBSPs) the blocks live in: the GPU path ships whole
  // segments (one large copy each) plus a per-MB offset table instead of gathering blocks.
  struct Segment {
    const u8* base;
    size_t len;
  };
  std::vector<Segment> segs;
  std::vector<u32> slot_seg;      // per slot: index into segs
  int nslots = 0;
  int frames = 0;                 // AUs folded in

  void reset(int wmbs, int hmbs) {
    width_mbs = wmbs;
    height_mbs = hmbs;
    slot.assign(size_t(wmbs) * hmbs, -1);
    clear_payload();
  }
  void clear_payload() {
    if (coded.size() * 8 < slot.size()) {
      for (i32 mb : coded) slot[size_t(mb)] = -1;  // sparse reset
    } else {
      std::fill(slot.begin(), slot.end(), -1);
    }
    src.clear();
    keep.clear();
    own.clear();
    coded.clear();
    segs.clear();
    slot_seg.clear();
    nslots = 0;
    frames = 0;
  }
  int mbs() const { return width_mbs * height_mbs; }
  // Pre-size the per-slot arrays (a slice of n bytes holds at most n / 384 PCM blocks) so a
  // keyframe's 8k+ blocks do not go through a chain of reallocations.
  void reserve_blocks(size_t n) {
    n = std::min(n, size_t(mbs()));
    src.reserve(src.size() + n);
    slot_seg.reserve(slot_seg.size() + n);
    coded.reserve(coded.size() + n);
  }
  void begin_segment(const u8* base, size_t len) { segs.push_back({base, len}); }
  // Latest writer wins: a MB coded again later in a collapsed GOP re-points its slot.
  // `p` must lie in the most recently begun segment.
  void set(int mb, const u8* p) { set_in(mb, p, u32(segs.size() - 1)); }
  // A run of blocks of consecutive MBs at a fixed stride (all in segment `seg`).
  void set_run(int mb0, int count, const u8* p, size_t stride, u32 seg) {
    bool fresh = true;  // common case (a keyframe slice): no MB of the run coded yet
    for (int k = 0; k < count && fresh; ++k) fresh = slot[size_t(mb0 + k)] < 0;
    if (!fresh) {
      for (int k = 0; k < count; ++k) set_in(mb0 + k, p + size_t(k) * stride, seg);
      return;
    }
    const size_t base = src.size();
    src.resize(base + size_t(count));
    slot_seg.resize(base + size_t(count), seg);
    coded.resize(base + size_t(count));
    for (int k = 0; k < count; ++k) {
      slot[size_t(mb0 + k)] = nslots + k;
      src[base + size_t(k)] = p + size_t(k) * stride;
      coded[base + size_t(k)] = mb0 + k;
    }
    nslots += count;
  }
  void set_in(int mb, const u8* p, u32 seg) {
    int s = slot[size_t(mb)];
    if (s < 0) {
      slot[size_t(mb)] = nslots++;
      src.push_back(p);
      slot_seg.push_back(seg);
      coded.push_back(mb);
    } else {
      src[size_t(s)] = p;
      slot_seg[size_t(s)] = seg;
    }
  }
  const u8* block(int s) const { return src[size_t(s)]; }
};

// Picture-level metadata produced by the parser (fills VideoFrame fields).
struct PictureInfo {
  int width = 0, height = 0;          // cropped output size
  int coded_width = 0, coded_height = 0;
  int crop_left = 0, crop_top = 0;
  char pict_type = '?';
  bool idr = false;
  int frame_num = 0;
  int coded_mbs = 0;                  // non-skipped MBs in this AU
  double fps = 0;
  // Speculative I-slice walk (H264Parser::set_speculate): payload slots [spec_lo, spec_hi) were
  // placed by arithmetic (uniform 386-byte I_PCM records, byte-exact slice length) without
  // reading their headers; the consumer (GPU kernel / CPU path) must check that each such
  // block is preceded by the I_PCM header bytes 0D 00 before the frame is published.
  int spec_lo = 0, spec_hi = 0;
  bool speculative() const { return spec_hi > spec_lo; }
};

class UnsupportedStream : public Error {
 public:
  using Error::Error;
};

struct BlockSink;  // per-slice PCM block collector (codec.cpp)

// Stateful H.264 AU parser (keeps SPS/PPS tables across AUs).
class H264Parser {
 public:
  // Parse one AU; macroblock updates are folded into `upd` (resized to the stream when
  // needed). `upd.src` points into `au`'s bytes: the caller keeps the AU alive (upd.keep).
  // Throws UnsupportedStream for syntax outside the subset.
  PictureInfo parse(const AccessUnit& au, MbUpdate& upd);
  // Parameter sets only (no slice walk) — cheap keyframe/size probe.
  void absorb_parameter_sets(const AccessUnit& au);
  bool has_sps() const { return !sps_.empty(); }
  const h264::Sps& active_sps() const;
  const std::vector<u8>& last_sps_nal() const { return sps_nal_; }
  const std::vector<u8>& last_pps_nal() const { return pps_nal_; }
  // Allow the header-free I-slice walk for the next parse (single-AU jobs whose consumer
  // verifies the headers, see PictureInfo::spec_lo).
  void set_speculate(bool on) { speculate_ = on; }

 private:
  bool speculate_ = false;
  int spec_lo_ = 0, spec_hi_ = 0;
  void walk_slice(const u8* rbsp, size_t n, const h264::SliceHeader& sh, BitReader& br,
                  const h264::Sps& sps, BlockSink& upd, int& coded);
  std::map<int, h264::Sps> sps_;
  std::map<int, h264::Pps> pps_;
  int active_sps_id_ = -1;
  std::vector<u8> sps_nal_, pps_nal_;
  std::vector<u8> rbsp_scratch_;
  std::vector<u32> epb_;
};

// Stateful H.265 AU parser: the CABAC coding-tree walk of the native HEVC subset — 16x16 CTBs
// (= minimum CU = PCM CU size), PCM intra CUs, skipped inter CUs with a single reference and
// zero merge candidates, no SAO/deblocking. PCM CU samples are laid out exactly like an H.264
// I_PCM macroblock (256 luma, 64 Cb, 64 Cr), so the same MbUpdate / GPU kernel reconstructs
// both codecs. Everything else throws UnsupportedStream.
class H265Parser {
 public:
  PictureInfo parse(const AccessUnit& au, MbUpdate& upd);
  void absorb_parameter_sets(const AccessUnit& au);
  bool has_sps() const { return !sps_.empty(); }
  const hevc::Sps& active_sps() const;

 private:
  void store_parameter_set(int type, const u8* p, size_t n);
  void walk_slice(const u8* rbsp, size_t n, const hevc::SliceHeader& sh, const hevc::Sps& sps,
                  const hevc::Pps& pps, BlockSink& upd, int& coded);
  std::map<int, hevc::Vps> vps_;
  std::map<int, hevc::Sps> sps_;
  std::map<int, hevc::Pps> pps_;
  int active_sps_id_ = -1;
  std::vector<u8> rbsp_scratch_;
  std::vector<u32> epb_;
  std::vector<u8> skip_;  // per-CTB cu_skip_flag of the current picture (ctxInc derivation)
};

// Codec dispatcher used by cameras (the codec comes from the SDP / AU).
class StreamParser {
 public:
  PictureInfo parse(const AccessUnit& au, MbUpdate& upd, bool speculate = false) {
    codec_ = au.codec;
    if (au.codec == Codec::kH265) return h265_.parse(au, upd);
    h264_.set_speculate(speculate);
    return h264_.parse(au, upd);
  }
  void absorb_parameter_sets(const AccessUnit& au) {
    codec_ = au.codec;
    if (au.codec == Codec::kH265) h265_.absorb_parameter_sets(au);
    else h264_.absorb_parameter_sets(au);
  }
  bool has_sps() const { return codec_ == Codec::kH265 ? h265_.has_sps() : h264_.has_sps(); }
  Codec codec() const { return codec_; }
  H264Parser& h264() { return h264_; }
  H265Parser& h265() { return h265_; }

 private:
  Codec codec_ = Codec::kH264;
  H264Parser h264_;
  H265Parser h265_;
};

// Host NV12 surface (CPU backend / test oracle).
struct HostSurface {
  int coded_w = 0, coded_h = 0;
  std::vector<u8> y, uv;  // NV12
  // High bit depth (HEVC Main10): the same NV12 layout with one u16 per sample (LSB-aligned);
  // y / uv stay empty. bd = the sample bit depth of the storage (8: u8 planes).
  int bd = 8;
  std::vector<u16> y16, uv16;
  // chroma format: 1 (and 0, grey chroma) NV12; 2 = 4:2:2 (H.264 High 4:2:2): NV16, the
  // interleaved chroma plane has coded_h rows
  int cf = 1;
  bool wide() const { return bd > 8; }
  int chroma_rows() const { return cf == 2 ? coded_h : coded_h / 2; }
  void alloc(int w, int h, int bit_depth = 8, int chroma_format = 1) {
    coded_w = w;
    coded_h = h;
    bd = bit_depth;
    cf = chroma_format == 2 ? 2 : 1;
    const size_t nc = size_t(w) * size_t(chroma_rows());
    if (bd > 8) {
      y.clear();
      uv.clear();
      y16.assign(size_t(w) * h, u16(16 << (bd - 8)));
      uv16.assign(nc, u16(128 << (bd - 8)));
    } else {
      y16.clear();
      uv16.clear();
      y.assign(size_t(w) * h, 16);
      uv.assign(nc, 128);
    }
  }
  // sample of component c (0 Y, 1 Cb, 2 Cr) at component coordinates (x, y)
  int get(int c, int x, int yy) const {
    const size_t i = c == 0 ? size_t(yy) * coded_w + size_t(x) : size_t(yy) * coded_w + size_t(2 * x + c - 1);
    if (bd > 8) return c == 0 ? y16[i] : uv16[i];
    return c == 0 ? y[i] : uv[i];
  }
  void set(int c, int x, int yy, int v) {
    const size_t i = c == 0 ? size_t(yy) * coded_w + size_t(x) : size_t(yy) * coded_w + size_t(2 * x + c - 1);
    if (bd > 8) (c == 0 ? y16 : uv16)[i] = u16(v);
    else (c == 0 ? y : uv)[i] = u8(v);
  }
};

// 8-bit NV12 copy of a high bit depth and / or 4:2:2 surface: the form the BGR24 conversion and
// the letterbox read. 4:2:2 chroma rows are averaged in pairs, (a + b + 1) >> 1 at the source
// depth; then samples above 8 bits are rounded to nearest, saturating. An 8-bit 4:2:0 surface is
// copied as is.
void narrow_surface(const HostSurface& s, HostSurface& out);

// CPU reference of the fused GPU kernel: apply MB update to the NV12 surface, then convert the
// cropped picture to packed BGR24 (out must hold width*height*3 bytes).
void cpu_apply_update(const MbUpdate& upd, HostSurface& s);
void cpu_nv12_to_bgr(const HostSurface& s, int crop_left, int crop_top, int width, int height,
                     u8* out);

}  // namespace vep
