// Native H.264 macroblock-layer parser (CAVLC, I_PCM + P_Skip subset) and CPU reference
// reconstruction. See codec.h for the CPU/GPU split.
#include <algorithm>
#include "codec.h"

#include "cabac.h"
#include "color.h"

namespace vep {

using namespace h264;

// ------------------------------------------------------------------------------ AccessUnit

bool AccessUnit::pin() {
  if (pinned_) return true;
  std::shared_ptr<u8> b = hostmem::pinned_block(data.size());
  u8* dst = b ? b.get() : nullptr;
  constexpr size_t kChunk = size_t(256) << 10;
  std::vector<u32> tmp;
  epb_.clear();
  epb_idx_.assign(1, 0);
  for (size_t i = 0; i < nals.size(); ++i) {
    const size_t off = nals[i].first, n = nals[i].second;
    for (size_t c = 0; c < n; c += kChunk) {
      const size_t len = std::min(kChunk, n - c);
      const u8* src = data.data() + off + c;
      if (dst) std::memcpy(dst + off + c, src, len);
      // window reaches 2 bytes back so a 00 00 03 split by the chunk edge is still seen; an
      // EPB needs its two zero bytes right before it, so windows cannot disagree with a
      // sequential scan
      const size_t back = std::min<size_t>(c, 2);
      find_epb(data.data() + off + c - back, len + back, tmp);
      for (u32 e : tmp)
        if (e >= back) epb_.push_back(u32(c + e - back));
    }
    epb_idx_.push_back(u32(epb_.size()));
  }
  if (!b) return false;
  pinned_len_ = data.size();
  pinned_ = std::move(b);
  std::vector<u8>().swap(data);
  return true;
}

static const u8* rbsp_of(const u8* nal, size_t n, std::vector<u32>& epb,
                         std::vector<u8>& scratch, size_t& out_n, const u32* known_b = nullptr,
                         const u32* known_e = nullptr) {
  if (known_b) epb.assign(known_b, known_e);  // scanned at ingest (AccessUnit::pin)
  else find_epb(nal, n, epb);
  if (epb.empty()) {
    out_n = n;
    return nal;
  }
  // unescape with one memcpy per run between emulation-prevention bytes
  scratch.resize(n);
  size_t o = 0, from = 0;
  for (u32 e : epb) {
    std::memcpy(scratch.data() + o, nal + from, e - from);
    o += e - from;
    from = size_t(e) + 1;
  }
  std::memcpy(scratch.data() + o, nal + from, n - from);
  out_n = o + (n - from);
  return scratch.data();
}

// Collects the PCM blocks of one slice NAL. Without emulation-prevention bytes the RBSP is the
// NAL itself and blocks are referenced in place. With EPBs the walk runs on the unescaped
// scratch copy; resolve() maps each block back into the escaped NAL (RBSP offset + number of
// EPBs before it) — still in place — unless an EPB falls inside the block, in which case its
// 384 bytes go to a small owned buffer. No whole-slice copy survives the parse.
struct BlockSink {
  MbUpdate& upd;
  const u8* rbsp;
  bool direct;
  std::vector<std::pair<int, u32>> pending;  // (mb, RBSP offset), increasing offsets

  void add(int mb, const u8* p) {
    if (direct) upd.set(mb, p);
    else pending.emplace_back(mb, u32(p - rbsp));
  }
  void add_run(int mb0, int count, const u8* p, size_t stride) {
    if (direct) {
      upd.set_run(mb0, count, p, stride, u32(upd.segs.size() - 1));
    } else {
      for (int k = 0; k < count; ++k) add(mb0 + k, p + size_t(k) * stride);
    }
  }
  void resolve(const u8* nal, const std::vector<u32>& epb) {
    if (direct || pending.empty()) return;
    const u32 seg = u32(upd.segs.size() - 1);  // the NAL's segment (begun by the caller)
    size_t k = 0, straddle = 0;
    // pass 1: count blocks an EPB splits (their RBSP bytes are not contiguous in the NAL)
    auto q = [&](size_t i) { return size_t(epb[i]) - i; };  // RBSP position after EPB i
    for (auto& [mb, off] : pending) {
      while (k < epb.size() && q(k) <= off) ++k;
      if (k < epb.size() && q(k) < size_t(off) + kPcmMbBytes) ++straddle;
    }
    std::shared_ptr<std::vector<u8>> own;
    u32 own_seg = 0;
    if (straddle) {
      own = std::make_shared<std::vector<u8>>(straddle * kPcmMbBytes);
      upd.own.push_back(own);
      upd.begin_segment(own->data(), own->size());
      own_seg = u32(upd.segs.size() - 1);
    }
    k = 0;
    size_t o = 0;
    for (auto& [mb, off] : pending) {
      while (k < epb.size() && q(k) <= off) ++k;
      if (k < epb.size() && q(k) < size_t(off) + kPcmMbBytes) {
        u8* dst = own->data() + o * kPcmMbBytes;
        std::memcpy(dst, rbsp + off, kPcmMbBytes);
        upd.set_in(mb, dst, own_seg);
        ++o;
      } else {
        upd.set_in(mb, nal + off + k, seg);
      }
    }
  }
};

void H264Parser::absorb_parameter_sets(const AccessUnit& au) {
  for (size_t i = 0; i < au.nals.size(); ++i) {
    const u8* p = au.nal(i);
    size_t n = au.nal_size(i);
    if (n < 2) continue;
    int t = nal_type(p[0]);
    if (t != kNalSps && t != kNalPps) continue;
    size_t rn;
    const u8* r = rbsp_of(p, n, epb_, rbsp_scratch_, rn);
    if (t == kNalSps) {
      Sps s = parse_sps(r, rn);
      sps_[s.sps_id] = s;
      sps_nal_.assign(p, p + n);
    } else {
      Pps q = parse_pps(r, rn);
      pps_[q.pps_id] = q;
      pps_nal_.assign(p, p + n);
    }
  }
}

const Sps& H264Parser::active_sps() const {
  auto it = sps_.find(active_sps_id_ < 0 ? sps_.begin()->first : active_sps_id_);
  VEP_CHECK(it != sps_.end(), "no active SPS");
  return it->second;
}

void H264Parser::walk_slice(const u8* rbsp, size_t n, const SliceHeader& sh, BitReader& br,
                            const Sps& sps, BlockSink& upd, int& coded) {
  (void)rbsp;
  (void)n;
  const int total = sps.width_mbs * sps.height_mbs();
  const size_t stop = br.stop_bit_pos();
  const int st = sh.slice_type % 5;
  const bool is_i = (st == kI);
  VEP_CHECK(is_i || st == kP, "only I and P slices are supported by the native decoder");
  const u32 pcm_type = is_i ? 25u : 30u;  // I_PCM (Table 7-11) / offset by 5 in P slices
  // Byte-aligned fast path: after a PCM macroblock the reader is byte aligned, and the next
  // macroblock header is a fixed 2-byte pattern — I slice: ue(25) + 7 alignment zeros = 0D 00;
  // P slice: ue(0) skip run + ue(30) + 6 zeros = 87 C0. Peeking two bytes replaces the bit-level
  // Exp-Golomb walk for the common case; anything else takes the general path below.
  const u8 f0 = is_i ? 0x0D : 0x87, f1 = is_i ? 0x00 : 0xC0;
  const u8* base = br.data();
  const size_t nbytes = br.size();
  int mb = sh.first_mb;
  bool more = true;
  do {
    if (br.byte_aligned()) {
      size_t off = br.bytepos();
      // Speculative walk: an I slice whose remaining bytes are exactly k I_PCM records plus
      // the one-byte trailing 0x80 is taken as k PCM MBs without touching the 2-byte headers
      // in between (each would be a cold cache miss). Only the first and last headers are
      // read here; the consumer checks every other one (spec_lo/spec_hi) before publishing.
      constexpr size_t rec = 2 + kPcmMbBytes;
      if (is_i && speculate_ && upd.direct && spec_hi_ == spec_lo_ && (stop & 7) == 0) {
        const size_t end = stop >> 3;
        if (end > off && (end - off) % rec == 0 && base[end] == 0x80 && base[off] == f0 &&
            base[off + 1] == f1 && base[end - rec] == f0 && base[end - rec + 1] == f1) {
          const int k = int((end - off) / rec);
          VEP_CHECK(mb + k <= total, "macroblock address past end of picture");
          spec_lo_ = upd.upd.nslots;
          upd.add_run(mb, k, base + off + 2, rec);
          spec_hi_ = upd.upd.nslots;
          if (spec_hi_ - spec_lo_ != k)  // a slice re-coding MBs of an earlier slice
            throw UnsupportedStream("overlapping slices in one picture");
          coded += k;
          br.seek_byte(end);
          break;
        }
      }
      while (off + 2 + kPcmMbBytes <= nbytes && base[off] == f0 && base[off + 1] == f1 &&
             (off + 2) * 8 < stop) {
        VEP_CHECK(mb < total, "macroblock address past end of picture");
        // the headers sit 386 B apart: a cold slice is one DRAM miss per MB, so keep ~16 in
        // flight (prefetch past the end of the buffer is harmless on x86 and never faults)
        __builtin_prefetch(base + off + 64 * (2 + kPcmMbBytes));
        upd.add(mb, base + off + 2);
        ++coded;
        ++mb;
        off += 2 + kPcmMbBytes;
      }
      br.seek_byte(off);
      if (br.bitpos() >= stop) break;
    }
    int run = 0;
    if (!is_i) {
      run = int(br.ue());
      VEP_CHECK(mb + run <= total, "mb_skip_run past end of picture");
      mb += run;  // P_Skip with zero MV on an all-skip neighbourhood == keep reference MB
      if (run > 0) more = br.bitpos() < stop;
    }
    if (more) {
      VEP_CHECK(mb < total, "macroblock address past end of picture");
      u32 mbt = br.ue();
      if (mbt != pcm_type)
        throw UnsupportedStream("unsupported mb_type " + std::to_string(mbt) +
                                " (native subset decoder handles I_PCM and P_Skip only)");
      br.align();
      size_t off = br.bytepos();
      VEP_CHECK(off + kPcmMbBytes <= br.size(), "truncated PCM macroblock");
      upd.add(mb, base + off);
      br.skip(kPcmMbBytes * 8);
      ++coded;
    }
    more = br.bitpos() < stop;
    ++mb;
  } while (more);
}

PictureInfo H264Parser::parse(const AccessUnit& au, MbUpdate& upd) {
  PictureInfo pi;
  bool got_slice = false;
  spec_lo_ = spec_hi_ = 0;
  for (size_t i = 0; i < au.nals.size(); ++i) {
    const u8* p = au.nal(i);
    size_t n = au.nal_size(i);
    if (n < 2) continue;
    int t = nal_type(p[0]);
    if (t == kNalSps || t == kNalPps) {
      size_t rn;
      const u8* r = rbsp_of(p, n, epb_, rbsp_scratch_, rn);
      if (t == kNalSps) {
        Sps s = parse_sps(r, rn);
        sps_[s.sps_id] = s;
        sps_nal_.assign(p, p + n);
      } else {
        Pps q = parse_pps(r, rn);
        pps_[q.pps_id] = q;
        pps_nal_.assign(p, p + n);
      }
      continue;
    }
    if (t != kNalSlice && t != kNalIdr) continue;
    size_t rn;
    const u32 *kb = nullptr, *ke = nullptr;
    au.epb_of(i, &kb, &ke);
    const u8* r = rbsp_of(p, n, epb_, rbsp_scratch_, rn, kb, ke);
    BitReader br(r + 1, rn - 1);
    // peek pps id to locate parameter sets
    BitReader peek(r + 1, rn - 1);
    peek.ue();
    peek.ue();
    int pps_id = int(peek.ue());
    auto pit = pps_.find(pps_id);
    if (pit == pps_.end()) throw UnsupportedStream("slice references unknown PPS");
    auto sit = sps_.find(pit->second.sps_id);
    if (sit == sps_.end()) throw UnsupportedStream("slice references unknown SPS");
    const Sps& sps = sit->second;
    const Pps& pps = pit->second;
    // anything beyond the I_PCM / P_Skip subset goes to the general decoder (avc.h)
    if (pps.cabac) throw UnsupportedStream("CABAC slices (general decoder)");
    if (pps.transform_8x8_mode || sps.scaling_matrix_present || pps.scaling_matrix_present)
      throw UnsupportedStream("High-profile tools (general decoder)");
    if (!sps.frame_mbs_only) throw UnsupportedStream("interlaced H.264 is not supported");
    if (sps.chroma_format_idc != 1 || sps.bit_depth_luma != 8 || sps.bit_depth_chroma != 8)
      throw UnsupportedStream("only 8-bit 4:2:0 is supported");
    active_sps_id_ = sps.sps_id;
    SliceHeader sh = parse_slice_header(br, p[0], sps, pps);
    if (!got_slice) {
      pi.coded_width = sps.coded_width();
      pi.coded_height = sps.coded_height();
      pi.width = sps.width();
      pi.height = sps.height();
      pi.crop_left = sps.crop_left;
      pi.crop_top = sps.crop_top;
      pi.pict_type = sh.pict_char();
      pi.idr = sh.idr();
      pi.frame_num = sh.frame_num;
      pi.fps = sps.fps();
      if (upd.width_mbs != sps.width_mbs || upd.height_mbs != sps.height_mbs())
        upd.reset(sps.width_mbs, sps.height_mbs());
      got_slice = true;
    }  // mixed-slice pictures report the first slice's type, as PyAV's pict_type does
    upd.begin_segment(p, n);
    upd.reserve_blocks(n / kPcmMbBytes + 1);
    BlockSink sink{upd, r, r == p, {}};
    walk_slice(r, rn, sh, br, sps, sink, pi.coded_mbs);
    sink.resolve(p, epb_);
  }
  pi.spec_lo = spec_lo_;
  pi.spec_hi = spec_hi_;
  speculate_ = false;  // one parse only
  VEP_CHECK(got_slice, "access unit has no slice");
  upd.frames += 1;
  return pi;
}

// ------------------------------------------------------------------------------------ H.265

void H265Parser::store_parameter_set(int t, const u8* p, size_t n) {
  size_t rn;
  const u8* r = rbsp_of(p, n, epb_, rbsp_scratch_, rn);
  if (t == hevc::kVps) {
    hevc::Vps v = hevc::parse_vps(r, rn);
    vps_[v.vps_id] = v;
  } else if (t == hevc::kSps) {
    hevc::Sps s = hevc::parse_sps(r, rn);
    sps_[s.sps_id] = s;
  } else {
    hevc::Pps q = hevc::parse_pps(r, rn);
    pps_[q.pps_id] = q;
  }
}

void H265Parser::absorb_parameter_sets(const AccessUnit& au) {
  for (size_t i = 0; i < au.nals.size(); ++i) {
    const u8* p = au.nal(i);
    size_t n = au.nal_size(i);
    if (n < 3) continue;
    int t = hevc::nal_type(p);
    if (t == hevc::kVps || t == hevc::kSps || t == hevc::kPps) store_parameter_set(t, p, n);
  }
}

const hevc::Sps& H265Parser::active_sps() const {
  VEP_CHECK(!sps_.empty(), "no active SPS");
  auto it = sps_.find(active_sps_id_ < 0 ? sps_.begin()->first : active_sps_id_);
  VEP_CHECK(it != sps_.end(), "no active SPS");
  return it->second;
}

// Coding-tree walk of one slice segment (H.265 §7.3.8). With CtbLog2SizeY == MinCbLog2SizeY
// every CTB is one CU and split_cu_flag is absent; per CU:
//   P/B: cu_skip_flag (ctxInc = left skip + above skip, §9.3.4.2.2)
//        skip -> merge_idx (TR, first bin context-coded) — every merge candidate is the zero
//        MV on reference 0 in this subset, so a skipped CU keeps the reference samples;
//        else pred_mode_flag must be MODE_INTRA
//   part_mode bin 0 must be PART_2Nx2N, then pcm_flag (terminating bin) must be 1;
//   PCM: alignment zeros, 384 raw sample bytes (16x16 Y, 8x8 Cb, 8x8 Cr), CABAC re-init;
//   end_of_slice_segment_flag (terminating bin).
void H265Parser::walk_slice(const u8* rbsp, size_t n, const hevc::SliceHeader& sh,
                            const hevc::Sps& sps, const hevc::Pps& pps, BlockSink& upd,
                            int& coded) {
  const int wctb = sps.width_ctbs(), total = wctb * sps.height_ctbs();
  const bool inter = sh.slice_type != hevc::kI;
  const int init_type = !inter ? 0 : (sh.slice_type == hevc::kP ? (sh.cabac_init ? 2 : 1)
                                                                 : (sh.cabac_init ? 1 : 2));
  const int qp = pps.init_qp + sh.qp_delta;
  cabac::Ctx skip_ctx[3], pred_ctx, part_ctx, merge_ctx;
  for (auto& c : skip_ctx) c.init(0, qp);
  if (inter) {
    const int skip_init[3] = {197, 185, 201};
    for (int k = 0; k < 3; ++k) skip_ctx[k].init(skip_init[k], qp);
    pred_ctx.init(init_type == 1 ? 149 : 134, qp);
    merge_ctx.init(init_type == 1 ? 122 : 137, qp);
  }
  part_ctx.init(init_type == 0 ? 184 : 154, qp);
  const int slice_addr = sh.segment_address;  // no dependent segments: slice == segment
  cabac::Decoder dec(rbsp, n, sh.data_bytepos);
  for (int ctb = sh.segment_address;; ++ctb) {
    VEP_CHECK(ctb < total, "coding tree unit past end of picture");
    bool skip = false;
    if (inter) {
      const int x = ctb % wctb;
      const int l = (x > 0 && ctb - 1 >= slice_addr) ? skip_[size_t(ctb - 1)] : 0;
      const int a = (ctb - wctb >= slice_addr) ? skip_[size_t(ctb - wctb)] : 0;
      skip = dec.decision(skip_ctx[l + a]);
    }
    skip_[size_t(ctb)] = u8(skip);
    if (skip) {
      if (sh.max_num_merge_cand > 1 && dec.decision(merge_ctx))
        for (int k = 1; k < sh.max_num_merge_cand - 1 && dec.bypass(); ++k) {
        }
    } else {
      if (inter && !dec.decision(pred_ctx))
        throw UnsupportedStream("inter-coded HEVC CU (native subset decodes PCM + skip only)");
      if (!dec.decision(part_ctx)) throw UnsupportedStream("intra NxN HEVC CU is not supported");
      if (!dec.terminate())
        throw UnsupportedStream("regular intra HEVC CU (native subset decodes PCM + skip only)");
      const size_t off = dec.aligned_bytepos();
      VEP_CHECK(off + kPcmMbBytes <= n, "truncated PCM coding unit");
      upd.add(ctb, rbsp + off);
      ++coded;
      dec.start(off + kPcmMbBytes);
    }
    if (dec.terminate()) break;  // end_of_slice_segment_flag
  }
}

PictureInfo H265Parser::parse(const AccessUnit& au, MbUpdate& upd) {
  PictureInfo pi;
  bool got_slice = false;
  for (size_t i = 0; i < au.nals.size(); ++i) {
    const u8* p = au.nal(i);
    size_t n = au.nal_size(i);
    if (n < 3) continue;
    const int t = hevc::nal_type(p);
    if (t == hevc::kVps || t == hevc::kSps || t == hevc::kPps) {
      store_parameter_set(t, p, n);
      continue;
    }
    if (!hevc::is_vcl(t)) continue;
    if (t > hevc::kTrailR && t < hevc::kBlaWLp)
      throw UnsupportedStream("HEVC leading / sub-layer pictures are not supported");
    size_t rn;
    const u32 *kb = nullptr, *ke = nullptr;
    au.epb_of(i, &kb, &ke);
    const u8* r = rbsp_of(p, n, epb_, rbsp_scratch_, rn, kb, ke);
    const int pps_id = hevc::peek_slice_pps_id(r, rn);
    auto pit = pps_.find(pps_id);
    if (pit == pps_.end()) throw UnsupportedStream("slice references unknown PPS");
    auto sit = sps_.find(pit->second.sps_id);
    if (sit == sps_.end()) throw UnsupportedStream("slice references unknown SPS");
    const hevc::Sps& sps = sit->second;
    const hevc::Pps& pps = pit->second;
    if (sps.chroma_format_idc != 1 || sps.bit_depth_luma != 8 || sps.bit_depth_chroma != 8)
      throw UnsupportedStream("only 8-bit 4:2:0 HEVC is supported");
    if (sps.log2_ctb != 4 || sps.log2_min_cb != 4 || !sps.pcm || sps.log2_min_pcm > 4 ||
        sps.log2_max_pcm < 4 || sps.pcm_bit_depth_luma != 8 || sps.pcm_bit_depth_chroma != 8)
      throw UnsupportedStream("native HEVC subset needs 16x16 CTBs coded as 8-bit PCM CUs");
    if (pps.transquant_bypass || pps.tiles || pps.entropy_coding_sync)
      throw UnsupportedStream("HEVC tiles / WPP / transquant bypass are not supported");
    hevc::SliceHeader sh;
    try {
      sh = hevc::parse_slice_header(r, rn, sps, pps);
    } catch (const UnsupportedStream&) {
      throw;
    } catch (const Error& e) {
      throw UnsupportedStream(e.what());
    }
    if (sh.slice_type == hevc::kB) throw UnsupportedStream("HEVC B slices are not supported");
    if (sh.sao_luma || sh.sao_chroma || !sh.deblocking_disabled)
      throw UnsupportedStream("HEVC in-loop filters (SAO / deblocking) are not supported");
    if (sh.slice_type == hevc::kP && sh.num_ref_idx_l0 != 1)
      throw UnsupportedStream("HEVC P slices with more than one reference are not supported");
    active_sps_id_ = sps.sps_id;
    if (!got_slice) {
      pi.coded_width = sps.width;
      pi.coded_height = sps.height;
      pi.width = sps.out_width();
      pi.height = sps.out_height();
      pi.crop_left = sps.conf_left;
      pi.crop_top = sps.conf_top;
      pi.pict_type = sh.pict_char();
      pi.idr = hevc::is_irap(t);
      pi.frame_num = sh.poc_lsb;
      pi.fps = sps.fps();
      const int w = sps.width_ctbs(), h = sps.height_ctbs();
      if (upd.width_mbs != w || upd.height_mbs != h) upd.reset(w, h);
      skip_.assign(size_t(w) * h, 0);
      got_slice = true;
    }
    upd.begin_segment(p, n);
    upd.reserve_blocks(n / kPcmMbBytes + 1);
    BlockSink sink{upd, r, r == p, {}};
    walk_slice(r, rn, sh, sps, pps, sink, pi.coded_mbs);
    sink.resolve(p, epb_);
  }
  VEP_CHECK(got_slice, "access unit has no slice");
  upd.frames += 1;
  return pi;
}

// ------------------------------------------------------------------------------ ParamSets

void ParamSets::absorb(const u8* p, size_t n) {
  if (n < 2) return;
  if (codec == Codec::kH264) {
    const int t = nal_type(p[0]);
    if (t == kNalSps) sps.assign(p, p + n);
    else if (t == kNalPps) pps.assign(p, p + n);
  } else {
    const int t = hevc::nal_type(p);
    if (t == hevc::kVps) vps.assign(p, p + n);
    else if (t == hevc::kSps) sps.assign(p, p + n);
    else if (t == hevc::kPps) pps.assign(p, p + n);
  }
}

std::pair<int, int> ParamSets::size() const {
  if (sps.empty()) return {0, 0};
  std::vector<u8> r(sps.size());
  const size_t n = ebsp_to_rbsp(sps.data(), sps.size(), r.data());
  try {
    if (codec == Codec::kH264) {
      const Sps s = parse_sps(r.data(), n);
      return {s.width(), s.height()};
    }
    const hevc::Sps s = hevc::parse_sps(r.data(), n);
    return {s.out_width(), s.out_height()};
  } catch (const std::exception&) {
    return {0, 0};
  }
}

void cpu_apply_update(const MbUpdate& upd, HostSurface& s) {
  const int W = upd.width_mbs;
  VEP_CHECK(s.coded_w == W * 16 && s.coded_h == upd.height_mbs * 16, "surface size mismatch");
  for (int mb = 0; mb < upd.mbs(); ++mb) {
    int sl = upd.slot[mb];
    if (sl < 0) continue;
    const u8* src = upd.block(sl);
    int mx = mb % W, my = mb / W;
    for (int r = 0; r < 16; ++r)
      std::memcpy(&s.y[size_t(my * 16 + r) * s.coded_w + mx * 16], src + r * 16, 16);
    for (int r = 0; r < 8; ++r) {
      u8* d = &s.uv[size_t(my * 8 + r) * s.coded_w + mx * 16];
      for (int c = 0; c < 8; ++c) {
        d[2 * c] = src[256 + r * 8 + c];
        d[2 * c + 1] = src[320 + r * 8 + c];
      }
    }
  }
}

void narrow_surface(const HostSurface& s, HostSurface& out) {
  if (!s.wide() && s.cf != 2) {
    out = s;
    return;
  }
  out.coded_w = s.coded_w;
  out.coded_h = s.coded_h;
  out.bd = 8;
  out.cf = 1;
  out.y16.clear();
  out.uv16.clear();
  const int sh = s.bd - 8, rnd = (1 << sh) >> 1;
  auto n8 = [&](int v) { return u8(std::min(255, (v + rnd) >> sh)); };
  const size_t w = size_t(s.coded_w), ny = w * size_t(s.coded_h);
  out.y.resize(ny);
  out.uv.resize(ny / 2);
  for (size_t i = 0; i < ny; ++i) out.y[i] = n8(s.wide() ? int(s.y16[i]) : int(s.y[i]));
  auto c = [&](size_t i) { return s.wide() ? int(s.uv16[i]) : int(s.uv[i]); };
  for (size_t r = 0; r < size_t(s.coded_h / 2); ++r)
    for (size_t x = 0; x < w; ++x)
      out.uv[r * w + x] = n8(s.cf == 2 ? (c(2 * r * w + x) + c((2 * r + 1) * w + x) + 1) >> 1 : c(r * w + x));
}

void cpu_nv12_to_bgr(const HostSurface& s8, int crop_left, int crop_top, int width, int height,
                     u8* out) {
  HostSurface tmp;
  const bool conv = s8.wide() || s8.cf == 2;
  if (conv) narrow_surface(s8, tmp);
  const HostSurface& s = conv ? tmp : s8;
  for (int y = 0; y < height; ++y) {
    int sy = y + crop_top;
    const u8* yr = &s.y[size_t(sy) * s.coded_w];
    const u8* cr = &s.uv[size_t(sy >> 1) * s.coded_w];
    u8* o = out + size_t(y) * width * 3;
    for (int x = 0; x < width; ++x) {
      int sx = x + crop_left;
      int ci = (sx >> 1) * 2;
      yuv_to_bgr(yr[sx], cr[ci], cr[ci + 1], o + 3 * x, o + 3 * x + 1, o + 3 * x + 2);
    }
  }
}

}  // namespace vep
