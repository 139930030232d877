// Native H.264 macroblock-layer parser (CAVLC, I_PCM + P_Skip subset) and CPU reference
// reconstruction. See codec.h for the CPU/GPU split.
#include "codec.h"

#include "color.h"

namespace vep {

using namespace h264;

static const u8* rbsp_of(const u8* nal, size_t n, std::vector<u32>& epb,
                         std::vector<u8>& scratch, size_t& out_n) {
  find_epb(nal, n, epb);
  if (epb.empty()) {
    out_n = n;
    return nal;
  }
  scratch.resize(n);
  out_n = ebsp_to_rbsp(nal, n, scratch.data());
  return scratch.data();
}

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
                            const Sps& sps, MbUpdate& upd, int& coded) {
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
      while (off + 2 + kPcmMbBytes <= nbytes && base[off] == f0 && base[off + 1] == f1 &&
             (off + 2) * 8 < stop) {
        VEP_CHECK(mb < total, "macroblock address past end of picture");
        upd.set(mb, base + off + 2);
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
      upd.set(mb, base + off);
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
    const u8* r = rbsp_of(p, n, epb_, rbsp_scratch_, rn);
    std::shared_ptr<std::vector<u8>> owned;
    if (r != p) {
      // emulation-prevention bytes present: the MB samples are referenced from an owned
      // unescaped copy (kept alive by the update) instead of the shared parser scratch
      owned = std::make_shared<std::vector<u8>>(r, r + rn);
      r = owned->data();
    }
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
    if (pps.cabac) throw UnsupportedStream("CABAC streams need the RocDecode backend");
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
    if (owned) upd.own.push_back(owned);
    upd.begin_segment(r, rn);
    walk_slice(r, rn, sh, br, sps, upd, pi.coded_mbs);
  }
  VEP_CHECK(got_slice, "access unit has no slice");
  upd.frames += 1;
  return pi;
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

void cpu_nv12_to_bgr(const HostSurface& s, int crop_left, int crop_top, int width, int height,
                     u8* out) {
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
