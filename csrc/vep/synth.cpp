// Synthetic H.264 camera encoder (I_PCM / P_Skip). See synth.h.
#include "synth.h"

#include "hevc_dec.h"

#include <algorithm>
#include <cmath>

#include "cabac.h"

namespace vep {

using namespace h264;

SynthH264::SynthH264(const SynthConfig& cfg) : cfg_(cfg) {
  VEP_CHECK(cfg.width >= 16 && cfg.height >= 16 && cfg.width % 2 == 0 && cfg.height % 2 == 0,
            "synthetic size must be even and >= 16");
  wmbs_ = (cfg.width + 15) / 16;
  hmbs_ = (cfg.height + 15) / 16;
  sps_.profile_idc = 66;
  sps_.constraint_flags = 0xC0;
  sps_.level_idc = 51;
  sps_.log2_max_frame_num = 8;
  sps_.poc_type = 2;
  sps_.max_num_ref_frames = 1;
  sps_.width_mbs = wmbs_;
  sps_.height_map_units = hmbs_;
  sps_.crop_right = wmbs_ * 16 - cfg.width;
  sps_.crop_bottom = hmbs_ * 16 - cfg.height;
  sps_.timing_info = true;
  sps_.num_units_in_tick = 1;
  sps_.time_scale = u32(2 * cfg.fps);
  pps_.deblocking_filter_control = true;
  if (cfg.codec == Codec::kH265) {
    VEP_CHECK(cfg.merge_cands >= 1 && cfg.merge_cands <= 5, "merge_cands must be 1..5");
    hvps_.timing_info = true;
    hvps_.num_units_in_tick = 1;
    hvps_.time_scale = u32(cfg.fps);
    hsps_.width = wmbs_ * 16;
    hsps_.height = hmbs_ * 16;
    hsps_.conf_right = wmbs_ * 16 - cfg.width;
    hsps_.conf_bottom = hmbs_ * 16 - cfg.height;
    hsps_.ptl.level_idc = (cfg.width * cfg.height > 2228224) ? 153 : 123;  // 5.1 / 4.1
    hevc::ShortTermRps rps;
    rps.num_negative = 1;
    rps.delta_poc[0] = -1;
    rps.used[0] = true;
    hsps_.st_rps = {rps};
    hsps_.vui = true;
    hsps_.video_signal_type = true;
    hsps_.timing_info = true;
    hsps_.num_units_in_tick = 1;
    hsps_.time_scale = u32(cfg.fps);
    for (auto* pr : {&vps_nal_, &sps_nal_, &pps_nal_}) pr->clear();
    std::vector<u8> r = hevc::write_vps(hvps_);
    rbsp_to_ebsp(r.data(), r.size(), vps_nal_);
    r = hevc::write_sps(hsps_);
    rbsp_to_ebsp(r.data(), r.size(), sps_nal_);
    r = hevc::write_pps(hpps_);
    rbsp_to_ebsp(r.data(), r.size(), pps_nal_);
    skip_.assign(size_t(wmbs_) * hmbs_, 0);
  } else {
    std::vector<u8> r = write_sps(sps_);
    rbsp_to_ebsp(r.data(), r.size(), sps_nal_);
    r = write_pps(pps_);
    rbsp_to_ebsp(r.data(), r.size(), pps_nal_);
  }
  pic_.alloc(wmbs_ * 16, hmbs_ * 16);
  bg_.alloc(wmbs_ * 16, hmbs_ * 16);
  state_ = cfg.seed * 0x9E3779B97F4A7C15ull + 0x1234567ull;
  double area = std::max(1.0, cfg.motion * wmbs_ * hmbs_);
  bw_ = std::clamp(int(std::lround(std::sqrt(area * 4.0 / 3.0))), 1, wmbs_);
  bh_ = std::clamp(int(std::lround(area / bw_)), 1, hmbs_);
  if (cfg.motion <= 0) bw_ = bh_ = 0;
  if (cfg.compressed && cfg.codec == Codec::kH265) {  // general HEVC Main stream
    hevc::HevcEncConfig hc;
    hc.width = cfg.width;
    hc.height = cfg.height;
    hc.fps = cfg.fps;
    hc.gop = cfg.gop;
    hc.idr_phase = cfg.idr_phase;
    hc.qp = cfg.qp;
    hc.slices = cfg.slices;
    hc.bframes = cfg.bframes;
    hc.objects = cfg.objects;
    hc.seed = cfg.seed;
    hc.deblock = cfg.deblock_idc != 1;
    hc.coverage = cfg.coverage;
    hc.noise = cfg.noise;
    hc.temporal_noise = cfg.temporal_noise;
    hc.tile_cols = cfg.tile_cols;
    hc.tile_rows = cfg.tile_rows;
    hc.wpp = cfg.wpp;
    hc.segments = cfg.segments;
    hc.scaling_lists = cfg.scaling_lists;
    hc.weighted = cfg.weighted_p || cfg.weighted_b;
    hc.long_term = cfg.long_term;
    hc.open_gop = cfg.open_gop;
    hc.lossless = cfg.lossless;
    hc.bit_depth = cfg.bit_depth;
    auto enc = std::make_unique<hevc::HevcEncoder>(hc);
    vps_nal_ = enc->vps_nal();
    avc_ = std::move(enc);
    sps_nal_ = avc_->sps_nal();
    pps_nal_ = avc_->pps_nal();
  } else if (cfg.compressed) {
    if (cfg.profile == "main" || cfg.profile == "high") {
      avc::AvcHighConfig hc;
      hc.width = cfg.width;
      hc.height = cfg.height;
      hc.fps = cfg.fps;
      hc.gop = cfg.gop;
      hc.idr_phase = cfg.idr_phase;
      hc.qp = cfg.qp;
      hc.slices = cfg.slices;
      hc.refs = cfg.refs;
      hc.bframes = cfg.bframes;
      hc.cabac = cfg.cabac;
      hc.t8x8 = cfg.profile == "high";
      hc.weighted_p = cfg.weighted_p;
      hc.weighted_b = cfg.weighted_b;
      hc.direct_spatial = cfg.direct_spatial;
      hc.objects = cfg.objects;
      hc.seed = cfg.seed;
      hc.deblock_idc = cfg.deblock_idc;
      hc.coverage = cfg.coverage;
      hc.noise = cfg.noise;
      hc.temporal_noise = cfg.temporal_noise;
      hc.interlaced = cfg.interlaced >= 1;
      hc.mono = cfg.mono;
      hc.bit_depth = cfg.bit_depth;
      hc.chroma_format = cfg.chroma_format;
      if (cfg.interlaced == 2) {
        hc.fields = true;
        hc.cabac = false;
      }
      avc_ = std::make_unique<avc::AvcHighEncoder>(hc);
    } else {
      VEP_CHECK(cfg.profile == "baseline", "profile must be baseline, main or high");
      avc::AvcEncConfig ac;
      ac.width = cfg.width;
      ac.height = cfg.height;
      ac.fps = cfg.fps;
      ac.gop = cfg.gop;
      ac.idr_phase = cfg.idr_phase;
      ac.qp = cfg.qp;
      ac.slices = cfg.slices;
      ac.refs = cfg.refs;
      ac.objects = cfg.objects;
      ac.seed = cfg.seed;
      ac.deblock_idc = cfg.deblock_idc;
      ac.coverage = cfg.coverage;
      ac.noise = cfg.noise;
      ac.temporal_noise = cfg.temporal_noise;
      if (cfg.coverage) {
        ac.pcm_rate = 3;
        ac.nonref_rate = 15;
      }
      avc_ = std::make_unique<avc::AvcEncoder>(ac);
    }
    sps_nal_ = avc_->sps_nal();
    pps_nal_ = avc_->pps_nal();
  }
}

u64 SynthH264::rnd() {
  u64 x = state_;
  x ^= x << 13;
  x ^= x >> 7;
  x ^= x << 17;
  return state_ = x;
}

void SynthH264::paint_background() {
  const int W = bg_.coded_w, H = bg_.coded_h;
  const int lo = cfg_.zero_samples ? 0 : 16;
  for (int y = 0; y < H; ++y) {
    u8* row = &bg_.y[size_t(y) * W];
    for (int x = 0; x < W; x += 8) {
      u64 r = rnd();
      for (int k = 0; k < 8; ++k) {
        int v = 16 + ((x + k) * 3 + y * 2) % 160 + int((r >> (8 * k)) & 63);
        row[x + k] = u8(std::clamp(v, lo, 235));
      }
    }
  }
  for (int y = 0; y < H / 2; ++y) {
    u8* row = &bg_.uv[size_t(y) * W];
    for (int x = 0; x < W; x += 8) {
      u64 r = rnd();
      for (int k = 0; k < 8; ++k) {
        int base = (k & 1) ? 96 + (y % 64) : 96 + ((x / 2) % 64);
        row[x + k] = u8(std::clamp(base + int((r >> (8 * k)) & 15), lo, 240));
      }
    }
  }
  if (cfg_.zero_samples) {  // plant explicit 00 00 runs so EPBs appear in the NAL
    for (int y = 0; y < H; y += 7) bg_.y[size_t(y) * W + (y % W)] = 0, bg_.y[size_t(y) * W + ((y + 1) % W)] = 0;
  }
}

SynthH264::Rect SynthH264::box_at(i64 f) const {
  if (bw_ == 0) return {0, 0, 0, 0};
  int span_x = std::max(1, wmbs_ - bw_ + 1), span_y = std::max(1, hmbs_ - bh_ + 1);
  i64 px = f % (2 * span_x);
  int x = int(px < span_x ? px : 2 * span_x - 1 - px);
  i64 py = (f / 2) % (2 * span_y);
  int y = int(py < span_y ? py : 2 * span_y - 1 - py);
  return {x, y, x + bw_, y + bh_};
}

void SynthH264::paint_box(const Rect& r) {
  const int W = pic_.coded_w;
  u8 cb = u8(64 + (rnd() & 127)), cr = u8(64 + (rnd() & 127));
  for (int y = r.y0 * 16; y < r.y1 * 16; ++y) {
    u8* row = &pic_.y[size_t(y) * W];
    for (int x = r.x0 * 16; x < r.x1 * 16; x += 8) {
      u64 q = rnd();
      for (int k = 0; k < 8; ++k) row[x + k] = u8(180 + ((q >> (8 * k)) & 31));
    }
  }
  for (int y = r.y0 * 8; y < r.y1 * 8; ++y) {
    u8* row = &pic_.uv[size_t(y) * W];
    for (int x = r.x0 * 16; x < r.x1 * 16; x += 2) {
      row[x] = cb;
      row[x + 1] = cr;
    }
  }
}

void SynthH264::pcm_payload(int mb, u8* out) const {
  const int W = pic_.coded_w;
  int mx = mb % wmbs_, my = mb / wmbs_;
  for (int r = 0; r < 16; ++r)
    std::memcpy(out + r * 16, &pic_.y[size_t(my * 16 + r) * W + mx * 16], 16);
  for (int r = 0; r < 8; ++r) {
    const u8* s = &pic_.uv[size_t(my * 8 + r) * W + mx * 16];
    for (int c = 0; c < 8; ++c) {
      out[256 + r * 8 + c] = s[2 * c];
      out[320 + r * 8 + c] = s[2 * c + 1];
    }
  }
}

std::vector<u8> SynthH264::encode_slice(bool idr, int mb0, int mb1,
                                        const std::vector<u8>& coded) {
  BitWriter bw;
  SliceHeader sh;
  sh.nal_type = idr ? kNalIdr : kNalSlice;
  sh.nal_ref_idc = 3;
  sh.first_mb = mb0;
  sh.slice_type = idr ? 7 : 5;
  sh.frame_num = frame_num_;
  sh.idr_pic_id = idr_id_;
  sh.disable_deblocking = 1;
  write_slice_header(bw, sh, sps_, pps_);
  u8 buf[kPcmMbBytes];
  int run = 0;
  for (int mb = mb0; mb < mb1; ++mb) {
    if (!idr && !coded[mb]) {
      ++run;
      continue;
    }
    if (!idr) {
      bw.ue(u32(run));
      run = 0;
    }
    bw.ue(idr ? 25u : 30u);
    bw.align_zero();
    pcm_payload(mb, buf);
    bw.bytes(buf, kPcmMbBytes);
  }
  if (!idr && run > 0) bw.ue(u32(run));
  bw.trailing();
  std::vector<u8> nal;
  rbsp_to_ebsp(bw.buf().data(), bw.buf().size(), nal);
  return nal;
}

// HEVC slice segment: one CU per 16x16 CTB; see H265Parser::walk_slice for the syntax.
std::vector<u8> SynthH264::encode_slice_hevc(bool idr, int ctb0, int ctb1,
                                             const std::vector<u8>& coded) {
  BitWriter bw;
  hevc::SliceHeader sh;
  sh.nal_type = idr ? hevc::kIdrWRadl : hevc::kTrailR;
  sh.first_slice_in_pic = ctb0 == 0;
  sh.segment_address = ctb0;
  sh.slice_type = idr ? hevc::kI : hevc::kP;
  sh.poc_lsb = poc_;
  sh.max_num_merge_cand = cfg_.merge_cands;
  hevc::write_slice_header(bw, sh, hsps_, hpps_);
  std::vector<u8> out = std::move(bw.buf());
  const int qp = hpps_.init_qp + sh.qp_delta;
  cabac::Ctx skip_ctx[3], pred_ctx, part_ctx, merge_ctx;
  const int skip_init[3] = {197, 185, 201};
  for (int k = 0; k < 3; ++k) skip_ctx[k].init(skip_init[k], qp);
  pred_ctx.init(149, qp);
  merge_ctx.init(122, qp);
  part_ctx.init(idr ? 184 : 154, qp);
  cabac::Encoder enc(out);
  u8 buf[kPcmMbBytes];
  for (int ctb = ctb0; ctb < ctb1; ++ctb) {
    const bool pcm = idr || coded[size_t(ctb)];
    if (!idr) {
      const int x = ctb % wmbs_;
      const int l = (x > 0 && ctb - 1 >= ctb0) ? skip_[size_t(ctb - 1)] : 0;
      const int a = (ctb - wmbs_ >= ctb0) ? skip_[size_t(ctb - wmbs_)] : 0;
      enc.decision(skip_ctx[l + a], pcm ? 0 : 1);
      skip_[size_t(ctb)] = u8(!pcm);
      if (!pcm && cfg_.merge_cands > 1) {
        const int idx = ctb % cfg_.merge_cands;  // any candidate: all are the zero MV
        enc.decision(merge_ctx, idx > 0);
        for (int k = 1; k < cfg_.merge_cands - 1 && idx > 0; ++k) {
          enc.bypass(idx > k);
          if (idx <= k) break;
        }
      }
      if (pcm) enc.decision(pred_ctx, 1);  // MODE_INTRA
    }
    if (pcm) {
      enc.decision(part_ctx, 1);  // PART_2Nx2N
      enc.terminate(1);           // pcm_flag
      enc.align_zero();           // pcm_alignment_zero_bit
      pcm_payload(ctb, buf);
      enc.raw_bytes(buf, kPcmMbBytes);
      enc.start();
    }
    enc.terminate(ctb + 1 == ctb1 ? 1 : 0);  // end_of_slice_segment_flag
  }
  enc.align_zero();  // rbsp_slice_segment_trailing_bits (the stop bit ends the flush)
  std::vector<u8> nal;
  rbsp_to_ebsp(out.data(), out.size(), nal);
  return nal;
}

std::shared_ptr<AccessUnit> SynthH264::next() {
  ++frame_;
  if (avc_) {
    auto au = avc_->next();
    au->arrival_ms = now_ms();
    return au;
  }
  // frame 0 is always an IDR; later IDRs fall where (frame + phase) % gop == 0 so that a fleet
  // of cameras does not refresh in lock-step
  const bool idr = frame_ == 0 || ((frame_ + cfg_.idr_phase) % cfg_.gop) == 0;
  auto au = std::make_shared<AccessUnit>();
  const bool h265 = cfg_.codec == Codec::kH265;
  au->codec = cfg_.codec;
  au->pts = au->dts = frame_ * 90000 / cfg_.fps;
  au->duration = 90000 / cfg_.fps;
  au->keyframe = idr;
  au->seq = u64(frame_);
  au->arrival_ms = now_ms();
  const int total = wmbs_ * hmbs_;
  std::vector<u8> coded(size_t(total), 0);
  Rect box = box_at(frame_);
  if (idr) {
    paint_background();
    pic_.y = bg_.y;
    pic_.uv = bg_.uv;
    if (bw_) paint_box(box);
    frame_num_ = 0;
    poc_ = 0;
    idr_id_ = (idr_id_ + 1) & 0xffff;
    if (h265) au->add_nal(vps_nal_.data(), vps_nal_.size());
    au->add_nal(sps_nal_.data(), sps_nal_.size());
    au->add_nal(pps_nal_.data(), pps_nal_.size());
  } else {
    frame_num_ = (frame_num_ + 1) % (1 << sps_.log2_max_frame_num);
    ++poc_;
    // restore background under the previous box, paint the new one
    const int W = pic_.coded_w;
    const Rect& o = prev_box_;
    for (int y = o.y0 * 16; y < o.y1 * 16; ++y)
      std::memcpy(&pic_.y[size_t(y) * W + o.x0 * 16], &bg_.y[size_t(y) * W + o.x0 * 16],
                  size_t(o.x1 - o.x0) * 16);
    for (int y = o.y0 * 8; y < o.y1 * 8; ++y)
      std::memcpy(&pic_.uv[size_t(y) * W + o.x0 * 16], &bg_.uv[size_t(y) * W + o.x0 * 16],
                  size_t(o.x1 - o.x0) * 16);
    if (bw_) paint_box(box);
    for (const Rect& r : {o, box})
      for (int y = r.y0; y < r.y1; ++y)
        for (int x = r.x0; x < r.x1; ++x) coded[size_t(y) * wmbs_ + x] = 1;
  }
  prev_box_ = box;
  const int ns = std::max(1, std::min(cfg_.slices, hmbs_));
  for (int s = 0; s < ns; ++s) {
    int r0 = hmbs_ * s / ns, r1 = hmbs_ * (s + 1) / ns;
    std::vector<u8> nal = h265 ? encode_slice_hevc(idr, r0 * wmbs_, r1 * wmbs_, coded)
                               : encode_slice(idr, r0 * wmbs_, r1 * wmbs_, coded);
    au->add_nal(nal.data(), nal.size());
  }
  return au;
}

}  // namespace vep
