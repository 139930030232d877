// H.264 parameter-set / slice-header parsing and writing (ITU-T H.264 §7.3.2.1, §7.3.2.2, §7.3.3).
#include "h264.h"
#include "codec.h"

#include <algorithm>

namespace vep::h264 {

const u8 kDefault4x4[2][16] = {
    {6, 13, 13, 20, 20, 20, 28, 28, 28, 28, 32, 32, 32, 37, 37, 42},
    {10, 14, 14, 20, 20, 20, 24, 24, 24, 24, 27, 27, 27, 30, 30, 34}};
const u8 kDefault8x8[2][64] = {
    {6,  10, 10, 13, 11, 13, 16, 16, 16, 16, 18, 18, 18, 18, 18, 23, 23, 23, 23, 23, 23, 25,
     25, 25, 25, 25, 25, 25, 27, 27, 27, 27, 27, 27, 27, 27, 29, 29, 29, 29, 29, 29, 29, 31,
     31, 31, 31, 31, 31, 33, 33, 33, 33, 33, 36, 36, 36, 36, 38, 38, 38, 40, 40, 42},
    {9,  13, 13, 15, 13, 15, 17, 17, 17, 17, 19, 19, 19, 19, 19, 21, 21, 21, 21, 21, 21, 22,
     22, 22, 22, 22, 22, 22, 24, 24, 24, 24, 24, 24, 24, 24, 25, 25, 25, 25, 25, 25, 25, 27,
     27, 27, 27, 27, 27, 28, 28, 28, 28, 28, 30, 30, 30, 30, 32, 32, 32, 33, 33, 35}};

// scaling_list() (§7.3.2.1.1.1): returns useDefaultScalingMatrixFlag.
static bool read_scaling_list(BitReader& br, u8* list, int size) {
  int last = 8, next = 8;
  bool use_default = false;
  for (int j = 0; j < size; ++j) {
    if (next != 0) {
      const int delta = br.se();
      VEP_CHECK(delta >= -128 && delta <= 127, "delta_scale out of range");
      next = (last + delta + 256) % 256;
      use_default = j == 0 && next == 0;
    }
    list[j] = u8(next == 0 ? last : next);
    last = list[j];
  }
  return use_default;
}

// Parse up to `count` lists with the fall-back rule: rule A (SPS, `base` = nullptr) falls back
// to the defaults, rule B (PPS) to the SPS's lists for lists 0, 3, 6, 7.
static void read_scaling_matrix(BitReader& br, int count, ScalingLists& out, const ScalingLists* base,
                                bool* present, bool* use_default) {
  for (int i = 0; i < 8; ++i) {
    const bool pr = i < count && br.u1();
    if (present) present[i] = pr;
    bool def = false;
    if (pr) def = read_scaling_list(br, i < 6 ? out.l4[i] : out.l8[i - 6], i < 6 ? 16 : 64);
    if (use_default) use_default[i] = def;
    if (pr && !def) continue;
    if (i < 6) {
      u8* l = out.l4[i];
      if (pr && def) std::memcpy(l, kDefault4x4[i >= 3], 16);
      else if (i == 0 || i == 3) std::memcpy(l, base ? base->l4[i] : kDefault4x4[i >= 3], 16);
      else std::memcpy(l, out.l4[i - 1], 16);
    } else {
      u8* l = out.l8[i - 6];
      if (pr && def) std::memcpy(l, kDefault8x8[i - 6], 64);
      else std::memcpy(l, base ? base->l8[i - 6] : kDefault8x8[i - 6], 64);
    }
  }
}

static void read_hrd(BitReader& br) {
  const u32 cnt = br.ue() + 1;
  VEP_CHECK(cnt <= 32, "cpb_cnt out of range");
  br.u(4);
  br.u(4);
  for (u32 i = 0; i < cnt; ++i) {
    br.ue();
    br.ue();
    br.u1();
  }
  br.u(5);
  br.u(5);
  br.u(5);
  br.u(5);
}

int Sps::max_dpb_frames() const {
  int mbs;  // MaxDpbMbs (Table A-1)
  switch (level_idc) {
    case 9: case 10: mbs = 396; break;
    case 11: mbs = (constraint_flags & 0x10) && profile_idc != 100 ? 396 : 900; break;
    case 12: case 13: case 20: mbs = 2376; break;
    case 21: mbs = 4752; break;
    case 22: case 30: mbs = 8100; break;
    case 31: mbs = 18000; break;
    case 32: mbs = 20480; break;
    case 40: case 41: mbs = 32768; break;
    case 42: mbs = 34816; break;
    case 50: mbs = 110400; break;
    case 51: case 52: mbs = 184320; break;
    default: mbs = 696320; break;
  }
  const int pic = width_mbs * height_mbs();
  return std::max(1, std::min(16, pic > 0 ? mbs / pic : 16));
}

Sps parse_sps(const u8* rbsp, size_t n) {
  VEP_CHECK(n >= 4 && nal_type(rbsp[0]) == kNalSps, "not an SPS NAL");
  BitReader br(rbsp + 1, n - 1);
  Sps s;
  s.scaling.flat();
  s.profile_idc = br.u(8);
  s.constraint_flags = br.u(8);
  s.level_idc = br.u(8);
  s.sps_id = br.ue();
  VEP_CHECK(s.sps_id < 32, "sps_id out of range");
  switch (s.profile_idc) {
    case 100: case 110: case 122: case 244: case 44: case 83: case 86: case 118:
    case 128: case 138: case 139: case 134: case 135: {
      s.chroma_format_idc = br.ue();
      VEP_CHECK(s.chroma_format_idc <= 3, "bad chroma_format_idc");
      if (s.chroma_format_idc == 3) br.u1();  // separate_colour_plane_flag
      s.bit_depth_luma = 8 + br.ue();
      s.bit_depth_chroma = 8 + br.ue();
      VEP_CHECK(s.bit_depth_luma <= 14 && s.bit_depth_chroma <= 14, "bad bit depth");
      s.transform_bypass = br.u1();
      s.scaling_matrix_present = br.u1();
      if (s.scaling_matrix_present)
        read_scaling_matrix(br, s.chroma_format_idc != 3 ? 8 : 12, s.scaling, nullptr, nullptr, nullptr);
      break;
    }
    default: break;
  }
  s.log2_max_frame_num = br.ue() + 4;
  VEP_CHECK(s.log2_max_frame_num <= 16, "log2_max_frame_num out of range");
  s.poc_type = br.ue();
  VEP_CHECK(s.poc_type <= 2, "bad pic_order_cnt_type");
  if (s.poc_type == 0) {
    s.log2_max_poc_lsb = br.ue() + 4;
    VEP_CHECK(s.log2_max_poc_lsb <= 16, "log2_max_pic_order_cnt_lsb out of range");
  } else if (s.poc_type == 1) {
    s.delta_pic_order_always_zero = br.u1();
    s.offset_for_non_ref_pic = br.se();
    s.offset_for_top_to_bottom_field = br.se();
    const u32 cyc = br.ue();
    VEP_CHECK(cyc < 256, "poc cycle too long");
    for (u32 i = 0; i < cyc; ++i) s.offset_for_ref_frame.push_back(br.se());
  }
  s.max_num_ref_frames = br.ue();
  VEP_CHECK(s.max_num_ref_frames <= 16, "max_num_ref_frames out of range");
  s.gaps_in_frame_num_allowed = br.u1();
  s.width_mbs = br.ue() + 1;
  s.height_map_units = br.ue() + 1;
  s.frame_mbs_only = br.u1();
  if (!s.frame_mbs_only) s.mbaff = br.u1();
  s.direct_8x8 = br.u1();
  if (br.u1()) {  // frame_cropping_flag
    const int cx = (s.chroma_format_idc == 0 || s.chroma_format_idc == 3) ? 1 : 2;
    const int cy = ((s.chroma_format_idc == 1) ? 2 : 1) * (s.frame_mbs_only ? 1 : 2);
    s.crop_left = br.ue() * cx;
    s.crop_right = br.ue() * cx;
    s.crop_top = br.ue() * cy;
    s.crop_bottom = br.ue() * cy;
  }
  if (br.bits_left() > 0 && br.u1()) {  // vui_parameters_present_flag
    if (br.u1()) {  // aspect_ratio_info_present_flag
      if (br.u(8) == 255) br.u(32);
    }
    if (br.u1()) br.u1();  // overscan
    if (br.u1()) {         // video_signal_type_present_flag
      br.u(4);
      if (br.u1()) br.u(24);
    }
    if (br.u1()) {  // chroma_loc_info_present_flag
      br.ue();
      br.ue();
    }
    s.timing_info = br.u1();
    if (s.timing_info) {
      s.num_units_in_tick = br.u(32);
      s.time_scale = br.u(32);
      br.u1();
    }
    const bool nal_hrd = br.u1();
    if (nal_hrd) read_hrd(br);
    const bool vcl_hrd = br.u1();
    if (vcl_hrd) read_hrd(br);
    if (nal_hrd || vcl_hrd) br.u1();  // low_delay_hrd_flag
    br.u1();                          // pic_struct_present_flag
    if (br.u1()) {                    // bitstream_restriction_flag
      br.u1();
      br.ue();
      br.ue();
      br.ue();
      br.ue();
      s.max_num_reorder_frames = int(br.ue());
      s.max_dec_frame_buffering = int(br.ue());
      VEP_CHECK(s.max_num_reorder_frames <= 16 && s.max_dec_frame_buffering <= 16,
                "bitstream_restriction out of range");
    }
  }
  VEP_CHECK(s.width_mbs > 0 && s.width_mbs <= 1024 && s.height_mbs() <= 1024, "bad SPS size");
  return s;
}

Pps parse_pps(const u8* rbsp, size_t n) {
  VEP_CHECK(n >= 2 && nal_type(rbsp[0]) == kNalPps, "not a PPS NAL");
  BitReader br(rbsp + 1, n - 1);
  Pps p;
  p.pps_id = br.ue();
  p.sps_id = br.ue();
  VEP_CHECK(p.pps_id < 256 && p.sps_id < 32, "pps ids out of range");
  p.cabac = br.u1();
  p.bottom_field_pic_order = br.u1();
  p.num_slice_groups = br.ue() + 1;
  VEP_CHECK(p.num_slice_groups == 1, "FMO slice groups are not supported");
  p.num_ref_idx_l0_default = br.ue() + 1;
  p.num_ref_idx_l1_default = br.ue() + 1;
  VEP_CHECK(p.num_ref_idx_l0_default <= 32 && p.num_ref_idx_l1_default <= 32, "num_ref_idx out of range");
  p.weighted_pred = br.u1();
  p.weighted_bipred_idc = br.u(2);
  VEP_CHECK(p.weighted_bipred_idc <= 2, "bad weighted_bipred_idc");
  p.pic_init_qp = 26 + br.se();
  p.pic_init_qs = 26 + br.se();
  p.chroma_qp_index_offset = br.se();
  VEP_CHECK(p.chroma_qp_index_offset >= -12 && p.chroma_qp_index_offset <= 12, "chroma_qp_index_offset out of range");
  p.deblocking_filter_control = br.u1();
  p.constrained_intra_pred = br.u1();
  p.redundant_pic_cnt_present = br.u1();
  p.second_chroma_qp_index_offset = p.chroma_qp_index_offset;
  p.scaling.flat();
  if (br.bitpos() < br.stop_bit_pos()) {  // more_rbsp_data(): the High-profile tail
    p.transform_8x8_mode = br.u1();
    p.scaling_matrix_present = br.u1();
    if (p.scaling_matrix_present)
      for (int i = 0; i < 6 + 2 * int(p.transform_8x8_mode); ++i) {
        p.scaling_list_present[i] = br.u1();
        if (p.scaling_list_present[i])
          p.scaling_use_default[i] = read_scaling_list(br, i < 6 ? p.scaling.l4[i] : p.scaling.l8[i - 6], i < 6 ? 16 : 64);
      }
    p.second_chroma_qp_index_offset = br.se();
    VEP_CHECK(p.second_chroma_qp_index_offset >= -12 && p.second_chroma_qp_index_offset <= 12,
              "second_chroma_qp_index_offset out of range");
  }
  return p;
}

ScalingLists resolve_scaling(const Sps& sps, const Pps& pps) {
  if (!pps.scaling_matrix_present) return sps.scaling;  // flat when the SPS has none
  // rule B when the SPS carries a matrix, rule A otherwise
  const ScalingLists* base = sps.scaling_matrix_present ? &sps.scaling : nullptr;
  ScalingLists out = pps.scaling;
  for (int i = 0; i < 8; ++i) {
    const bool pr = pps.scaling_list_present[i], def = pps.scaling_use_default[i];
    if (pr && !def) continue;
    if (i < 6) {
      u8* l = out.l4[i];
      if (pr && def) std::memcpy(l, kDefault4x4[i >= 3], 16);
      else if (i == 0 || i == 3) std::memcpy(l, base ? base->l4[i] : kDefault4x4[i >= 3], 16);
      else std::memcpy(l, out.l4[i - 1], 16);
    } else {
      u8* l = out.l8[i - 6];
      if (pr && def) std::memcpy(l, kDefault8x8[i - 6], 64);
      else std::memcpy(l, base ? base->l8[i - 6] : kDefault8x8[i - 6], 64);
    }
  }
  return out;
}

SliceHeader parse_slice_header(BitReader& br, u8 nal_hdr, const Sps& sps, const Pps& pps) {
  SliceHeader sh;
  sh.nal_type = nal_type(nal_hdr);
  sh.nal_ref_idc = nal_ref_idc(nal_hdr);
  sh.first_mb = br.ue();
  sh.slice_type = br.ue();
  sh.pps_id = br.ue();
  sh.frame_num = br.u(sps.log2_max_frame_num);
  if (!sps.frame_mbs_only && br.u1()) throw UnsupportedStream("interlaced H.264: field pictures (PAFF) are not supported");
  if (sh.idr()) sh.idr_pic_id = br.ue();
  if (sps.poc_type == 0) {
    sh.poc_lsb = br.u(sps.log2_max_poc_lsb);
    if (pps.bottom_field_pic_order) br.se();
  } else if (sps.poc_type == 1 && !sps.delta_pic_order_always_zero) {
    br.se();
    if (pps.bottom_field_pic_order) br.se();
  }
  if (pps.redundant_pic_cnt_present) br.ue();
  int st = sh.slice_type % 5;
  if (st == kB) br.u1();  // direct_spatial_mv_pred_flag
  sh.num_ref_idx_l0 = pps.num_ref_idx_l0_default;
  int num_l1 = pps.num_ref_idx_l1_default;
  if (st == kP || st == kSP || st == kB) {
    if (br.u1()) {
      sh.num_ref_idx_l0 = br.ue() + 1;
      if (st == kB) num_l1 = int(br.ue()) + 1;
    }
  }
  VEP_CHECK(sh.num_ref_idx_l0 <= 32 && num_l1 <= 32, "num_ref_idx out of range");
  // ref_pic_list_modification()
  if (st != kI && st != kSI) {
    if (br.u1()) {
      for (;;) {
        u32 idc = br.ue();
        if (idc == 3) break;
        VEP_CHECK(idc <= 5, "bad modification_of_pic_nums_idc");
        br.ue();
      }
    }
  }
  if (st == kB) {
    if (br.u1()) {
      for (;;) {
        u32 idc = br.ue();
        if (idc == 3) break;
        br.ue();
      }
    }
  }
  if ((pps.weighted_pred && (st == kP || st == kSP)) || (pps.weighted_bipred_idc == 1 && st == kB)) {
    // pred_weight_table(): skipped here (the general decoder, avc.cpp, applies it)
    br.ue();
    if (sps.chroma_format_idc != 0) br.ue();
    for (int l = 0; l < (st == kB ? 2 : 1); ++l) {
      const int nref = l == 0 ? sh.num_ref_idx_l0 : num_l1;
      for (int i = 0; i < nref; ++i) {
        if (br.u1()) {
          br.se();
          br.se();
        }
        if (sps.chroma_format_idc != 0 && br.u1())
          for (int k = 0; k < 4; ++k) br.se();
      }
    }
  }
  if (sh.nal_ref_idc != 0) {  // dec_ref_pic_marking()
    if (sh.idr()) {
      br.u1();
      br.u1();
    } else if (br.u1()) {
      for (;;) {
        u32 op = br.ue();
        if (op == 0) break;
        if (op == 1 || op == 3) br.ue();
        if (op == 2) br.ue();
        if (op == 3 || op == 6) br.ue();
        if (op == 4) br.ue();
      }
    }
  }
  if (pps.cabac && st != kI && st != kSI) br.ue();
  sh.slice_qp_delta = br.se();
  if (st == kSP || st == kSI) {
    if (st == kSP) br.u1();
    br.se();
  }
  if (pps.deblocking_filter_control) {
    sh.disable_deblocking = br.ue();
    if (sh.disable_deblocking != 1) {
      br.se();
      br.se();
    }
  }
  sh.data_bitpos = br.bitpos();
  return sh;
}

std::vector<u8> write_sps(const Sps& s) {
  BitWriter bw;
  bw.u(8, (0 << 7) | (3 << 5) | kNalSps);
  bw.u(8, s.profile_idc);
  bw.u(8, s.constraint_flags);
  bw.u(8, s.level_idc);
  bw.ue(s.sps_id);
  if (s.profile_idc >= 100) {
    bw.ue(s.chroma_format_idc);  // 4:2:0, or 4:0:0 (monochrome)
    bw.ue(u32(s.bit_depth_luma - 8));    // (High 10: 2)
    bw.ue(u32(s.bit_depth_chroma - 8));
    bw.u1(0);   // qpprime_y_zero_transform_bypass_flag
    bw.u1(s.scaling_matrix_present);
    if (s.scaling_matrix_present) {  // all eight lists explicit (delta-coded, §7.3.2.1.1.1)
      auto list = [&](const u8* v, int n) {
        bw.u1(1);
        int last = 8;
        for (int k = 0; k < n; ++k) {
          int d = (int(v[k]) - last + 256) % 256;
          if (d > 127) d -= 256;
          bw.se(d);
          last = v[k];
        }
      };
      for (int l = 0; l < 6; ++l) list(s.scaling.l4[l], 16);
      for (int l = 0; l < 2; ++l) list(s.scaling.l8[l], 64);
    }
  }
  bw.ue(s.log2_max_frame_num - 4);
  bw.ue(s.poc_type);
  if (s.poc_type == 0) bw.ue(s.log2_max_poc_lsb - 4);
  bw.ue(s.max_num_ref_frames);
  bw.u1(0);
  bw.ue(s.width_mbs - 1);
  bw.ue(s.height_map_units - 1);
  bw.u1(s.frame_mbs_only);
  if (!s.frame_mbs_only) bw.u1(s.mbaff);  // mb_adaptive_frame_field_flag
  bw.u1(s.direct_8x8 || !s.frame_mbs_only);  // direct_8x8_inference (1 for interlaced streams)
  bool crop = s.crop_left || s.crop_right || s.crop_top || s.crop_bottom;
  bw.u1(crop);
  if (crop) {
    // CropUnitX / Y (§7.4.2.1.1): SubWidthC / SubHeightC (4:2:2: 2 / 1; 4:0:0 and 4:4:4: 1 / 1)
    const int cx = s.chroma_format_idc == 0 || s.chroma_format_idc == 3 ? 1 : 2;
    const int cy = (s.chroma_format_idc == 1 ? 2 : 1) * (s.frame_mbs_only ? 1 : 2);
    bw.ue(s.crop_left / cx);
    bw.ue(s.crop_right / cx);
    bw.ue(s.crop_top / cy);
    VEP_CHECK(s.crop_bottom % cy == 0, "crop must be a multiple of CropUnitY rows");
    bw.ue(s.crop_bottom / cy);
  }
  bw.u1(1);  // vui
  bw.u1(0);  // aspect ratio
  bw.u1(0);  // overscan
  bw.u1(1);  // video_signal_type_present: BT.601 limited range (SMPTE 170M)
  bw.u(3, 5);
  bw.u1(0);
  bw.u1(1);
  bw.u(8, 6);
  bw.u(8, 6);
  bw.u(8, 6);
  bw.u1(0);  // chroma loc
  bw.u1(s.timing_info);
  if (s.timing_info) {
    bw.u(32, s.num_units_in_tick);
    bw.u(32, s.time_scale);
    bw.u1(1);
  }
  bw.u1(0);  // nal hrd
  bw.u1(0);  // vcl hrd
  bw.u1(0);  // pic_struct_present
  const bool restrict = s.max_num_reorder_frames >= 0;
  bw.u1(restrict);  // bitstream_restriction
  if (restrict) {
    bw.u1(1);   // motion_vectors_over_pic_boundaries_flag
    bw.ue(0);   // max_bytes_per_pic_denom
    bw.ue(0);   // max_bits_per_mb_denom
    bw.ue(16);  // log2_max_mv_length_horizontal
    bw.ue(16);  // log2_max_mv_length_vertical
    bw.ue(u32(s.max_num_reorder_frames));
    bw.ue(u32(std::max(s.max_dec_frame_buffering, s.max_num_ref_frames)));
  }
  bw.trailing();
  return bw.buf();
}

std::vector<u8> write_pps(const Pps& p) {
  BitWriter bw;
  bw.u(8, (0 << 7) | (3 << 5) | kNalPps);
  bw.ue(p.pps_id);
  bw.ue(p.sps_id);
  bw.u1(p.cabac);
  bw.u1(p.bottom_field_pic_order);  // bottom_field_pic_order_in_frame_present_flag
  bw.ue(0);
  bw.ue(p.num_ref_idx_l0_default - 1);
  bw.ue(p.num_ref_idx_l1_default - 1);
  bw.u1(p.weighted_pred);
  bw.u(2, u32(p.weighted_bipred_idc));
  bw.se(p.pic_init_qp - 26);
  bw.se(p.pic_init_qs - 26);
  bw.se(p.chroma_qp_index_offset);
  bw.u1(p.deblocking_filter_control);
  bw.u1(p.constrained_intra_pred);
  bw.u1(0);
  if (p.transform_8x8_mode || p.second_chroma_qp_index_offset != p.chroma_qp_index_offset) {
    bw.u1(p.transform_8x8_mode);
    bw.u1(0);  // pic_scaling_matrix_present_flag
    bw.se(p.second_chroma_qp_index_offset);
  }
  bw.trailing();
  return bw.buf();
}

void write_slice_header(BitWriter& bw, const SliceHeader& sh, const Sps& sps, const Pps& pps) {
  bw.u(8, (0 << 7) | (u32(sh.nal_ref_idc) << 5) | u32(sh.nal_type));
  bw.ue(sh.first_mb);
  bw.ue(sh.slice_type);
  bw.ue(sh.pps_id);
  bw.u(sps.log2_max_frame_num, sh.frame_num);
  if (sh.idr()) bw.ue(sh.idr_pic_id);
  if (sps.poc_type == 0) bw.u(sps.log2_max_poc_lsb, sh.poc_lsb);
  int st = sh.slice_type % 5;
  if (st == kP) {
    bw.u1(0);  // num_ref_idx_active_override_flag
    bw.u1(0);  // ref_pic_list_modification_flag_l0
  }
  if (sh.nal_ref_idc) {
    if (sh.idr()) {
      bw.u1(0);
      bw.u1(0);
    } else {
      bw.u1(0);
    }
  }
  bw.se(sh.slice_qp_delta);
  if (pps.deblocking_filter_control) {
    bw.ue(sh.disable_deblocking);
    if (sh.disable_deblocking != 1) {
      bw.se(0);
      bw.se(0);
    }
  }
}

std::vector<std::pair<size_t, size_t>> split_annexb(const u8* p, size_t n) {
  std::vector<std::pair<size_t, size_t>> out;
  size_t i = 0, start = SIZE_MAX;
  while (i + 2 < n) {
    if (p[i] == 0 && p[i + 1] == 0 && p[i + 2] == 1) {
      if (start != SIZE_MAX) {
        size_t end = i;
        while (end > start && p[end - 1] == 0) --end;  // trailing_zero_8bits / 4-byte code
        out.emplace_back(start, end - start);
      }
      i += 3;
      start = i;
    } else {
      ++i;
    }
  }
  if (start != SIZE_MAX && start < n) {
    size_t end = n;
    while (end > start && p[end - 1] == 0) --end;  // trailing_zero_8bits
    if (end > start) out.emplace_back(start, end - start);
  }
  return out;
}

std::vector<u8> avcc_record(const std::vector<u8>& sps, const std::vector<u8>& pps) {
  VEP_CHECK(sps.size() >= 4 && !pps.empty(), "avcC needs SPS and PPS");
  std::vector<u8> r;
  r.push_back(1);
  r.push_back(sps[1]);
  r.push_back(sps[2]);
  r.push_back(sps[3]);
  r.push_back(0xFF);  // lengthSizeMinusOne = 3
  r.push_back(0xE1);  // 1 SPS
  r.push_back(u8(sps.size() >> 8));
  r.push_back(u8(sps.size()));
  r.insert(r.end(), sps.begin(), sps.end());
  r.push_back(1);
  r.push_back(u8(pps.size() >> 8));
  r.push_back(u8(pps.size()));
  r.insert(r.end(), pps.begin(), pps.end());
  return r;
}

}  // namespace vep::h264
