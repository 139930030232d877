// H.264/AVC NAL, parameter-set and slice-header layer (ITU-T H.264 §7.3).
//
// Replaces libavcodec's h264 parser used behind PyAV in the reference
// (python/read_image.py:87, python/rtsp_to_rtmp.py:92 `demux`).
#pragma once

#include "bits.h"
#include "common.h"

namespace vep::h264 {

enum NalType : int {
  kNalSlice = 1,
  kNalIdr = 5,
  kNalSei = 6,
  kNalSps = 7,
  kNalPps = 8,
  kNalAud = 9,
  kNalStapA = 24,  // RTP aggregation (RFC 6184)
  kNalFuA = 28,    // RTP fragmentation (RFC 6184)
};

inline int nal_type(u8 hdr) { return hdr & 0x1f; }
inline int nal_ref_idc(u8 hdr) { return (hdr >> 5) & 3; }

// Scaling matrices (§7.4.2.1.1): 6 4x4 lists (Intra Y/Cb/Cr, Inter Y/Cb/Cr) and, for 4:2:0,
// 2 8x8 lists (Intra Y, Inter Y), each in zig-zag scan order as coded.
struct ScalingLists {
  u8 l4[6][16];
  u8 l8[2][64];
  void flat() {
    std::memset(l4, 16, sizeof l4);
    std::memset(l8, 16, sizeof l8);
  }
};
// Default_4x4_Intra / _Inter and Default_8x8_Intra / _Inter (Tables 7-3, 7-4), scan order.
extern const u8 kDefault4x4[2][16];
extern const u8 kDefault8x8[2][64];

struct Sps {
  int profile_idc = 0, constraint_flags = 0, level_idc = 0, sps_id = 0;
  int chroma_format_idc = 1, bit_depth_luma = 8, bit_depth_chroma = 8;
  bool transform_bypass = false;
  bool scaling_matrix_present = false;
  ScalingLists scaling;  // resolved (fall-back rule A; flat when not present)
  int log2_max_frame_num = 4, poc_type = 0, log2_max_poc_lsb = 4;
  // pic_order_cnt_type 1
  int offset_for_non_ref_pic = 0, offset_for_top_to_bottom_field = 0;
  std::vector<int> offset_for_ref_frame;
  int max_num_ref_frames = 1;
  bool gaps_in_frame_num_allowed = false;
  int width_mbs = 0, height_map_units = 0;
  bool frame_mbs_only = true, mbaff = false, direct_8x8 = true;
  int crop_left = 0, crop_right = 0, crop_top = 0, crop_bottom = 0;  // in luma samples
  bool timing_info = false;
  u32 num_units_in_tick = 0, time_scale = 0;
  bool delta_pic_order_always_zero = false;
  // VUI bitstream_restriction (-1 when absent)
  int max_num_reorder_frames = -1, max_dec_frame_buffering = -1;

  int height_mbs() const { return height_map_units * (frame_mbs_only ? 1 : 2); }
  int coded_width() const { return width_mbs * 16; }
  int coded_height() const { return height_mbs() * 16; }
  int width() const { return coded_width() - crop_left - crop_right; }
  int height() const { return coded_height() - crop_top - crop_bottom; }
  double fps() const {
    return (timing_info && num_units_in_tick) ? double(time_scale) / (2.0 * num_units_in_tick)
                                              : 0.0;
  }
  // MaxDpbFrames of the level (Table A-1) for this picture size, at most 16.
  int max_dpb_frames() const;
};

struct Pps {
  int pps_id = 0, sps_id = 0;
  bool cabac = false, bottom_field_pic_order = false;
  int num_slice_groups = 1;
  int num_ref_idx_l0_default = 1, num_ref_idx_l1_default = 1;
  bool weighted_pred = false;
  int weighted_bipred_idc = 0;
  int pic_init_qp = 26, pic_init_qs = 26, chroma_qp_index_offset = 0;
  bool deblocking_filter_control = false, constrained_intra_pred = false,
       redundant_pic_cnt_present = false;
  // High-profile tail
  bool transform_8x8_mode = false;
  bool scaling_matrix_present = false;
  ScalingLists scaling;  // resolved against the SPS at activation (resolve_scaling)
  bool scaling_list_present[8] = {};
  bool scaling_use_default[8] = {};
  int second_chroma_qp_index_offset = 0;
};

// The scaling lists in force for a picture: the PPS's (fall-back rule B against the SPS) when
// the PPS carries a matrix, else the SPS's (flat when neither does).
ScalingLists resolve_scaling(const Sps& sps, const Pps& pps);

enum SliceType : int { kP = 0, kB = 1, kI = 2, kSP = 3, kSI = 4 };

struct SliceHeader {
  int nal_type = 0, nal_ref_idc = 0;
  int first_mb = 0, slice_type = 0, pps_id = 0, frame_num = 0, idr_pic_id = 0;
  int poc_lsb = 0;
  int num_ref_idx_l0 = 1;
  int slice_qp_delta = 0, disable_deblocking = 0;
  size_t data_bitpos = 0;  // bit offset of slice_data() within the RBSP
  bool idr() const { return nal_type == kNalIdr; }
  char pict_char() const {  // PyAV pict_type.name analog
    switch (slice_type % 5) {
      case kI: return 'I';
      case kP: return 'P';
      case kB: return 'B';
      case kSP: return 'S';
      default: return 'i';
    }
  }
};

// Parse an SPS / PPS from the RBSP *including* the 1-byte NAL header.
Sps parse_sps(const u8* rbsp, size_t n);
Pps parse_pps(const u8* rbsp, size_t n);
// Parse slice header; reader is left at the start of slice_data().
SliceHeader parse_slice_header(BitReader& br, u8 nal_hdr, const Sps& sps, const Pps& pps);

// Writers for the synthetic encoder (RBSP including NAL header byte). The High-profile fields
// (profile_idc >= 100: chroma format / bit depth / no scaling matrix; PPS transform_8x8_mode,
// second_chroma_qp_index_offset; CABAC; weighted bi-prediction idc; VUI reorder depth) are
// written from the structs.
std::vector<u8> write_sps(const Sps& s);
std::vector<u8> write_pps(const Pps& p);
void write_slice_header(BitWriter& bw, const SliceHeader& sh, const Sps& sps, const Pps& pps);

// Annex-B byte stream splitter: returns [offset, size) of each NAL (start codes stripped).
std::vector<std::pair<size_t, size_t>> split_annexb(const u8* p, size_t n);

// AVCDecoderConfigurationRecord (ISO/IEC 14496-15) from escaped SPS/PPS NALs; used by FLV + MP4.
std::vector<u8> avcc_record(const std::vector<u8>& sps_nal, const std::vector<u8>& pps_nal);

}  // namespace vep::h264
