// H.265/HEVC NAL, parameter-set and slice-segment-header layer (ITU-T H.265 §7.3) plus the
// HEVCDecoderConfigurationRecord (ISO/IEC 14496-15 §8.3.3) used by MP4 (hvcC) and enhanced-RTMP.
//
// The parsers read the general syntax (profile_tier_level with sub-layers, scaling lists,
// inter-predicted short-term RPS, long-term refs, VUI timing) so any real camera's parameter
// sets can be probed for size / frame rate; the native subset *decoder* (H265Parser in codec.h)
// then accepts the subset the synthetic farm emits and reports everything else as
// UnsupportedStream (the RocDecode/VCN backend's job — SURVEY.md §7.4 hard part 1).
//
// Reference parity: libavcodec hevc parser/decoder behind PyAV (python/read_image.py:87,
// python/rtsp_to_rtmp.py:92); BASELINE.json config 5 ("64x 4K30 H.265").
#pragma once

#include "bits.h"
#include "common.h"

namespace vep::hevc {

enum NalType : int {
  kTrailN = 0,
  kTrailR = 1,
  kRaslN = 8,
  kRaslR = 9,
  kBlaWLp = 16,
  kIdrWRadl = 19,
  kIdrNLp = 20,
  kCra = 21,
  kRsvIrap23 = 23,
  kVps = 32,
  kSps = 33,
  kPps = 34,
  kAud = 35,
  kSeiPrefix = 39,
  kSeiSuffix = 40,
  kAp = 48,  // RTP aggregation packet (RFC 7798)
  kFu = 49,  // RTP fragmentation unit (RFC 7798)
};

inline int nal_type(const u8* hdr) { return (hdr[0] >> 1) & 0x3f; }
inline bool is_irap(int t) { return t >= kBlaWLp && t <= kRsvIrap23; }
inline bool is_idr(int t) { return t == kIdrWRadl || t == kIdrNLp; }
inline bool is_vcl(int t) { return t < 32; }

struct ProfileTierLevel {
  int profile_space = 0, tier = 0, profile_idc = 1;
  u32 compat_flags = 0x60000000;     // Main + Main-compatible bits (1 and 2)
  u64 constraint_flags = 0x900000000000ull;  // 48 bits: progressive_source + frame_only
  int level_idc = 153;               // level 5.1 (x30)
};

struct ShortTermRps {
  int num_negative = 0, num_positive = 0;
  int delta_poc[32] = {};            // negatives then positives
  bool used[32] = {};
  int num_delta() const { return num_negative + num_positive; }
};

// Scaling lists (§7.3.4 scaling_list_data, §7.4.5): the coded lists in up-right diagonal order.
// matrixId 0..2 intra Y / Cb / Cr, 3..5 inter; sizeId 3 (32x32) uses matrixId 0 and 3 only.
struct ScalingList {
  u8 list[4][6][64] = {};
  u8 dc[4][6] = {};  // sizeId 2, 3: scaling_list_dc_coef_minus8 + 8
  ScalingList() { set_default(); }
  void set_default();  // Table 7-5 / 7-6 (flat 16 for 4x4)
  // ScalingFactor m of an n x n block (n = 4 << size_id), raster: out[y * n + x] = m[x][y].
  void factors(int size_id, int matrix_id, u8* out) const;
  bool operator==(const ScalingList& o) const;
};

struct Vps {
  int vps_id = 0;
  int max_sub_layers = 1;
  ProfileTierLevel ptl;
  bool timing_info = false;
  u32 num_units_in_tick = 0, time_scale = 0;
};

struct Sps {
  int vps_id = 0, sps_id = 0, max_sub_layers = 1;
  ProfileTierLevel ptl;
  int chroma_format_idc = 1;
  bool separate_colour_plane = false;
  int width = 0, height = 0;                 // pic_{width,height}_in_luma_samples (coded)
  int conf_left = 0, conf_right = 0, conf_top = 0, conf_bottom = 0;  // in luma samples
  int bit_depth_luma = 8, bit_depth_chroma = 8;
  int log2_max_poc_lsb = 8;
  int max_dec_pic_buffering = 2, max_num_reorder = 0, max_latency_increase_plus1 = 0;
  int log2_min_cb = 4, log2_ctb = 4;
  int log2_min_tb = 2, log2_max_tb = 4;
  int max_th_depth_inter = 0, max_th_depth_intra = 0;
  bool scaling_list = false, amp = false, sao = false;
  bool scaling_list_data = false;  // sps_scaling_list_data_present_flag (else the default lists)
  ScalingList sl;
  bool pcm = true;
  int pcm_bit_depth_luma = 8, pcm_bit_depth_chroma = 8;
  int log2_min_pcm = 4, log2_max_pcm = 4;
  bool pcm_loop_filter_disabled = true;
  std::vector<ShortTermRps> st_rps;
  bool long_term_refs = false;
  int num_long_term_ref_pics_sps = 0;
  std::vector<int> lt_poc_lsb_sps;    // lt_ref_pic_poc_lsb_sps[]
  std::vector<bool> lt_used_sps;      // used_by_curr_pic_lt_sps_flag[]
  bool temporal_mvp = false, strong_intra_smoothing = false;
  bool vui = false, video_signal_type = false;
  int video_format = 5, matrix_coeffs = 6;
  bool full_range = false;
  bool timing_info = false;
  u32 num_units_in_tick = 0, time_scale = 0;

  int ctb_size() const { return 1 << log2_ctb; }
  int width_ctbs() const { return (width + ctb_size() - 1) >> log2_ctb; }
  int height_ctbs() const { return (height + ctb_size() - 1) >> log2_ctb; }
  int out_width() const { return width - conf_left - conf_right; }
  int out_height() const { return height - conf_top - conf_bottom; }
  double fps() const {
    return (timing_info && num_units_in_tick) ? double(time_scale) / num_units_in_tick : 0.0;
  }
};

struct Pps {
  int pps_id = 0, sps_id = 0;
  bool dependent_slice_segments = false, output_flag_present = false;
  int num_extra_slice_header_bits = 0;
  bool sign_data_hiding = false, cabac_init_present = false;
  int num_ref_idx_l0_default = 1, num_ref_idx_l1_default = 1;
  int init_qp = 26;
  bool constrained_intra_pred = false, transform_skip = false, cu_qp_delta = false;
  int diff_cu_qp_delta_depth = 0;
  int beta_offset = 0, tc_offset = 0;        // pps_{beta,tc}_offset_div2 * 2
  int cb_qp_offset = 0, cr_qp_offset = 0;
  bool slice_chroma_qp_offsets_present = false;
  bool weighted_pred = false, weighted_bipred = false, transquant_bypass = false;
  bool tiles = false, entropy_coding_sync = false;
  int tile_cols = 1, tile_rows = 1;   // num_tile_{columns,rows}_minus1 + 1
  bool uniform_spacing = true;
  std::vector<int> col_width, row_height;  // explicit spacing: column_width_minus1 + 1 (cols - 1 entries)
  bool loop_filter_across_tiles = true;
  bool loop_filter_across_slices = false;
  bool deblocking_control = true, deblocking_override_enabled = false, deblocking_disabled = true;
  bool scaling_list = false, lists_modification = false;  // scaling_list: pps_scaling_list_data_present
  ScalingList sl;
  int log2_parallel_merge_level = 2;
  bool slice_header_extension = false;
  // Tile column / row boundaries in CTBs (§6.5.1, size cols + 1 / rows + 1).
  void tile_bounds(int wctbs, int hctbs, std::vector<int>& col_bd, std::vector<int>& row_bd) const;
};

// pred_weight_table (§7.3.6.3) with the derived weights / offsets (§7.4.7.3) per list and
// reference index: [list][ref][0 luma, 1 Cb, 2 Cr].
struct PredWeights {
  int luma_log2_denom = 0, chroma_log2_denom = 0;
  bool luma_flag[2][16] = {}, chroma_flag[2][16] = {};
  int w[2][16][3] = {}, o[2][16][3] = {};
  int log2_denom(int c) const { return c ? chroma_log2_denom : luma_log2_denom; }
};

enum SliceType : int { kB = 0, kP = 1, kI = 2 };

struct SliceHeader {
  int nal_type = 0;
  bool first_slice_in_pic = true;
  bool no_output_of_prior_pics = false;
  int pps_id = 0;
  bool dependent = false;
  int segment_address = 0;                   // CTB raster address
  int slice_type = kI;
  int poc_lsb = 0;
  ShortTermRps rps;                          // the picture's short-term RPS (non-IDR)
  int short_term_rps_idx = -1;               // -1: coded in the header, else the SPS set used
  // long-term entries (§7.3.6.1, derived per §7.4.7.1): num_long_term_sps come first
  int num_long_term = 0, num_long_term_sps = 0;
  int lt_idx_sps[32] = {};
  int lt_poc_lsb[32] = {};                   // PocLsbLt
  bool lt_used[32] = {};                     // UsedByCurrPicLt
  bool lt_msb_present[32] = {};              // delta_poc_msb_present_flag
  int lt_msb_cycle[32] = {};                 // DeltaPocMsbCycleLt (accumulated)
  int num_pic_total_curr = 0;
  bool weighted = false;                     // explicit weighted prediction in this slice
  PredWeights pwt;
  int num_ref_idx_l0 = 1, num_ref_idx_l1 = 1;
  bool list_mod[2] = {false, false};
  int list_entry[2][16] = {};                // ref_pic_list_modification entries
  bool mvd_l1_zero = false;
  bool cabac_init = false;
  bool collocated_from_l0 = true;
  int collocated_ref_idx = 0;
  int max_num_merge_cand = 5;
  int qp_delta = 0;
  int cb_qp_offset = 0, cr_qp_offset = 0;
  bool deblocking_disabled = true;
  int beta_offset = 0, tc_offset = 0;        // slice_{beta,tc}_offset_div2 * 2
  bool loop_filter_across_slices = false;
  bool sao_luma = false, sao_chroma = false;
  bool temporal_mvp = false;
  int num_entry_points = 0;
  std::vector<u32> entry_points;             // entry_point_offset_minus1 + 1 (bytes incl. emulation prevention)
  size_t data_bytepos = 0;                   // slice_segment_data() start within the RBSP
  char pict_char() const { return slice_type == kI ? 'I' : slice_type == kP ? 'P' : 'B'; }
};

// Parsers take the RBSP *including* the 2-byte NAL header.
Vps parse_vps(const u8* rbsp, size_t n);
Sps parse_sps(const u8* rbsp, size_t n);
Pps parse_pps(const u8* rbsp, size_t n);
// pps_id of a slice segment (first fields of the header) without full parsing.
int peek_slice_pps_id(const u8* rbsp, size_t n);
// `prev`: the header of the picture's previous slice segment (a dependent slice segment takes
// every slice-level field from it); may be null when the segment is independent.
SliceHeader parse_slice_header(const u8* rbsp, size_t n, const Sps& sps, const Pps& pps,
                               const SliceHeader* prev = nullptr);

// Writers (RBSP including the NAL header) for the synthetic encoder.
std::vector<u8> write_vps(const Vps& v);
std::vector<u8> write_sps(const Sps& s);
std::vector<u8> write_pps(const Pps& p);
// Writes the slice segment header through byte_alignment(); CABAC data follows.
void write_slice_header(BitWriter& bw, const SliceHeader& sh, const Sps& sps, const Pps& pps);
// General form (any slice type, explicit short-term RPS, SAO / reference / deblocking fields)
// for the closed-loop Main encoder.
void write_slice_header_full(BitWriter& bw, const SliceHeader& sh, const Sps& sps, const Pps& pps);
std::vector<u8> nal_header(int type, int tid_plus1 = 1);

// HEVCDecoderConfigurationRecord from escaped VPS/SPS/PPS NALs (MP4 hvcC, enhanced-RTMP).
std::vector<u8> hvcc_record(const std::vector<u8>& vps, const std::vector<u8>& sps,
                            const std::vector<u8>& pps);

}  // namespace vep::hevc
