// H.265 parameter sets / slice segment header: parsers, writers and the hvcC record. See hevc.h.
#include "hevc.h"

#include <algorithm>
#include <cstring>

namespace vep::hevc {

namespace {

int ceil_log2(int v) {
  int n = 0;
  while ((1 << n) < v) ++n;
  return n;
}

void parse_ptl(BitReader& br, ProfileTierLevel& p, int max_sub_layers_minus1) {
  p.profile_space = int(br.u(2));
  p.tier = int(br.u1());
  p.profile_idc = int(br.u(5));
  p.compat_flags = br.u(32);
  p.constraint_flags = (u64(br.u(16)) << 32) | br.u(32);
  p.level_idc = int(br.u(8));
  bool prof[8] = {}, lvl[8] = {};
  for (int i = 0; i < max_sub_layers_minus1; ++i) {
    prof[i] = br.u1();
    lvl[i] = br.u1();
  }
  if (max_sub_layers_minus1 > 0)
    for (int i = max_sub_layers_minus1; i < 8; ++i) br.skip(2);
  for (int i = 0; i < max_sub_layers_minus1; ++i) {
    if (prof[i]) br.skip(88);
    if (lvl[i]) br.skip(8);
  }
}

void write_ptl(BitWriter& bw, const ProfileTierLevel& p) {
  bw.u(2, u32(p.profile_space));
  bw.u1(u32(p.tier));
  bw.u(5, u32(p.profile_idc));
  bw.u(32, p.compat_flags);
  bw.u(16, u32(p.constraint_flags >> 32));
  bw.u(32, u32(p.constraint_flags));
  bw.u(8, u32(p.level_idc));
}

// Table 7-6: default 8x8 (and up-sampled 16x16 / 32x32) lists, up-right diagonal order.
constexpr u8 kSlIntra[64] = {16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 17, 16, 17, 16, 17, 18, 17, 18, 18, 17, 18, 21,
                             19, 20, 21, 20, 19, 21, 24, 22, 22, 24, 24, 22, 22, 24, 25, 25, 27, 30, 27, 25, 25, 29,
                             31, 35, 35, 31, 29, 36, 41, 44, 41, 36, 47, 54, 54, 47, 65, 70, 65, 88, 88, 115};
constexpr u8 kSlInter[64] = {16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 17, 17, 17, 17, 17, 18, 18, 18, 18, 18, 18, 20,
                             20, 20, 20, 20, 20, 20, 24, 24, 24, 24, 24, 24, 24, 24, 25, 25, 25, 25, 25, 25, 25, 28,
                             28, 28, 28, 28, 28, 33, 33, 33, 33, 33, 41, 41, 41, 41, 54, 54, 54, 71, 71, 91};

void set_default_list(ScalingList& sl, int size_id, int matrix_id) {
  for (int i = 0; i < 64; ++i)
    sl.list[size_id][matrix_id][i] = size_id == 0 ? 16 : (matrix_id < 3 ? kSlIntra[i] : kSlInter[i]);
  sl.dc[size_id][matrix_id] = 16;
}

// §7.3.4 (matrixId numbering of the range extensions: sizeId 3 uses 0 and 3)
void parse_scaling_list_data(BitReader& br, ScalingList& sl) {
  for (int size_id = 0; size_id < 4; ++size_id) {
    const int step = size_id == 3 ? 3 : 1;
    for (int matrix_id = 0; matrix_id < 6; matrix_id += step) {
      if (!br.u1()) {  // scaling_list_pred_mode_flag
        const int delta = int(br.ue());
        if (delta == 0) {
          set_default_list(sl, size_id, matrix_id);
        } else {
          const int ref = matrix_id - delta * step;
          VEP_CHECK(ref >= 0, "bad scaling_list_pred_matrix_id_delta");
          std::memcpy(sl.list[size_id][matrix_id], sl.list[size_id][ref], 64);
          sl.dc[size_id][matrix_id] = sl.dc[size_id][ref];
        }
      } else {
        int next = 8;
        const int num = std::min(64, 1 << (4 + (size_id << 1)));
        if (size_id > 1) {
          const int dc = br.se() + 8;
          VEP_CHECK(dc >= 1 && dc <= 255, "bad scaling_list_dc_coef_minus8");
          next = dc;
          sl.dc[size_id][matrix_id] = u8(dc);
        }
        for (int i = 0; i < num; ++i) {
          const int delta = br.se();
          VEP_CHECK(delta >= -128 && delta <= 127, "bad scaling_list_delta_coef");
          next = (next + delta + 256) % 256;
          VEP_CHECK(next > 0, "scaling list entry 0");
          sl.list[size_id][matrix_id][i] = u8(next);
        }
      }
    }
  }
  for (int m = 0; m < 6; ++m)  // (4:2:0 never uses the 32x32 chroma matrices: keep them defined)
    if (m % 3) {
      std::memcpy(sl.list[3][m], sl.list[2][m], 64);
      sl.dc[3][m] = sl.dc[2][m];
    }
}

// Writes every list explicitly (pred_mode_flag 1), or as "default" when it is the default.
void write_scaling_list_data(BitWriter& bw, const ScalingList& sl) {
  ScalingList def;
  for (int size_id = 0; size_id < 4; ++size_id) {
    const int step = size_id == 3 ? 3 : 1;
    for (int matrix_id = 0; matrix_id < 6; matrix_id += step) {
      const int num = std::min(64, 1 << (4 + (size_id << 1)));
      const bool is_def = std::memcmp(sl.list[size_id][matrix_id], def.list[size_id][matrix_id], size_t(num)) == 0 &&
                          (size_id < 2 || sl.dc[size_id][matrix_id] == 16);
      if (is_def) {
        bw.u1(0);
        bw.ue(0);
        continue;
      }
      bw.u1(1);
      int next = 8;
      if (size_id > 1) {
        bw.se(sl.dc[size_id][matrix_id] - 8);
        next = sl.dc[size_id][matrix_id];
      }
      for (int i = 0; i < num; ++i) {
        int d = int(sl.list[size_id][matrix_id][i]) - next;
        if (d > 127) d -= 256;
        if (d < -128) d += 256;
        bw.se(d);
        next = sl.list[size_id][matrix_id][i];
      }
    }
  }
}

// Up-right diagonal scan of a blk x blk block (§6.5.3): (x, y) of scan position i.
void diag_scan(int blk, int* xs, int* ys) {
  int i = 0, x = 0, y = 0;
  while (i < blk * blk) {
    while (y >= 0) {
      if (x < blk && y < blk) xs[i] = x, ys[i] = y, ++i;
      --y;
      ++x;
    }
    y = x;
    x = 0;
  }
}

// §7.3.7 + the inter-RPS derivation of §7.4.8 (eqs 7-61, 7-62).
ShortTermRps parse_st_rps(BitReader& br, int idx, const std::vector<ShortTermRps>& sets) {
  ShortTermRps r;
  const int num_sets = int(sets.size());
  bool inter = false;
  if (idx != 0) inter = br.u1();
  if (inter) {
    int delta_idx = 1;
    if (idx == num_sets) delta_idx = int(br.ue()) + 1;
    VEP_CHECK(delta_idx <= idx, "bad delta_idx_minus1 in st_ref_pic_set");
    const int sign = int(br.u1());
    const int delta_rps = (1 - 2 * sign) * (int(br.ue()) + 1);
    const ShortTermRps& ref = sets[size_t(idx - delta_idx)];
    const int nref = ref.num_delta();
    bool used[33] = {}, use_delta[33] = {};
    for (int j = 0; j <= nref; ++j) {
      used[j] = br.u1();
      use_delta[j] = used[j] ? true : bool(br.u1());
    }
    std::vector<std::pair<int, bool>> s0, s1;
    const int rn = ref.num_negative, rp = ref.num_positive;
    for (int j = rp - 1; j >= 0; --j) {
      int d = ref.delta_poc[rn + j] + delta_rps;
      if (d < 0 && use_delta[rn + j]) s0.push_back({d, used[rn + j]});
    }
    if (delta_rps < 0 && use_delta[nref]) s0.push_back({delta_rps, used[nref]});
    for (int j = 0; j < rn; ++j) {
      int d = ref.delta_poc[j] + delta_rps;
      if (d < 0 && use_delta[j]) s0.push_back({d, used[j]});
    }
    for (int j = rn - 1; j >= 0; --j) {
      int d = ref.delta_poc[j] + delta_rps;
      if (d > 0 && use_delta[j]) s1.push_back({d, used[j]});
    }
    if (delta_rps > 0 && use_delta[nref]) s1.push_back({delta_rps, used[nref]});
    for (int j = 0; j < rp; ++j) {
      int d = ref.delta_poc[rn + j] + delta_rps;
      if (d > 0 && use_delta[rn + j]) s1.push_back({d, used[rn + j]});
    }
    VEP_CHECK(s0.size() + s1.size() <= 32, "too many pictures in st_ref_pic_set");
    r.num_negative = int(s0.size());
    r.num_positive = int(s1.size());
    for (size_t i = 0; i < s0.size(); ++i) r.delta_poc[i] = s0[i].first, r.used[i] = s0[i].second;
    for (size_t i = 0; i < s1.size(); ++i)
      r.delta_poc[s0.size() + i] = s1[i].first, r.used[s0.size() + i] = s1[i].second;
  } else {
    r.num_negative = int(br.ue());
    r.num_positive = int(br.ue());
    VEP_CHECK(r.num_negative + r.num_positive <= 32, "too many pictures in st_ref_pic_set");
    int poc = 0;
    for (int i = 0; i < r.num_negative; ++i) {
      poc -= int(br.ue()) + 1;
      r.delta_poc[i] = poc;
      r.used[i] = br.u1();
    }
    poc = 0;
    for (int i = 0; i < r.num_positive; ++i) {
      poc += int(br.ue()) + 1;
      r.delta_poc[r.num_negative + i] = poc;
      r.used[r.num_negative + i] = br.u1();
    }
  }
  return r;
}

void write_st_rps(BitWriter& bw, int idx, const ShortTermRps& r) {
  if (idx != 0) bw.u1(0);  // no inter-RPS prediction
  bw.ue(u32(r.num_negative));
  bw.ue(u32(r.num_positive));
  int prev = 0;
  for (int i = 0; i < r.num_negative; ++i) {
    bw.ue(u32(prev - r.delta_poc[i] - 1));
    prev = r.delta_poc[i];
    bw.u1(r.used[i]);
  }
  prev = 0;
  for (int i = 0; i < r.num_positive; ++i) {
    const int d = r.delta_poc[r.num_negative + i];
    bw.ue(u32(d - prev - 1));
    prev = d;
    bw.u1(r.used[r.num_negative + i]);
  }
}

void parse_pred_weights(BitReader& br, SliceHeader& sh) {
  PredWeights& w = sh.pwt;
  w = PredWeights{};
  w.luma_log2_denom = int(br.ue());
  VEP_CHECK(w.luma_log2_denom <= 7, "bad luma_log2_weight_denom");
  w.chroma_log2_denom = w.luma_log2_denom + br.se();
  VEP_CHECK(w.chroma_log2_denom >= 0 && w.chroma_log2_denom <= 7, "bad delta_chroma_log2_weight_denom");
  for (int l = 0; l < (sh.slice_type == kB ? 2 : 1); ++l) {
    const int nref = l == 0 ? sh.num_ref_idx_l0 : sh.num_ref_idx_l1;
    for (int i = 0; i < nref; ++i) w.luma_flag[l][i] = br.u1();
    for (int i = 0; i < nref; ++i) w.chroma_flag[l][i] = br.u1();
    for (int i = 0; i < nref; ++i) {
      w.w[l][i][0] = 1 << w.luma_log2_denom;
      w.o[l][i][0] = 0;
      if (w.luma_flag[l][i]) {
        const int dw = br.se(), off = br.se();
        VEP_CHECK(dw >= -128 && dw <= 127 && off >= -128 && off <= 127, "bad luma weight / offset");
        w.w[l][i][0] += dw;
        w.o[l][i][0] = off;
      }
      for (int c = 1; c <= 2; ++c) {
        w.w[l][i][c] = 1 << w.chroma_log2_denom;
        w.o[l][i][c] = 0;
        if (w.chroma_flag[l][i]) {
          const int dw = br.se(), doff = br.se();
          VEP_CHECK(dw >= -128 && dw <= 127 && doff >= -512 && doff <= 511, "bad chroma weight / offset");
          w.w[l][i][c] += dw;
          w.o[l][i][c] = std::clamp(128 + doff - ((128 * w.w[l][i][c]) >> w.chroma_log2_denom), -128, 127);
        }
      }
    }
  }
}

void write_pred_weights(BitWriter& bw, const SliceHeader& sh) {
  const PredWeights& w = sh.pwt;
  bw.ue(u32(w.luma_log2_denom));
  bw.se(w.chroma_log2_denom - w.luma_log2_denom);
  for (int l = 0; l < (sh.slice_type == kB ? 2 : 1); ++l) {
    const int nref = l == 0 ? sh.num_ref_idx_l0 : sh.num_ref_idx_l1;
    for (int i = 0; i < nref; ++i) bw.u1(w.luma_flag[l][i]);
    for (int i = 0; i < nref; ++i) bw.u1(w.chroma_flag[l][i]);
    for (int i = 0; i < nref; ++i) {
      if (w.luma_flag[l][i]) {
        bw.se(w.w[l][i][0] - (1 << w.luma_log2_denom));
        bw.se(w.o[l][i][0]);
      }
      if (w.chroma_flag[l][i])
        for (int c = 1; c <= 2; ++c) {
          bw.se(w.w[l][i][c] - (1 << w.chroma_log2_denom));
          const int doff = w.o[l][i][c] - 128 + ((128 * w.w[l][i][c]) >> w.chroma_log2_denom);
          VEP_CHECK(doff >= -512 && doff <= 511, "chroma offset not codable with this weight");
          bw.se(doff);
        }
    }
  }
}

void check_nal(const u8* rbsp, size_t n, int want) {
  VEP_CHECK(n >= 3, "NAL too short");
  VEP_CHECK(nal_type(rbsp) == want, "unexpected HEVC NAL type");
}

}  // namespace

void ScalingList::set_default() {
  for (int size_id = 0; size_id < 4; ++size_id)
    for (int m = 0; m < 6; ++m) set_default_list(*this, size_id, m);
}

bool ScalingList::operator==(const ScalingList& o) const {
  return std::memcmp(list, o.list, sizeof list) == 0 && std::memcmp(dc, o.dc, sizeof dc) == 0;
}

void ScalingList::factors(int size_id, int matrix_id, u8* out) const {
  const int n = 4 << size_id;
  const int blk = size_id == 0 ? 4 : 8, rep = n / blk;
  int xs[64], ys[64];
  diag_scan(blk, xs, ys);
  for (int i = 0; i < blk * blk; ++i)
    for (int j = 0; j < rep; ++j)
      for (int k = 0; k < rep; ++k) out[(ys[i] * rep + j) * n + xs[i] * rep + k] = list[size_id][matrix_id][i];
  if (size_id >= 2) out[0] = dc[size_id][matrix_id];
}

void Pps::tile_bounds(int wctbs, int hctbs, std::vector<int>& col_bd, std::vector<int>& row_bd) const {
  auto make = [&](int count, int total, const std::vector<int>& sizes, std::vector<int>& bd) {
    bd.assign(size_t(count) + 1, 0);
    for (int i = 0; i < count; ++i) {
      int size;
      if (!tiles || count == 1) size = total;
      else if (uniform_spacing) size = ((i + 1) * total) / count - (i * total) / count;
      else size = i < count - 1 ? sizes[size_t(i)] : total - bd[size_t(i)];
      VEP_CHECK(size > 0, "HEVC: empty tile column / row");
      bd[size_t(i) + 1] = bd[size_t(i)] + size;
    }
    VEP_CHECK(bd[size_t(count)] == total, "HEVC: tile sizes do not cover the picture");
  };
  make(tiles ? tile_cols : 1, wctbs, col_width, col_bd);
  make(tiles ? tile_rows : 1, hctbs, row_height, row_bd);
}

std::vector<u8> nal_header(int type, int tid_plus1) {
  return {u8((type & 0x3f) << 1), u8(tid_plus1 & 7)};
}

Vps parse_vps(const u8* rbsp, size_t n) {
  check_nal(rbsp, n, kVps);
  BitReader br(rbsp + 2, n - 2);
  Vps v;
  v.vps_id = int(br.u(4));
  br.skip(2);  // base_layer_internal / available
  br.skip(6);  // max_layers_minus1
  v.max_sub_layers = int(br.u(3)) + 1;
  br.skip(1 + 16);
  parse_ptl(br, v.ptl, v.max_sub_layers - 1);
  const bool ordering = br.u1();
  for (int i = ordering ? 0 : v.max_sub_layers - 1; i < v.max_sub_layers; ++i) {
    br.ue();
    br.ue();
    br.ue();
  }
  const int max_layer_id = int(br.u(6));
  const int num_layer_sets = int(br.ue()) + 1;
  for (int i = 1; i < num_layer_sets; ++i) br.skip(size_t(max_layer_id) + 1);
  v.timing_info = br.u1();
  if (v.timing_info) {
    v.num_units_in_tick = br.u(32);
    v.time_scale = br.u(32);
  }
  return v;  // hrd parameters / extensions are not needed
}

Sps parse_sps(const u8* rbsp, size_t n) {
  check_nal(rbsp, n, kSps);
  BitReader br(rbsp + 2, n - 2);
  Sps s;
  s.vps_id = int(br.u(4));
  s.max_sub_layers = int(br.u(3)) + 1;
  br.skip(1);
  parse_ptl(br, s.ptl, s.max_sub_layers - 1);
  s.sps_id = int(br.ue());
  VEP_CHECK(s.sps_id < 16, "sps id out of range");
  s.chroma_format_idc = int(br.ue());
  if (s.chroma_format_idc == 3) s.separate_colour_plane = br.u1();
  s.width = int(br.ue());
  s.height = int(br.ue());
  VEP_CHECK(s.width > 0 && s.height > 0 && s.width <= 16888 && s.height <= 16888,
            "bad HEVC picture size");
  if (br.u1()) {
    const int sw = (s.chroma_format_idc == 1 || s.chroma_format_idc == 2) ? 2 : 1;
    const int sh = (s.chroma_format_idc == 1) ? 2 : 1;
    s.conf_left = int(br.ue()) * sw;
    s.conf_right = int(br.ue()) * sw;
    s.conf_top = int(br.ue()) * sh;
    s.conf_bottom = int(br.ue()) * sh;
  }
  s.bit_depth_luma = int(br.ue()) + 8;
  s.bit_depth_chroma = int(br.ue()) + 8;
  s.log2_max_poc_lsb = int(br.ue()) + 4;
  VEP_CHECK(s.log2_max_poc_lsb <= 16, "bad log2_max_pic_order_cnt_lsb");
  const bool ordering = br.u1();
  for (int i = ordering ? 0 : s.max_sub_layers - 1; i < s.max_sub_layers; ++i) {
    s.max_dec_pic_buffering = int(br.ue()) + 1;
    s.max_num_reorder = int(br.ue());
    s.max_latency_increase_plus1 = int(br.ue());
  }
  s.log2_min_cb = int(br.ue()) + 3;
  s.log2_ctb = s.log2_min_cb + int(br.ue());
  s.log2_min_tb = int(br.ue()) + 2;
  s.log2_max_tb = s.log2_min_tb + int(br.ue());
  VEP_CHECK(s.log2_ctb <= 6 && s.log2_max_tb <= 5, "bad HEVC block sizes");
  s.max_th_depth_inter = int(br.ue());
  s.max_th_depth_intra = int(br.ue());
  s.scaling_list = br.u1();
  if (s.scaling_list) {
    s.scaling_list_data = br.u1();
    if (s.scaling_list_data) parse_scaling_list_data(br, s.sl);
  }
  s.amp = br.u1();
  s.sao = br.u1();
  s.pcm = br.u1();
  if (s.pcm) {
    s.pcm_bit_depth_luma = int(br.u(4)) + 1;
    s.pcm_bit_depth_chroma = int(br.u(4)) + 1;
    s.log2_min_pcm = int(br.ue()) + 3;
    s.log2_max_pcm = s.log2_min_pcm + int(br.ue());
    s.pcm_loop_filter_disabled = br.u1();
  }
  const int nsets = int(br.ue());
  VEP_CHECK(nsets <= 64, "too many short-term RPS");
  s.st_rps.clear();
  for (int i = 0; i < nsets; ++i) s.st_rps.push_back(parse_st_rps(br, i, s.st_rps));
  s.long_term_refs = br.u1();
  if (s.long_term_refs) {
    s.num_long_term_ref_pics_sps = int(br.ue());
    VEP_CHECK(s.num_long_term_ref_pics_sps <= 32, "too many SPS long-term pictures");
    for (int i = 0; i < s.num_long_term_ref_pics_sps; ++i) {
      s.lt_poc_lsb_sps.push_back(int(br.u(s.log2_max_poc_lsb)));
      s.lt_used_sps.push_back(br.u1());
    }
  }
  s.temporal_mvp = br.u1();
  s.strong_intra_smoothing = br.u1();
  s.vui = br.u1();
  if (s.vui) {
    if (br.u1()) {  // aspect_ratio_info
      if (br.u(8) == 255) br.skip(32);
    }
    if (br.u1()) br.skip(1);  // overscan
    s.video_signal_type = br.u1();
    if (s.video_signal_type) {
      s.video_format = int(br.u(3));
      s.full_range = br.u1();
      if (br.u1()) {
        br.skip(16);
        s.matrix_coeffs = int(br.u(8));
      }
    }
    if (br.u1()) {  // chroma_loc_info
      br.ue();
      br.ue();
    }
    br.skip(3);      // neutral_chroma, field_seq, frame_field_info
    if (br.u1()) {   // default display window
      for (int i = 0; i < 4; ++i) br.ue();
    }
    s.timing_info = br.u1();
    if (s.timing_info) {
      s.num_units_in_tick = br.u(32);
      s.time_scale = br.u(32);
    }
    // hrd parameters / bitstream restriction / extensions are not needed
  }
  return s;
}

Pps parse_pps(const u8* rbsp, size_t n) {
  check_nal(rbsp, n, kPps);
  BitReader br(rbsp + 2, n - 2);
  Pps p;
  p.pps_id = int(br.ue());
  VEP_CHECK(p.pps_id < 64, "pps id out of range");
  p.sps_id = int(br.ue());
  p.dependent_slice_segments = br.u1();
  p.output_flag_present = br.u1();
  p.num_extra_slice_header_bits = int(br.u(3));
  p.sign_data_hiding = br.u1();
  p.cabac_init_present = br.u1();
  p.num_ref_idx_l0_default = int(br.ue()) + 1;
  p.num_ref_idx_l1_default = int(br.ue()) + 1;
  p.init_qp = 26 + br.se();
  p.constrained_intra_pred = br.u1();
  p.transform_skip = br.u1();
  p.cu_qp_delta = br.u1();
  if (p.cu_qp_delta) p.diff_cu_qp_delta_depth = int(br.ue());
  p.cb_qp_offset = br.se();
  p.cr_qp_offset = br.se();
  p.slice_chroma_qp_offsets_present = br.u1();
  p.weighted_pred = br.u1();
  p.weighted_bipred = br.u1();
  p.transquant_bypass = br.u1();
  p.tiles = br.u1();
  p.entropy_coding_sync = br.u1();
  if (p.tiles) {
    p.tile_cols = int(br.ue()) + 1;
    p.tile_rows = int(br.ue()) + 1;
    VEP_CHECK(p.tile_cols <= 64 && p.tile_rows <= 64, "too many tiles");
    p.uniform_spacing = br.u1();
    if (!p.uniform_spacing) {
      for (int i = 0; i < p.tile_cols - 1; ++i) p.col_width.push_back(int(br.ue()) + 1);
      for (int i = 0; i < p.tile_rows - 1; ++i) p.row_height.push_back(int(br.ue()) + 1);
    }
    p.loop_filter_across_tiles = br.u1();
  }
  p.loop_filter_across_slices = br.u1();
  p.deblocking_control = br.u1();
  p.deblocking_override_enabled = false;
  p.deblocking_disabled = false;
  if (p.deblocking_control) {
    p.deblocking_override_enabled = br.u1();
    p.deblocking_disabled = br.u1();
    if (!p.deblocking_disabled) {
      p.beta_offset = br.se() * 2;
      p.tc_offset = br.se() * 2;
    }
  }
  p.scaling_list = br.u1();
  if (p.scaling_list) parse_scaling_list_data(br, p.sl);
  p.lists_modification = br.u1();
  p.log2_parallel_merge_level = int(br.ue()) + 2;
  p.slice_header_extension = br.u1();
  return p;
}

int peek_slice_pps_id(const u8* rbsp, size_t n) {
  VEP_CHECK(n >= 3, "slice NAL too short");
  BitReader br(rbsp + 2, n - 2);
  br.u1();                                       // first_slice_segment_in_pic_flag
  if (is_irap(nal_type(rbsp))) br.u1();          // no_output_of_prior_pics_flag
  return int(br.ue());
}

SliceHeader parse_slice_header(const u8* rbsp, size_t n, const Sps& sps, const Pps& pps, const SliceHeader* prev) {
  VEP_CHECK(n >= 3, "slice NAL too short");
  BitReader br(rbsp + 2, n - 2);
  SliceHeader sh;
  sh.nal_type = nal_type(rbsp);
  sh.first_slice_in_pic = br.u1();
  if (is_irap(sh.nal_type)) sh.no_output_of_prior_pics = br.u1();
  sh.pps_id = int(br.ue());
  if (!sh.first_slice_in_pic) {
    if (pps.dependent_slice_segments) sh.dependent = br.u1();
    const int ctbs = sps.width_ctbs() * sps.height_ctbs();
    sh.segment_address = int(br.u(ceil_log2(ctbs)));
    VEP_CHECK(sh.segment_address < ctbs, "slice_segment_address out of range");
  }
  if (sh.dependent) {  // every slice-level field comes from the slice's independent segment
    VEP_CHECK(prev != nullptr, "dependent slice segment without a preceding slice segment");
    SliceHeader d = *prev;
    d.nal_type = sh.nal_type;
    d.first_slice_in_pic = false;
    d.pps_id = sh.pps_id;
    d.dependent = true;
    d.segment_address = sh.segment_address;
    d.num_entry_points = 0;
    d.entry_points.clear();
    sh = std::move(d);
  } else {
    br.skip(size_t(pps.num_extra_slice_header_bits));
    sh.slice_type = int(br.ue());
    VEP_CHECK(sh.slice_type <= 2, "bad slice_type");
    if (pps.output_flag_present) br.u1();
    if (sps.separate_colour_plane) br.skip(2);
    int num_pic_total_curr = 0;
    sh.deblocking_disabled = pps.deblocking_disabled;
    if (!is_idr(sh.nal_type)) {
      sh.poc_lsb = int(br.u(sps.log2_max_poc_lsb));
      const int nsets = int(sps.st_rps.size());
      ShortTermRps rps;
      if (!br.u1()) {
        rps = parse_st_rps(br, nsets, sps.st_rps);
      } else {
        VEP_CHECK(nsets > 0, "slice selects an SPS RPS but the SPS has none");
        int idx = nsets > 1 ? int(br.u(ceil_log2(nsets))) : 0;
        VEP_CHECK(idx < nsets, "short_term_ref_pic_set_idx out of range");
        rps = sps.st_rps[size_t(idx)];
        sh.short_term_rps_idx = idx;
      }
      sh.rps = rps;
      for (int i = 0; i < rps.num_delta(); ++i) num_pic_total_curr += rps.used[i];
      if (sps.long_term_refs) {  // §7.3.6.1 long-term entries, §7.4.7.1 derivations
        if (sps.num_long_term_ref_pics_sps > 0) sh.num_long_term_sps = int(br.ue());
        VEP_CHECK(sh.num_long_term_sps <= sps.num_long_term_ref_pics_sps, "num_long_term_sps out of range");
        sh.num_long_term = sh.num_long_term_sps + int(br.ue());
        VEP_CHECK(sh.num_long_term + rps.num_delta() <= 32, "too many reference pictures");
        for (int i = 0; i < sh.num_long_term; ++i) {
          if (i < sh.num_long_term_sps) {
            int idx = 0;
            if (sps.num_long_term_ref_pics_sps > 1) idx = int(br.u(ceil_log2(sps.num_long_term_ref_pics_sps)));
            VEP_CHECK(idx < sps.num_long_term_ref_pics_sps, "lt_idx_sps out of range");
            sh.lt_idx_sps[i] = idx;
            sh.lt_poc_lsb[i] = sps.lt_poc_lsb_sps[size_t(idx)];
            sh.lt_used[i] = sps.lt_used_sps[size_t(idx)];
          } else {
            sh.lt_poc_lsb[i] = int(br.u(sps.log2_max_poc_lsb));
            sh.lt_used[i] = br.u1();
          }
          sh.lt_msb_present[i] = br.u1();
          const int cycle = sh.lt_msb_present[i] ? int(br.ue()) : 0;
          sh.lt_msb_cycle[i] = (i == 0 || i == sh.num_long_term_sps) ? cycle : cycle + sh.lt_msb_cycle[i - 1];
          num_pic_total_curr += sh.lt_used[i];
        }
      }
      if (sps.temporal_mvp) sh.temporal_mvp = br.u1();
    }
    sh.num_pic_total_curr = num_pic_total_curr;
    if (sps.sao) {
      sh.sao_luma = br.u1();
      if (sps.chroma_format_idc != 0) sh.sao_chroma = br.u1();
    }
    if (sh.slice_type != kI) {
      sh.num_ref_idx_l0 = pps.num_ref_idx_l0_default;
      int l1 = pps.num_ref_idx_l1_default;
      if (br.u1()) {
        sh.num_ref_idx_l0 = int(br.ue()) + 1;
        if (sh.slice_type == kB) l1 = int(br.ue()) + 1;
      }
      VEP_CHECK(sh.num_ref_idx_l0 <= 15 && l1 <= 15, "num_ref_idx out of range");
      sh.num_ref_idx_l1 = sh.slice_type == kB ? l1 : 0;
      if (pps.lists_modification && num_pic_total_curr > 1) {
        const int bits = ceil_log2(num_pic_total_curr);
        sh.list_mod[0] = br.u1();
        if (sh.list_mod[0])
          for (int i = 0; i < sh.num_ref_idx_l0; ++i) sh.list_entry[0][i] = int(br.u(bits));
        if (sh.slice_type == kB) {
          sh.list_mod[1] = br.u1();
          if (sh.list_mod[1])
            for (int i = 0; i < l1; ++i) sh.list_entry[1][i] = int(br.u(bits));
        }
      }
      if (sh.slice_type == kB) sh.mvd_l1_zero = br.u1();
      if (pps.cabac_init_present) sh.cabac_init = br.u1();
      if (sh.temporal_mvp) {
        bool from_l0 = true;
        if (sh.slice_type == kB) from_l0 = br.u1();
        sh.collocated_from_l0 = from_l0;
        if ((from_l0 && sh.num_ref_idx_l0 > 1) || (!from_l0 && l1 > 1)) sh.collocated_ref_idx = int(br.ue());
        VEP_CHECK(sh.collocated_ref_idx < (from_l0 ? sh.num_ref_idx_l0 : l1), "collocated_ref_idx out of range");
      }
      sh.weighted = (pps.weighted_pred && sh.slice_type == kP) || (pps.weighted_bipred && sh.slice_type == kB);
      if (sh.weighted) parse_pred_weights(br, sh);
      sh.max_num_merge_cand = 5 - int(br.ue());
      VEP_CHECK(sh.max_num_merge_cand >= 1 && sh.max_num_merge_cand <= 5, "bad merge candidates");
    }
    sh.qp_delta = br.se();
    if (pps.slice_chroma_qp_offsets_present) {
      sh.cb_qp_offset = br.se();
      sh.cr_qp_offset = br.se();
    }
    sh.beta_offset = pps.beta_offset;
    sh.tc_offset = pps.tc_offset;
    bool override_flag = false;
    if (pps.deblocking_override_enabled) override_flag = br.u1();
    if (override_flag) {
      sh.deblocking_disabled = br.u1();
      if (!sh.deblocking_disabled) {
        sh.beta_offset = br.se() * 2;
        sh.tc_offset = br.se() * 2;
      }
    }
    sh.loop_filter_across_slices = pps.loop_filter_across_slices;
    if (pps.loop_filter_across_slices && (sh.sao_luma || sh.sao_chroma || !sh.deblocking_disabled))
      sh.loop_filter_across_slices = br.u1();
  }
  if (pps.tiles || pps.entropy_coding_sync) {
    sh.num_entry_points = int(br.ue());
    VEP_CHECK(sh.num_entry_points <= 4096, "too many entry points");
    if (sh.num_entry_points > 0) {
      const int len = int(br.ue()) + 1;
      VEP_CHECK(len <= 32, "bad entry point offset length");
      for (int i = 0; i < sh.num_entry_points; ++i) sh.entry_points.push_back(br.u(len) + 1);
    }
  }
  if (pps.slice_header_extension) {
    const int len = int(br.ue());
    br.skip(size_t(len) * 8);
  }
  VEP_CHECK(br.u1() == 1, "slice header byte_alignment() must start with 1");
  br.align();
  sh.data_bytepos = br.bytepos() + 2;
  return sh;
}

std::vector<u8> write_vps(const Vps& v) {
  BitWriter bw;
  for (u8 b : nal_header(kVps)) bw.u(8, b);
  bw.u(4, u32(v.vps_id));
  bw.u1(1);
  bw.u1(1);
  bw.u(6, 0);
  bw.u(3, 0);      // one sub-layer
  bw.u1(1);        // temporal_id_nesting
  bw.u(16, 0xFFFF);
  write_ptl(bw, v.ptl);
  bw.u1(1);        // sub_layer_ordering_info_present
  bw.ue(1);        // max_dec_pic_buffering_minus1
  bw.ue(0);
  bw.ue(0);
  bw.u(6, 0);      // max_layer_id
  bw.ue(0);        // num_layer_sets_minus1
  bw.u1(v.timing_info);
  if (v.timing_info) {
    bw.u(32, v.num_units_in_tick);
    bw.u(32, v.time_scale);
    bw.u1(0);      // poc_proportional_to_timing
    bw.ue(0);      // num_hrd_parameters
  }
  bw.u1(0);        // vps_extension
  bw.trailing();
  return std::move(bw.buf());
}

std::vector<u8> write_sps(const Sps& s) {
  BitWriter bw;
  for (u8 b : nal_header(kSps)) bw.u(8, b);
  bw.u(4, u32(s.vps_id));
  bw.u(3, 0);
  bw.u1(1);
  write_ptl(bw, s.ptl);
  bw.ue(u32(s.sps_id));
  bw.ue(u32(s.chroma_format_idc));
  bw.ue(u32(s.width));
  bw.ue(u32(s.height));
  const bool conf = s.conf_left || s.conf_right || s.conf_top || s.conf_bottom;
  bw.u1(conf);
  if (conf) {
    bw.ue(u32(s.conf_left / 2));
    bw.ue(u32(s.conf_right / 2));
    bw.ue(u32(s.conf_top / 2));
    bw.ue(u32(s.conf_bottom / 2));
  }
  bw.ue(u32(s.bit_depth_luma - 8));
  bw.ue(u32(s.bit_depth_chroma - 8));
  bw.ue(u32(s.log2_max_poc_lsb - 4));
  bw.u1(1);
  bw.ue(u32(s.max_dec_pic_buffering - 1));
  bw.ue(u32(s.max_num_reorder));
  bw.ue(u32(s.max_latency_increase_plus1));
  bw.ue(u32(s.log2_min_cb - 3));
  bw.ue(u32(s.log2_ctb - s.log2_min_cb));
  bw.ue(u32(s.log2_min_tb - 2));
  bw.ue(u32(s.log2_max_tb - s.log2_min_tb));
  bw.ue(u32(s.max_th_depth_inter));
  bw.ue(u32(s.max_th_depth_intra));
  bw.u1(s.scaling_list);
  if (s.scaling_list) {
    bw.u1(s.scaling_list_data);
    if (s.scaling_list_data) write_scaling_list_data(bw, s.sl);
  }
  bw.u1(s.amp);
  bw.u1(s.sao);
  bw.u1(s.pcm);
  if (s.pcm) {
    bw.u(4, u32(s.pcm_bit_depth_luma - 1));
    bw.u(4, u32(s.pcm_bit_depth_chroma - 1));
    bw.ue(u32(s.log2_min_pcm - 3));
    bw.ue(u32(s.log2_max_pcm - s.log2_min_pcm));
    bw.u1(s.pcm_loop_filter_disabled);
  }
  bw.ue(u32(s.st_rps.size()));
  for (size_t i = 0; i < s.st_rps.size(); ++i) write_st_rps(bw, int(i), s.st_rps[i]);
  bw.u1(s.long_term_refs);
  if (s.long_term_refs) {
    bw.ue(u32(s.lt_poc_lsb_sps.size()));
    for (size_t i = 0; i < s.lt_poc_lsb_sps.size(); ++i) {
      bw.u(s.log2_max_poc_lsb, u32(s.lt_poc_lsb_sps[i]));
      bw.u1(s.lt_used_sps[i]);
    }
  }
  bw.u1(s.temporal_mvp);
  bw.u1(s.strong_intra_smoothing);
  bw.u1(s.vui);
  if (s.vui) {
    bw.u1(0);  // aspect_ratio_info
    bw.u1(0);  // overscan
    bw.u1(s.video_signal_type);
    if (s.video_signal_type) {
      bw.u(3, u32(s.video_format));
      bw.u1(s.full_range);
      bw.u1(1);  // colour_description_present
      bw.u(8, u32(s.matrix_coeffs));  // colour_primaries (6 = SMPTE 170M, matches BT.601)
      bw.u(8, u32(s.matrix_coeffs));  // transfer_characteristics
      bw.u(8, u32(s.matrix_coeffs));  // matrix_coeffs
    }
    bw.u1(0);  // chroma_loc_info
    bw.u(3, 0);
    bw.u1(0);  // default display window
    bw.u1(s.timing_info);
    if (s.timing_info) {
      bw.u(32, s.num_units_in_tick);
      bw.u(32, s.time_scale);
      bw.u1(0);  // poc_proportional_to_timing
      bw.u1(0);  // hrd_parameters_present
    }
    bw.u1(0);  // bitstream_restriction
  }
  bw.u1(0);  // sps_extension_present
  bw.trailing();
  return std::move(bw.buf());
}

std::vector<u8> write_pps(const Pps& p) {
  BitWriter bw;
  for (u8 b : nal_header(kPps)) bw.u(8, b);
  bw.ue(u32(p.pps_id));
  bw.ue(u32(p.sps_id));
  bw.u1(p.dependent_slice_segments);
  bw.u1(0);  // output_flag_present
  bw.u(3, 0);
  bw.u1(p.sign_data_hiding);
  bw.u1(p.cabac_init_present);
  bw.ue(u32(p.num_ref_idx_l0_default - 1));
  bw.ue(u32(p.num_ref_idx_l1_default - 1));
  bw.se(p.init_qp - 26);
  bw.u1(p.constrained_intra_pred);
  bw.u1(p.transform_skip);
  bw.u1(p.cu_qp_delta);
  if (p.cu_qp_delta) bw.ue(u32(p.diff_cu_qp_delta_depth));
  bw.se(p.cb_qp_offset);
  bw.se(p.cr_qp_offset);
  bw.u1(p.slice_chroma_qp_offsets_present);
  bw.u1(p.weighted_pred);
  bw.u1(p.weighted_bipred);
  bw.u1(p.transquant_bypass);
  bw.u1(p.tiles);
  bw.u1(p.entropy_coding_sync);
  if (p.tiles) {
    bw.ue(u32(p.tile_cols - 1));
    bw.ue(u32(p.tile_rows - 1));
    bw.u1(p.uniform_spacing);
    if (!p.uniform_spacing) {
      for (int i = 0; i < p.tile_cols - 1; ++i) bw.ue(u32(p.col_width[size_t(i)] - 1));
      for (int i = 0; i < p.tile_rows - 1; ++i) bw.ue(u32(p.row_height[size_t(i)] - 1));
    }
    bw.u1(p.loop_filter_across_tiles);
  }
  bw.u1(p.loop_filter_across_slices);
  bw.u1(1);  // deblocking_filter_control_present
  bw.u1(p.deblocking_override_enabled);
  bw.u1(p.deblocking_disabled);
  if (!p.deblocking_disabled) {
    bw.se(p.beta_offset / 2);
    bw.se(p.tc_offset / 2);
  }
  bw.u1(p.scaling_list);
  if (p.scaling_list) write_scaling_list_data(bw, p.sl);
  bw.u1(0);  // lists_modification_present
  bw.ue(u32(p.log2_parallel_merge_level - 2));
  bw.u1(0);  // slice_segment_header_extension_present
  bw.u1(0);  // pps_extension_present
  bw.trailing();
  return std::move(bw.buf());
}

void write_slice_header(BitWriter& bw, const SliceHeader& sh, const Sps& sps, const Pps& pps) {
  for (u8 b : nal_header(sh.nal_type)) bw.u(8, b);
  bw.u1(sh.first_slice_in_pic);
  if (is_irap(sh.nal_type)) bw.u1(0);
  bw.ue(u32(sh.pps_id));
  if (!sh.first_slice_in_pic)
    bw.u(ceil_log2(sps.width_ctbs() * sps.height_ctbs()), u32(sh.segment_address));
  bw.ue(u32(sh.slice_type));
  if (!is_idr(sh.nal_type)) {
    bw.u(sps.log2_max_poc_lsb, u32(sh.poc_lsb) & ((1u << sps.log2_max_poc_lsb) - 1));
    bw.u1(1);  // short_term_ref_pic_set_sps_flag (idx 0, not coded when there is one set)
    VEP_CHECK(sps.st_rps.size() == 1, "writer expects exactly one SPS RPS");
    if (sps.temporal_mvp) bw.u1(0);
  }
  if (sps.sao) {
    bw.u1(0);
    bw.u1(0);
  }
  if (sh.slice_type != kI) {
    bw.u1(0);  // num_ref_idx_active_override
    if (pps.cabac_init_present) bw.u1(sh.cabac_init);
    bw.ue(u32(5 - sh.max_num_merge_cand));
  }
  bw.se(sh.qp_delta);
  if (pps.loop_filter_across_slices && !pps.deblocking_disabled) bw.u1(0);
  bw.u1(1);  // byte_alignment()
  bw.align_zero();
}

void write_slice_header_full(BitWriter& bw, const SliceHeader& sh, const Sps& sps, const Pps& pps) {
  for (u8 b : nal_header(sh.nal_type)) bw.u(8, b);
  bw.u1(sh.first_slice_in_pic);
  if (is_irap(sh.nal_type)) bw.u1(sh.no_output_of_prior_pics);
  bw.ue(u32(sh.pps_id));
  if (!sh.first_slice_in_pic) {
    if (pps.dependent_slice_segments) bw.u1(sh.dependent);
    bw.u(ceil_log2(sps.width_ctbs() * sps.height_ctbs()), u32(sh.segment_address));
  }
  if (!sh.dependent) {
    bw.ue(u32(sh.slice_type));
    if (!is_idr(sh.nal_type)) {
      bw.u(sps.log2_max_poc_lsb, u32(sh.poc_lsb) & ((1u << sps.log2_max_poc_lsb) - 1));
      bw.u1(0);  // short_term_ref_pic_set_sps_flag: the RPS is coded in the header
      write_st_rps(bw, int(sps.st_rps.size()), sh.rps);
      if (sps.long_term_refs) {
        if (sps.num_long_term_ref_pics_sps > 0) bw.ue(u32(sh.num_long_term_sps));
        bw.ue(u32(sh.num_long_term - sh.num_long_term_sps));
        for (int i = 0; i < sh.num_long_term; ++i) {
          if (i < sh.num_long_term_sps) {
            if (sps.num_long_term_ref_pics_sps > 1)
              bw.u(ceil_log2(sps.num_long_term_ref_pics_sps), u32(sh.lt_idx_sps[i]));
          } else {
            bw.u(sps.log2_max_poc_lsb, u32(sh.lt_poc_lsb[i]));
            bw.u1(sh.lt_used[i]);
          }
          bw.u1(sh.lt_msb_present[i]);
          if (sh.lt_msb_present[i]) {
            const int prev = (i == 0 || i == sh.num_long_term_sps) ? 0 : sh.lt_msb_cycle[i - 1];
            VEP_CHECK(sh.lt_msb_cycle[i] >= prev, "DeltaPocMsbCycleLt must not decrease");
            bw.ue(u32(sh.lt_msb_cycle[i] - prev));
          }
        }
      }
      if (sps.temporal_mvp) bw.u1(sh.temporal_mvp);
    }
    if (sps.sao) {
      bw.u1(sh.sao_luma);
      bw.u1(sh.sao_chroma);
    }
    if (sh.slice_type != kI) {
      const bool override_refs = sh.num_ref_idx_l0 != pps.num_ref_idx_l0_default ||
                                 (sh.slice_type == kB && sh.num_ref_idx_l1 != pps.num_ref_idx_l1_default);
      bw.u1(override_refs);
      if (override_refs) {
        bw.ue(u32(sh.num_ref_idx_l0 - 1));
        if (sh.slice_type == kB) bw.ue(u32(sh.num_ref_idx_l1 - 1));
      }
      if (sh.slice_type == kB) bw.u1(sh.mvd_l1_zero);
      if (pps.cabac_init_present) bw.u1(sh.cabac_init);
      if (sh.temporal_mvp) {
        if (sh.slice_type == kB) bw.u1(sh.collocated_from_l0);
        const int n = sh.collocated_from_l0 ? sh.num_ref_idx_l0 : sh.num_ref_idx_l1;
        if (n > 1) bw.ue(u32(sh.collocated_ref_idx));
      }
      if ((pps.weighted_pred && sh.slice_type == kP) || (pps.weighted_bipred && sh.slice_type == kB))
        write_pred_weights(bw, sh);
      bw.ue(u32(5 - sh.max_num_merge_cand));
    }
    bw.se(sh.qp_delta);
    if (pps.slice_chroma_qp_offsets_present) {
      bw.se(sh.cb_qp_offset);
      bw.se(sh.cr_qp_offset);
    }
    bool override_flag = false;
    if (pps.deblocking_override_enabled) {
      override_flag = sh.deblocking_disabled != pps.deblocking_disabled || sh.beta_offset != pps.beta_offset ||
                      sh.tc_offset != pps.tc_offset;
      bw.u1(override_flag);
    }
    if (override_flag) {
      bw.u1(sh.deblocking_disabled);
      if (!sh.deblocking_disabled) {
        bw.se(sh.beta_offset / 2);
        bw.se(sh.tc_offset / 2);
      }
    }
    if (pps.loop_filter_across_slices && (sh.sao_luma || sh.sao_chroma || !sh.deblocking_disabled))
      bw.u1(sh.loop_filter_across_slices);
  }
  if (pps.tiles || pps.entropy_coding_sync) {
    bw.ue(u32(sh.entry_points.size()));
    if (!sh.entry_points.empty()) {
      u32 mx = 1;
      for (u32 e : sh.entry_points) mx = std::max(mx, e - 1);
      const int len = std::max(1, 32 - __builtin_clz(mx));
      bw.ue(u32(len - 1));
      for (u32 e : sh.entry_points) bw.u(len, e - 1);
    }
  }
  bw.u1(1);  // byte_alignment()
  bw.align_zero();
}

std::vector<u8> hvcc_record(const std::vector<u8>& vps, const std::vector<u8>& sps,
                            const std::vector<u8>& pps) {
  VEP_CHECK(!sps.empty(), "hvcC needs an SPS");
  std::vector<u8> r(sps.size());
  const size_t rn = ebsp_to_rbsp(sps.data(), sps.size(), r.data());
  const Sps s = parse_sps(r.data(), rn);
  std::vector<u8> o;
  o.push_back(1);  // configurationVersion
  o.push_back(u8((s.ptl.profile_space << 6) | (s.ptl.tier << 5) | s.ptl.profile_idc));
  for (int i = 3; i >= 0; --i) o.push_back(u8(s.ptl.compat_flags >> (8 * i)));
  for (int i = 5; i >= 0; --i) o.push_back(u8(s.ptl.constraint_flags >> (8 * i)));
  o.push_back(u8(s.ptl.level_idc));
  o.push_back(0xF0);  // min_spatial_segmentation_idc = 0
  o.push_back(0x00);
  o.push_back(0xFC);  // parallelismType = 0
  o.push_back(u8(0xFC | (s.chroma_format_idc & 3)));
  o.push_back(u8(0xF8 | ((s.bit_depth_luma - 8) & 7)));
  o.push_back(u8(0xF8 | ((s.bit_depth_chroma - 8) & 7)));
  const u32 fr = s.fps() > 0 ? u32(s.fps() * 256.0 + 0.5) : 0;  // avgFrameRate (frames/256 s)
  o.push_back(u8(fr >> 8));
  o.push_back(u8(fr));
  // constantFrameRate(2)=0 | numTemporalLayers(3)=1 | temporalIdNested(1)=1 | lengthSizeMinusOne(2)=3
  o.push_back(u8((0 << 6) | (1 << 3) | (1 << 2) | 3));
  const std::vector<u8>* arrays[3] = {&vps, &sps, &pps};
  const int types[3] = {kVps, kSps, kPps};
  int narr = 0;
  for (auto* a : arrays) narr += a->empty() ? 0 : 1;
  o.push_back(u8(narr));
  for (int i = 0; i < 3; ++i) {
    const std::vector<u8>& n = *arrays[i];
    if (n.empty()) continue;
    o.push_back(u8(0x80 | types[i]));  // array_completeness = 1
    o.push_back(0);
    o.push_back(1);
    o.push_back(u8(n.size() >> 8));
    o.push_back(u8(n.size()));
    o.insert(o.end(), n.begin(), n.end());
  }
  return o;
}

}  // namespace vep::hevc
