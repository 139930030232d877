// General H.265 Main decoder: parameter sets, picture order count (§8.3.1), reference picture
// set marking (§8.3.2), reference list construction (§8.3.4), slice decoding through the CTU
// layer (hevc_ctu.cpp), the in-loop filters and output in POC order with the bumping process of
// C.5.2. See hevc_dec.h for the supported feature set.
#include <algorithm>
#include <cstdio>
#include <cstring>

#include "bits.h"
#include "fanout.h"
#include "hevc_ctu.h"
#include "hevc_recon.h"

namespace vep::hevc {

namespace {
bool is_rasl(int t) { return t == 8 || t == 9; }
bool is_radl(int t) { return t == 6 || t == 7; }
bool is_sub_layer_non_ref(int t) { return t <= 14 && (t % 2) == 0; }
bool is_bla(int t) { return t >= 16 && t <= 18; }

void check_supported(const Sps& sps, const Pps& pps) {
  if (sps.chroma_format_idc != 1 || sps.separate_colour_plane) throw UnsupportedStream("HEVC: only 4:2:0 is supported");
  if (sps.bit_depth_luma < 8 || sps.bit_depth_luma > 10 || sps.bit_depth_chroma < 8 || sps.bit_depth_chroma > 10)
    throw UnsupportedStream("HEVC: bit depth above 10 (only Main / Main10) is not supported");
  if (sps.bit_depth_luma != sps.bit_depth_chroma)
    throw UnsupportedStream("HEVC: different luma and chroma bit depths are not supported");
  if (sps.pcm && (sps.pcm_bit_depth_luma > sps.bit_depth_luma || sps.pcm_bit_depth_chroma > sps.bit_depth_chroma))
    throw Error("HEVC: PCM bit depth above the sample bit depth");
  VEP_CHECK(sps.width > 0 && sps.height > 0 && sps.width % (1 << sps.log2_min_cb) == 0 &&
                sps.height % (1 << sps.log2_min_cb) == 0,
            "HEVC: picture size must be a multiple of the minimum CU");
  VEP_CHECK(sps.log2_ctb >= 4 && sps.log2_ctb <= 6 && sps.log2_min_cb >= 3 && sps.log2_min_cb <= sps.log2_ctb,
            "HEVC: CTB / CU sizes out of range");
  VEP_CHECK(sps.log2_min_tb >= 2 && sps.log2_max_tb <= 5 && sps.log2_min_tb < sps.log2_min_cb &&
                sps.log2_max_tb <= sps.log2_ctb,
            "HEVC: transform sizes out of range");
}
}  // namespace

Decoder::Decoder() : pc_(std::make_unique<PicCtx>()), gpu_pool_(Recycler<GpuPicture>::make(12)) {
  if (const char* e = std::getenv("VEP_HEVC_SLICE_THREADS")) parallel_slices_ = e[0] != '0';
}
Decoder::~Decoder() = default;

void Decoder::bump(std::vector<FramePtr>& out) {
  FramePtr best;
  for (const FramePtr& f : dpb_)
    if (f->needed_for_output && (!best || f->poc < best->poc)) best = f;
  if (!best) return;
  best->needed_for_output = false;
  last_out_slot_ = best->slot;  // (its surface is converted after the job: not reused before)
  out.push_back(best);
  dpb_.erase(std::remove_if(dpb_.begin(), dpb_.end(), [](const FramePtr& f) { return !f->is_ref && !f->needed_for_output; }),
             dpb_.end());
}

void Decoder::start_picture(const SliceHeader& sh, int tid, const Sps& sps, const Pps& pps, const AccessUnit& au,
                            i64 tag, std::vector<FramePtr>& out) {
  check_supported(sps, pps);
  const int t = sh.nal_type;
  const bool irap = is_irap(t);
  if (irap) {
    no_rasl_output_ = is_idr(t) || is_bla(t) || first_;
    irap_tag_ = tag;
  }
  skip_pic_ = false;
  if (is_rasl(t) && no_rasl_output_) {  // leading pictures of a CRA we started at: not decodable
    skip_pic_ = true;
    return;
  }
  // only a picture that starts a new coded video sequence may change the picture size (a mid-GOP
  // SPS with another size would have the picture predict from surfaces of the old size)
  if (!(irap && no_rasl_output_) && act_w_ && (sps.width != act_w_ || sps.height != act_h_ || sps.bit_depth_luma != act_bd_))
    throw Error("HEVC: picture size or bit depth changed outside an IRAP picture");
  act_w_ = sps.width;  // (by value: a repeated SPS NAL replaces the map entry sps_act_ points at)
  act_h_ = sps.height;
  act_bd_ = sps.bit_depth_luma;
  // picture order count (§8.3.1)
  const int max_lsb = 1 << sps.log2_max_poc_lsb;
  int msb = 0;
  if (!(irap && no_rasl_output_)) {
    const int prev_lsb = prev_tid0_poc_ & (max_lsb - 1);
    const int prev_msb = prev_tid0_poc_ - prev_lsb;
    if (sh.poc_lsb < prev_lsb && prev_lsb - sh.poc_lsb >= max_lsb / 2) msb = prev_msb + max_lsb;
    else if (sh.poc_lsb > prev_lsb && sh.poc_lsb - prev_lsb > max_lsb / 2) msb = prev_msb - max_lsb;
    else msb = prev_msb;
  }
  const int poc = msb + (is_idr(t) ? 0 : sh.poc_lsb);
  if (tid == 0 && !is_rasl(t) && !is_radl(t) && !is_sub_layer_non_ref(t)) prev_tid0_poc_ = poc;
  // reference picture set (§8.3.2): long-term entries first (any reference picture, by POC LSBs
  // or full POC), then the short-term ones (short-term reference pictures only)
  st_before_.clear();
  st_after_.clear();
  lt_curr_.clear();
  if (is_idr(t)) {
    for (FramePtr& f : dpb_) f->is_ref = f->long_term = false;
  } else {
    std::vector<FramePtr> keep;
    const bool tolerate = irap && no_rasl_output_;  // (CRA / BLA start: references are not needed)
    for (int i = 0; i < sh.num_long_term; ++i) {
      int plt = sh.lt_poc_lsb[i];
      if (sh.lt_msb_present[i]) plt += poc - sh.lt_msb_cycle[i] * max_lsb - (poc & (max_lsb - 1));
      FramePtr hit;
      for (const FramePtr& f : dpb_)
        if (f->is_ref && (sh.lt_msb_present[i] ? f->poc == plt : (f->poc & (max_lsb - 1)) == plt)) hit = f;
      if (hit) {
        keep.push_back(hit);
        if (sh.lt_used[i]) lt_curr_.push_back(hit);
      } else if (sh.lt_used[i] && !tolerate) {
        throw Error("HEVC: missing long-term reference picture (poc " + std::to_string(plt) + ")");
      }
    }
    for (const FramePtr& f : keep) f->long_term = true;
    const ShortTermRps& r = sh.rps;
    for (int i = 0; i < r.num_delta(); ++i) {
      FramePtr hit;
      for (const FramePtr& f : dpb_)
        if (f->is_ref && !f->long_term && f->poc == poc + r.delta_poc[i]) hit = f;
      if (hit) keep.push_back(hit);
      if (!r.used[i]) continue;
      if (!hit) {
        if (tolerate) continue;
        throw Error("HEVC: missing reference picture (poc " + std::to_string(poc + r.delta_poc[i]) + ")");
      }
      (i < r.num_negative ? st_before_ : st_after_).push_back(hit);
    }
    for (FramePtr& f : dpb_)
      if (std::find(keep.begin(), keep.end(), f) == keep.end()) f->is_ref = f->long_term = false;
  }
  // output and removal of pictures from the DPB (C.5.2.2)
  if (irap && no_rasl_output_ && !first_) {
    if (!sh.no_output_of_prior_pics) {
      while (true) {
        const size_t before = out.size();
        bump(out);
        if (out.size() == before) break;
      }
    }
    dpb_.clear();
  } else {
    dpb_.erase(std::remove_if(dpb_.begin(), dpb_.end(), [](const FramePtr& f) { return !f->is_ref && !f->needed_for_output; }),
               dpb_.end());
    while (true) {
      int waiting = 0;
      bool late = false;
      const int max_latency = sps.max_latency_increase_plus1 ? sps.max_num_reorder + sps.max_latency_increase_plus1 - 1 : 0;
      for (const FramePtr& f : dpb_)
        if (f->needed_for_output) {
          ++waiting;
          if (sps.max_latency_increase_plus1 && f->latency >= max_latency) late = true;
        }
      if (!(waiting > sps.max_num_reorder || late || int(dpb_.size()) >= sps.max_dec_pic_buffering) || !waiting) break;
      bump(out);
    }
  }
  first_ = false;
  // the new picture
  cur_ = std::make_shared<HevcFrame>();
  if (gpu_mode_) {  // a DPB surface slot no kept or just-output picture uses
    gpu_slots_ = std::max(gpu_slots_, sps.max_dec_pic_buffering + 2);
    std::vector<bool> used(size_t(gpu_slots_), false);
    for (const FramePtr& f : dpb_) used[size_t(f->slot)] = true;
    if (last_out_slot_ >= 0 && last_out_slot_ < gpu_slots_) used[size_t(last_out_slot_)] = true;
    int slot = 0;
    while (slot < gpu_slots_ && used[size_t(slot)]) ++slot;
    VEP_CHECK(slot < gpu_slots_, "HEVC: no free DPB surface");
    cur_->slot = slot;
  } else {
    cur_->s.alloc(sps.width, sps.height, sps.bit_depth_luma);
  }
  cur_->poc = poc;
  cur_->uid = next_uid_++;
  cur_->pts = au.pts;
  cur_->dts = au.dts;
  cur_->tag = tag;
  cur_->keyframe = irap;
  cur_->rasl_of = is_rasl(t) ? irap_tag_ : -1;
  cur_->type = sh.pict_char();
  cur_->width = sps.out_width();
  cur_->height = sps.out_height();
  cur_->crop_left = sps.conf_left;
  cur_->crop_top = sps.conf_top;
  sps_act_ = &sps;
  pps_act_ = &pps;
  pc_->init(sps, pps, &cur_->s);
  pc_->poc = poc;
  pc_->prefilled = false;
  deferred_.clear();
  // independent slices in parallel: no WPP (rows share contexts) and no dependent segments
  // (decode_slice switches deferral off when one arrives)
  // (tiles and wavefront rows together: parsed slice by slice)
  defer_ = parallel_slices_ && !(pps.entropy_coding_sync && pps.tiles) && FanOut::shared().size() > 0;
  if (gpu_mode_) {
    cur_gpu_ = gpu_pool_->acquire([](GpuPicture& g) {  // default state, capacities kept
      GpuPicture fresh;
      auto keep = [](auto& from, auto& to) {
        from.clear();
        to.swap(from);
      };
      keep(g.pus, fresh.pus);
      keep(g.tus, fresh.tus);
      keep(g.level_begin, fresh.level_begin);
      keep(g.coefs, fresh.coefs);
      keep(g.pcm, fresh.pcm);
      keep(g.bs_v, fresh.bs_v);
      keep(g.bs_h, fresh.bs_h);
      keep(g.qp, fresh.qp);
      keep(g.pcm_map, fresh.pcm_map);
      keep(g.intra_map, fresh.intra_map);
      keep(g.avail, fresh.avail);
      keep(g.ctb_slice, fresh.ctb_slice);
      keep(g.ctb_tile, fresh.ctb_tile);
      keep(g.wp, fresh.wp);
      keep(g.slices, fresh.slices);
      keep(g.sao_params, fresh.sao_params);
      g = std::move(fresh);
    });
    cur_gpu_->target = cur_->slot;
    cur_gpu_->pts = au.pts;
    cur_gpu_->tag = tag;
    cur_gpu_->cra = irap && !no_rasl_output_;
    cur_gpu_->bd_y = sps.bit_depth_luma;
    cur_gpu_->bd_c = sps.bit_depth_chroma;
    pc_->init_gpu(cur_gpu_.get());
  }
}

std::vector<std::shared_ptr<GpuPicture>> Decoder::take_gpu_pictures() {
  std::vector<std::shared_ptr<GpuPicture>> v;
  v.swap(gpu_out_);
  return v;
}

namespace {
// RBSP offsets of the 2nd.. substreams of a slice segment: the entry point offsets count bytes of
// the NAL as sent (emulation prevention bytes included, §7.4.7.1) from the first slice data byte.
std::vector<size_t> substream_starts(const SliceHeader& sh, const u8* ebsp, size_t en) {
  std::vector<size_t> ep;  // EBSP positions of the removed emulation prevention bytes
  int zeros = 0;
  for (size_t i = 0; i < en; ++i) {
    if (zeros >= 2 && ebsp[i] == 3) {
      ep.push_back(i);
      zeros = 0;
      continue;
    }
    zeros = ebsp[i] == 0 ? zeros + 1 : 0;
  }
  // EBSP position of the first slice data byte (RBSP data_bytepos)
  size_t e0 = sh.data_bytepos, k = 0;
  for (; k < ep.size() && ep[k] <= e0; ++k) ++e0;
  std::vector<size_t> out;
  size_t e = e0;
  for (u32 off : sh.entry_points) {
    e += off;
    if (e >= en) return {};
    const size_t removed = size_t(std::lower_bound(ep.begin(), ep.end(), e) - ep.begin());
    out.push_back(e - removed);
  }
  return out;
}
}  // namespace

void Decoder::decode_slice(const SliceHeader& sh, const u8* rbsp, size_t n, const u8* ebsp, size_t en) {
  SliceInfo si;
  si.sh = sh;
  if (!sh.first_slice_in_pic) {
    VEP_CHECK(!pc_->slices.empty(), "HEVC: slice segment before the first slice of the picture");
    VEP_CHECK(pc_->slice[size_t(sh.segment_address)] == 0xFFFF, "HEVC: slice segment overlaps decoded CTUs");
  }
  if (sh.dependent) {  // a further segment of the previous slice: its lists, QP and identity
    const SliceInfo& p = pc_->slices.back();
    si.qp = p.qp;
    si.ord = p.ord;
    si.addr_rs = p.addr_rs;
    for (int l = 0; l < 2; ++l) {
      si.list[l] = p.list[l];
      si.list_poc[l] = p.list_poc[l];
      si.list_lt[l] = p.list_lt[l];
    }
    pc_->slices.push_back(std::move(si));
    run_deferred(false);  // (a dependent segment continues the previous one's contexts: sequential)
    defer_ = false;
    decode_slice_data(*pc_, int(pc_->slices.size()) - 1, rbsp, n, sh.data_bytepos);
    return;
  }
  si.qp = pps_act_->init_qp + sh.qp_delta;  // SliceQpY, -QpBdOffsetY .. 51
  VEP_CHECK(si.qp >= -pc_->qp_off_y && si.qp <= 51, "HEVC: slice QP out of range");
  si.ord = pc_->slices.empty() ? 0 : pc_->slices.back().ord + 1;
  si.addr_rs = sh.segment_address;
  if (si.ord > 0) pc_->multi = true;
  if (sh.slice_type != kI) {  // reference picture lists (§8.3.4)
    const int total = int(st_before_.size() + st_after_.size() + lt_curr_.size());
    VEP_CHECK(total > 0, "HEVC: inter slice without reference pictures");
    for (int l = 0; l < (sh.slice_type == kB ? 2 : 1); ++l) {
      std::vector<std::pair<FramePtr, bool>> temp;  // (picture, long-term)
      const int nref = l == 0 ? sh.num_ref_idx_l0 : sh.num_ref_idx_l1;
      const std::vector<FramePtr>& a = l == 0 ? st_before_ : st_after_;
      const std::vector<FramePtr>& b = l == 0 ? st_after_ : st_before_;
      while (int(temp.size()) < std::max(nref, total)) {
        for (const FramePtr& f : a) temp.push_back({f, false});
        for (const FramePtr& f : b) temp.push_back({f, false});
        for (const FramePtr& f : lt_curr_) temp.push_back({f, true});
      }
      for (int i = 0; i < nref; ++i) {
        const int e = sh.list_mod[l] ? sh.list_entry[l][i] : i;
        VEP_CHECK(e < int(temp.size()), "HEVC: list_entry out of range");
        si.list[l].push_back(temp[size_t(e)].first);
        si.list_poc[l].push_back(temp[size_t(e)].first->poc);
        si.list_lt[l].push_back(u8(temp[size_t(e)].second));
      }
    }
  }
  pc_->slices.push_back(std::move(si));
  if (defer_) {  // kept until the picture's last slice: then every slice runs in parallel
    const size_t k = deferred_.size();
    if (slice_rbsp_.size() <= k) slice_rbsp_.resize(k + 1);
    slice_rbsp_[k].assign(rbsp, rbsp + n);
    deferred_.push_back({pc_->slices.size() - 1, n, sh.data_bytepos});
    if (slice_subs_.size() <= k) slice_subs_.resize(k + 1);
    slice_subs_[k].clear();
    if ((pps_act_->tiles || pps_act_->entropy_coding_sync) && !sh.entry_points.empty())
      slice_subs_[k] = substream_starts(sh, ebsp, en);
    return;
  }
  decode_slice_data(*pc_, int(pc_->slices.size()) - 1, rbsp, n, sh.data_bytepos);
}

void Decoder::run_deferred(bool parallel) {
  if (deferred_.empty()) return;
  std::vector<std::array<size_t, 3>> work;
  work.swap(deferred_);
  PicCtx& pc = *pc_;
  size_t subs = 0;
  for (size_t k = 0; k < work.size(); ++k) subs += k < slice_subs_.size() ? slice_subs_[k].size() : 0;
  if ((work.size() == 1 && subs == 0) || !parallel) {  // the sequential path, nothing to merge
    for (size_t k = 0; k < work.size(); ++k)
      decode_slice_data(pc, int(work[k][0]), slice_rbsp_[k].data(), work[k][1], work[k][2]);
    return;
  }
  // The CTB -> slice maps for the whole picture first: slice k covers tile-scan addresses from its
  // segment address up to the next slice's.
  const int total = pc.wctb * pc.hctb;
  for (size_t k = 0; k < work.size(); ++k) {
    const SliceInfo& sl = pc.slices[work[k][0]];
    const int b = pc.rs2ts[size_t(sl.sh.segment_address)];
    const int e = k + 1 < work.size() ? pc.rs2ts[size_t(pc.slices[work[k + 1][0]].sh.segment_address)] : total;
    VEP_CHECK(b < e, "HEVC: slice segment addresses out of order");
    for (int ts = b; ts < e; ++ts) {
      const int rs = pc.ts2rs[size_t(ts)];
      pc.slice[size_t(rs)] = u16(work[k][0]);
      pc.sord[size_t(rs)] = u16(sl.ord);
    }
  }
  pc.prefilled = true;
  pc.multi = true;
  // units: whole slices, or (tiles with entry points) each substream of a slice: slice k,
  // substream start (RBSP), tile-scan range, last substream of the slice
  struct Unit {
    size_t k, pos;
    int first_ts, end_ts;
    bool last;
  };
  std::vector<Unit> units;
  for (size_t k = 0; k < work.size(); ++k) {
    const int b = pc.rs2ts[size_t(pc.slices[work[k][0]].sh.segment_address)];
    const int e = k + 1 < work.size() ? pc.rs2ts[size_t(pc.slices[work[k + 1][0]].sh.segment_address)] : total;
    std::vector<int> cuts;  // substream starts inside the slice: tiles, or CTB rows (WPP)
    const bool wpp = pc.pps->entropy_coding_sync;
    for (int ts = b + 1; ts < e; ++ts) {
      const int rs = pc.ts2rs[size_t(ts)];
      if (wpp ? pc.ctb_row_start(rs) : pc.tile[size_t(rs)] != pc.tile[size_t(pc.ts2rs[size_t(ts - 1)])]) cuts.push_back(ts);
    }
    const std::vector<size_t>* sub = k < slice_subs_.size() ? &slice_subs_[k] : nullptr;
    if (!sub || sub->empty() || sub->size() != cuts.size()) {
      units.push_back({k, work[k][2], -1, -1, true});  // the whole slice (decode_slice_data)
      continue;
    }
    int from = b;
    size_t pos = work[k][2];
    for (size_t j = 0; j <= cuts.size(); ++j) {
      const int to = j < cuts.size() ? cuts[j] : e;
      units.push_back({k, pos, from, to, j == cuts.size()});
      if (j < cuts.size()) pos = (*sub)[j], from = to;
    }
  }
  while (shards_.size() < units.size()) shards_.push_back(std::make_unique<SliceShard>());
  for (size_t k = 0; k < units.size(); ++k) {  // (records buffers keep their capacity)
    SliceShard& sh = *shards_[k];
    sh.g.tus.clear();
    sh.g.pus.clear();
    sh.g.coefs.clear();
    sh.g.pcm.clear();
    sh.g.wp.clear();
    sh.g.bd_y = pc.bd_y;
    sh.g.bd_c = pc.bd_c;
    sh.stats = {};
    sh.any_bypass = false;
    sh.ctus = 0;
  }
  parallel_units_ += units.size();

  // wavefront rows: each waits for the CTBs above it (units are taken in order, so a waited-on
  // row was claimed by a running thread: FanOut hands out indices in increasing order)
  bool rows = false;
  for (const Unit& x : units) rows |= x.first_ts >= 0 && pc.pps->entropy_coding_sync;
  if (rows) {
    if (!wpp_sync_) wpp_sync_ = std::make_unique<WppSync>();
    wpp_sync_->reset(pc.wctb, pc.hctb);
    pc.wpp_sync = wpp_sync_.get();
  }
  struct Clear {
    PicCtx& pc;
    ~Clear() { pc.wpp_sync = nullptr; }
  } clear{pc};
  FanOut::shared().run(int(units.size()), [&](int u) {
    const Unit& x = units[size_t(u)];
    const auto& w = work[x.k];
    try {
      if (x.first_ts < 0)
        decode_slice_data(pc, int(w[0]), slice_rbsp_[x.k].data(), w[1], w[2], shards_[size_t(u)].get());
      else
        decode_substream(pc, int(w[0]), slice_rbsp_[x.k].data(), w[1], x.pos, x.first_ts, x.end_ts, x.last,
                         shards_[size_t(u)].get());
    } catch (...) {
      if (pc.wpp_sync) pc.wpp_sync->abort.store(true);
      throw;
    }
  });
  // merge in decoding order (slices, then their tiles): the records equal a sequential parse's
  int ctus = 0;
  for (size_t k = 0; k < units.size(); ++k) {
    SliceShard& sh = *shards_[k];
    ctus += sh.ctus;
    pc.any_bypass |= sh.any_bypass;
    Stats& st = pc.stats;
    st.intra += sh.stats.intra, st.inter += sh.stats.inter, st.skip += sh.stats.skip, st.pcm += sh.stats.pcm;
    st.merge += sh.stats.merge, st.bi += sh.stats.bi, st.tskip += sh.stats.tskip, st.amp += sh.stats.amp;
    GpuPicture* g = pc.gpu;
    if (!g) continue;
    const u32 coef0 = u32(g->coefs.size()), pcm0 = u32(g->pcm.size());
    g->coefs.insert(g->coefs.end(), sh.g.coefs.begin(), sh.g.coefs.end());
    g->pcm.insert(g->pcm.end(), sh.g.pcm.begin(), sh.g.pcm.end());
    for (GpuTu t : sh.g.tus) {
      if (t.flags & kTuPcm) t.data += pcm0;
      else if (t.flags & kTuCoef) t.data += coef0;
      g->tus.push_back(t);
    }
    std::vector<u8> wmap(sh.g.wp.size() + 1, 0);  // shard weight index -> picture weight index
    for (size_t i = 0; i < sh.g.wp.size(); ++i) {
      size_t j = 0;
      while (j < g->wp.size() && std::memcmp(&g->wp[j], &sh.g.wp[i], sizeof(GpuWp)) != 0) ++j;
      if (j == g->wp.size()) {
        VEP_CHECK(g->wp.size() < 255, "HEVC: more than 255 distinct prediction weights in one picture");
        g->wp.push_back(sh.g.wp[i]);
      }
      wmap[i + 1] = u8(j + 1);
    }
    for (GpuPu u : sh.g.pus) {
      u.wp = wmap[u.wp];
      g->pus.push_back(u);
    }
  }
  VEP_CHECK(ctus == total, "HEVC: picture has undecoded CTUs");
}

void Decoder::finish_picture(std::vector<FramePtr>& out) {
  try {
    run_deferred(true);
  } catch (...) {  // the damaged picture is dropped
    deferred_.clear();
    cur_ = nullptr;
    cur_gpu_ = nullptr;
    throw;
  }
  FramePtr f = cur_;
  cur_ = nullptr;
  for (int k = 0; k < pc_->wctb * pc_->hctb; ++k)
    VEP_CHECK(pc_->slice[size_t(k)] != 0xFFFF, "HEVC: picture has undecoded CTUs");
  bool deblock = false, sao = false;
  for (const SliceInfo& s : pc_->slices) {
    deblock |= !s.sh.deblocking_disabled;
    sao |= s.sh.sao_luma || s.sh.sao_chroma;
  }
  if (gpu_mode_) {
    finish_gpu_picture(*pc_);
    gpu_out_.push_back(std::move(cur_gpu_));
  } else {
    if (deblock) deblock_picture(*pc_);
    if (sao) sao_picture(*pc_);
  }
  if (sps_act_->temporal_mvp) f->col = build_col(*pc_, f->col_w);
  stats = pc_->stats;
  // C.5.2.3: the current picture is a short-term reference and waits for output
  for (FramePtr& d : dpb_)
    if (d->needed_for_output) ++d->latency;
  f->is_ref = true;
  f->needed_for_output = true;
  f->latency = 0;
  dpb_.push_back(f);
  last_ = f;
  const Sps& sps = *sps_act_;
  const int max_latency = sps.max_latency_increase_plus1 ? sps.max_num_reorder + sps.max_latency_increase_plus1 - 1 : 0;
  while (true) {
    int waiting = 0;
    bool late = false;
    for (const FramePtr& d : dpb_)
      if (d->needed_for_output) {
        ++waiting;
        if (sps.max_latency_increase_plus1 && d->latency >= max_latency) late = true;
      }
    if (!waiting || !(waiting > sps.max_num_reorder || late)) break;
    bump(out);
  }
}

std::vector<FramePtr> Decoder::decode(const AccessUnit& au, i64 tag) {
  std::vector<FramePtr> out;
  for (size_t i = 0; i < au.nals.size(); ++i) {
    const u8* p = au.nal(i);
    const size_t n = au.nal_size(i);
    if (n < 2) continue;
    const int t = nal_type(p);
    const int tid = (p[1] & 7) - 1;
    if (t == 36 || t == 37) {  // end of sequence / bitstream: the next IRAP starts afresh
      if (cur_) finish_picture(out);
      first_ = true;
      continue;
    }
    if (!(t < 22 || (t >= kVps && t <= kPps))) continue;  // AUD, SEI, reserved
    if (t < 22 && t > 9 && t < 16) continue;              // reserved VCL types
    rbsp_.resize(n);
    const size_t rn = ebsp_to_rbsp(p, n, rbsp_.data());
    if (t == kVps) {
      Vps v = parse_vps(rbsp_.data(), rn);
      vps_[v.vps_id] = v;
      continue;
    }
    if (t == kSps) {
      Sps s = parse_sps(rbsp_.data(), rn);
      sps_[s.sps_id] = std::move(s);
      continue;
    }
    if (t == kPps) {
      Pps q = parse_pps(rbsp_.data(), rn);
      pps_[q.pps_id] = q;
      continue;
    }
    const int pps_id = peek_slice_pps_id(rbsp_.data(), rn);
    auto pit = pps_.find(pps_id);
    if (pit == pps_.end()) throw Error("HEVC: slice refers to a missing PPS");
    auto sit = sps_.find(pit->second.sps_id);
    if (sit == sps_.end()) throw Error("HEVC: PPS refers to a missing SPS");
    const SliceHeader sh = parse_slice_header(rbsp_.data(), rn, sit->second, pit->second, have_prev_sh_ ? &prev_sh_ : nullptr);
    prev_sh_ = sh;  // (a dependent segment of the next NAL takes its slice fields from here)
    have_prev_sh_ = true;
    try {
      if (sh.first_slice_in_pic) {
        if (cur_) finish_picture(out);
        start_picture(sh, tid, sit->second, pit->second, au, tag, out);
      } else if (!cur_ && !skip_pic_) {
        throw Error("HEVC: slice segment without the start of its picture");
      }
      if (skip_pic_) continue;
      decode_slice(sh, rbsp_.data(), rn, p, n);
    } catch (...) {
      cur_ = nullptr;  // the damaged picture is dropped
      cur_gpu_ = nullptr;
      throw;
    }
  }
  if (cur_) finish_picture(out);
  return out;
}

std::vector<FramePtr> Decoder::flush() {
  std::vector<FramePtr> out;
  if (cur_) finish_picture(out);
  while (true) {
    const size_t before = out.size();
    bump(out);
    if (out.size() == before) break;
  }
  dpb_.clear();
  first_ = true;
  return out;
}

}  // namespace vep::hevc
