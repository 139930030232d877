// ISO-BMFF (MP4) per-GOP segment writer and the background archiver thread.
//
// Reference parity: python/archive.py:21-100 (StoreMP4VideoChunks): one file per GOP named
// <start_timestamp_ms>_<segment_length_ms>.mp4 under <disk_path>/<device_id>/. Timestamps are
// rebased to the GOP's first DTS (the reference's "minimum_dts" rebase, without its -1 quirk,
// SURVEY.md Appendix A.7).
#include <sys/stat.h>

#include <algorithm>
#include <cstdio>

#include "h264.h"
#include "hevc.h"
#include "mux.h"

namespace vep::mux {

namespace {

struct Box {
  std::vector<u8> b;
  size_t start;
  explicit Box(const char* type) {
    b.resize(8);
    std::memcpy(&b[4], type, 4);
    start = 0;
  }
  void u8_(u8 v) { b.push_back(v); }
  void u16_(u32 v) { b.push_back(u8(v >> 8)); b.push_back(u8(v)); }
  void u32_(u32 v) { for (int i = 3; i >= 0; --i) b.push_back(u8(v >> (8 * i))); }
  void full(u8 ver, u32 flags) { u8_(ver); b.push_back(u8(flags >> 16)); b.push_back(u8(flags >> 8)); b.push_back(u8(flags)); }
  void bytes(const void* p, size_t n) { const u8* q = static_cast<const u8*>(p); b.insert(b.end(), q, q + n); }
  void zeros(size_t n) { b.insert(b.end(), n, 0); }
  void add(const Box& c) { b.insert(b.end(), c.b.begin(), c.b.end()); }
  const std::vector<u8>& done() {
    u32 n = u32(b.size());
    b[0] = u8(n >> 24); b[1] = u8(n >> 16); b[2] = u8(n >> 8); b[3] = u8(n);
    return b;
  }
};

void matrix(Box& x) {
  const u32 m[9] = {0x00010000, 0, 0, 0, 0x00010000, 0, 0, 0, 0x40000000};
  for (u32 v : m) x.u32_(v);
}

}  // namespace

i64 segment_duration_ms(const std::vector<AuPtr>& aus) {
  i64 sum = 0;
  bool has = false;
  i64 mn = INT64_MAX, mx = INT64_MIN;
  for (auto& a : aus) {
    if (a->duration > 0) {
      has = true;
      sum += a->duration;
    }
    mn = std::min(mn, a->dts);
    mx = std::max(mx, a->dts);
  }
  i64 ticks = has ? sum : (aus.empty() ? 0 : mx - mn);
  return ticks * 1000 / 90000;
}

std::vector<u8> build_mp4(const std::vector<AuPtr>& aus, const Mp4Info& info) {
  VEP_CHECK(!aus.empty(), "empty GOP");
  VEP_CHECK(info.ps.complete(), "MP4 needs the stream's parameter sets");
  const bool hevc = info.ps.codec == Codec::kH265;
  const u32 ts = 90000;
  const i64 base = aus.front()->dts;
  std::vector<std::vector<u8>> samples;
  std::vector<u32> durs;
  std::vector<u32> sync;
  for (size_t i = 0; i < aus.size(); ++i) {
    samples.push_back(au_to_avcc(*aus[i]));
    i64 d = aus[i]->duration;
    if (d <= 0) d = (i + 1 < aus.size()) ? aus[i + 1]->dts - aus[i]->dts : (i ? i64(durs.back()) : 3000);
    durs.push_back(u32(std::max<i64>(d, 1)));
    if (aus[i]->keyframe) sync.push_back(u32(i + 1));
  }
  u64 total90 = 0;
  for (u32 d : durs) total90 += d;
  (void)base;

  Box ftyp("ftyp");
  ftyp.bytes("isom", 4);
  ftyp.u32_(0x200);
  ftyp.bytes(hevc ? "isomiso2hvc1mp41" : "isomiso2avc1mp41", 16);

  auto build_moov = [&](u32 chunk_offset) {
    Box mvhd("mvhd");
    mvhd.full(0, 0);
    mvhd.u32_(0);
    mvhd.u32_(0);
    mvhd.u32_(1000);
    mvhd.u32_(u32(total90 * 1000 / ts));
    mvhd.u32_(0x00010000);
    mvhd.u16_(0x0100);
    mvhd.zeros(10);
    matrix(mvhd);
    mvhd.zeros(24);
    mvhd.u32_(2);

    Box tkhd("tkhd");
    tkhd.full(0, 3);
    tkhd.u32_(0);
    tkhd.u32_(0);
    tkhd.u32_(1);
    tkhd.u32_(0);
    tkhd.u32_(u32(total90 * 1000 / ts));
    tkhd.zeros(8);
    tkhd.u16_(0);
    tkhd.u16_(0);
    tkhd.u16_(0);
    tkhd.u16_(0);
    matrix(tkhd);
    tkhd.u32_(u32(info.width) << 16);
    tkhd.u32_(u32(info.height) << 16);

    Box mdhd("mdhd");
    mdhd.full(0, 0);
    mdhd.u32_(0);
    mdhd.u32_(0);
    mdhd.u32_(ts);
    mdhd.u32_(u32(total90));
    mdhd.u16_(0x55C4);  // 'und'
    mdhd.u16_(0);

    Box hdlr("hdlr");
    hdlr.full(0, 0);
    hdlr.u32_(0);
    hdlr.bytes("vide", 4);
    hdlr.zeros(12);
    hdlr.bytes("VideoHandler", 13);

    Box vmhd("vmhd");
    vmhd.full(0, 1);
    vmhd.zeros(8);
    Box url("url ");
    url.full(0, 1);
    url.done();
    Box dref("dref");
    dref.full(0, 0);
    dref.u32_(1);
    dref.add(url);
    dref.done();
    Box dinf("dinf");
    dinf.add(dref);

    Box avcc(hevc ? "hvcC" : "avcC");
    std::vector<u8> rec = hevc ? hevc::hvcc_record(info.ps.vps, info.ps.sps, info.ps.pps)
                               : h264::avcc_record(info.ps.sps, info.ps.pps);
    avcc.bytes(rec.data(), rec.size());
    Box avc1(hevc ? "hvc1" : "avc1");
    avc1.zeros(6);
    avc1.u16_(1);
    avc1.zeros(16);
    avc1.u16_(u32(info.width));
    avc1.u16_(u32(info.height));
    avc1.u32_(0x00480000);
    avc1.u32_(0x00480000);
    avc1.u32_(0);
    avc1.u16_(1);
    avc1.zeros(32);
    avc1.u16_(0x18);
    avc1.u16_(0xFFFF);
    avcc.done();
    avc1.add(avcc);
    Box stsd("stsd");
    stsd.full(0, 0);
    stsd.u32_(1);
    avc1.done();
    stsd.add(avc1);

    Box stts("stts");
    stts.full(0, 0);
    std::vector<std::pair<u32, u32>> runs;
    for (u32 d : durs) {
      if (!runs.empty() && runs.back().second == d) ++runs.back().first;
      else runs.push_back({1, d});
    }
    stts.u32_(u32(runs.size()));
    for (auto& r : runs) {
      stts.u32_(r.first);
      stts.u32_(r.second);
    }
    Box stss("stss");
    stss.full(0, 0);
    stss.u32_(u32(sync.size()));
    for (u32 s : sync) stss.u32_(s);
    Box stsc("stsc");
    stsc.full(0, 0);
    stsc.u32_(1);
    stsc.u32_(1);
    stsc.u32_(u32(samples.size()));
    stsc.u32_(1);
    Box stsz("stsz");
    stsz.full(0, 0);
    stsz.u32_(0);
    stsz.u32_(u32(samples.size()));
    for (auto& s : samples) stsz.u32_(u32(s.size()));
    Box stco("stco");
    stco.full(0, 0);
    stco.u32_(1);
    stco.u32_(chunk_offset);

    Box stbl("stbl");
    stsd.done(); stts.done(); stss.done(); stsc.done(); stsz.done(); stco.done();
    stbl.add(stsd);
    stbl.add(stts);
    if (!sync.empty()) stbl.add(stss);
    stbl.add(stsc);
    stbl.add(stsz);
    stbl.add(stco);
    Box minf("minf");
    vmhd.done(); dinf.done(); stbl.done();
    minf.add(vmhd);
    minf.add(dinf);
    minf.add(stbl);
    Box mdia("mdia");
    mdhd.done(); hdlr.done(); minf.done();
    mdia.add(mdhd);
    mdia.add(hdlr);
    mdia.add(minf);
    Box trak("trak");
    tkhd.done(); mdia.done();
    trak.add(tkhd);
    trak.add(mdia);
    Box moov("moov");
    mvhd.done(); trak.done();
    moov.add(mvhd);
    moov.add(trak);
    return std::vector<u8>(moov.done());
  };
  const std::vector<u8>& fb = ftyp.done();
  std::vector<u8> moov = build_moov(0);
  const u32 off = u32(fb.size() + moov.size() + 8);
  moov = build_moov(off);
  size_t mdat_len = 8;
  for (auto& s : samples) mdat_len += s.size();
  std::vector<u8> out;
  out.reserve(fb.size() + moov.size() + mdat_len);
  out.insert(out.end(), fb.begin(), fb.end());
  out.insert(out.end(), moov.begin(), moov.end());
  out.push_back(u8(mdat_len >> 24));
  out.push_back(u8(mdat_len >> 16));
  out.push_back(u8(mdat_len >> 8));
  out.push_back(u8(mdat_len));
  out.insert(out.end(), {'m', 'd', 'a', 't'});
  for (auto& s : samples) out.insert(out.end(), s.begin(), s.end());
  return out;
}

// -------------------------------------------------------------------------------- Archiver

Archiver::Archiver() : th_([this] { loop(); }) {}

Archiver::~Archiver() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
}

void Archiver::enqueue(const std::string& dir, const std::string& device, i64 start_ms,
                       std::vector<AuPtr> gop, Mp4Info info) {
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(Job{dir, device, start_ms, std::move(gop), std::move(info)});
  }
  cv_.notify_one();
}

void Archiver::flush() {
  std::unique_lock<std::mutex> g(mu_);
  idle_.wait(g, [&] { return q_.empty() && !busy_; });
}

std::string Archiver::last_path() const {
  std::lock_guard<std::mutex> g(const_cast<std::mutex&>(mu_));
  return last_;
}

static void mkdirs(const std::string& p) {
  std::string cur;
  for (size_t i = 0; i < p.size(); ++i) {
    cur.push_back(p[i]);
    if (p[i] == '/' || i + 1 == p.size()) ::mkdir(cur.c_str(), 0755);
  }
}

void Archiver::loop() {
  for (;;) {
    Job j;
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) {
        if (stop_) return;
        continue;
      }
      j = std::move(q_.front());
      q_.pop_front();
      busy_ = true;
    }
    try {
      std::string dir = j.dir;
      if (!dir.empty() && dir.back() != '/') dir += '/';
      dir += j.device;
      mkdirs(dir);
      std::string path = dir + "/" + std::to_string(j.start_ms) + "_" +
                         std::to_string(segment_duration_ms(j.gop)) + ".mp4";
      std::vector<u8> bytes = build_mp4(j.gop, j.info);
      std::string tmp = path + ".part";
      FILE* f = std::fopen(tmp.c_str(), "wb");
      VEP_CHECK(f, "cannot open " + tmp);
      size_t w = std::fwrite(bytes.data(), 1, bytes.size(), f);
      std::fclose(f);
      VEP_CHECK(w == bytes.size(), "short write " + tmp);
      VEP_CHECK(std::rename(tmp.c_str(), path.c_str()) == 0, "rename failed " + path);
      written_.fetch_add(1);
      std::lock_guard<std::mutex> g(mu_);
      last_ = path;
    } catch (const std::exception&) {
      failed_.fetch_add(1);
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      busy_ = false;
    }
    idle_.notify_all();
  }
}

}  // namespace vep::mux
