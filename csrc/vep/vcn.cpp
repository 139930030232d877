// VCN decode backend (vcn.h): rocDecode loaded at run time, one parser + decoder per camera.
#include "vcn.h"

#include <dlfcn.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>

// The rocDecode API as ROCm ships it (the copy inside rocprofiler-sdk: rocdecode.h + rocparser.h).
#include <rocprofiler-sdk/rocdecode/details/rocparser.h>

#include "gpu.h"

namespace vep::vcn {

namespace {

struct Api {
  decltype(&rocDecCreateVideoParser) create_parser = nullptr;
  decltype(&rocDecParseVideoData) parse = nullptr;
  decltype(&rocDecParserMarkFrameForReuse) mark_reuse = nullptr;  // optional (older releases)
  decltype(&rocDecDestroyVideoParser) destroy_parser = nullptr;
  decltype(&rocDecCreateDecoder) create_decoder = nullptr;
  decltype(&rocDecDestroyDecoder) destroy_decoder = nullptr;
  decltype(&rocDecDecodeFrame) decode_frame = nullptr;
  decltype(&rocDecGetDecodeStatus) decode_status = nullptr;  // optional
  decltype(&rocDecGetVideoFrame) get_frame = nullptr;
  decltype(&rocDecGetErrorName) error_name = nullptr;  // optional
  std::string path, error;
};

Api try_load(const std::string& lib) {
  Api t;
  void* h = dlopen(lib.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    const char* e = dlerror();
    t.error = e ? e : (lib + ": cannot be loaded");
    return t;
  }
  auto sym = [&](auto& fn, const char* name) { fn = reinterpret_cast<std::decay_t<decltype(fn)>>(dlsym(h, name)); };
  sym(t.create_parser, "rocDecCreateVideoParser");
  sym(t.parse, "rocDecParseVideoData");
  sym(t.mark_reuse, "rocDecParserMarkFrameForReuse");
  sym(t.destroy_parser, "rocDecDestroyVideoParser");
  sym(t.create_decoder, "rocDecCreateDecoder");
  sym(t.destroy_decoder, "rocDecDestroyDecoder");
  sym(t.decode_frame, "rocDecDecodeFrame");
  sym(t.decode_status, "rocDecGetDecodeStatus");
  sym(t.get_frame, "rocDecGetVideoFrame");
  sym(t.error_name, "rocDecGetErrorName");
  if (t.create_parser && t.parse && t.destroy_parser && t.create_decoder && t.destroy_decoder && t.decode_frame &&
      t.get_frame) {
    t.path = lib;  // the handle stays open for the process lifetime
    return t;
  }
  dlclose(h);
  Api bad;
  bad.error = lib + ": missing rocDecode entry points";
  return bad;
}

std::mutex g_api_mu;
Api g_api;
bool g_api_tried = false;

const Api& api() {
  std::lock_guard<std::mutex> g(g_api_mu);
  if (!g_api_tried) {
    g_api_tried = true;
    std::vector<std::string> cands;
    if (const char* e = std::getenv("VEP_ROCDECODE_LIB"); e && *e) cands.push_back(e);
    for (const char* n : {"librocdecode.so.1", "librocdecode.so.0", "librocdecode.so",
                          "/opt/rocm/lib/librocdecode.so.1", "/opt/rocm/lib/librocdecode.so"})
      cands.push_back(n);
    std::string first_error;
    for (const std::string& lib : cands) {
      Api t = try_load(lib);
      if (t.create_parser) {
        g_api = std::move(t);
        break;
      }
      if (first_error.empty()) first_error = t.error;
    }
    if (!g_api.create_parser) g_api.error = first_error.empty() ? "librocdecode not found" : first_error;
  }
  return g_api;
}

std::string status_name(rocDecStatus s) {
  const Api& a = api();
  if (a.error_name)
    if (const char* n = a.error_name(s)) return n;
  return "rocDecStatus " + std::to_string(int(s));
}

// Pictures in flight beyond the parser's minimum: a displayed picture keeps its surface until
// the worker has copied it (lane stages + one queued job per camera).
constexpr int kSurfaceHeadroom = 6;
constexpr int kMaxSurfaces = 32;

struct DecoderBox {  // owned by the session and by every Frame mapped from it
  rocDecDecoderHandle h = nullptr;
  ~DecoderBox() {
    if (h) api().destroy_decoder(h);
  }
};

}  // namespace

struct Core : std::enable_shared_from_this<Core> {
  std::recursive_mutex mu;
  RocdecVideoParser parser = nullptr;
  std::shared_ptr<DecoderBox> dec;
  u64 generation = 0;
  int device = 0;
  int coded_w = 0, coded_h = 0, out_w = 0, out_h = 0;
  RocdecVideoFormat fmt{};
  struct Meta {
    i64 pts, dts, tag, arrival_ms;
    bool keyframe, corrupt;
    char type;
  };
  std::map<u64, Meta> meta;           // packet timestamp -> its access unit
  std::vector<FramePtr>* sink = nullptr;  // display callback output during a parse call
  std::string err;
  SessionStats st;

  ~Core() {
    if (parser) api().destroy_parser(parser);
    parser = nullptr;
  }

  static int ROCDECAPI on_sequence(void* ud, RocdecVideoFormat* f) {
    Core& c = *static_cast<Core*>(ud);
    if (f->chroma_format != rocDecVideoChromaFormat_420 || f->bit_depth_luma_minus8 != 0 ||
        f->bit_depth_chroma_minus8 != 0) {
      c.err = "VCN: only 8-bit 4:2:0 streams are supported";
      return 0;
    }
    const int surfaces = std::max<int>(f->min_num_decode_surfaces,
                                       std::min<int>(f->min_num_decode_surfaces + kSurfaceHeadroom, kMaxSurfaces));
    const int ow = f->display_area.right - f->display_area.left;
    const int oh = f->display_area.bottom - f->display_area.top;
    if (ow <= 0 || oh <= 0 || (ow & 1) || (oh & 1)) {
      c.err = "VCN: unsupported display area";
      return 0;
    }
    ++c.st.sequences;
    if (c.dec && c.coded_w == int(f->coded_width) && c.coded_h == int(f->coded_height) && c.out_w == ow &&
        c.out_h == oh)
      return surfaces;
    // new (or first) sequence geometry: a fresh decoder; frames still mapped from the old one
    // keep it alive until the worker has copied them
    RocDecoderCreateInfo ci{};
    ci.device_id = u8(std::max(c.device, 0));
    ci.width = f->coded_width;
    ci.height = f->coded_height;
    ci.num_decode_surfaces = u32(surfaces);
    ci.codec_type = f->codec;
    ci.chroma_format = rocDecVideoChromaFormat_420;
    ci.bit_depth_minus_8 = 0;
    ci.max_width = f->coded_width;
    ci.max_height = f->coded_height;
    ci.display_rect.left = i16(f->display_area.left);
    ci.display_rect.top = i16(f->display_area.top);
    ci.display_rect.right = i16(f->display_area.right);
    ci.display_rect.bottom = i16(f->display_area.bottom);
    ci.output_format = rocDecVideoSurfaceFormat_NV12;
    ci.target_width = u32(ow);
    ci.target_height = u32(oh);
    ci.num_output_surfaces = 2;
    auto box = std::make_shared<DecoderBox>();
    const rocDecStatus s = api().create_decoder(&box->h, &ci);
    if (s != ROCDEC_SUCCESS || !box->h) {
      box->h = nullptr;
      c.err = "VCN: rocDecCreateDecoder failed: " + status_name(s);
      return 0;
    }
    c.dec = std::move(box);
    ++c.generation;
    c.coded_w = int(f->coded_width);
    c.coded_h = int(f->coded_height);
    c.out_w = ow;
    c.out_h = oh;
    c.fmt = *f;
    return surfaces;
  }

  static int ROCDECAPI on_decode(void* ud, RocdecPicParams* p) {
    Core& c = *static_cast<Core*>(ud);
    if (!c.dec) {
      c.err = "VCN: picture before any sequence header";
      return 0;
    }
    const rocDecStatus s = api().decode_frame(c.dec->h, p);
    if (s != ROCDEC_SUCCESS) {
      ++c.st.errors;
      c.err = "VCN: rocDecDecodeFrame failed: " + status_name(s);
      return 0;
    }
    ++c.st.decoded;
    return 1;
  }

  static int ROCDECAPI on_display(void* ud, RocdecParserDispInfo* di) {
    Core& c = *static_cast<Core*>(ud);
    if (!di) return 1;  // end-of-stream notification
    if (!c.dec) return 0;
    void* planes[3] = {nullptr, nullptr, nullptr};
    u32 pitch[3] = {0, 0, 0};
    RocdecProcParams pp{};
    pp.progressive_frame = di->progressive_frame;
    pp.top_field_first = di->top_field_first;
    const rocDecStatus s = api().get_frame(c.dec->h, di->picture_index, planes, pitch, &pp);
    if (s != ROCDEC_SUCCESS || !planes[0] || !planes[1] || pitch[0] < u32(c.out_w)) {
      ++c.st.errors;
      c.err = "VCN: rocDecGetVideoFrame failed: " + status_name(s);
      if (api().mark_reuse && c.parser) api().mark_reuse(c.parser, di->picture_index);
      return 0;
    }
    auto f = std::make_shared<Frame>();
    f->y = static_cast<const u8*>(planes[0]);
    f->uv = static_cast<const u8*>(planes[1]);
    f->pitch_y = pitch[0];
    f->pitch_uv = pitch[1] ? pitch[1] : pitch[0];
    f->width = c.out_w;
    f->height = c.out_h;
    if (api().decode_status) {
      RocdecDecodeStatus ds{};
      if (api().decode_status(c.dec->h, di->picture_index, &ds) == ROCDEC_SUCCESS)
        f->corrupt = ds.decode_status == rocDecodeStatus_Error ||
                     ds.decode_status == rocDecodeStatus_Error_Concealed;
    }
    auto m = c.meta.find(u64(di->pts));
    if (m != c.meta.end()) {
      f->pts = m->second.pts;
      f->dts = m->second.dts;
      f->tag = m->second.tag;
      f->arrival_ms = m->second.arrival_ms;
      f->keyframe = m->second.keyframe;
      f->corrupt = f->corrupt || m->second.corrupt;
      f->type = m->second.type;
    }
    f->core_ = c.shared_from_this();
    f->dec_ = c.dec;
    f->pic_idx_ = di->picture_index;
    f->generation_ = c.generation;
    ++c.st.displayed;
    if (c.sink) c.sink->push_back(std::move(f));
    return 1;
  }
};

Frame::~Frame() {
  if (!core_ || pic_idx_ < 0) return;
  std::lock_guard<std::recursive_mutex> g(core_->mu);
  if (generation_ == core_->generation && core_->parser && api().mark_reuse)
    api().mark_reuse(core_->parser, pic_idx_);
}

bool available() {
  const Api& a = api();
  return a.create_parser != nullptr;
}

bool load(const std::string& path) {
  api();  // the default search first: a loaded library is never replaced
  std::lock_guard<std::mutex> g(g_api_mu);
  if (g_api.create_parser) return true;
  Api t = try_load(path);
  if (!t.create_parser) {
    g_api.error = t.error;
    return false;
  }
  g_api = std::move(t);
  return true;
}

std::string library() { return api().path; }
std::string load_error() { return available() ? std::string() : api().error; }

Session::Session(Codec codec, int device) : codec_(codec) {
  VEP_CHECK(available(), "VCN backend: " + api().error);
  core_ = std::make_shared<Core>();
  core_->device = device;
  RocdecParserParams pp{};
  pp.codec_type = codec == Codec::kH264 ? rocDecVideoCodec_AVC : rocDecVideoCodec_HEVC;
  pp.max_num_decode_surfaces = 1;  // the sequence callback returns the real count
  pp.clock_rate = 0;
  pp.error_threshold = 100;  // hand damaged pictures to VCN too (concealed, flagged corrupt)
  pp.max_display_delay = 0;  // display as soon as the reorder rules allow (live video)
  pp.user_data = core_.get();
  pp.pfn_sequence_callback = &Core::on_sequence;
  pp.pfn_decode_picture = &Core::on_decode;
  pp.pfn_display_picture = &Core::on_display;
  pp.pfn_get_sei_msg = nullptr;
  const rocDecStatus s = api().create_parser(&core_->parser, &pp);
  VEP_CHECK(s == ROCDEC_SUCCESS && core_->parser, "VCN: rocDecCreateVideoParser failed: " + status_name(s));
}

// Frames still held elsewhere keep the core (parser, decoder) alive past the session.
Session::~Session() = default;

namespace {
bool is_parameter_set(Codec c, const u8* nal, size_t n) {
  if (n == 0) return false;
  if (c == Codec::kH264) {
    const int t = nal[0] & 0x1F;
    return t == 7 || t == 8;
  }
  const int t = (nal[0] >> 1) & 0x3F;
  return t == 32 || t == 33 || t == 34;
}
void put_nal(std::vector<u8>& out, const u8* p, size_t n) {
  static const u8 sc[4] = {0, 0, 0, 1};
  out.insert(out.end(), sc, sc + 4);
  out.insert(out.end(), p, p + n);
}
}  // namespace

void Session::send(const u8* data, size_t n, u32 flags, u64 pts) {
  RocdecSourceDataPacket pkt{};
  pkt.flags = flags;
  pkt.payload_size = u32(n);
  pkt.payload = data;
  pkt.pts = pts;
  const rocDecStatus s = api().parse(core_->parser, &pkt);
  ++core_->st.packets;
  std::string err;
  std::swap(err, core_->err);
  if (!err.empty()) throw Error(err);
  if (s != ROCDEC_SUCCESS) {
    ++core_->st.errors;
    throw Error("VCN: rocDecParseVideoData failed: " + status_name(s));
  }
}

std::vector<FramePtr> Session::decode(const AccessUnit& au, i64 tag) {
  std::vector<FramePtr> out;
  pkt_.clear();
  bool has_ps = false;
  for (size_t i = 0; i < au.nals.size(); ++i)
    has_ps |= is_parameter_set(codec_, au.nal(i), au.nal_size(i));
  if (has_ps) {  // the stream's current parameter sets (IP cameras repeat them at every IDR)
    ps_.clear();
    for (size_t i = 0; i < au.nals.size(); ++i)
      if (is_parameter_set(codec_, au.nal(i), au.nal_size(i)))
        ps_.emplace_back(au.nal(i), au.nal(i) + au.nal_size(i));
  } else if (need_ps_) {
    for (const auto& p : ps_) put_nal(pkt_, p.data(), p.size());
  }
  for (size_t i = 0; i < au.nals.size(); ++i) put_nal(pkt_, au.nal(i), au.nal_size(i));
  if (has_ps || !ps_.empty()) need_ps_ = false;
  std::lock_guard<std::recursive_mutex> g(core_->mu);
  const u64 pts = next_pts_++;
  core_->meta[pts] = Core::Meta{au.pts, au.dts, tag, au.arrival_ms, au.keyframe, au.corrupt,
                                au.keyframe ? 'I' : '?'};
  while (core_->meta.size() > 256) core_->meta.erase(core_->meta.begin());
  core_->sink = &out;
  try {
    send(pkt_.data(), pkt_.size(), ROCDEC_PKT_ENDOFPICTURE | ROCDEC_PKT_TIMESTAMP, pts);
  } catch (...) {
    core_->sink = nullptr;
    throw;
  }
  core_->sink = nullptr;
  return out;
}

std::vector<FramePtr> Session::flush() {
  std::vector<FramePtr> out;
  std::lock_guard<std::recursive_mutex> g(core_->mu);
  core_->sink = &out;
  try {
    send(nullptr, 0, ROCDEC_PKT_ENDOFSTREAM, 0);
  } catch (...) {
    core_->sink = nullptr;
    throw;
  }
  core_->sink = nullptr;
  need_ps_ = true;
  return out;
}

SessionStats Session::stats() const {
  std::lock_guard<std::recursive_mutex> g(core_->mu);
  return core_->st;
}

int Session::coded_width() const {
  std::lock_guard<std::recursive_mutex> g(core_->mu);
  return core_->coded_w;
}

int Session::coded_height() const {
  std::lock_guard<std::recursive_mutex> g(core_->mu);
  return core_->coded_h;
}

}  // namespace vep::vcn

namespace vep::gpu {
bool rocdecode_available() { return vcn::available(); }
}  // namespace vep::gpu
