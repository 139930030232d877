// pybind11 bindings of the vep native data plane (module `video_edge_ai_proxy_amd._vep`).
// Every call that can block (decode, D2H, network) releases the GIL.
#include <malloc.h>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "vep/hostprof.h"
#include "vep/avc.h"
#include "vep/avc_cavlc.h"
#include "vep/avc_recon.h"
#include "vep/bench_driver.h"
#include "vep/cabac.h"
#include "vep/codec.h"
#include "vep/gpu.h"
#include "vep/h264.h"
#include "vep/hevc_ctu.h"
#include "vep/hevc_dec.h"
#include "vep/hevc_kern.h"
#include "bind_ext.h"
#include "vep/runtime.h"
#include "vep/synth.h"

namespace py = pybind11;
using namespace vep;

static py::bytes to_bytes(const u8* p, size_t n) {
  return py::bytes(reinterpret_cast<const char*>(p), n);
}

// (y, uv) coded NV12 planes of a surface: uint8, or uint16 for high bit depth (HEVC Main10,
// H.264 High 10); 4:2:2 (NV16): the uv plane has coded_h rows
static py::tuple surface_planes(const HostSurface& p) {
  if (p.wide()) {
    py::array_t<uint16_t> y({p.coded_h, p.coded_w});
    py::array_t<uint16_t> uv({p.chroma_rows(), p.coded_w});
    std::memcpy(y.mutable_data(), p.y16.data(), p.y16.size() * 2);
    std::memcpy(uv.mutable_data(), p.uv16.data(), p.uv16.size() * 2);
    return py::make_tuple(y, uv);
  }
  py::array_t<uint8_t> y({p.coded_h, p.coded_w});
  py::array_t<uint8_t> uv({p.chroma_rows(), p.coded_w});
  std::memcpy(y.mutable_data(), p.y.data(), p.y.size());
  std::memcpy(uv.mutable_data(), p.uv.data(), p.uv.size());
  return py::make_tuple(y, uv);
}

static py::dict meta_dict(const FrameMeta& m) {
  py::dict d;
  d["width"] = m.width;
  d["height"] = m.height;
  d["timestamp"] = m.timestamp;
  d["pts"] = m.pts;
  d["dts"] = m.dts;
  d["packet"] = m.packet;
  d["keyframe"] = m.keyframe;
  d["is_keyframe"] = m.is_keyframe;
  d["is_corrupt"] = m.is_corrupt;
  d["frame_type"] = std::string(1, m.frame_type);
  d["time_base"] = m.time_base;
  d["seq"] = m.seq;
  d["decoded_us"] = m.decoded_us;
  d["arrival_ms"] = m.arrival_ms;
  return d;
}

// Worst case of a VideoFrame's trailer (everything after the pixel data): 7 varint fields
// (<= 11 B each), 2 bools, frame_type, time_base, shape, device_id.
static py::dict pic_dict(const PictureInfo& p) {
  py::dict d;
  d["width"] = p.width;
  d["height"] = p.height;
  d["coded_width"] = p.coded_width;
  d["coded_height"] = p.coded_height;
  d["pict_type"] = std::string(1, p.pict_type);
  d["idr"] = p.idr;
  d["frame_num"] = p.frame_num;
  d["coded_mbs"] = p.coded_mbs;
  d["fps"] = p.fps;
  return d;
}

// Callers bind the result to a local (`auto cp = cam_ref(w, i)`) when the camera must outlive
// a GIL-released section; short accessors use cam_of.
static py::dict domain_dict(const HostDomain& d) {
  py::dict o;
  o["device"] = d.device;
  o["index"] = d.index;
  o["numa_node"] = d.numa_node;
  o["pci_bus_id"] = d.pci_bus_id;
  o["cpus"] = d.cpus;
  o["cpulist"] = format_cpulist(d.cpus);
  o["cpu_share"] = d.cpu_share;
  o["parse_threads"] = d.parse_threads;
  o["io_threads"] = d.io_threads;
  o["source"] = d.source;
  return o;
}

static HostDomain domain_from(const py::dict& o) {
  HostDomain d;
  auto get_i = [&](const char* k, int dflt) { return o.contains(k) ? o[k].cast<int>() : dflt; };
  d.device = get_i("device", -1);
  d.index = get_i("index", 0);
  d.numa_node = get_i("numa_node", -1);
  if (o.contains("pci_bus_id")) d.pci_bus_id = o["pci_bus_id"].cast<std::string>();
  if (o.contains("cpus")) d.cpus = o["cpus"].cast<std::vector<int>>();
  d.cpu_share = get_i("cpu_share", int(d.cpus.size()));
  d.parse_threads = get_i("parse_threads", 0);
  d.io_threads = get_i("io_threads", 1);
  if (o.contains("source")) d.source = o["source"].cast<std::string>();
  return d;
}

static std::shared_ptr<Camera> cam_ref(Worker& w, int idx) {
  std::shared_ptr<Camera> c = w.camera(idx);
  if (!c) throw py::index_error("no camera with index " + std::to_string(idx));
  return c;
}
static Camera& cam_of(Worker& w, int idx) { return *cam_ref(w, idx); }

// Stateful oracle: parse + CPU reconstruct a sequence of AUs, return the final BGR picture.
// Streams inside the I_PCM / P_Skip subset take the fast-path parser; anything else switches to
// the general H.264 decoder (avc.h) for good, like a Camera does.
struct CpuDecoder {
  StreamParser parser;
  MbUpdate upd;
  HostSurface surf;
  PictureInfo last;
  avc::Decoder avc;
  std::vector<HostSurface> slots;
  bool general = false;
  int target = 0;
  int coded = 0;
  bool fields_out = false;  // the newest output is a field pair (woven into `woven`)
  HostSurface woven;
  mutable HostSurface weave_tmp;
  const HostSurface& out() const { return general ? (fields_out ? woven : slots[size_t(target)]) : surf; }
  // samples of an output frame (a field pair: its two field slots woven)
  const HostSurface& frame_of(const avc::OutFrame& f) const {
    if (!f.fields) return slots[size_t(f.slot)];
    avc::weave_fields(slots[2 * size_t(f.slot)], slots[2 * size_t(f.slot) + 1], weave_tmp);
    return weave_tmp;
  }
  py::object decode(const AccessUnit& au) {
    bool no_output = false;
    {
      py::gil_scoped_release nogil;
      bool done = false;
      if (!general) {
        try {
          upd.clear_payload();  // `au` outlives this call: src pointers into it are safe
          last = parser.parse(au, upd);
          if (surf.coded_w != last.coded_width || surf.coded_h != last.coded_height)
            surf.alloc(last.coded_width, last.coded_height);
          cpu_apply_update(upd, surf);
          coded = upd.nslots;
          done = true;
        } catch (const UnsupportedStream&) {
          if (au.codec != Codec::kH264) throw;
          general = true;
        }
      }
      std::vector<avc::OutFrame> outs;
      size_t nal = 0;  // (a field pair may come as one access unit: one picture per field)
      while (!done) {
        avc::PicturePtr pic = avc.parse(au, 0, &nal);
        done = nal >= au.nals.size();
        if (slots.size() < size_t(pic->dpb_slots)) slots.resize(size_t(pic->dpb_slots));
        for (auto& h : slots)
          if (h.coded_w != pic->wmbs * 16 || h.coded_h != pic->hmbs * 16 || h.bd != pic->bd || h.cf != pic->cf)
            h.alloc(pic->wmbs * 16, pic->hmbs * 16, pic->bd, pic->cf);
        avc::cpu_reconstruct(*pic, slots);
        coded = pic->info.coded_mbs;
        pictures.push_back(pic->info);
        for (const avc::MbRec& m : pic->mbs) {
          ++kinds[m.kind];
          if (m.flags & avc::kMbT8x8) ++t8x8;
          if (m.flags & avc::kMbWp) ++weighted;
          if (m.kind <= avc::kInter) {
            bool bi = false, l1only = false;
            for (int k = 0; k < 4; ++k) {
              bi |= m.ref[k] != 0xFF && m.ref1[k] != 0xFF;
              l1only |= m.ref[k] == 0xFF && m.ref1[k] != 0xFF;
            }
            bipred += bi;
            list1_only += l1only;
          }
        }
        outs.insert(outs.end(), pic->outputs.begin(), pic->outputs.end());
        if (!done) continue;
        // B-frame reordering: the newest frame that left the reorder buffer, if any
        pending_outputs = outs;
        no_output = outs.empty();
        if (!no_output) {
          last = outs.back().info;
          target = outs.back().slot;
          fields_out = outs.back().fields;
          if (fields_out) woven = frame_of(outs.back());
          last_poc = outs.back().poc;
          last_pts = outs.back().au.pts;
        }
      }
    }
    if (no_output) return py::none();
    py::array_t<uint8_t> o({last.height, last.width, 3});
    cpu_nv12_to_bgr(out(), last.crop_left, last.crop_top, last.width, last.height, o.mutable_data());
    return o;
  }
  // Every frame that left the reorder buffer with the last decode() (or, after flush_frames(),
  // at end of stream): [(pts, (Y, UV) coded NV12 planes)] in output order.
  py::list frames_of(const std::vector<avc::OutFrame>& fs) const {
    py::list l;
    for (const auto& f : fs) {
      const HostSurface& s = frame_of(f);
      l.append(py::make_tuple(f.au.pts, surface_planes(s)));
    }
    return l;
  }
  // Frames still in the reorder buffer (end of stream), oldest first.
  py::list flush() {
    py::list out_list;
    for (const auto& f : avc.flush_output()) {
      py::array_t<uint8_t> o({f.info.height, f.info.width, 3});
      cpu_nv12_to_bgr(frame_of(f), f.info.crop_left, f.info.crop_top, f.info.width, f.info.height,
                      o.mutable_data());
      out_list.append(o);
    }
    return out_list;
  }
  std::vector<PictureInfo> pictures;      // every decoded picture (decoding order)
  // macroblock statistics over every decoded picture (coverage checks)
  u64 kinds[6] = {0, 0, 0, 0, 0, 0};
  u64 t8x8 = 0, weighted = 0, bipred = 0, list1_only = 0;
  std::vector<avc::OutFrame> pending_outputs;  // outputs of the last decode() (output order)
  int last_poc = 0;
  i64 last_pts = 0;
};

PYBIND11_MODULE(_vep, m) {
  m.doc() = "vep native data plane (gfx950 HIP kernels, H.264 subset decoder, RTSP/RTP, muxers)";
  py::register_exception<Error>(m, "NativeError");
  py::register_exception<UnsupportedStream>(m, "UnsupportedStream");

  m.def("device_count", &gpu::device_count);
  // Frame servers and clients allocate a new multi-MB buffer per frame: glibc would mmap each
  // one and the first touch of its pages then costs more than the copy itself. Keep such blocks
  // in the (per-thread) heaps instead, so freed frame buffers are reused without page faults.
  // The arenas are capped (M_ARENA_MAX): with hundreds of handler threads, per-thread arenas each
  // keeping freed frames plus the trim threshold would grow the resident set without bound.
  m.def("tune_malloc_for_frames", [](int mmap_threshold_mb, int arenas) {
    const int thr = std::max(1, mmap_threshold_mb) << 20;
    return mallopt(M_MMAP_THRESHOLD, thr) == 1 && mallopt(M_TRIM_THRESHOLD, 4 * thr) == 1 &&
           mallopt(M_TOP_PAD, thr) == 1 && (arenas <= 0 || mallopt(M_ARENA_MAX, arenas) == 1);
  }, py::arg("mmap_threshold_mb") = 64, py::arg("arenas") = 8);

  py::class_<SynthConfig>(m, "SynthConfig")
      .def(py::init<>())
      .def_readwrite("width", &SynthConfig::width)
      .def_readwrite("height", &SynthConfig::height)
      .def_readwrite("fps", &SynthConfig::fps)
      .def_readwrite("gop", &SynthConfig::gop)
      .def_readwrite("motion", &SynthConfig::motion)
      .def_readwrite("seed", &SynthConfig::seed)
      .def_readwrite("slices", &SynthConfig::slices)
      .def_readwrite("zero_samples", &SynthConfig::zero_samples)
      .def_readwrite("idr_phase", &SynthConfig::idr_phase)
      .def_readwrite("merge_cands", &SynthConfig::merge_cands)
      .def_readwrite("compressed", &SynthConfig::compressed)
      .def_readwrite("qp", &SynthConfig::qp)
      .def_readwrite("refs", &SynthConfig::refs)
      .def_readwrite("objects", &SynthConfig::objects)
      .def_readwrite("deblock_idc", &SynthConfig::deblock_idc)
      .def_readwrite("coverage", &SynthConfig::coverage)
      .def_readwrite("noise", &SynthConfig::noise)
      .def_readwrite("temporal_noise", &SynthConfig::temporal_noise)
      .def_readwrite("profile", &SynthConfig::profile)
      .def_readwrite("bframes", &SynthConfig::bframes)
      .def_readwrite("cabac", &SynthConfig::cabac)
      .def_readwrite("weighted_p", &SynthConfig::weighted_p)
      .def_readwrite("weighted_b", &SynthConfig::weighted_b)
      .def_readwrite("direct_spatial", &SynthConfig::direct_spatial)
      .def_readwrite("tile_cols", &SynthConfig::tile_cols)
      .def_readwrite("tile_rows", &SynthConfig::tile_rows)
      .def_readwrite("wpp", &SynthConfig::wpp)
      .def_readwrite("segments", &SynthConfig::segments)
      .def_readwrite("scaling_lists", &SynthConfig::scaling_lists)
      .def_readwrite("long_term", &SynthConfig::long_term)
      .def_readwrite("open_gop", &SynthConfig::open_gop)
      .def_readwrite("lossless", &SynthConfig::lossless)
      .def_readwrite("bit_depth", &SynthConfig::bit_depth)
      .def_readwrite("chroma_format", &SynthConfig::chroma_format)
      .def_readwrite("interlaced", &SynthConfig::interlaced)
      .def_readwrite("mono", &SynthConfig::mono)
      .def_property(
          "codec", [](const SynthConfig& c) { return c.codec == Codec::kH265 ? "h265" : "h264"; },
          [](SynthConfig& c, const std::string& v) {
            if (v == "h264" || v == "avc") c.codec = Codec::kH264;
            else if (v == "h265" || v == "hevc") c.codec = Codec::kH265;
            else throw Error("codec must be h264 or h265");
          });

  py::class_<AccessUnit, std::shared_ptr<AccessUnit>>(m, "AccessUnit")
      .def(py::init<>())
      .def_property_readonly("codec", [](const AccessUnit& a) { return int(a.codec); })
      .def_readwrite("pts", &AccessUnit::pts)
      .def_readwrite("dts", &AccessUnit::dts)
      .def_readwrite("duration", &AccessUnit::duration)
      .def_readwrite("keyframe", &AccessUnit::keyframe)
      .def_readwrite("corrupt", &AccessUnit::corrupt)
      .def_readwrite("arrival_ms", &AccessUnit::arrival_ms)
      .def_readwrite("seq", &AccessUnit::seq)
      .def_property_readonly("size", &AccessUnit::bytes)
      .def("pin", &AccessUnit::pin)
      .def_property_readonly("pinned", &AccessUnit::pinned)
      .def("nals",
           [](const AccessUnit& a) {
             py::list l;
             for (size_t i = 0; i < a.nals.size(); ++i) l.append(to_bytes(a.nal(i), a.nal_size(i)));
             return l;
           })
      .def("annexb",
           [](const AccessUnit& a) {
             std::string s;
             for (size_t i = 0; i < a.nals.size(); ++i) {
               s.append("\x00\x00\x00\x01", 4);
               s.append(reinterpret_cast<const char*>(a.nal(i)), a.nal_size(i));
             }
             return py::bytes(s);
           })
      .def_static(
          "from_nals",
          [](const std::vector<std::string>& nals, i64 pts, i64 dts, bool key, int codec) {
            auto a = std::make_shared<AccessUnit>();
            a->codec = Codec(codec);
            for (auto& n : nals) a->add_nal(reinterpret_cast<const u8*>(n.data()), n.size());
            a->pts = pts;
            a->dts = dts;
            a->keyframe = key;
            a->arrival_ms = now_ms();
            return a;
          },
          py::arg("nals"), py::arg("pts") = 0, py::arg("dts") = 0, py::arg("keyframe") = false,
          py::arg("codec") = 0);

  py::class_<SynthH264>(m, "SynthH264")
      .def(py::init<const SynthConfig&>())
      .def("next", [](SynthH264& s) { return std::shared_ptr<AccessUnit>(s.next()); },
           py::call_guard<py::gil_scoped_release>())
      .def("picture", [](const SynthH264& s) { return surface_planes(s.picture()); })
      .def_property_readonly("sps_nal", [](const SynthH264& s) { return to_bytes(s.sps_nal().data(), s.sps_nal().size()); })
      .def_property_readonly("pps_nal", [](const SynthH264& s) { return to_bytes(s.pps_nal().data(), s.pps_nal().size()); })
      .def_property_readonly("vps_nal", [](const SynthH264& s) { return to_bytes(s.vps_nal().data(), s.vps_nal().size()); })
      .def_property_readonly("frame_index", &SynthH264::frame_index)
      .def_property_readonly("last_pts", &SynthH264::last_pts);
  m.attr("SynthEncoder") = m.attr("SynthH264");

  auto surface_tuple = [](const HostSurface& p) { return surface_planes(p); };

  py::class_<avc::AvcHighConfig>(m, "AvcHighConfig")
      .def(py::init<>())
      .def_readwrite("width", &avc::AvcHighConfig::width)
      .def_readwrite("height", &avc::AvcHighConfig::height)
      .def_readwrite("fps", &avc::AvcHighConfig::fps)
      .def_readwrite("gop", &avc::AvcHighConfig::gop)
      .def_readwrite("idr_phase", &avc::AvcHighConfig::idr_phase)
      .def_readwrite("bframes", &avc::AvcHighConfig::bframes)
      .def_readwrite("pyramid", &avc::AvcHighConfig::pyramid)
      .def_readwrite("refs", &avc::AvcHighConfig::refs)
      .def_readwrite("qp", &avc::AvcHighConfig::qp)
      .def_readwrite("bit_depth", &avc::AvcHighConfig::bit_depth)
      .def_readwrite("chroma_format", &avc::AvcHighConfig::chroma_format)
      .def_readwrite("cabac", &avc::AvcHighConfig::cabac)
      .def_readwrite("t8x8", &avc::AvcHighConfig::t8x8)
      .def_readwrite("weighted_p", &avc::AvcHighConfig::weighted_p)
      .def_readwrite("weighted_b", &avc::AvcHighConfig::weighted_b)
      .def_readwrite("direct_spatial", &avc::AvcHighConfig::direct_spatial)
      .def_readwrite("scaling", &avc::AvcHighConfig::scaling)
      .def_readwrite("slices", &avc::AvcHighConfig::slices)
      .def_readwrite("deblock_idc", &avc::AvcHighConfig::deblock_idc)
      .def_readwrite("chroma_qp_offset", &avc::AvcHighConfig::chroma_qp_offset)
      .def_readwrite("second_chroma_qp_offset", &avc::AvcHighConfig::second_chroma_qp_offset)
      .def_readwrite("coverage", &avc::AvcHighConfig::coverage)
      .def_readwrite("interlaced", &avc::AvcHighConfig::interlaced)
      .def_readwrite("mono", &avc::AvcHighConfig::mono)
      .def_readwrite("fields", &avc::AvcHighConfig::fields)
      .def_readwrite("marking", &avc::AvcHighConfig::marking)
      .def_readwrite("objects", &avc::AvcHighConfig::objects)
      .def_readwrite("noise", &avc::AvcHighConfig::noise)
      .def_readwrite("temporal_noise", &avc::AvcHighConfig::temporal_noise)
      .def_readwrite("seed", &avc::AvcHighConfig::seed);
  py::class_<avc::AvcHighEncoder>(m, "AvcHighEncoder")
      .def(py::init<const avc::AvcHighConfig&>())
      .def("next", &avc::AvcHighEncoder::next, py::call_guard<py::gil_scoped_release>())
      .def("picture", [surface_tuple](const avc::AvcHighEncoder& e) { return surface_tuple(e.reconstruction()); })
      .def("source", [surface_tuple](const avc::AvcHighEncoder& e) { return surface_tuple(e.source()); })
      .def_property_readonly("last_pts", &avc::AvcHighEncoder::last_pts)
      .def_property_readonly("last_type", [](const avc::AvcHighEncoder& e) { return std::string(1, e.last_type()); })
      .def_property_readonly("last_display_index", &avc::AvcHighEncoder::last_display_index)
      .def_property_readonly("sps_nal", [](const avc::AvcHighEncoder& e) { return to_bytes(e.sps_nal().data(), e.sps_nal().size()); })
      .def_property_readonly("pps_nal", [](const avc::AvcHighEncoder& e) { return to_bytes(e.pps_nal().data(), e.pps_nal().size()); });

  py::class_<hevc::HevcEncConfig>(m, "HevcEncConfig")
      .def(py::init<>())
      .def_readwrite("width", &hevc::HevcEncConfig::width)
      .def_readwrite("height", &hevc::HevcEncConfig::height)
      .def_readwrite("fps", &hevc::HevcEncConfig::fps)
      .def_readwrite("gop", &hevc::HevcEncConfig::gop)
      .def_readwrite("idr_phase", &hevc::HevcEncConfig::idr_phase)
      .def_readwrite("bframes", &hevc::HevcEncConfig::bframes)
      .def_readwrite("qp", &hevc::HevcEncConfig::qp)
      .def_readwrite("log2_ctb", &hevc::HevcEncConfig::log2_ctb)
      .def_readwrite("log2_min_cb", &hevc::HevcEncConfig::log2_min_cb)
      .def_readwrite("amp", &hevc::HevcEncConfig::amp)
      .def_readwrite("sao", &hevc::HevcEncConfig::sao)
      .def_readwrite("deblock", &hevc::HevcEncConfig::deblock)
      .def_readwrite("tskip", &hevc::HevcEncConfig::tskip)
      .def_readwrite("sign_hiding", &hevc::HevcEncConfig::sign_hiding)
      .def_readwrite("cu_qp_delta", &hevc::HevcEncConfig::cu_qp_delta)
      .def_readwrite("pcm", &hevc::HevcEncConfig::pcm)
      .def_readwrite("tmvp", &hevc::HevcEncConfig::tmvp)
      .def_readwrite("slices", &hevc::HevcEncConfig::slices)
      .def_readwrite("tile_cols", &hevc::HevcEncConfig::tile_cols)
      .def_readwrite("tile_rows", &hevc::HevcEncConfig::tile_rows)
      .def_readwrite("wpp", &hevc::HevcEncConfig::wpp)
      .def_readwrite("segments", &hevc::HevcEncConfig::segments)
      .def_readwrite("scaling_lists", &hevc::HevcEncConfig::scaling_lists)
      .def_readwrite("weighted", &hevc::HevcEncConfig::weighted)
      .def_readwrite("long_term", &hevc::HevcEncConfig::long_term)
      .def_readwrite("open_gop", &hevc::HevcEncConfig::open_gop)
      .def_readwrite("lossless", &hevc::HevcEncConfig::lossless)
      .def_readwrite("bit_depth", &hevc::HevcEncConfig::bit_depth)
      .def_readwrite("coverage", &hevc::HevcEncConfig::coverage)
      .def_readwrite("objects", &hevc::HevcEncConfig::objects)
      .def_readwrite("noise", &hevc::HevcEncConfig::noise)
      .def_readwrite("temporal_noise", &hevc::HevcEncConfig::temporal_noise)
      .def_readwrite("seed", &hevc::HevcEncConfig::seed);
  py::class_<hevc::HevcEncoder>(m, "HevcEncoder")
      .def(py::init<const hevc::HevcEncConfig&>())
      .def("next", &hevc::HevcEncoder::next, py::call_guard<py::gil_scoped_release>())
      .def("picture", [surface_tuple](const hevc::HevcEncoder& e) { return surface_tuple(e.reconstruction()); })
      .def("source", [surface_tuple](const hevc::HevcEncoder& e) { return surface_tuple(e.source()); })
      .def_property_readonly("last_pts", &hevc::HevcEncoder::last_pts)
      .def_property_readonly("last_type", [](const hevc::HevcEncoder& e) { return std::string(1, e.last_type()); })
      .def_property_readonly("vps_nal", [](const hevc::HevcEncoder& e) { return to_bytes(e.vps_nal().data(), e.vps_nal().size()); })
      .def_property_readonly("sps_nal", [](const hevc::HevcEncoder& e) { return to_bytes(e.sps_nal().data(), e.sps_nal().size()); })
      .def_property_readonly("pps_nal", [](const hevc::HevcEncoder& e) { return to_bytes(e.pps_nal().data(), e.pps_nal().size()); });
  // General H.265 Main decoder (CPU): decode() / flush() return the frames leaving the output
  // queue as [(pts, poc, type, (Y, UV) coded NV12 planes)] in output order.
  py::class_<hevc::Decoder>(m, "HevcDecoder")
      .def(py::init<>())
      .def("decode",
           [surface_tuple](hevc::Decoder& d, const AccessUnit& au) {
             std::vector<hevc::FramePtr> fs;
             {
               py::gil_scoped_release nogil;
               fs = d.decode(au, 0);
             }
             py::list l;
             for (const auto& f : fs) l.append(py::make_tuple(f->pts, f->poc, std::string(1, f->type), surface_tuple(f->s)));
             return l;
           })
      .def("flush",
           [surface_tuple](hevc::Decoder& d) {
             py::list l;
             for (const auto& f : d.flush()) l.append(py::make_tuple(f->pts, f->poc, std::string(1, f->type), surface_tuple(f->s)));
             return l;
           })
      .def_property_readonly("stats", [](const hevc::Decoder& d) {
        py::dict s;
        s["intra"] = d.stats.intra;
        s["inter"] = d.stats.inter;
        s["skip"] = d.stats.skip;
        s["pcm"] = d.stats.pcm;
        s["merge"] = d.stats.merge;
        s["bi"] = d.stats.bi;
        s["tskip"] = d.stats.tskip;
        s["amp"] = d.stats.amp;
        return s;
      });

  // General H.265 decoder in records mode + the CPU mirror of the GPU reconstruction (tests):
  // same outputs as HevcDecoder, reconstructed from the GPU work lists.
  struct HevcRecords {
    hevc::Decoder d;
    std::vector<HostSurface> slots;
    u64 pictures = 0, pus = 0, tus = 0, intra_tus = 0, max_level = 0, exchange_violations = 0;
    bool execute = true;  // false: parse only (records are counted, not executed: parse timing)
    explicit HevcRecords(bool ex = true) : execute(ex) { d.set_gpu_mode(true); }
    py::list frames(const std::vector<hevc::FramePtr>& fs) {
      py::list l;
      for (const auto& f : fs) {
        const HostSurface& s = slots[size_t(f->slot)];
        const int W = f->width + f->crop_left, H = f->height + f->crop_top;
        (void)W;
        (void)H;
        const int cw = s.coded_w, ch = s.coded_h;
        (void)ch;
        // the coded picture (the decoder's surfaces are coded_w x coded_h, slots are 16-aligned)
        const int pw = coded_w_, ph = coded_h_;
        py::tuple planes;
        if (s.wide()) {  // Main10: uint16 planes
          py::array_t<uint16_t> y({ph, pw});
          py::array_t<uint16_t> uv({ph / 2, pw});
          for (int r = 0; r < ph; ++r) std::memcpy(y.mutable_data() + size_t(r) * pw, &s.y16[size_t(r) * cw], size_t(pw) * 2);
          for (int r = 0; r < ph / 2; ++r)
            std::memcpy(uv.mutable_data() + size_t(r) * pw, &s.uv16[size_t(r) * cw], size_t(pw) * 2);
          planes = py::make_tuple(y, uv);
        } else {
          py::array_t<uint8_t> y({ph, pw});
          py::array_t<uint8_t> uv({ph / 2, pw});
          for (int r = 0; r < ph; ++r) std::memcpy(y.mutable_data() + size_t(r) * pw, &s.y[size_t(r) * cw], size_t(pw));
          for (int r = 0; r < ph / 2; ++r)
            std::memcpy(uv.mutable_data() + size_t(r) * pw, &s.uv[size_t(r) * cw], size_t(pw));
          planes = py::make_tuple(y, uv);
        }
        l.append(py::make_tuple(f->pts, f->poc, std::string(1, f->type), planes, f->slot));
      }
      return l;
    }
    void run(std::vector<std::shared_ptr<hevc::GpuPicture>> ps) {
      for (auto& p : ps) {
        coded_w_ = p->width;
        coded_h_ = p->height;
        const int sw = (p->width + 15) & ~15, sh = (p->height + 15) & ~15;
        if (slots.size() < size_t(d.gpu_slots())) slots.resize(size_t(d.gpu_slots()));
        const int bd = std::max(p->bd_y, p->bd_c);
        for (auto& h : slots)
          if (h.coded_w != sw || h.coded_h != sh || h.bd != bd) h.alloc(sw, sh, bd);
        if (execute) hevc::cpu_execute(*p, slots);
        ++pictures;
        pus += p->pus.size();
        tus += p->tus.size();
        for (const auto& t : p->tus) intra_tus += (t.flags & hevc::kTuIntra) ? 1 : 0;
        exchange_violations += hevc::exchange_violations(*p);
        auto h = [](const void* d, size_t n) {  // FNV-1a of a record array (tests: records equality)
          u64 x = 1469598103934665603ull;
          for (size_t i = 0; i < n; ++i) x = (x ^ static_cast<const u8*>(d)[i]) * 1099511628211ull;
          return x;
        };
        last_qp.assign(p->qp.begin(), p->qp.end());
        last_digest = {h(p->pus.data(), p->pus.size() * sizeof(hevc::GpuPu)),
                       h(p->tus.data(), p->tus.size() * sizeof(hevc::GpuTu)),
                       h(p->coefs.data(), p->coefs.size() * 2), h(p->pcm.data(), p->pcm.size()),
                       h(p->bs_v.data(), p->bs_v.size()), h(p->bs_h.data(), p->bs_h.size()),
                       h(p->qp.data(), p->qp.size()), h(p->wp.data(), p->wp.size() * sizeof(hevc::GpuWp)),
                       h(p->sao_params.data(), p->sao_params.size() * sizeof(hevc::GpuSao))};
        max_level = std::max<u64>(max_level, p->level_begin.empty() ? 0 : p->level_begin.size() - 1);
      }
    }
    int coded_w_ = 0, coded_h_ = 0;
    std::vector<u64> last_digest;  // pus, tus, coefs, pcm, bs_v, bs_h, qp, wp, sao of the last picture
    std::vector<signed char> last_qp;       // QpY per 4x4 block of the last picture
  };
  py::class_<HevcRecords>(m, "HevcRecordsDecoder")
      .def(py::init<bool>(), py::arg("execute") = true)
      .def_property_readonly("parallel_units", [](const HevcRecords& r) { return r.d.parallel_units(); })
      .def_property_readonly("last_digest", [](const HevcRecords& r) { return r.last_digest; })
      .def_property_readonly("last_qp", [](const HevcRecords& r) { return std::vector<int>(r.last_qp.begin(), r.last_qp.end()); })
      .def("decode",
           [](HevcRecords& r, const AccessUnit& au) {
             std::vector<hevc::FramePtr> fs;
             {
               py::gil_scoped_release nogil;
               fs = r.d.decode(au, 0);
               r.run(r.d.take_gpu_pictures());
             }
             return r.frames(fs);
           })
      .def("flush",
           [](HevcRecords& r) {
             auto fs = r.d.flush();
             r.run(r.d.take_gpu_pictures());
             return r.frames(fs);
           })
      .def_property_readonly("stats", [](const HevcRecords& r) {
        py::dict s;
        s["pictures"] = r.pictures;
        s["pus"] = r.pus;
        s["tus"] = r.tus;
        s["intra_tus"] = r.intra_tus;
        s["max_levels"] = r.max_level;
        s["exchange_violations"] = r.exchange_violations;
        s["slots"] = r.d.gpu_slots();
        return s;
      });

  py::class_<CpuDecoder>(m, "CpuDecoder")
      .def(py::init<>())
      .def("decode", &CpuDecoder::decode)
      .def("flush", &CpuDecoder::flush)
      .def("frames", [](CpuDecoder& d) { return d.general ? d.frames_of(d.pending_outputs) : py::list(); })
      .def("flush_frames", [](CpuDecoder& d) { return d.frames_of(d.avc.flush_output()); })
      .def_property_readonly("last_poc", [](const CpuDecoder& d) { return d.last_poc; })
      .def_property_readonly("last_pts", [](const CpuDecoder& d) { return d.last_pts; })
      .def_property_readonly("mb_stats", [](const CpuDecoder& d) {
        py::dict r;
        const char* names[6] = {"skip", "inter", "i4x4", "i16x16", "pcm", "i8x8"};
        for (int k = 0; k < 6; ++k) r[names[k]] = d.kinds[k];
        r["t8x8"] = d.t8x8;
        r["weighted"] = d.weighted;
        r["bipred"] = d.bipred;
        r["list1_only"] = d.list1_only;
        std::string types;
        for (const auto& p : d.pictures) types += p.pict_type;
        r["types"] = types;
        return r;
      })
      .def_property_readonly("outputs_last", [](const CpuDecoder& d) { return int(d.pending_outputs.size()); })
      .def_property_readonly("info", [](const CpuDecoder& d) { return pic_dict(d.last); })
      .def_property_readonly("coded_mbs", [](const CpuDecoder& d) { return d.coded; })
      .def_property_readonly("pictures_decoded", [](const CpuDecoder& d) { return d.pictures.size(); })
      .def_property_readonly("marking_stats", [](const CpuDecoder& d) {
        py::dict s;
        for (int k = 1; k <= 6; ++k) s[py::str("mmco" + std::to_string(k))] = d.avc.mmco_ops[k];
        s["list_mods"] = d.avc.list_mods;
        s["long_term_marked"] = d.avc.long_term_marked;
        s["redundant_slices_skipped"] = d.avc.redundant_slices_skipped;
        return s;
      })
      .def_property_readonly("general", [](const CpuDecoder& d) { return d.general; })
      .def_property_readonly("parallel_slices", [](const CpuDecoder& d) { return d.avc.parallel_slices_run(); })
      .def("surface", [](const CpuDecoder& d) {
        const HostSurface& s = d.out();
        py::array_t<uint8_t> y({s.coded_h, s.coded_w});
        py::array_t<uint8_t> uv({s.coded_h / 2, s.coded_w});
        std::memcpy(y.mutable_data(), s.y.data(), s.y.size());
        std::memcpy(uv.mutable_data(), s.uv.data(), s.uv.size());
        return py::make_tuple(y, uv);
      });

  // Reconstruction primitives of avc_recon.h (shared by the CPU decoder, the gfx950 kernels and
  // the encoders), exposed one by one for tests/test_spec_oracle.py, which checks them against
  // independent implementations written from the H.264 text.
  auto rc = m.def_submodule("recon", "H.264 reconstruction primitives (avc_recon.h)");
  rc.def("idct4", [](std::vector<int> d) {
    VEP_CHECK(d.size() == 16, "16 coefficients");
    i16 c[16];
    for (int k = 0; k < 16; ++k) c[k] = i16(d[size_t(k)]);
    std::vector<int> r(16);
    avc::idct4x4(c, r.data());
    return r;
  });
  rc.def("idct8", [](std::vector<int> d) {
    VEP_CHECK(d.size() == 64, "64 coefficients");
    i16 c[64];
    for (int k = 0; k < 64; ++k) c[k] = i16(d[size_t(k)]);
    std::vector<int> r(64);
    avc::idct8x8(c, r.data());
    return r;
  });
  rc.def("dequant4", [](int c, int qp, int i, int j) { return avc::dequant4x4(c, qp, i, j); });
  // top = p[-1..7, -1] (9, top-right already substituted), left = p[-1, 0..3]
  rc.def("intra4x4", [](std::vector<int> top, std::vector<int> left, bool has_top, bool has_left, int mode, int bd) {
    VEP_CHECK(top.size() == 9 && left.size() == 4, "9 top + 4 left samples");
    avc::Intra4Nb n{};
    for (int k = 0; k < 9; ++k) n.t[k] = top[size_t(k)];
    for (int k = 0; k < 4; ++k) n.l[k] = left[size_t(k)];
    n.has_top = has_top;
    n.has_left = has_left;
    std::vector<int> r(16);
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x) r[size_t(y * 4 + x)] = avc::intra4x4_pred(n, mode, x, y, bd);
    return r;
  }, py::arg("top"), py::arg("left"), py::arg("has_top"), py::arg("has_left"), py::arg("mode"), py::arg("bd") = 8);
  // top = p[-1..15, -1] (17, top-right substituted), left = p[-1, 0..7]: reference filtering +
  // prediction
  rc.def("intra8x8", [](std::vector<int> top, std::vector<int> left, bool has_top, bool has_left, bool has_tl,
                        int mode, int bd) {
    VEP_CHECK(top.size() == 17 && left.size() == 8, "17 top + 8 left samples");
    int f[25];
    avc::intra8x8_filter([&](int x) { return top[size_t(x + 1)]; }, [&](int y) { return left[size_t(y)]; },
                         has_top, has_left, has_tl, f);
    std::vector<int> r(64);
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) r[size_t(y * 8 + x)] = avc::intra8x8_pred(f, has_top, has_left, mode, x, y, bd);
    return r;
  }, py::arg("top"), py::arg("left"), py::arg("has_top"), py::arg("has_left"), py::arg("has_tl"), py::arg("mode"),
     py::arg("bd") = 8);
  rc.def("intra16x16", [](std::vector<int> top, std::vector<int> left, bool has_top, bool has_left, int mode, int bd) {
    VEP_CHECK(top.size() == 17 && left.size() == 16, "17 top + 16 left samples");
    avc::Intra16Nb n{};
    for (int k = 0; k < 17; ++k) n.top[k] = top[size_t(k)];
    for (int k = 0; k < 16; ++k) n.left[k] = left[size_t(k)];
    n.has_top = has_top;
    n.has_left = has_left;
    n.has_tl = has_top && has_left;
    const avc::PredConst k = avc::intra16x16_const(n, mode, bd);
    std::vector<int> r(256);
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) r[size_t(y * 16 + x)] = avc::intra16x16_pred(n, k, mode, x, y, bd);
    return r;
  }, py::arg("top"), py::arg("left"), py::arg("has_top"), py::arg("has_left"), py::arg("mode"), py::arg("bd") = 8);
  // (cf 2: 4:2:2, 16 left samples, 8x16 prediction)
  rc.def("intra_chroma", [](std::vector<int> top, std::vector<int> left, bool has_top, bool has_left, int mode, int bd,
                            int cf) {
    const int ch = cf == 2 ? 16 : 8;
    VEP_CHECK(top.size() == 9 && left.size() == size_t(ch), "9 top + 8 (4:2:2: 16) left samples");
    avc::IntraChromaNb n{};
    for (int k = 0; k < 9; ++k) n.top[k] = top[size_t(k)];
    for (int k = 0; k < ch; ++k) n.left[k] = left[size_t(k)];
    n.has_top = has_top;
    n.has_left = has_left;
    n.has_tl = has_top && has_left;
    const avc::PredConst k = mode == 3 ? avc::chroma_plane_const(n, cf) : avc::PredConst{0, 0, 0, 0};
    std::vector<int> r(size_t(8 * ch));
    for (int y = 0; y < ch; ++y)
      for (int x = 0; x < 8; ++x) r[size_t(y * 8 + x)] = avc::chroma_pred(n, k, mode, x, y, bd, cf);
    return r;
  }, py::arg("top"), py::arg("left"), py::arg("has_top"), py::arg("has_left"), py::arg("mode"), py::arg("bd") = 8,
     py::arg("cf") = 1);
  // 4:2:2 chroma DC: 8 levels (parsing order) -> dcC per chroma block (raster, 2 wide)
  rc.def("chroma422_dc", [](std::vector<int> lv, int qpdc, int ls) {
    VEP_CHECK(lv.size() == 8, "8 levels");
    std::vector<int> r(8);
    avc::chroma422_dc(lv.data(), qpdc, ls, r.data());
    return r;
  });
  rc.def("luma_qpel", [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> plane, int xi, int yi,
                         int fx, int fy) {
    VEP_CHECK(plane.ndim() == 2, "2-D plane");
    const int h = int(plane.shape(0)), w = int(plane.shape(1));
    return avc::luma_qpel(plane.data(), w, w, h, xi, yi, fx, fy);
  });
  rc.def("chroma_epel", [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> uv, int c, int xi,
                           int yi, int fx, int fy) {
    VEP_CHECK(uv.ndim() == 2 && uv.shape(1) % 2 == 0, "interleaved UV plane");
    const int h = int(uv.shape(0)), pitch = int(uv.shape(1));
    return avc::chroma_epel(uv.data(), pitch, pitch / 2, h, c, xi, yi, fx, fy);
  });
  // High 10 planes: u16 samples at bit depth bd
  rc.def("luma_qpel16", [](py::array_t<uint16_t, py::array::c_style | py::array::forcecast> plane, int xi, int yi,
                           int fx, int fy, int bd) {
    VEP_CHECK(plane.ndim() == 2, "2-D plane");
    const int h = int(plane.shape(0)), w = int(plane.shape(1));
    return avc::luma_qpel(plane.data(), w, w, h, xi, yi, fx, fy, bd);
  });
  rc.def("chroma_epel16", [](py::array_t<uint16_t, py::array::c_style | py::array::forcecast> uv, int c, int xi,
                             int yi, int fx, int fy) {
    VEP_CHECK(uv.ndim() == 2 && uv.shape(1) % 2 == 0, "interleaved UV plane");
    const int h = int(uv.shape(0)), pitch = int(uv.shape(1));
    return avc::chroma_epel(uv.data(), pitch, pitch / 2, h, c, xi, yi, fx, fy);
  });
  rc.def("edge_params", [](int qp_p, int qp_q, int off_a, int off_b, int bd) {
    const avc::EdgeParams e = avc::edge_params(qp_p, qp_q, off_a, off_b, bd);
    return py::make_tuple(e.alpha, e.beta, std::vector<int>{e.tc0[0], e.tc0[1], e.tc0[2]});
  }, py::arg("qp_p"), py::arg("qp_q"), py::arg("off_a"), py::arg("off_b"), py::arg("bd") = 8);
  // QPC of Table 8-15 from QPY (QpBdOffsetC: High 10 QPs below 0)
  rc.def("chroma_qp_bd", [](int qpy, int offset, int qpbd_c) { return avc::chroma_qp_bd(qpy, offset, qpbd_c); });
  // one sample line across an edge: p = p0..p3, q = q0..q3 -> filtered (p, q)
  // (unified: filter_samples_u, the one-stream luma / chroma form of the GPU High 10 / 4:2:2 filter)
  rc.def("filter_line", [](std::vector<int> p, std::vector<int> q, int bs, int alpha, int beta, int tc0,
                           bool chroma, int bd, bool unified) {
    VEP_CHECK(p.size() == 4 && q.size() == 4, "4 + 4 samples");
    if (unified) avc::filter_samples_u(p.data(), q.data(), bs, alpha, beta, tc0, chroma, bd);
    else avc::filter_samples(p.data(), q.data(), bs, alpha, beta, tc0, chroma, bd);
    return py::make_tuple(p, q);
  }, py::arg("p"), py::arg("q"), py::arg("bs"), py::arg("alpha"), py::arg("beta"), py::arg("tc0"),
     py::arg("chroma"), py::arg("bd") = 8, py::arg("unified") = false);

  m.def("cavlc_roundtrip", [](int nc, int max_coeff, const std::vector<int>& c) {
    // write_residual_block -> read_residual_block (table self-consistency, tests only)
    VEP_CHECK(int(c.size()) == max_coeff, "coefficient count mismatch");
    BitWriter bw;
    avc::write_residual_block(bw, nc, max_coeff, c.data());
    bw.u1(1);
    bw.align_zero();
    avc::Bits br(bw.buf().data(), bw.buf().size());
    std::vector<int> out(16, 0);
    const int total = avc::read_residual_block(br, nc, max_coeff, out.data());
    out.resize(size_t(max_coeff));
    return py::make_tuple(out, total);
  });
  m.def("avc_source_luma", [](const SynthH264& s) {
    const HostSurface& p = s.source();
    py::array_t<uint8_t> y({p.coded_h, p.coded_w});
    std::memcpy(y.mutable_data(), p.y.data(), p.y.size());
    return y;
  });
  m.def("parse_sps", [](const std::string& nal) {
    std::vector<u8> r(nal.size());
    size_t n = ebsp_to_rbsp(reinterpret_cast<const u8*>(nal.data()), nal.size(), r.data());
    h264::Sps s = h264::parse_sps(r.data(), n);
    py::dict d;
    d["profile_idc"] = s.profile_idc;
    d["level_idc"] = s.level_idc;
    d["width"] = s.width();
    d["height"] = s.height();
    d["coded_width"] = s.coded_width();
    d["coded_height"] = s.coded_height();
    d["fps"] = s.fps();
    d["poc_type"] = s.poc_type;
    d["max_num_ref_frames"] = s.max_num_ref_frames;
    d["chroma_format_idc"] = s.chroma_format_idc;
    d["bit_depth_luma"] = s.bit_depth_luma;
    d["bit_depth_chroma"] = s.bit_depth_chroma;
    return d;
  });
  m.def("parse_hevc_sps", [](const std::string& nal) {
    std::vector<u8> r(nal.size());
    size_t n = ebsp_to_rbsp(reinterpret_cast<const u8*>(nal.data()), nal.size(), r.data());
    hevc::Sps s = hevc::parse_sps(r.data(), n);
    py::dict d;
    d["profile_idc"] = s.ptl.profile_idc;
    d["level_idc"] = s.ptl.level_idc;
    d["width"] = s.out_width();
    d["height"] = s.out_height();
    d["coded_width"] = s.width;
    d["coded_height"] = s.height;
    d["fps"] = s.fps();
    d["ctb_size"] = s.ctb_size();
    d["pcm"] = s.pcm;
    d["num_short_term_rps"] = int(s.st_rps.size());
    d["scaling_list"] = s.scaling_list;
    d["scaling_list_data"] = s.scaling_list_data;
    d["long_term_refs"] = s.long_term_refs;
    d["num_long_term_ref_pics_sps"] = s.num_long_term_ref_pics_sps;
    return d;
  });
  auto hevc_rbsp = [](const std::string& nal) {
    std::vector<u8> r(nal.size());
    r.resize(ebsp_to_rbsp(reinterpret_cast<const u8*>(nal.data()), nal.size(), r.data()));
    return r;
  };
  m.def("parse_hevc_pps", [hevc_rbsp](const std::string& nal) {
    const std::vector<u8> r = hevc_rbsp(nal);
    hevc::Pps p = hevc::parse_pps(r.data(), r.size());
    py::dict d;
    d["tiles"] = p.tiles;
    d["tile_cols"] = p.tile_cols;
    d["tile_rows"] = p.tile_rows;
    d["uniform_spacing"] = p.uniform_spacing;
    d["loop_filter_across_tiles"] = p.loop_filter_across_tiles;
    d["entropy_coding_sync"] = p.entropy_coding_sync;
    d["dependent_slice_segments"] = p.dependent_slice_segments;
    d["weighted_pred"] = p.weighted_pred;
    d["weighted_bipred"] = p.weighted_bipred;
    d["transquant_bypass"] = p.transquant_bypass;
    d["scaling_list"] = p.scaling_list;
    return d;
  });
  // ScalingFactor matrix (raster n x n, n = 4 << size_id) of the default lists, or of the lists an
  // SPS / PPS carries (the PPS ones win, as in decoding).
  m.def("hevc_scaling_factors", [hevc_rbsp](int size_id, int matrix_id, py::object sps_nal, py::object pps_nal) {
    VEP_CHECK(size_id >= 0 && size_id < 4 && matrix_id >= 0 && matrix_id < 6, "bad sizeId / matrixId");
    hevc::ScalingList sl;
    if (!sps_nal.is_none()) {
      const std::vector<u8> r = hevc_rbsp(sps_nal.cast<std::string>());
      sl = hevc::parse_sps(r.data(), r.size()).sl;
    }
    if (!pps_nal.is_none()) {
      const std::vector<u8> r = hevc_rbsp(pps_nal.cast<std::string>());
      hevc::Pps p = hevc::parse_pps(r.data(), r.size());
      if (p.scaling_list) sl = p.sl;
    }
    const int n = 4 << size_id;
    std::vector<u8> f(size_t(n) * n);
    sl.factors(size_id, matrix_id, f.data());
    return std::vector<int>(f.begin(), f.end());
  }, py::arg("size_id"), py::arg("matrix_id"), py::arg("sps_nal") = py::none(), py::arg("pps_nal") = py::none());
  // Slice segment header fields of an escaped slice NAL: entry point offsets and the byte offset
  // of slice_segment_data() within the escaped NAL.
  m.def("hevc_slice_entry_points", [hevc_rbsp](const std::string& nal, const std::string& sps_nal,
                                               const std::string& pps_nal) {
    const std::vector<u8> rs = hevc_rbsp(sps_nal), rp = hevc_rbsp(pps_nal), r = hevc_rbsp(nal);
    const hevc::Sps sps = hevc::parse_sps(rs.data(), rs.size());
    const hevc::Pps pps = hevc::parse_pps(rp.data(), rp.size());
    const hevc::SliceHeader prev;  // (a dependent segment's slice fields are not needed here)
    const hevc::SliceHeader sh = hevc::parse_slice_header(r.data(), r.size(), sps, pps, &prev);
    // RBSP offset -> escaped offset: count the emulation prevention bytes before it
    size_t ebsp = 0, rbsp = 0;
    int zeros = 0;
    const u8* p = reinterpret_cast<const u8*>(nal.data());
    while (rbsp < sh.data_bytepos && ebsp < nal.size()) {
      const u8 b = p[ebsp++];
      if (zeros >= 2 && b == 3) {
        zeros = 0;
        continue;
      }
      ++rbsp;
      zeros = b == 0 ? zeros + 1 : 0;
    }
    py::dict d;
    d["entry_points"] = std::vector<u32>(sh.entry_points.begin(), sh.entry_points.end());
    d["data_offset_ebsp"] = ebsp;
    d["dependent"] = sh.dependent;
    d["segment_address"] = sh.segment_address;
    return d;
  });
  // Record-size statistics of H.264 access units parsed in records mode (the bytes the GPU pulls
  // over PCIe per picture): macroblocks, coefficient-pool entries (sparse groups: mask words +
  // values), non-zero coefficients, motion-vector entries.
  // Sparse coefficient records against the dense blocks they encode: random blocks (any density,
  // int16 extremes, 4x4 and 8x8 transforms, any coded pattern) through store_mb -> expand_coefs
  // (H.264, avc_recon.h) and through hk_sparse_store -> hk_sparse_expand for every H.265 TB size
  // (hevc_kern.h). Returns (H.264 mismatches, H.265 mismatches).
  m.def("sparse_coef_fuzz", [](u64 seed, int trials) {
    u64 x = seed * 0x9E3779B97F4A7C15ull + 1;
    auto rnd = [&]() {
      x ^= x << 13;
      x ^= x >> 7;
      x ^= x << 17;
      return x;
    };
    auto val = [&](int density) -> i16 {  // non-zero with probability density / 16
      if (int(rnd() & 15) >= density) return 0;
      const int r = int(rnd() % 8);
      if (r == 0) return i16(-32768);
      if (r == 1) return i16(32767);
      const int v = int(rnd() % 64) - 32;
      return i16(v ? v : 1);
    };
    int bad_avc = 0, bad_hevc = 0;
    for (int t = 0; t < trials; ++t) {
      const int dens = int(rnd() % 17);
      avc::MbResidual res;
      res.t8 = rnd() & 1;
      i16 want[avc::kDenseCoefs] = {};
      if (res.t8) {
        for (int q = 0; q < 4; ++q) {
          const bool coded = rnd() & 1;
          for (int i = 0; i < 64; ++i) want[64 * q + i] = res.b8[q][i] = coded ? val(dens) : 0;
          if (coded) res.luma |= u16(0x33u << ((q & 1) * 2 + (q >> 1) * 8));
        }
      } else {
        for (int b = 0; b < 16; ++b) {
          const bool coded = rnd() & 1;
          for (int i = 0; i < 16; ++i) want[16 * b + i] = res.blk[b][i] = coded ? val(dens) : 0;
          if (coded) res.luma |= u16(1u << b);
        }
      }
      for (int k = 0; k < 8; ++k) {
        const bool coded = rnd() & 1;
        for (int i = 0; i < 16; ++i) want[256 + 16 * k + i] = res.blk[16 + k][i] = coded ? val(dens) : 0;
        if (coded) res.chroma |= u8(1u << k);
      }
      avc::Picture pic;
      pic.wmbs = pic.hmbs = 1;
      pic.mbs.resize(1);
      avc::MbRec rec{};
      rec.kind = res.t8 ? avc::kI8x8 : avc::kI16x16;
      rec.flags = res.t8 ? u8(avc::kMbT8x8) : u8(0);
      avc::MbState s;
      avc::store_mb(pic, 0, rec, s, &res, nullptr);
      i16 got[avc::kDenseCoefs];
      avc::expand_coefs(pic.coefs.data(), pic.mbs[0], got);
      bad_avc += std::memcmp(got, want, sizeof got) != 0 ||
                 pic.coefs.size() != size_t(avc::coef_words(pic.mbs[0])) + avc::coef_values(pic.coefs.data(), pic.mbs[0]);
      // H.265: one TB per size, positions listed in random order
      for (int log2 = 2; log2 <= 5; ++log2) {
        const int nn = 1 << (2 * log2);
        std::vector<i16> dense(size_t(nn), 0), val_list, out(size_t(nn + nn / 16)), back(static_cast<size_t>(nn));
        std::vector<u16> pos;
        for (int k = 0; k < nn; ++k)
          if ((dense[size_t(k)] = val(dens))) pos.push_back(u16(k));
        for (size_t i = pos.size(); i > 1; --i) std::swap(pos[i - 1], pos[size_t(rnd() % i)]);
        for (u16 k : pos) val_list.push_back(dense[k]);
        const int n = hevc::hk_sparse_store(log2, pos.data(), val_list.data(), int(pos.size()), out.data());
        hevc::hk_sparse_expand(out.data(), log2, back.data());
        bad_hevc += back != dense || n != hevc::hk_sparse_words(log2) + int(pos.size());
      }
    }
    return std::make_pair(bad_avc, bad_hevc);
  });
  // Parse-only timing of an access-unit sequence (the host cost per picture; tools/bench).
  m.def("avc_parse_seconds", [](const std::vector<std::shared_ptr<AccessUnit>>& aus, int reps) {
    py::gil_scoped_release r;
    double best = 1e30;
    for (int k = 0; k < std::max(1, reps); ++k) {
      avc::Decoder dec;
      const i64 t0 = mono_us();
      for (const auto& au : aus) {
        size_t nal = 0;
        do dec.parse(*au, 0, &nal);
        while (nal < au->nals.size());
      }
      best = std::min(best, double(mono_us() - t0) * 1e-6);
    }
    return best;
  }, py::arg("aus"), py::arg("reps") = 3);
  m.def("avc_record_stats", [](const std::vector<std::shared_ptr<AccessUnit>>& aus) {
    py::gil_scoped_release r;
    avc::Decoder dec;
    u64 mbs = 0, coefs = 0, nz = 0, mvs = 0, pics = 0;
    for (const auto& au : aus) {
      auto p = dec.parse(*au);
      if (!p) continue;
      ++pics;
      mbs += p->mbs.size();
      coefs += p->coefs.size();
      mvs += p->mvs.size();
      for (const avc::MbRec& m : p->mbs)
        if (m.kind != avc::kIPcm) nz += avc::coef_values(p->coefs.data(), m);
    }
    py::gil_scoped_acquire g;
    py::dict d;
    d["pictures"] = pics;
    d["mbs"] = mbs;
    d["coefs"] = coefs;
    d["nonzero"] = nz;
    d["mvs"] = mvs;
    return d;
  });
  // Same for H.265 access units (records mode): pictures, transform blocks, coefficient-pool
  // entries (sparse: mask words + stored values per coded block), non-zero entries, prediction
  // blocks.
  m.def("hevc_record_stats", [](const std::vector<std::shared_ptr<AccessUnit>>& aus) {
    py::gil_scoped_release r;
    hevc::Decoder dec;
    dec.set_gpu_mode(true);
    u64 pics = 0, tus = 0, coefs = 0, nz = 0, pus = 0;
    for (const auto& au : aus) {
      dec.decode(*au);
      for (const auto& p : dec.take_gpu_pictures()) {
        ++pics;
        tus += p->tus.size();
        pus += p->pus.size();
        coefs += p->coefs.size();
        for (i16 c : p->coefs) nz += c != 0;
      }
    }
    py::gil_scoped_acquire g;
    py::dict d;
    d["pictures"] = pics;
    d["tus"] = tus;
    d["coefs"] = coefs;
    d["nonzero"] = nz;
    d["pus"] = pus;
    return d;
  });
  // Intra_8x8 tap forms (intra8x8_pred_tap / intra8x8_filter_tap, the GPU kernel's branch-free
  // form) against the direct formulas (intra8x8_pred_g / intra8x8_filter_at) on random samples:
  // every mode but DC, every sample position, every availability combination. Returns the
  // number of mismatching samples.
  m.def("avc_intra8x8_tap_check", [](u64 seed, int trials) {
    u64 st = seed * 0x9E3779B97F4A7C15ull + 7;
    auto rnd = [&]() {
      st ^= st << 13;
      st ^= st >> 7;
      st ^= st << 17;
      return int(st & 255);
    };
    int bad = 0;
    for (int t = 0; t < trials; ++t) {
      int s[25];
      for (int k = 0; k < 25; ++k) s[k] = (t & 3) == 0 ? (rnd() & 1) * 255 : rnd();  // extremes too
      auto T = [&](int i) { return s[1 + i]; };
      auto L = [&](int j) { return j < 0 ? s[0] : s[17 + j]; };
      for (int mode = 0; mode < 9; ++mode) {
        if (mode == 2) continue;
        for (int y = 0; y < 8; ++y)
          for (int x = 0; x < 8; ++x) {
            const u32 tw = avc::intra8x8_pred_tap(mode, x, y);
            const int got = avc::eval_tap8(tw, s[tw & 31], s[(tw >> 5) & 31], s[(tw >> 10) & 31]);
            bad += got != avc::intra8x8_pred_g(T, L, true, true, mode, x, y);
          }
      }
      for (int av = 0; av < 8; ++av) {
        const bool top = av & 1, left = av & 2, tl = av & 4;
        for (int k = 0; k < 25; ++k) {
          const u32 tw = avc::intra8x8_filter_tap(top, left, tl, k);
          const int got =
              (tw & avc::kTap8Const) ? 128 : avc::eval_tap8(tw, s[tw & 31], s[(tw >> 5) & 31], s[(tw >> 10) & 31]);
          bad += got != avc::intra8x8_filter_at(T, [&](int j) { return s[17 + j]; }, top, left, tl, k);
        }
      }
    }
    return bad;
  });
  // Random-bin CABAC engine round trip (context-coded with skewed and flipping statistics,
  // bypass, terminate-0 and a final terminate-1 flush). Returns (ok, coded_bytes).
  m.def("cabac_roundtrip", [](u64 seed, int n, int qp) {
    u64 st = seed * 0x9E3779B97F4A7C15ull + 1;
    auto rnd = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; };
    const size_t nn = static_cast<size_t>(n);
    std::vector<u8> kind(nn), ctx(nn), bin(nn);
    for (int i = 0; i < n; ++i) {
      u64 r = rnd();
      kind[size_t(i)] = u8((r & 15) == 0 ? 1 : ((r & 63) == 1 ? 2 : 0));  // 0 ctx, 1 bypass, 2 term0
      ctx[size_t(i)] = u8((r >> 8) % 4);
      const int p = ctx[size_t(i)] == 0 ? 2 : ctx[size_t(i)] == 1 ? 50 : ctx[size_t(i)] == 2 ? 97 : ((i / 500) & 1) ? 90 : 10;
      bin[size_t(i)] = kind[size_t(i)] == 2 ? 0 : u8(int((r >> 20) % 100) < p);
    }
    std::vector<u8> buf;
    cabac::Ctx ce[4], cd[4];
    const int init[4] = {197, 154, 122, 139};
    for (int k = 0; k < 4; ++k) ce[k].init(init[k], qp), cd[k].init(init[k], qp);
    {
      cabac::Encoder e(buf);
      for (int i = 0; i < n; ++i) {
        if (kind[size_t(i)] == 0) e.decision(ce[ctx[size_t(i)]], bin[size_t(i)]);
        else if (kind[size_t(i)] == 1) e.bypass(bin[size_t(i)]);
        else e.terminate(0);
      }
      e.terminate(1);
      e.align_zero();
    }
    cabac::Decoder d(buf.data(), buf.size(), 0);
    bool ok = true;
    for (int i = 0; i < n && ok; ++i) {
      u32 b;
      if (kind[size_t(i)] == 0) b = d.decision(cd[ctx[size_t(i)]]);
      else if (kind[size_t(i)] == 1) b = d.bypass();
      else b = d.terminate();
      ok = b == bin[size_t(i)];
    }
    ok = ok && d.terminate() == 1 && d.aligned_bytepos() == buf.size();
    return py::make_tuple(ok, buf.size());
  });
  // Host parse cost of one AU (µs, mean over iters) and of its emulation-prevention scan alone.
  m.def("parse_cost_us", [](const AccessUnit& au, int iters, std::shared_ptr<AccessUnit> prime) {
    py::gil_scoped_release r;
    StreamParser p;
    MbUpdate u;
    if (prime) p.absorb_parameter_sets(*prime);
    p.parse(au, u);
    i64 t0 = mono_us();
    for (int k = 0; k < iters; ++k) {
      u.clear_payload();
      p.parse(au, u);
    }
    const double parse_us = double(mono_us() - t0) / iters;
    std::vector<u32> epb;
    t0 = mono_us();
    for (int k = 0; k < iters; ++k)
      for (size_t i = 0; i < au.nals.size(); ++i) find_epb(au.nal(i), au.nal_size(i), epb);
    const double scan_us = double(mono_us() - t0) / iters;
    return std::make_pair(parse_us, scan_us);
  }, py::arg("au"), py::arg("iters") = 100, py::arg("prime") = nullptr);
  m.def("rocdecode_available", [] { return gpu::rocdecode_available(); });
  m.def("cabac_bins_decoded", [] { return cabac::bins_decoded().load(); },
        "CABAC bins decoded by this process so far (H.264 and H.265 slices, counted as each ends)");
  m.def("tsc_now", [] { return u64(__builtin_ia32_rdtsc()); }, "the x86 time-stamp counter");
  m.def("hostprof_start", &hostprof::start, py::arg("interval_us") = 1000,
        "start sampling host CPU time (SIGPROF, every thread of the process)");
  m.def("hostprof_stop", &hostprof::stop, py::arg("path"), "stop sampling; write 'count object offset symbol' lines");
  // VCN backend (vcn.h): which librocdecode is loaded, why none is, load a specific build
  m.def("vcn_library", [] { return vcn::library(); });
  m.def("vcn_load_error", [] { return vcn::load_error(); });
  m.def("vcn_load", [](const std::string& path) { return vcn::load(path); }, py::arg("path"));
  m.def("pinned_pool_stats", [] {
    hostmem::PoolStats st = hostmem::pool_stats();
    py::dict d;
    d["enabled"] = hostmem::pool_enabled();
    d["chunks"] = st.chunks;
    d["bytes_reserved"] = st.bytes_reserved;
    d["blocks_live"] = st.blocks_live;
    d["blocks_reused"] = st.blocks_reused;
    d["fallbacks"] = st.fallbacks;
    return d;
  });
  m.def("hvcc_record", [](const std::string& vps, const std::string& sps, const std::string& pps) {
    auto v = [](const std::string& x) { return std::vector<u8>(x.begin(), x.end()); };
    std::vector<u8> r = hevc::hvcc_record(v(vps), v(sps), v(pps));
    return to_bytes(r.data(), r.size());
  });
  m.def("rbsp_to_ebsp", [](const std::string& r) {
    std::vector<u8> out;
    rbsp_to_ebsp(reinterpret_cast<const u8*>(r.data()), r.size(), out);
    return to_bytes(out.data(), out.size());
  });
  m.def("ebsp_to_rbsp", [](const std::string& e) {
    std::vector<u8> out(e.size());
    size_t n = ebsp_to_rbsp(reinterpret_cast<const u8*>(e.data()), e.size(), out.data());
    return to_bytes(out.data(), n);
  });
  m.def("find_epb", [](const std::string& e) {
    std::vector<u32> out;
    find_epb(reinterpret_cast<const u8*>(e.data()), e.size(), out);
    return out;
  });
  m.def("split_annexb", [](const std::string& b) {
    auto v = h264::split_annexb(reinterpret_cast<const u8*>(b.data()), b.size());
    py::list l;
    for (auto& [o, n] : v) l.append(py::bytes(b.data() + o, n));
    return l;
  });
  m.def("bitwriter_roundtrip", [](const std::vector<u32>& ue_vals, const std::vector<i32>& se_vals) {
    BitWriter bw;
    for (u32 v : ue_vals) bw.ue(v);
    for (i32 v : se_vals) bw.se(v);
    bw.trailing();
    BitReader br(bw.buf().data(), bw.buf().size());
    std::vector<u32> u;
    std::vector<i32> s;
    for (size_t i = 0; i < ue_vals.size(); ++i) u.push_back(br.ue());
    for (size_t i = 0; i < se_vals.size(); ++i) s.push_back(br.se());
    bool at_stop = br.bitpos() == br.stop_bit_pos();
    return py::make_tuple(u, s, at_stop);
  });

  m.def(
      "plan_host_domains",
      [](const std::vector<int>& devices, const std::vector<std::string>& explicit_cpus, int reserve) {
        py::list out;
        for (const HostDomain& d : plan_host_domains(devices, explicit_cpus, reserve)) out.append(domain_dict(d));
        return out;
      },
      py::arg("devices"), py::arg("explicit_cpus") = std::vector<std::string>{}, py::arg("reserve") = 1,
      "Per-worker host domains (hostplan.h): CPUs, NUMA node, parse / io thread counts");
  m.def("affinity_cpus", &affinity_cpus);
  m.def("parse_cpulist", &parse_cpulist);
  m.def("format_cpulist", &format_cpulist);
  m.def("cpu_budget", &cpu_budget);
  py::class_<Worker>(m, "Worker")
      .def(py::init([](int device, int letterbox_size, int chw_dtype, std::vector<float> mean,
                       std::vector<float> stdv, int max_cameras, int pack_threads,
                       int letterbox_format, int lanes, int stages, int queue, bool lane_threads,
                       const std::string& decoder, int kf_window_us, py::object host_domain,
                       bool ref_copies, bool backpressure) {
             WorkerOptions o;
             o.device = device;
             if (!host_domain.is_none()) {
               o.domain = domain_from(host_domain.cast<py::dict>());
               VEP_CHECK(o.domain.device == device, "host_domain belongs to another device");
             }
             if (decoder == "native") o.decoder = kDecoderNative;
             else if (decoder == "vcn") o.decoder = kDecoderVcn;
             else if (decoder == "auto") o.decoder = kDecoderAuto;
             else throw Error("decoder must be native, vcn or auto (got '" + decoder + "')");
             o.lanes = lanes;
             o.stages = stages;
             o.queue = queue;
             o.lane_threads = lane_threads;
             o.kf_window_us = kf_window_us;
             o.ref_copies = ref_copies;
             o.backpressure = backpressure;
             o.pack_threads = pack_threads;
             o.letterbox_format = letterbox_format;
             o.letterbox_size = letterbox_size;
             o.chw_dtype = chw_dtype;
             for (int k = 0; k < 3; ++k) {
               o.mean[k] = mean.size() == 3 ? mean[size_t(k)] : 0.f;
               o.std[k] = stdv.size() == 3 ? stdv[size_t(k)] : 1.f;
             }
             o.max_cameras = max_cameras;
             return std::make_unique<Worker>(o);
           }),
           py::arg("device") = 0, py::arg("letterbox_size") = 0, py::arg("chw_dtype") = 0,
           py::arg("mean") = std::vector<float>{}, py::arg("std") = std::vector<float>{},
           py::arg("max_cameras") = 256, py::arg("pack_threads") = 4,
           py::arg("letterbox_format") = 0, py::arg("lanes") = 0, py::arg("stages") = 0,
           py::arg("queue") = 0, py::arg("lane_threads") = false, py::arg("decoder") = "native",
           py::arg("kf_window_us") = -1, py::arg("host_domain") = py::none(), py::arg("ref_copies") = false,
           py::arg("backpressure") = false)
      .def_property_readonly("ref_copy_bytes", &Worker::ref_copy_bytes)
      .def_property_readonly("kf_window_us", &Worker::kf_window_us)
      .def_property_readonly("host_domain", [](Worker& w) { return domain_dict(w.host_domain()); })
      .def_property_readonly("ingest_parse_threads", &Worker::ingest_parse_threads)
      .def_property_readonly("device", [](Worker& w) { return w.device().id(); })
      .def_property_readonly("decoder", [](Worker& w) { return std::string(w.vcn() ? "vcn" : "native"); })
      .def_property_readonly("lanes", &Worker::lanes)
      .def_property_readonly("stages", &Worker::stages)
      .def_property_readonly("inflight", &Worker::inflight)
      .def_property_readonly("launch_seq", &Worker::launch_seq)
      .def("wait_published", &Worker::wait_published, py::arg("seq"),
           py::call_guard<py::gil_scoped_release>())
      .def("add_camera", &Worker::add_camera, py::arg("name"), py::arg("ring_slots") = 2)
      .def("remove_camera", &Worker::remove_camera, py::call_guard<py::gil_scoped_release>())
      .def("find", [](Worker& w, const std::string& n) { auto c = w.find(n); return c ? c->index() : -1; })
      .def("num_cameras", &Worker::num_cameras)
      .def("start", &Worker::start)
      .def("stop", &Worker::stop, py::call_guard<py::gil_scoped_release>())
      .def("flush", &Worker::flush, py::call_guard<py::gil_scoped_release>())
      .def("complete_all", &Worker::complete_all, py::call_guard<py::gil_scoped_release>())
      .def("set_last_query", [](Worker& w, int i, i64 ms) { cam_of(w, i).last_query_ms.store(ms); })
      .def("last_query", [](Worker& w, int i) { return cam_of(w, i).last_query_ms.load(); })
      .def("set_keyframe_only", [](Worker& w, int i, bool v) { cam_of(w, i).keyframe_only.store(v); })
      .def("keyframe_only", [](Worker& w, int i) { return cam_of(w, i).keyframe_only.load(); })
      .def("set_proxy", [](Worker& w, int i, bool v) { cam_of(w, i).proxy_rtmp.store(v); })
      .def("proxy", [](Worker& w, int i) { return cam_of(w, i).proxy_rtmp.load(); })
      .def("set_idle_cutoff_ms", [](Worker& w, int i, i64 v) { cam_of(w, i).idle_cutoff_ms.store(v); })
      .def("submit_au",
           [](Worker& w, int i, std::shared_ptr<AccessUnit> au) {
             Camera& c = cam_of(w, i);
             py::gil_scoped_release r;
             return c.on_access_unit(au);
           })
      .def("read_surface",
           [](Worker& w, int i) -> py::object {
             HostSurface s;
             i64 pts = 0;
             bool ok;
             {
               py::gil_scoped_release r;
               ok = w.read_surface(i, s, &pts);
             }
             if (!ok) return py::none();
             return py::make_tuple(pts, surface_planes(s));
           },
           py::arg("cam"),
           "(pts, (y, uv)) of the DPB surface holding the camera's newest published picture at full "
           "sample depth (uint16 above 8 bits), coded size; None when none. Call with the camera idle.")
      .def("decode_now",
           [](Worker& w, int i, std::shared_ptr<AccessUnit> au) {
             Camera& c = cam_of(w, i);
             py::gil_scoped_release r;
             DecodeJob job;
             if (!c.make_job(au, job)) return false;
             std::vector<DecodeJob> v;
             v.push_back(std::move(job));
             w.run_batch(v);
             return true;
           })
      .def("decode_many",
           [](Worker& w, const std::vector<std::pair<int, std::vector<std::shared_ptr<AccessUnit>>>>& work,
              bool sync) {
             // one batch: per camera all given AUs (merged into one job, GOP catch-up style)
             std::vector<std::shared_ptr<Camera>> keep;
             for (auto& [idx, aus] : work) keep.push_back(cam_ref(w, idx));
             py::gil_scoped_release r;
             std::vector<DecodeJob> jobs;
             for (size_t k = 0; k < work.size(); ++k) {
               DecodeJob merged;
               bool have = false;
               for (auto& au : work[k].second) {
                 DecodeJob j;
                 if (!keep[k]->make_job(au, j)) continue;
                 if (!have) merged = std::move(j);
                 else merge_job(merged, std::move(j));
                 have = true;
               }
               if (have) jobs.push_back(std::move(merged));
             }
             const size_t n = jobs.size();
             if (sync) w.run_batch(jobs);
             else w.launch_async(jobs);  // published later (launch_seq / wait_published)
             return n;
           },
           py::arg("work"), py::arg("sync") = true)
      .def("avc_profile", [](Worker& w) {
        static const char* kNames[gpu::kAvcProfSlots] = {
            "intra_wait", "intra_load", "intra_luma", "intra_chroma", "intra_store", "intra_mbs",
            "dbk_wait", "dbk_load", "dbk_filter", "dbk_store", "dbk_mbs", "intra_residual",
            "hbd_intra", "hbd_dbk", "hbd_barrier", "hbd_pictures", "hbd_dbk_load", "hbd_dbk_edges",
            "hbd_dbk_store", "hbd_dbk_mbs"};
        const std::vector<u64> v = w.avc_profile();
        py::dict d;
        for (int i = 0; i < gpu::kAvcProfSlots; ++i) d[kNames[i]] = v[size_t(i)];
        return d;
      })
      .def("stats",
           [](Worker& w, int i) {
             Camera& c = cam_of(w, i);
             py::dict d;
             d["packets"] = c.packets.load();
             d["decoded"] = c.decoded.load();
             d["skipped"] = c.skipped.load();
             d["shed"] = c.shed.load();
             d["errors"] = c.errors.load();
             d["bytes_in"] = c.bytes_in.load();
             d["last_packet_ms"] = c.last_packet_ms.load();
             d["decoder"] = c.general_decoder() ? "general" : "fast";
             d["backend"] = c.backend();
             auto ring = c.ring();
             d["published"] = ring ? ring->published() : 0;
             d["width"] = ring ? ring->width() : 0;
             d["height"] = ring ? ring->height() : 0;
             d["ring_slots"] = ring ? ring->slots() : c.ring_slots_cfg;
             py::list hist;
             for (auto& h : c.lat_hist) hist.append(h.load());
             d["latency_hist"] = hist;
             d["latency_sum_ms"] = c.lat_sum_ms.load();
             py::list bounds;
             for (double b : Camera::kLatBucketsMs) bounds.append(b);
             d["latency_bounds_ms"] = bounds;
             return d;
           })
      .def("log", [](Worker& w, int i, bool err, const std::string& line) { cam_of(w, i).logs.add(err, line); })
      .def("logs", [](Worker& w, int i, bool err, int last) { return cam_of(w, i).logs.dump(err, size_t(last)); },
           py::arg("idx"), py::arg("err") = false, py::arg("last") = 100)
      .def("read_latest",
           [](Worker& w, int i, i64 after) -> py::object {
             std::shared_ptr<FrameRing> ring = cam_of(w, i).ring();
             if (!ring) return py::none();
             size_t n = ring->slot_bytes();
             py::array_t<uint8_t> out({ring->height(), ring->width(), 3});
             FrameMeta m;
             bool ok;
             u8* dst = out.mutable_data();
             {
               py::gil_scoped_release r;
               ok = w.read_latest(*ring, after, &m, dst, n);
             }
             if (!ok) return py::none();
             return py::make_tuple(meta_dict(m), out);
           },
           py::arg("idx"), py::arg("after") = 0)
      .def("video_frame_bound",
           // Upper bound of the serialized VideoFrame of this camera's current ring (0: no ring).
           [](Worker& w, int i, const std::string& device_id) -> size_t {
             std::shared_ptr<FrameRing> ring = cam_of(w, i).ring();
             if (!ring) return 0;
             FrameMeta probe{};
             probe.width = ring->width();
             probe.height = ring->height();
             return encode_video_frame(probe, ring->slot_bytes(), device_id).first.size() +
                    ring->slot_bytes() + video_frame_suffix_max(device_id);
           },
           py::arg("idx"), py::arg("device_id") = "")
      .def("video_frame_into",
           // The serialized VideoFrame written into caller memory at `addr` (e.g. a shared-memory
           // segment the front-end process maps): (seq, length, meta), None if no newer frame, or
           // the needed size (int) if `cap` is too small. pinned: the range is register_host()ed,
           // so the pixels arrive by one DMA with no staging copy.
           [](Worker& w, int i, i64 after, const std::string& device_id, uintptr_t addr, size_t cap,
              bool pinned) -> py::object {
             std::shared_ptr<Camera> cp = cam_ref(w, i);
             std::shared_ptr<FrameRing> ring = cp->ring();
             if (!ring) return py::none();
             const size_t n = ring->slot_bytes();
             FrameMeta probe;
             int slot;
             if (!ring->latest(after, &probe, &slot)) return py::none();
             const std::string pre = encode_video_frame(probe, n, device_id).first;
             const size_t need = pre.size() + n + video_frame_suffix_max(device_id);
             if (cap < need) return py::int_(need);
             char* buf = reinterpret_cast<char*>(addr);
             std::memcpy(buf, pre.data(), pre.size());
             FrameMeta m;
             bool ok;
             {
               py::gil_scoped_release r;
               ok = w.read_latest(*ring, after, &m, reinterpret_cast<u8*>(buf) + pre.size(), n, pinned);
             }
             if (!ok) return py::none();
             auto [pre2, suf] = encode_video_frame(m, n, device_id);
             VEP_CHECK(pre2 == pre && suf.size() <= video_frame_suffix_max(device_id),
                       "VideoFrame header changed while serving");
             std::memcpy(buf + pre.size() + n, suf.data(), suf.size());
             return py::make_tuple(m.seq, pre.size() + n + suf.size(), meta_dict(m));
           },
           py::arg("idx"), py::arg("after"), py::arg("device_id"), py::arg("addr"), py::arg("cap"),
           py::arg("pinned") = false)
      .def("register_host",
           [](Worker& w, uintptr_t addr, size_t n) { return w.register_host(reinterpret_cast<void*>(addr), n); })
      .def("unregister_host", [](Worker& w, uintptr_t addr) { w.unregister_host(reinterpret_cast<void*>(addr)); })
      .def("video_frame",
           // Serialized VideoFrame proto, built in place in its final bytes object: header, the
           // slot's pixels (D2H through a pinned pool buffer, GIL released), trailer; the object
           // is then shrunk to the exact length (no second copy of the frame).
           [](Worker& w, int i, i64 after, const std::string& device_id) -> py::object {
             Camera& c = cam_of(w, i);
             std::shared_ptr<FrameRing> ring = c.ring();
             if (!ring) return py::none();
             const size_t n = ring->slot_bytes();
             FrameMeta probe;
             int slot;
             if (!ring->latest(after, &probe, &slot)) return py::none();
             // the prefix holds width, height and the data length: fixed for this ring
             const std::string pre = encode_video_frame(probe, n, device_id).first;
             const size_t suf_max = video_frame_suffix_max(device_id);
             PyObject* b = PyBytes_FromStringAndSize(nullptr, Py_ssize_t(pre.size() + n + suf_max));
             if (!b) throw py::error_already_set();
             char* buf = PyBytes_AS_STRING(b);
             std::memcpy(buf, pre.data(), pre.size());
             FrameMeta m;
             bool ok;
             {
               py::gil_scoped_release r;
               try {
                 ok = w.read_latest(*ring, after, &m, reinterpret_cast<u8*>(buf) + pre.size(), n);
               } catch (...) {
                 py::gil_scoped_acquire a;
                 Py_DECREF(b);
                 throw;
               }
             }
             if (!ok) {
               Py_DECREF(b);
               return py::none();
             }
             auto [pre2, suf] = encode_video_frame(m, n, device_id);
             VEP_CHECK(pre2 == pre && suf.size() <= suf_max, "VideoFrame header changed while serving");
             std::memcpy(buf + pre.size() + n, suf.data(), suf.size());
             if (_PyBytes_Resize(&b, Py_ssize_t(pre.size() + n + suf.size())) != 0) throw py::error_already_set();
             py::object res = py::reinterpret_steal<py::object>(b);
             return py::make_tuple(m.seq, res, meta_dict(m));
           },
           py::arg("idx"), py::arg("after") = 0, py::arg("device_id") = "")
      .def("set_consumer_buffers",
           [](Worker& w, uintptr_t hwc, uintptr_t chw, int rows) {
             w.set_consumer_buffers(reinterpret_cast<u8*>(hwc), reinterpret_cast<void*>(chw), rows);
           })
      .def("snapshot_consumer",
           // Consistent copy of consumer rows [0, rows) into dst (device pointer on a GPU worker),
           // enqueued on `stream` (a hipStream_t as int, e.g. torch.cuda.current_stream().cuda_stream;
           // 0 = wait on the host): after every letterbox write already enqueued, before any later.
           [](Worker& w, uintptr_t dst, size_t cap, int rows, uintptr_t stream) {
             py::gil_scoped_release nogil;
             return w.snapshot_consumer(reinterpret_cast<void*>(dst), cap, rows, reinterpret_cast<hipStream_t>(stream));
           },
           py::arg("dst"), py::arg("cap"), py::arg("rows"), py::arg("stream") = 0)
      .def_property_readonly("snapshots", &Worker::snapshots)
      .def("wait_frame",
           // Block (GIL released) until the camera publishes a frame with seq > after.
           [](Worker& w, int i, i64 after, int timeout_ms) {
             std::shared_ptr<Camera> cp = cam_ref(w, i);
             Camera& c = *cp;
             py::gil_scoped_release r;
             const i64 deadline = mono_us() + i64(timeout_ms) * 1000;
             std::shared_ptr<FrameRing> ring;
             while (!(ring = c.ring())) {  // ring appears with the first decoded frame
               if (mono_us() >= deadline) return false;
               std::this_thread::sleep_for(std::chrono::milliseconds(2));
             }
             int left = int(std::max<i64>(0, (deadline - mono_us()) / 1000));
             return ring->wait_newer(after, left);
           },
           py::arg("idx"), py::arg("after"), py::arg("timeout_ms"))
      .def("published", [](Worker& w, int i) {
        auto ring = cam_of(w, i).ring();
        return ring ? ring->published() : i64(0);
      })
      .def("consumer_hwc_ptr", [](Worker& w) { return reinterpret_cast<uintptr_t>(w.consumer_hwc()); })
      .def("consumer_chw_ptr", [](Worker& w) { return reinterpret_cast<uintptr_t>(w.consumer_chw()); })
      .def("ring_slot_ptr", [](Worker& w, int i, int s) {
        auto ring = cam_of(w, i).ring();
        if (!ring) return uintptr_t(0);
        return reinterpret_cast<uintptr_t>(ring->slot_ptr(s));
      })
      .def("latest_slot", [](Worker& w, int i) -> py::object {
        auto ring = cam_of(w, i).ring();
        FrameMeta m;
        int slot;
        if (!ring || !ring->latest(0, &m, &slot)) return py::none();
        return py::make_tuple(slot, meta_dict(m));
      })
      .def("timings",
           [](Worker& w) {
             py::dict d;
             d["prepare_ms"] = w.timers.prepare / 1000.0;
             d["index_ms"] = w.timers.index / 1000.0;
             d["copy_ms"] = w.timers.copy / 1000.0;
             d["enqueue_ms"] = w.timers.enqueue / 1000.0;
             d["wait_ms"] = w.timers.wait / 1000.0;
             return d;
           })
      .def_property_readonly("batches", &Worker::batches)
      .def_property_readonly("frames", &Worker::frames)
      .def_property_readonly("dropped", &Worker::dropped)
      .def_property_readonly("shed", &Worker::shed)
      .def_property_readonly("merged", &Worker::merged)
      .def("hold_lanes", &Worker::hold_lanes, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("pictures", &Worker::pictures)
      .def_property_readonly("gpu_ms_total", &Worker::gpu_ms_total)
      .def_property_readonly("bytes_inplace", &Worker::bytes_inplace)
      .def_property_readonly("records_gathered", &Worker::records_gathered)
      .def_property_readonly("direct_reads", &Worker::direct_reads)
      .def_property_readonly("bytes_staged", &Worker::bytes_staged)
      .def("compute_stream_ptr", [](Worker& w) { return reinterpret_cast<uintptr_t>(w.compute_stream()); });

  py::class_<ReplayBench>(m, "ReplayBench")
      .def(py::init([](Worker& w, int ncams, const SynthConfig& cfg, int cached, int threads,
                       int ring_slots, const std::string& prefix, int window, bool records) {
             py::gil_scoped_release r;
             return std::make_unique<ReplayBench>(w, ncams, cfg, cached, threads, ring_slots, prefix,
                                                  window, records);
           }),
           py::arg("worker"), py::arg("ncams"), py::arg("cfg"), py::arg("cached_frames") = 30,
           py::arg("threads") = 8, py::arg("ring_slots") = 2, py::arg("prefix") = "cam",
           py::arg("window") = 2, py::arg("records") = false, py::keep_alive<1, 2>())
      .def("step", &ReplayBench::step, py::call_guard<py::gil_scoped_release>())
      .def("parse_only_ms", &ReplayBench::parse_only_ms, py::call_guard<py::gil_scoped_release>())
      .def("drain", &ReplayBench::drain, py::call_guard<py::gil_scoped_release>())
      .def("quiesce", &ReplayBench::quiesce, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("parse_failures", &ReplayBench::parse_failures)
      .def_property_readonly("frames", &ReplayBench::frames)
      .def_property_readonly("payload_bytes", &ReplayBench::bitstream_bytes)
      .def_property_readonly("stream_bytes", &ReplayBench::stream_bytes)
      .def_property_readonly("stream_frames", &ReplayBench::stream_frames)
      .def_property_readonly("parse_ms", &ReplayBench::parse_ms)
      .def_property_readonly("parse_wait_ms", &ReplayBench::parse_wait_ms)
      .def_property_readonly("batch_ms", &ReplayBench::batch_ms)
      .def_property_readonly("cameras", &ReplayBench::cameras);

  // CPU reference of the colour conversion (coded NV12 planes -> cropped BGR24).
  m.def("nv12_to_bgr_cpu", [](py::array_t<uint8_t, py::array::c_style> y, py::array_t<uint8_t, py::array::c_style> uv,
                              int crop_left, int crop_top, int width, int height) {
    VEP_CHECK(y.ndim() == 2 && uv.ndim() == 2 && uv.shape(0) * 2 == y.shape(0) && uv.shape(1) == y.shape(1),
              "nv12_to_bgr_cpu: Y (H, W) and UV (H / 2, W) planes expected");
    VEP_CHECK(crop_left + width <= y.shape(1) && crop_top + height <= y.shape(0), "crop window outside the planes");
    HostSurface s;
    s.coded_w = int(y.shape(1));
    s.coded_h = int(y.shape(0));
    s.y.assign(y.data(), y.data() + y.size());
    s.uv.assign(uv.data(), uv.data() + uv.size());
    py::array_t<uint8_t> o({height, width, 3});
    cpu_nv12_to_bgr(s, crop_left, crop_top, width, height, o.mutable_data());
    return o;
  });

  // ---- op API on caller-owned device buffers (torch tensors pass data_ptr / stream) ----
  m.def("nv12_to_bgr",
        [](uintptr_t y, uintptr_t uv, uintptr_t mask, uintptr_t prefix, uintptr_t offsets,
           uintptr_t payload, int wmbs, int hmbs, int out_w, int out_h, int crop_left,
           int crop_top, uintptr_t out, uintptr_t stream) {
          gpu::DecodeDesc d{};
          d.y = reinterpret_cast<u8*>(y);
          d.uv = reinterpret_cast<u8*>(uv);
          d.mask = reinterpret_cast<const u32*>(mask);
          d.prefix = reinterpret_cast<const u32*>(prefix);
          d.offsets = reinterpret_cast<const u32*>(offsets);
          d.payload = reinterpret_cast<const u8*>(payload);
          d.bgr = reinterpret_cast<u8*>(out);
          d.wmbs = wmbs;
          d.hmbs = hmbs;
          d.out_w = out_w;
          d.out_h = out_h;
          d.crop_left = crop_left;
          d.crop_top = crop_top;
          d.tiles_x = (wmbs + gpu::kTileMbW - 1) / gpu::kTileMbW;
          d.tile_begin = 0;
          gpu::launch_decode_convert_one(d, reinterpret_cast<hipStream_t>(stream));
        });
  m.def("letterbox",
        [](uintptr_t y, uintptr_t uv, int pitch, int src_w, int src_h, int crop_left, int crop_top,
           int size, uintptr_t out_hwc, uintptr_t out_chw, int chw_dtype, std::vector<float> mean,
           std::vector<float> stdv, int pad, uintptr_t stream, int format) {
          gpu::LetterboxDesc d{};
          d.y = reinterpret_cast<const u8*>(y);
          d.uv = reinterpret_cast<const u8*>(uv);
          d.pitch = pitch;
          d.src_w = src_w;
          d.src_h = src_h;
          d.crop_left = crop_left;
          d.crop_top = crop_top;
          d.out_hwc = reinterpret_cast<u8*>(out_hwc);
          d.out_chw = reinterpret_cast<void*>(out_chw);
          gpu::fill_letterbox_geometry(d, size, format == gpu::kLbNV12);
          gpu::LetterboxParams p{};
          p.format = format;
          p.size = size;
          p.chw_dtype = chw_dtype;
          for (int k = 0; k < 3; ++k) {
            p.mean[k] = mean.size() == 3 ? mean[size_t(k)] : 0.f;
            p.inv_std[k] = 1.f / (stdv.size() == 3 ? stdv[size_t(k)] : 1.f);
          }
          p.pad_value = u8(pad);
          gpu::launch_letterbox_one(d, p, reinterpret_cast<hipStream_t>(stream));
        },
        py::arg("y"), py::arg("uv"), py::arg("pitch"), py::arg("src_w"), py::arg("src_h"),
        py::arg("crop_left"), py::arg("crop_top"), py::arg("size"), py::arg("out_hwc"),
        py::arg("out_chw"), py::arg("chw_dtype"), py::arg("mean"), py::arg("std"), py::arg("pad"),
        py::arg("stream"), py::arg("format") = 0);
  m.def("nv12_to_chw",
        [](uintptr_t in, uintptr_t out, int n, int size, int chw_dtype, std::vector<float> mean,
           std::vector<float> stdv, uintptr_t stream) {
          float m3[3], is3[3];
          for (int k = 0; k < 3; ++k) {
            m3[k] = mean.size() == 3 ? mean[size_t(k)] : 0.f;
            is3[k] = 1.f / (stdv.size() == 3 ? stdv[size_t(k)] : 1.f);
          }
          gpu::launch_nv12_to_chw(reinterpret_cast<const u8*>(in), reinterpret_cast<void*>(out), n,
                                  size, chw_dtype, m3, is3, reinterpret_cast<hipStream_t>(stream));
        });
  m.def("letterbox_geometry", [](int src_w, int src_h, int size, bool even) {
    gpu::LetterboxDesc d{};
    d.src_w = src_w;
    d.src_h = src_h;
    gpu::fill_letterbox_geometry(d, size, even);
    return py::make_tuple(d.nw, d.nh, d.pad_x, d.pad_y);
  }, py::arg("src_w"), py::arg("src_h"), py::arg("size"), py::arg("even") = false);

  bind_net(m);
  bind_mux(m);
  bind_hevc(m);
  bind_bus(m);
  bind_rpc(m);
}
