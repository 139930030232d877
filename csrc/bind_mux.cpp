// Bindings: FLV / RTMP / MP4 muxers and the archiver.
#include <pybind11/stl.h>

#include "bind_ext.h"
#include "vep/mux.h"

namespace py = pybind11;
using namespace vep;

static py::bytes B(const std::vector<u8>& v) {
  return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
}
static std::vector<u8> V(const std::string& s) { return std::vector<u8>(s.begin(), s.end()); }
static std::vector<AuPtr> aus_of(const std::vector<std::shared_ptr<AccessUnit>>& v) {
  return std::vector<AuPtr>(v.begin(), v.end());
}

static ParamSets PS(int codec, const std::string& vps, const std::string& sps,
                    const std::string& pps) {
  ParamSets p;
  p.codec = Codec(codec);
  p.vps = V(vps);
  p.sps = V(sps);
  p.pps = V(pps);
  return p;
}

void bind_mux(py::module_& m) {
  m.def("au_to_avcc", [](const AccessUnit& a) { return B(mux::au_to_avcc(a)); });
  m.def("flv_file_header", [] { return B(mux::flv_file_header()); });
  m.def(
      "flv_sequence_header",
      [](const std::string& sps, const std::string& pps, const std::string& vps, int codec) {
        return B(mux::flv_sequence_header(PS(codec, vps, sps, pps)));
      },
      py::arg("sps"), py::arg("pps"), py::arg("vps") = "", py::arg("codec") = 0);
  m.def("flv_video_body", [](const AccessUnit& a) { return B(mux::flv_video(a)); });
  m.def("flv_tag", [](int type, u32 ts, const std::string& body) {
    return B(mux::flv_tag(u8(type), ts, V(body)));
  });
  m.def(
      "build_mp4",
      [](const std::vector<std::shared_ptr<AccessUnit>>& aus, int w, int h, const std::string& sps,
         const std::string& pps, const std::string& vps, int codec) {
        mux::Mp4Info i;
        i.width = w;
        i.height = h;
        i.ps = PS(codec, vps, sps, pps);
        return B(mux::build_mp4(aus_of(aus), i));
      },
      py::arg("aus"), py::arg("width"), py::arg("height"), py::arg("sps"), py::arg("pps"),
      py::arg("vps") = "", py::arg("codec") = 0);
  m.def("segment_duration_ms", [](const std::vector<std::shared_ptr<AccessUnit>>& aus) {
    return mux::segment_duration_ms(aus_of(aus));
  });

  py::class_<mux::RtmpPublisher>(m, "RtmpPublisher")
      .def(py::init<std::string, int>(), py::arg("url"), py::arg("timeout_ms") = 5000)
      .def("connect", &mux::RtmpPublisher::connect, py::call_guard<py::gil_scoped_release>())
      .def(
          "send_sequence_header",
          [](mux::RtmpPublisher& p, const std::string& sps, const std::string& pps,
             const std::string& vps, int codec) { p.send_sequence_header(PS(codec, vps, sps, pps)); },
          py::arg("sps"), py::arg("pps"), py::arg("vps") = "", py::arg("codec") = 0)
      .def("send_au", &mux::RtmpPublisher::send_au, py::call_guard<py::gil_scoped_release>())
      .def("close", &mux::RtmpPublisher::close)
      .def_property_readonly("connected", &mux::RtmpPublisher::connected)
      .def_property_readonly("messages", &mux::RtmpPublisher::messages)
      .def_property_readonly("bytes_sent", &mux::RtmpPublisher::bytes_sent);

  py::class_<mux::RtmpSink>(m, "RtmpSink")
      .def(py::init<const std::string&, int>(), py::arg("bind") = "127.0.0.1", py::arg("port") = 0)
      .def("start", &mux::RtmpSink::start)
      .def("stop", &mux::RtmpSink::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &mux::RtmpSink::port)
      .def_property_readonly("video_messages", &mux::RtmpSink::video_messages)
      .def_property_readonly("keyframes", &mux::RtmpSink::keyframes)
      .def_property_readonly("hevc_messages", &mux::RtmpSink::hevc_messages)
      .def_property_readonly("sequence_headers", &mux::RtmpSink::sequence_headers)
      .def_property_readonly("stream_key", &mux::RtmpSink::last_stream_key)
      .def_property_readonly("video_bytes", &mux::RtmpSink::video_bytes)
      .def("set_keep_bodies", &mux::RtmpSink::set_keep_bodies)
      .def("video_bodies", [](const mux::RtmpSink& s) {
        py::list l;
        for (auto& b : s.video_bodies()) l.append(B(b));
        return l;
      });

  py::class_<mux::Archiver, std::shared_ptr<mux::Archiver>>(m, "Archiver")
      .def(py::init<>())
      .def("flush", &mux::Archiver::flush, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("written", &mux::Archiver::written)
      .def_property_readonly("failed", &mux::Archiver::failed)
      .def_property_readonly("last_path", &mux::Archiver::last_path);
}
