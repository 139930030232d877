// Bindings: RTP/RTSP layer, ingest sessions.
#include <pybind11/functional.h>
#include <pybind11/stl.h>

#include "bind_ext.h"
#include "vep/ingest.h"
#include "vep/net.h"

namespace py = pybind11;
using namespace vep;

static py::bytes B(const std::vector<u8>& v) {
  return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
}

static py::dict state_dict(const SessionState& s) {
  py::dict d;
  d["status"] = s.status;
  d["running"] = s.running;
  d["restarting"] = s.restarting;
  d["dead"] = s.dead;
  d["paused"] = s.paused;
  d["oomkilled"] = s.oomkilled;
  d["pid"] = s.pid;
  d["exit_code"] = s.exit_code;
  d["error"] = s.error;
  d["started_at_ms"] = s.started_at_ms;
  d["finished_at_ms"] = s.finished_at_ms;
  d["restart_count"] = s.restart_count;
  d["failing_streak"] = s.failing_streak;
  d["health"] = s.health;
  d["aus"] = s.aus;
  d["bytes"] = s.bytes;
  d["lost"] = s.lost;
  d["rtmp_messages"] = s.rtmp_messages;
  d["rtmp_error"] = s.rtmp_error;
  d["fps"] = s.fps;
  return d;
}

void bind_net(py::module_& m) {
  py::enum_<net::Fault>(m, "Fault")
      .value("NONE", net::Fault::kNone)
      .value("DROP_CONNECTION", net::Fault::kDropConnection)
      .value("STALL", net::Fault::kStall)
      .value("CORRUPT_NAL", net::Fault::kCorruptNal)
      .value("SKIP_KEYFRAME", net::Fault::kSkipKeyframe)
      .value("REFUSE", net::Fault::kRefuse);

  m.def("packetize_nal",
        [](const std::string& nal, int codec, size_t mtu) {
          std::vector<std::vector<u8>> out;
          net::packetize_nal(Codec(codec), reinterpret_cast<const u8*>(nal.data()), nal.size(), mtu, out);
          py::list l;
          for (auto& p : out) l.append(B(p));
          return l;
        },
        py::arg("nal"), py::arg("codec") = 0, py::arg("mtu") = 1400);
  m.def("aggregate_nals", [](const std::vector<std::string>& nals, int codec) {
    std::vector<std::vector<u8>> v;
    for (auto& n : nals) v.emplace_back(n.begin(), n.end());
    return B(net::aggregate_nals(Codec(codec), v));
  }, py::arg("nals"), py::arg("codec") = 0);
  m.def("rtp_packet", [](const std::string& payload, int seq, u32 ts, bool marker, int pt, u32 ssrc) {
    std::vector<u8> o(net::kRtpHeader + payload.size());
    net::RtpHeader h;
    h.seq = u16(seq);
    h.ts = ts;
    h.marker = marker;
    h.pt = u8(pt);
    h.ssrc = ssrc;
    net::write_rtp_header(o.data(), h);
    std::memcpy(o.data() + net::kRtpHeader, payload.data(), payload.size());
    return B(o);
  }, py::arg("payload"), py::arg("seq"), py::arg("ts"), py::arg("marker") = false,
     py::arg("pt") = 96, py::arg("ssrc") = 1);
  m.def("base64_encode", [](const std::string& s) {
    return net::base64_encode(reinterpret_cast<const u8*>(s.data()), s.size());
  });
  m.def("base64_decode", [](const std::string& s) { return B(net::base64_decode(s)); });
  m.def("parse_url", [](const std::string& s) {
    net::Url u = net::parse_url(s);
    py::dict d;
    d["scheme"] = u.scheme;
    d["user"] = u.user;
    d["password"] = u.pass;
    d["host"] = u.host;
    d["port"] = u.port;
    d["path"] = u.path;
    return d;
  });

  py::class_<net::Depacketizer>(m, "Depacketizer")
      .def(py::init([](int codec) { return std::make_unique<net::Depacketizer>(Codec(codec)); }),
           py::arg("codec") = 0)
      .def("push",
           [](net::Depacketizer& d, const std::string& pkt) {
             net::RtpHeader h;
             const u8* pl;
             size_t n;
             if (!net::parse_rtp(reinterpret_cast<const u8*>(pkt.data()), pkt.size(), h, &pl, &n))
               throw Error("malformed RTP packet");
             std::vector<AuPtr> out;
             d.push(h, pl, n, out);
             std::vector<std::shared_ptr<AccessUnit>> r;
             for (auto& a : out) r.push_back(std::const_pointer_cast<AccessUnit>(a));
             return r;
           })
      .def("flush", [](net::Depacketizer& d) {
        std::vector<AuPtr> out;
        d.flush(out);
        std::vector<std::shared_ptr<AccessUnit>> r;
        for (auto& a : out) r.push_back(std::const_pointer_cast<AccessUnit>(a));
        return r;
      })
      .def_property_readonly("lost", &net::Depacketizer::lost)
      .def_property_readonly("aus", &net::Depacketizer::aus);

  py::class_<net::RtspServer>(m, "RtspServer")
      .def(py::init<const std::string&, int>(), py::arg("bind") = "127.0.0.1", py::arg("port") = 0)
      .def("add_stream",
           [](net::RtspServer& s, const std::string& path, const SynthConfig& cfg, bool realtime,
              int cached_frames, const std::string& user, const std::string& pass) {
             net::ServedStream st;
             st.cfg = cfg;
             st.realtime = realtime;
             st.cached_frames = cached_frames;
             st.user = user;
             st.pass = pass;
             py::gil_scoped_release r;
             s.add_stream(path, st);
           },
           py::arg("path"), py::arg("cfg"), py::arg("realtime") = true, py::arg("cached_frames") = 0,
           py::arg("user") = "", py::arg("password") = "")
      .def("start", &net::RtspServer::start)
      .def("stop", &net::RtspServer::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &net::RtspServer::port)
      .def("inject", &net::RtspServer::inject)
      .def("set_pacing", &net::RtspServer::set_pacing, py::arg("mode"))
      .def_property_readonly("sessions", &net::RtspServer::sessions)
      .def_property_readonly("aus_sent", &net::RtspServer::aus_sent);

  py::class_<net::RtspClient>(m, "RtspClient")
      .def(py::init([](const std::string& url, int timeout_ms) {
             net::RtspClientOptions o;
             o.timeout_ms = timeout_ms;
             return std::make_unique<net::RtspClient>(url, o);
           }),
           py::arg("url"), py::arg("timeout_ms") = 5000)
      .def("open",
           [](net::RtspClient& c) {
             net::RtspStreamInfo i;
             {
               py::gil_scoped_release r;
               i = c.open();
             }
             py::dict d;
             d["codec"] = i.codec == Codec::kH264 ? "h264" : "h265";
             d["payload_type"] = i.payload_type;
             d["clock_rate"] = i.clock_rate;
             py::list ps;
             for (auto& p : i.param_sets) ps.append(B(p));
             d["param_sets"] = ps;
             d["control"] = i.control;
             d["framerate"] = i.framerate;
             d["sdp"] = i.sdp;
             return d;
           })
      .def("read",
           // Collect up to n access units (or until the stream ends / timeout_s elapses).
           [](net::RtspClient& c, int n, double timeout_s) {
             std::vector<std::shared_ptr<AccessUnit>> got;
             std::atomic<bool> stop{false};
             std::string why;
             {
               py::gil_scoped_release r;
               const i64 deadline = mono_us() + i64(timeout_s * 1e6);
               std::thread watchdog([&] {
                 while (!stop.load() && mono_us() < deadline)
                   std::this_thread::sleep_for(std::chrono::milliseconds(10));
                 stop = true;
               });
               why = c.run([&](const AuPtr& a) {
                 if (int(got.size()) < n) got.push_back(std::const_pointer_cast<AccessUnit>(a));
                 if (int(got.size()) >= n) stop = true;
               }, stop);
               stop = true;
               watchdog.join();
             }
             return py::make_tuple(got, why);
           },
           py::arg("n"), py::arg("timeout_s") = 10.0)
      .def("close", &net::RtspClient::close)
      .def_property_readonly("bytes", &net::RtspClient::bytes)
      .def_property_readonly("lost", &net::RtspClient::lost);

  py::class_<IngestSession>(m, "IngestSession")
      .def(py::init([](Worker& w, int cam, const std::string& name, const std::string& rtsp,
                       const std::string& rtmp, const std::string& disk,
                       std::shared_ptr<mux::Archiver> arch, int timeout_ms, int reconnect_ms,
                       int max_backoff_ms, bool lossless) {
             IngestConfig c;
             c.lossless = lossless;
             c.name = name;
             c.rtsp_url = rtsp;
             c.rtmp_url = rtmp;
             c.disk_path = disk;
             c.timeout_ms = timeout_ms;
             c.reconnect_delay_ms = reconnect_ms;
             c.max_backoff_ms = max_backoff_ms;
             return std::make_unique<IngestSession>(w, cam, c, arch);
           }),
           py::arg("worker"), py::arg("cam"), py::arg("name"), py::arg("rtsp_url"),
           py::arg("rtmp_url") = "", py::arg("disk_path") = "", py::arg("archiver") = nullptr,
           py::arg("timeout_ms") = 5000, py::arg("reconnect_delay_ms") = 1000,
           py::arg("max_backoff_ms") = 30000, py::arg("lossless") = false, py::keep_alive<1, 2>())
      .def("start", &IngestSession::start)
      .def("stop", &IngestSession::stop, py::call_guard<py::gil_scoped_release>())
      .def("state", [](IngestSession& s) { return state_dict(s.state()); })
      .def("set_lossless", &IngestSession::set_lossless)
      .def_property_readonly("lossless", &IngestSession::lossless)
      .def("log", &IngestSession::log);
}
