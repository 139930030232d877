// Python bindings of the native gRPC endpoint (csrc/vep/rpcsrv.h): the serving processes run it
// on the public port; its non-frame methods call back into Python (the forwarding to the hub).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "bind_ext.h"
#include "vep/h2load.h"
#include "vep/rpcsrv.h"

namespace py = pybind11;
using namespace vep;

namespace {
// The server joins threads that may be waiting for the GIL (the Python callback): it is always
// destroyed with the GIL released.
struct ServerDeleter {
  void operator()(rpc::Server* s) const {
    py::gil_scoped_release g;
    delete s;
  }
};
}  // namespace

void bind_rpc(py::module_& m) {
  py::class_<rpc::Server, std::unique_ptr<rpc::Server, ServerDeleter>>(m, "RpcServer")
      .def(py::init([](const std::string& host, int port, const std::string& bus_tag, int io_threads,
                       int wait_threads, int slow_threads, py::object handler, bool reuseport,
                       int stream_deadline_ms, u32 max_streams, u32 max_queued_requests,
                       u32 max_resets_per_s, bool zero_copy) {
             rpc::ServerOptions o;
             o.host = host;
             o.port = port;
             o.bus_tag = bus_tag;
             o.io_threads = io_threads;
             o.wait_threads = wait_threads;
             o.slow_threads = slow_threads;
             o.reuseport = reuseport;
             o.stream_deadline_ms = stream_deadline_ms;
             o.max_streams = max_streams;
             o.max_queued_requests = max_queued_requests;
             o.max_resets_per_s = max_resets_per_s;
             o.zero_copy = zero_copy;
             rpc::SlowHandler h;
             if (!handler.is_none()) {
               // (the callable is released with the GIL held, whichever thread drops it last)
               auto fn = std::shared_ptr<py::object>(new py::object(handler), [](py::object* p) {
                 py::gil_scoped_acquire g;
                 delete p;
               });
               h = [fn](const std::string& method, const std::string& req, const std::string& peer) {
                 py::gil_scoped_acquire g;
                 rpc::Reply r;
                 py::tuple t = (*fn)(method, py::bytes(req), peer).cast<py::tuple>();
                 r.status = t[0].cast<int>();
                 r.message = t[1].cast<std::string>();
                 for (auto x : t[2]) r.msgs.push_back(x.cast<std::string>());
                 return r;
               };
             }
             py::gil_scoped_release nogil;
             return std::unique_ptr<rpc::Server, ServerDeleter>(new rpc::Server(o, std::move(h)));
           }),
           py::arg("host") = "0.0.0.0", py::arg("port") = 0, py::arg("bus_tag") = "", py::arg("io_threads") = 2,
           py::arg("wait_threads") = 256, py::arg("slow_threads") = 8, py::arg("handler") = py::none(),
           py::arg("reuseport") = true, py::arg("stream_deadline_ms") = 15000, py::arg("max_streams") = 1000,
           py::arg("max_queued_requests") = 16, py::arg("max_resets_per_s") = 200, py::arg("zero_copy") = true,
           "Native gRPC endpoint: VideoLatestImage from the frame bus `bus_tag`; the other Image methods "
           "call handler(method, request_bytes, peer) -> (status, message, [response_bytes, ...])")
      .def_property_readonly("port", &rpc::Server::port)
      .def("stop", &rpc::Server::stop, py::call_guard<py::gil_scoped_release>())
      .def("take_latencies", &rpc::Server::take_latencies)
      .def("stats", [](const rpc::Server& s) {
        const rpc::ServerStats st = s.stats();
        py::dict d;
        d["connections"] = st.connections;
        d["connections_open"] = st.connections_open;
        d["streams"] = st.streams;
        d["frames_served"] = st.frames_served;
        d["empty_frames"] = st.empty_frames;
        d["bytes_sent"] = st.bytes_sent;
        d["slow_calls"] = st.slow_calls;
        d["frame_copies"] = st.frame_copies;
        d["protocol_errors"] = st.protocol_errors;
        d["goaways"] = st.goaways;
        d["refused_streams"] = st.refused_streams;
        d["cancelled_waits"] = st.cancelled_waits;
        d["deadline_streams"] = st.deadline_streams;
        d["zero_copy_frames"] = st.zero_copy_frames;
        d["slow_readers"] = st.slow_readers;
        d["p50_ms"] = st.p50_ms;
        d["p99_ms"] = st.p99_ms;
        return d;
      });

  // Native load generator (csrc/vep/h2load.h): back-to-back VideoLatestImage clients, one TCP
  // connection each, on `threads` epoll threads; latencies of the measured window in ms.
  m.def(
      "h2_load",
      [](const std::string& host, int port, const std::vector<std::string>& names, int clients, int threads,
         double start_at, double duration_s, bool key_frame_only) {
        h2load::Options o;
        o.host = host;
        o.port = port;
        o.names = names;
        o.clients = clients;
        o.threads = threads;
        o.start_at = start_at;
        o.duration_s = duration_s;
        o.key_frame_only = key_frame_only;
        h2load::Result r;
        {
          py::gil_scoped_release g;
          r = h2load::run(o);
        }
        py::dict d;
        d["lat_ms"] = r.lat_ms;
        d["ok"] = r.ok;
        d["errors"] = r.errors;
        d["bytes"] = r.bytes;
        d["cpu_s"] = r.cpu_s;
        d["first_error"] = r.first_error;
        return d;
      },
      py::arg("host"), py::arg("port"), py::arg("names"), py::arg("clients"), py::arg("threads") = 2,
      py::arg("start_at") = 0.0, py::arg("duration_s") = 3.0, py::arg("key_frame_only") = false);
  m.def("hpack_huffman_encode", [](const py::bytes& b) { return py::bytes(rpc::huffman_encode(std::string(b))); });
  m.def("hpack_huffman_decode", [](const py::bytes& b) -> py::object {
    const std::string s = b;
    std::string out;
    if (!rpc::huffman_decode(reinterpret_cast<const u8*>(s.data()), s.size(), out)) return py::none();
    return py::bytes(out);
  });
  py::class_<rpc::HpackDecoder>(m, "HpackDecoder")
      .def(py::init<>())
      .def("decode",
           [](rpc::HpackDecoder& d, const py::bytes& b) -> py::object {
             const std::string s = b;
             std::vector<std::pair<std::string, std::string>> out;
             if (!d.decode(reinterpret_cast<const u8*>(s.data()), s.size(), out)) return py::none();
             py::list l;
             for (auto& [k, v] : out) l.append(py::make_tuple(k, v));
             return l;
           })
      .def_property_readonly("table_size", &rpc::HpackDecoder::table_size)
      .def_property_readonly("table_entries", &rpc::HpackDecoder::table_entries);
}
