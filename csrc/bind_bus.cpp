// Python bindings of the frame bus (csrc/vep/bus.h): the owner side runs in the process that
// decodes (Hub / isolated worker), the reader side in the serving processes.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "bind_ext.h"
#include "vep/bus.h"
#include "vep/runtime.h"

namespace py = pybind11;
using namespace vep;

void bind_bus(py::module_& m) {
  py::class_<bus::Owner>(m, "BusOwner")
      .def(py::init<const std::string&, int, int>(), py::arg("tag"), py::arg("owner"), py::arg("max_cams"))
      .def("attach", &bus::Owner::attach, py::keep_alive<1, 2>(), py::call_guard<py::gil_scoped_release>())
      .def("add", &bus::Owner::add)
      .def("remove", &bus::Owner::remove)
      .def("stop", &bus::Owner::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("path", &bus::Owner::path)
      .def_property_readonly("published", &bus::Owner::published)
      .def_property_readonly("dma_bytes", &bus::Owner::dma_bytes);

  py::class_<bus::Reader>(m, "BusReader")
      .def(py::init<const std::string&>(), py::arg("tag"))
      .def("has", &bus::Reader::has, py::call_guard<py::gil_scoped_release>())
      .def("names", &bus::Reader::names, py::call_guard<py::gil_scoped_release>())
      .def("touch", &bus::Reader::touch, py::arg("name"), py::arg("key_frame_only") = -1,
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("rescans", &bus::Reader::rescans)
      .def("mapped_data_segments", &bus::Reader::mapped_data_segments, py::call_guard<py::gil_scoped_release>())
      .def("info",
           [](bus::Reader& r, const std::string& name) -> py::object {
             bus::Reader::Info i;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = r.info(name, &i);
             }
             if (!ok) return py::none();
             py::dict d;
             d["owner_pid"] = i.owner_pid;
             d["pinned"] = i.pinned;
             d["ring_seq"] = i.ring_seq;
             d["bus_seq"] = i.bus_seq;
             d["owner_published"] = i.published;
             return d;
           })
      .def("frame",
           // (seq, serialized VideoFrame bytes) of the newest bus frame with seq > after (waiting up
           // to wait_ms for it), (seq, None) when that frame's seq is `have` (the caller holds its
           // bytes), None on timeout / unknown camera. key_frame_only < 0 leaves the mode as is;
           // touch = False reads without marking the camera's demand (last_query).
           [](bus::Reader& r, const std::string& name, i64 after, int wait_ms, int key_frame_only,
              i64 have, bool touch) -> py::object {
             bus::Reader::Ticket t;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = r.wait(name, after, wait_ms, key_frame_only, &t, touch);
             }
             if (!ok) return py::none();
             const i64 ns = r.newest_seq(t);
             if (have > 0 && ns == have) return py::make_tuple(ns, py::none());
             PyObject* b = PyBytes_FromStringAndSize(nullptr, Py_ssize_t(t.cap));
             if (!b) throw py::error_already_set();
             size_t len;
             i64 seq = 0;
             {
               py::gil_scoped_release nogil;
               len = r.copy(t, reinterpret_cast<u8*>(PyBytes_AS_STRING(b)), t.cap, &seq);
             }
             if (!len) {
               Py_DECREF(b);
               return py::none();
             }
             if (_PyBytes_Resize(&b, Py_ssize_t(len)) != 0) throw py::error_already_set();
             return py::make_tuple(seq, py::reinterpret_steal<py::object>(b));
           },
           py::arg("name"), py::arg("after") = 0, py::arg("wait_ms") = 0, py::arg("key_frame_only") = -1,
           py::arg("have") = -1, py::arg("touch") = true);

  m.def("bus_remove_segments", &bus::remove_segments_of, py::arg("pid"),
        "Unlink the frame-bus segments a (dead) process left in /dev/shm.");
}
