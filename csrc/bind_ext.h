// Binding entry points of the network (RTSP/RTP) and muxer (FLV/RTMP/MP4) layers.
#pragma once
#include <pybind11/pybind11.h>

void bind_net(pybind11::module_& m);
void bind_mux(pybind11::module_& m);
void bind_hevc(pybind11::module_& m);
void bind_bus(pybind11::module_& m);
void bind_rpc(pybind11::module_& m);
