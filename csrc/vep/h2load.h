// Native VideoLatestImage load generator: many concurrent gRPC-over-HTTP/2 clients on a few epoll
// threads, for measuring the serving endpoints (native csrc/vep/rpcsrv.cpp or grpcio) under the
// reference's client pattern (examples/opencv_display.py:43-45: each viewer loops on
// VideoLatestImage for one camera) without the client side being the bottleneck: the Python gRPC
// clients (vep_bench/latency_clients.py) spend ~10 ms of CPU parsing each 6.2 MB 1080p frame,
// which on a 16-CPU box competes with the server they measure. These clients count the DATA bytes
// of each response and discard them (the kernel's socket copy is the only per-byte work), answer
// SETTINGS / PING, and keep the connection window open.
//
// Reference: server/grpcapi/grpc_api.go:133-235 (the handler being measured).
#pragma once

#include <string>
#include <vector>

#include "common.h"

namespace vep::h2load {

struct Options {
  std::string host = "127.0.0.1";
  int port = 50001;
  std::vector<std::string> names;  // client k asks for camera names[k % names.size()]
  int clients = 1;                 // connections (one client each, its own TCP connection)
  int threads = 2;                 // epoll threads
  double start_at = 0;             // wall-clock (time(nullptr)-based, seconds) start of the measured window
  double duration_s = 3.0;         // measured window
  bool key_frame_only = false;
  double connect_timeout_s = 20.0;
};

struct Result {
  std::vector<double> lat_ms;  // request sent -> response complete (END_STREAM), measured window
  u64 ok = 0;                  // responses with a message, measured window
  u64 errors = 0;              // failed connections / reset or empty responses
  u64 bytes = 0;               // DATA bytes of those responses
  double cpu_s = 0;            // this process's CPU time over the measured window (user + sys)
  std::string first_error;
};

// Connects every client, sends one warm-up request each (the server-side cursor then sits at the
// camera's current frame), waits for start_at, then issues back-to-back requests for duration_s.
Result run(const Options& o);

}  // namespace vep::h2load
