// Native gRPC endpoint of the Image service (HTTP/2, RFC 7540 + HPACK, RFC 7541): serves
// VideoLatestImage straight from the node's frame bus (bus.h) with no Python and no interpreter
// lock on the path, and hands the other methods (ListStreams, Annotate, Proxy, Storage: registry,
// queue and cloud calls, not a hot path) to a callback.
//
// Reference parity: the Go server answers every VideoLatestImage stream on its own goroutine
// (server/grpcapi/grpc_api.go:133-235, server/main.go:142-154): per received request it marks
// the camera's demand (keyframe-only mode + last_query), waits up to 3 x 1 s for a frame newer
// than the caller's cursor and sends it (an empty VideoFrame when none arrives), within a 15 s
// deadline on the stream. Same here, with the cursor kept per (client connection, camera) as the
// Python server does (the reference shared one per camera across clients).
//
// Design: a few epoll I/O threads own the connections (framing, HPACK, flow control, writev of
// DATA frames that point into one shared copy of each camera's newest frame: the bus slot is
// copied out once per frame per serving process, whatever the number of clients); a pool of
// waiter threads blocks on the bus futexes; a small pool runs the other methods' callback.
#pragma once

#include <atomic>
#include <functional>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "common.h"

namespace vep::rpc {

// One reply of a non-frame method: gRPC status (0 = OK), message, and the response messages
// (serialized protobufs; several for a server-streaming method).
struct Reply {
  int status = 0;
  std::string message;
  std::vector<std::string> msgs;
};
// (method name, serialized request, peer "ipv4:host:port") -> reply. Runs on the slow pool.
using SlowHandler = std::function<Reply(const std::string& method, const std::string& request, const std::string& peer)>;

struct ServerOptions {
  std::string host = "0.0.0.0";
  int port = 0;                 // 0: any free port
  bool reuseport = true;        // several serving processes on one port (SO_REUSEPORT)
  int io_threads = 2;
  int wait_threads = 256;       // concurrent VideoLatestImage requests waiting for a frame
  int slow_threads = 8;
  std::string bus_tag;          // frame source (bus::Reader)
  std::string service = "chrys.cloud.videostreaming.v1beta1.Image";
  int stream_deadline_ms = 15000;  // grpc_api.go:135
  int wait_attempts = 3;           // grpc_api.go:187 (XREAD BLOCK 1 s, 3 attempts)
  int wait_block_ms = 1000;
  size_t max_cursors = 65536;
  // Send frames straight from the frame bus's shared memory under a slot lease (bus.h) instead of
  // copying each new frame once per serving process.
  bool zero_copy = true;
  // Protocol limits (what grpc-go's server bounds for the reference, server/main.go:142-153).
  // Violations end the connection with GOAWAY (or refuse / fail the one stream) before any
  // unbounded buffering happens.
  u32 max_streams = 1000;            // SETTINGS_MAX_CONCURRENT_STREAMS; more: RST_STREAM REFUSED_STREAM
  u32 max_header_list = 16384;       // SETTINGS_MAX_HEADER_LIST_SIZE (decoded, RFC 7540 6.5.2 accounting)
  u32 max_header_block = 65536;      // encoded header block incl. CONTINUATION; more: ENHANCE_YOUR_CALM
  u32 max_queued_requests = 16;      // per stream, not yet answered; more: RESOURCE_EXHAUSTED on the stream
  size_t max_request_bytes = 8u << 20;   // buffered request bytes per connection; more: ENHANCE_YOUR_CALM
  u32 max_resets_per_s = 200;        // client resets of unanswered streams (rapid-reset defence)
  size_t read_budget = 256u << 10;   // bytes read from one connection per readiness event
  size_t out_high_water = 64u << 20; // queued output above which the connection's input is paused
  // HTTP/2 inbound frame payloads above 16384 bytes (the SETTINGS_MAX_FRAME_SIZE this server
  // never raises) are FRAME_SIZE_ERROR.
};

struct ServerStats {
  u64 connections = 0, connections_open = 0, streams = 0, frames_served = 0, empty_frames = 0;
  u64 bytes_sent = 0, slow_calls = 0, frame_copies = 0, protocol_errors = 0;
  u64 goaways = 0;           // connections ended by the server for a protocol or limit violation
  u64 refused_streams = 0;   // RST_STREAM REFUSED_STREAM (over max_streams)
  u64 cancelled_waits = 0;   // frame waits ended early because the client reset the stream
  u64 deadline_streams = 0;  // streams ended with DEADLINE_EXCEEDED
  u64 zero_copy_frames = 0;  // frames sent straight from a leased bus slot (no copy)
  u64 slow_readers = 0;      // connections closed with leased bytes unsent for bus::kLeaseSendMs
  double p50_ms = 0, p99_ms = 0;  // request received -> response queued (recent requests)
};

class Server {
 public:
  Server(const ServerOptions& o, SlowHandler slow);
  ~Server();
  Server(const Server&) = delete;
  Server& operator=(const Server&) = delete;
  int port() const;
  void stop();
  ServerStats stats() const;
  // server-side request latencies (ms) recorded since the last call (bounded to the newest 8192)
  std::vector<float> take_latencies();

  struct Impl;

 private:
  std::unique_ptr<Impl> p_;
};

// ---- HPACK pieces (exposed for tests)
// Huffman code of RFC 7541 Appendix B (canonical: generated from the code lengths).
bool huffman_decode(const u8* p, size_t n, std::string& out);
std::string huffman_encode(const std::string& s);

class HpackDecoder {
 public:
  // Decodes one header block; false on a malformed block (a connection error) or when the decoded
  // header list exceeds max_list (sum of name + value + 32 per field, RFC 7540 6.5.2): indexed
  // fields can expand a small block, so the bound applies to the output, not the input.
  bool decode(const u8* p, size_t n, std::vector<std::pair<std::string, std::string>>& out);
  void set_max_list(size_t n) { max_list_ = n; }
  bool list_too_large() const { return over_; }
  size_t table_size() const { return size_; }
  size_t table_entries() const { return dyn_.size(); }

 private:
  bool entry(size_t idx, std::string& name, std::string& value) const;
  void add(const std::string& name, const std::string& value);
  void evict();
  std::vector<std::pair<std::string, std::string>> dyn_;  // newest first
  size_t size_ = 0, max_ = 4096, limit_ = 4096;
  size_t max_list_ = size_t(-1);
  bool over_ = false;
};

}  // namespace vep::rpc
