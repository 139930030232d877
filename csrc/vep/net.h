// Network ingest layer: RTP (RFC 3550) H.264/H.265 packetization (RFC 6184 / RFC 7798), an
// RTSP 1.0 client over TCP-interleaved transport, and an RTSP server that serves synthetic
// cameras (the test/bench "camera farm").
//
// Reference parity: replaces FFmpeg's rtsp demuxer opened by PyAV with
// rtsp_transport=tcp, stimeout=5 s, max_delay=5 s (python/rtsp_to_rtmp.py:61-68, :92) and the
// reconnect loop (rtsp_to_rtmp.py:186-187). SURVEY.md §2.2 N1.
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "codec.h"
#include "synth.h"

namespace vep::net {

// ------------------------------------------------------------------------------------- RTP

struct RtpHeader {
  u8 pt = 96;
  bool marker = false;
  u16 seq = 0;
  u32 ts = 0;
  u32 ssrc = 0;
};
constexpr size_t kRtpHeader = 12;
void write_rtp_header(u8* out, const RtpHeader& h);
// Returns false on a malformed packet; payload excludes CSRCs, extension and padding.
bool parse_rtp(const u8* p, size_t n, RtpHeader& h, const u8** payload, size_t* plen);

// Split one NAL into RTP payloads of at most `mtu` bytes (single NAL unit or FU-A / FU).
void packetize_nal(Codec c, const u8* nal, size_t n, size_t mtu,
                   std::vector<std::vector<u8>>& out);
// Aggregate small NALs (e.g. SPS+PPS) into one STAP-A (H.264) / AP (H.265) payload.
std::vector<u8> aggregate_nals(Codec c, const std::vector<std::vector<u8>>& nals);

// Reassembles NAL units and access units from RTP payloads.
class Depacketizer {
 public:
  explicit Depacketizer(Codec c) : codec_(c) {}
  // Feed one packet. Completed AUs (marker bit or timestamp change) are appended to `out`.
  void push(const RtpHeader& h, const u8* payload, size_t n, std::vector<AuPtr>& out);
  void flush(std::vector<AuPtr>& out);
  u64 lost() const { return lost_; }
  u64 aus() const { return aus_; }
  void set_clock(u32 clock_rate) { clock_ = clock_rate; }

 private:
  void add_nal(const u8* p, size_t n);
  void finish(std::vector<AuPtr>& out);
  Codec codec_;
  std::shared_ptr<AccessUnit> cur_;
  std::vector<u8> frag_;
  bool in_frag_ = false, frag_bad_ = false, corrupt_ = false;
  bool have_seq_ = false, have_ts_ = false;
  u16 last_seq_ = 0;
  u32 cur_ts_ = 0;
  i64 ts_base_ = 0, ts_ext_ = 0;
  u32 last_ts_ = 0;
  u32 clock_ = 90000;
  u64 lost_ = 0, aus_ = 0, seq_counter_ = 0;
};

bool is_keyframe_nal(Codec c, const u8* nal, size_t n);

// ----------------------------------------------------------------------------------- base64
std::string base64_encode(const u8* p, size_t n);
std::vector<u8> base64_decode(const std::string& s);

// ------------------------------------------------------------------------------------- URL
struct Url {
  std::string scheme, user, pass, host, path;
  int port = 0;
};
Url parse_url(const std::string& u);

// ---------------------------------------------------------------------------- RTSP client

struct RtspStreamInfo {
  Codec codec = Codec::kH264;
  int payload_type = 96;
  u32 clock_rate = 90000;
  std::vector<std::vector<u8>> param_sets;  // sprop-parameter-sets / sprop-vps,sps,pps
  std::string control;
  double framerate = 0;
  std::string sdp;
};

struct RtspClientOptions {
  int timeout_ms = 5000;    // stimeout=5000000 us (rtsp_to_rtmp.py:63)
  std::string user_agent = "vep/0.1";
};

// Blocking RTSP session: connect, OPTIONS/DESCRIBE/SETUP(TCP interleaved)/PLAY, then deliver
// access units until `stop` is set, the server closes, or the socket times out.
class RtspClient {
 public:
  void touch_rx() { last_rx_us_ = mono_us(); }  // reading paused on purpose (flow control)
  using AuCallback = std::function<void(const AuPtr&)>;
  RtspClient(std::string url, RtspClientOptions opt = {});
  ~RtspClient();
  // Connect + handshake. Throws vep::Error on failure.
  RtspStreamInfo open();
  // Read loop; returns the reason the stream ended.
  std::string run(const AuCallback& cb, const std::atomic<bool>& stop);
  // Event-driven use (IoLoop): after open(), read whatever the socket holds without blocking and
  // deliver the completed access units; false (with the reason) when the stream ended.
  bool read_available(const AuCallback& cb, std::string& why);
  // Periodic upkeep between reads: session keep-alive, stall timeout (false = timed out).
  bool maintain(std::string& why);
  int fd() const { return fd_; }
  void close();
  u64 bytes() const { return bytes_; }
  u64 lost() const { return dep_ ? dep_->lost() : 0; }

 private:
  bool parse_buffer(std::vector<AuPtr>& aus, std::string& why);
  void emit(std::vector<AuPtr>& aus, const AuCallback& cb);
  bool params_sent_ = false;
  i64 last_ka_us_ = 0;
  std::string request(const std::string& method, const std::string& uri,
                      const std::string& extra, std::string* body);
  std::string url_;
  Url u_;
  RtspClientOptions opt_;
  int fd_ = -1;
  int cseq_ = 0;
  std::string session_, base_;
  std::string auth_;  // Authorization header value (Basic/Digest)
  std::string realm_, nonce_;
  bool digest_ = false;
  std::vector<u8> rbuf_;
  size_t rpos_ = 0;
  RtspStreamInfo info_;
  std::unique_ptr<Depacketizer> dep_;
  u64 bytes_ = 0;
  i64 last_rx_us_ = 0;
};

// ---------------------------------------------------------------------------- RTSP server

enum class Fault : int { kNone = 0, kDropConnection = 1, kStall = 2, kCorruptNal = 3,
                          kSkipKeyframe = 4, kRefuse = 5 };

struct ServedStream {
  SynthConfig cfg;
  bool realtime = true;     // pace at cfg.fps; false = as fast as the socket drains
  int cached_frames = 0;    // >0: pre-encode this many AUs and loop them
  std::string user, pass;   // optional Basic auth
};

class RtspServer {
 public:
  explicit RtspServer(const std::string& bind = "127.0.0.1", int port = 0);
  ~RtspServer();
  void add_stream(const std::string& path, const ServedStream& s);
  void start();
  void stop();
  int port() const { return port_; }
  void inject(const std::string& path, Fault f);  // applies to the stream's live sessions
  int sessions() const { return live_.load(); }
  u64 aus_sent() const { return aus_sent_.load(); }
  // Override every stream's pacing: 1 = real time at cfg.fps, 0 = as fast as the socket
  // drains, -1 = each stream's own ServedStream::realtime. Takes effect at the next frame.
  void set_pacing(int mode) { pace_.store(mode); }

 private:
  struct Stream {
    ServedStream cfg;
    std::vector<AuPtr> cache;
    // RTP payloads (FU-A / single NAL) of each cached AU, packetized once: (payload, marker)
    std::vector<std::vector<std::pair<std::vector<u8>, bool>>> cache_pk;
    std::vector<u8> sps, pps, vps;
    std::atomic<int> fault{0};
  };
  void accept_loop();
  void serve(int fd);
  std::string bind_;
  int port_;
  int lfd_ = -1;
  std::atomic<bool> stop_{false};
  std::thread acc_;
  std::mutex mu_;
  std::map<std::string, std::shared_ptr<Stream>> streams_;
  std::vector<int> conn_fds_;
  std::atomic<int> live_{0};
  std::atomic<u64> aus_sent_{0};
  std::atomic<int> pace_{-1};
};

}  // namespace vep::net
