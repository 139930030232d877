// Pass-through muxers: FLV tags, an RTMP publisher (+ a minimal RTMP ingest sink for tests) and
// per-GOP ISO-BMFF (MP4) segments. No transcoding: access units are re-framed as AVCC.
//
// Reference parity: FFmpeg's flv muxer + rtmp protocol opened via
// av.open(rtmp, format="flv", mode='w') (python/rtsp_to_rtmp.py:84-89, :162-182) and the mp4
// muxer of python/archive.py:45-100. SURVEY.md §2.2 N8/N9.
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>

#include "codec.h"

namespace vep::mux {

// NAL units of an AU re-framed as 4-byte-length AVCC, dropping SPS/PPS/AUD (carried in avcC).
std::vector<u8> au_to_avcc(const AccessUnit& au);

// FLV VIDEODATA bodies (without the 11-byte tag header). H.264 uses the classic AVC tags
// (CodecID 7); H.265 uses enhanced RTMP (IsExHeader, FourCC 'hvc1', SequenceStart /
// CodedFramesX), which FFmpeg >= 6.1, OBS and the major ingest services accept.
std::vector<u8> flv_avc_sequence_header(const std::vector<u8>& sps, const std::vector<u8>& pps);
std::vector<u8> flv_avc_nalu(const AccessUnit& au);
std::vector<u8> flv_sequence_header(const ParamSets& ps);
std::vector<u8> flv_video(const AccessUnit& au);
// Complete FLV tag (header + body + PreviousTagSize).
std::vector<u8> flv_tag(u8 type, u32 ts_ms, const std::vector<u8>& body);
std::vector<u8> flv_file_header();

// RTMP publisher (simple handshake, AMF0 connect/createStream/publish, chunked messages).
class RtmpPublisher {
 public:
  explicit RtmpPublisher(std::string url, int timeout_ms = 5000);
  ~RtmpPublisher();
  void connect();
  bool connected() const { return fd_ >= 0; }
  void send_sequence_header(const ParamSets& ps);
  void send_au(const AccessUnit& au, u32 ts_ms);
  void close();
  // From another thread: unblocks a connect / handshake / send in progress (shutdown of the
  // socket) and makes later connects fail; the owning thread still closes.
  void interrupt();
  u64 bytes_sent() const { return sent_; }
  u64 messages() const { return msgs_; }

 private:
  void send_message(int csid, u8 type, u32 stream, u32 ts, const std::vector<u8>& body);
  std::string url_, app_, key_, tc_url_;
  std::string host_;
  int port_ = 1935, timeout_ms_;
  int fd_ = -1;
  std::mutex fd_mu_;  // fd_ open/close vs interrupt()
  bool interrupted_ = false;
  u32 out_chunk_ = 128;
  u32 stream_id_ = 1;
  u64 sent_ = 0, msgs_ = 0;
};

// Minimal RTMP ingest server: accepts publishers, answers the command flow, records video.
class RtmpSink {
 public:
  explicit RtmpSink(const std::string& bind = "127.0.0.1", int port = 0);
  ~RtmpSink();
  void start();
  void stop();
  int port() const { return port_; }
  u64 video_messages() const { return video_.load(); }
  u64 keyframes() const { return keys_.load(); }
  u64 sequence_headers() const { return seqhdr_.load(); }
  u64 hevc_messages() const { return hevc_.load(); }  // enhanced-RTMP 'hvc1' video messages
  std::string last_stream_key() const;
  std::vector<std::vector<u8>> video_bodies() const;  // FLV VIDEODATA bodies in arrival order
  u64 video_bytes() const { return bytes_.load(); }
  // false: count the video messages only (long-running loads; bodies are not retained)
  void set_keep_bodies(bool on) { keep_bodies_ = on; }

 private:
  void serve(int fd);
  std::string bind_;
  int port_, lfd_ = -1;
  std::atomic<bool> stop_{false};
  std::thread acc_;
  std::atomic<int> live_{0};
  std::atomic<u64> video_{0}, keys_{0}, seqhdr_{0}, hevc_{0}, bytes_{0};
  std::atomic<bool> keep_bodies_{true};
  mutable std::mutex mu_;
  std::string key_;
  std::vector<std::vector<u8>> bodies_;
};

// One MP4 file for a GOP of access units (timestamps rebased to the first DTS).
struct Mp4Info {
  int width = 0, height = 0;
  ParamSets ps;  // avc1/avcC for H.264, hvc1/hvcC for H.265
};
std::vector<u8> build_mp4(const std::vector<AuPtr>& aus, const Mp4Info& info);
// Segment length in ms per archive.py:45-73 (sum of durations, else DTS span).
i64 segment_duration_ms(const std::vector<AuPtr>& aus);

// Background per-GOP writer: <dir>/<device>/<start_ms>_<duration_ms>.mp4
class Archiver {
 public:
  Archiver();
  ~Archiver();
  void enqueue(const std::string& dir, const std::string& device, i64 start_ms,
               std::vector<AuPtr> gop, Mp4Info info);
  void flush();
  u64 written() const { return written_.load(); }
  u64 failed() const { return failed_.load(); }
  std::string last_path() const;

 private:
  struct Job { std::string dir, device; i64 start_ms; std::vector<AuPtr> gop; Mp4Info info; };
  void loop();
  std::mutex mu_;
  std::condition_variable cv_, idle_;
  std::deque<Job> q_;
  bool stop_ = false, busy_ = false;
  std::atomic<u64> written_{0}, failed_{0};
  std::string last_;
  std::thread th_;
};

}  // namespace vep::mux
