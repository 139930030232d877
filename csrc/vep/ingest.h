// Per-camera ingest session + supervisor: RTSP client thread that feeds the camera's lazy
// decoder, the RTMP pass-through (proxy) and the per-GOP MP4 archiver, with restart-always
// semantics and container-like state for ListStreams / REST Info.
//
// Reference parity (one Docker container + Python worker per camera):
//  * connect / demux / reconnect-after-1 s: python/rtsp_to_rtmp.py:49-187
//  * proxy rising edge flushes the current GOP, then muxes every packet: :127-139, :162-182
//  * GOP -> archiver queue on every keyframe: :97-110; archive.py
//  * Docker `restart: always` + ContainerState (Status/Running/Restarting/ExitCode/Error/Pid/
//    StartedAt/FinishedAt/Health.FailingStreak): services/rtsp_process_manager.go:70-81, :283-335
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

#include "ioloop.h"
#include "mux.h"
#include "net.h"
#include "runtime.h"

namespace vep {

struct IngestConfig {
  std::string name;
  std::string rtsp_url;
  std::string rtmp_url;     // empty: no pass-through possible
  std::string disk_path;    // empty: no archive
  int timeout_ms = 5000;
  int reconnect_delay_ms = 1000;
  int max_backoff_ms = 30000;
  // Lossless ingest: while the camera's parse backlog is deep, stop reading its socket (TCP
  // back-pressure to the camera) instead of dropping access units until the next keyframe.
  // For sources that can be slowed down (files, replay farms, benchmarks); a live camera that
  // outruns the decoder is better served by the default, which stays at the live edge.
  bool lossless = false;
};

struct SessionState {
  std::string status = "created";  // created | running | restarting | exited | dead
  bool running = false, restarting = false, dead = false, paused = false, oomkilled = false;
  int pid = 0;
  int exit_code = 0;
  std::string error;
  i64 started_at_ms = 0, finished_at_ms = 0;
  int restart_count = 0;
  int failing_streak = 0;
  std::string health = "starting";
  u64 aus = 0, bytes = 0, lost = 0;
  u64 rtmp_messages = 0;
  std::string rtmp_error;
  double fps = 0;
  int width = 0, height = 0;
};

// RTMP pass-through off the ingest thread: the ingest thread enqueues access units, a sender
// thread owns the connection (connect / retry every 2 s / send). The queue is bounded: when the
// RTMP server is slow or dead it overflows, everything queued is dropped and sending resumes at
// the next keyframe (with the sequence header), so ingest and decode never wait on RTMP.
class RtmpSender {
 public:
  RtmpSender(std::string url, int timeout_ms, size_t max_bytes = size_t(32) << 20);
  ~RtmpSender();
  // Start (or restart after an overflow / error) at a keyframe: the parameter sets and the
  // current GOP (rtsp_to_rtmp.py:127-139 flushes the GOP on the proxy's rising edge).
  void start_gop(const ParamSets& ps, const std::vector<AuPtr>& gop);
  void push(const AuPtr& au);  // one more AU of the running stream (dropped until a keyframe)
  u64 messages() const { return msgs_.load(); }
  u64 dropped() const { return dropped_.load(); }
  bool needs_keyframe() const { return need_key_.load(); }
  std::string error() const;

 private:
  struct Item {
    AuPtr au;          // null: sequence header
    ParamSets ps;
  };
  void run();
  void drop_all_locked();
  // Replaces the live publisher (registering it for interrupt()); false once stopping.
  bool publish(std::unique_ptr<mux::RtmpPublisher>& pub, std::unique_ptr<mux::RtmpPublisher> np);
  const std::string url_;
  const int timeout_ms_;
  const size_t max_bytes_;
  std::thread th_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Item> q_;
  size_t q_bytes_ = 0;
  bool stop_ = false;
  mux::RtmpPublisher* cur_ = nullptr;  // the live publisher (under mu_), for interrupt()
  std::atomic<bool> need_key_{true};
  std::atomic<u64> msgs_{0}, dropped_{0};
  std::string err_;
  i64 ts0_ = -1;
};

// Two execution modes. Pooled (the default): the RTSP handshake runs on the shared connector
// pool, the socket is then served by the shared epoll loop (IngestServices::io) and access units
// are parsed on the camera's strand of the shared parse pool; reconnect back-off is a timer, so a
// session owns no thread. Threaded (VEP_INGEST_THREADS=1): one blocking thread per camera that
// receives and parses, as in round 1.
class IngestSession {
 public:
  IngestSession(Worker& w, int cam, IngestConfig cfg, std::shared_ptr<mux::Archiver> archiver);
  ~IngestSession();
  void start();
  // Synchronous: when it returns no callback of this session runs, and every parse task it
  // posted to the shared strand pool has finished or been cancelled (so the camera slot can be
  // removed and reused).
  void stop();
  SessionState state() const;
  const IngestConfig& config() const { return cfg_; }
  // Switch lossless ingest (IngestConfig::lossless) on or off while running.
  void set_lossless(bool on) { lossless_.store(on, std::memory_order_relaxed); }
  bool lossless() const { return lossless_.load(std::memory_order_relaxed); }
  void log(bool err, const std::string& s);
  bool pooled() const { return pooled_; }

 private:
  struct Guard;  // liveness token of the pooled mode's timers / connector tasks
  class Handler;
  bool backlogged() const;  // lossless mode: parse backlog above the high-water mark
  bool drained() const;     // parse backlog at or below the low-water mark
  void run();
  void on_au(const AuPtr& au);
  void decode(const std::shared_ptr<Camera>& cam, const AuPtr& au);
  bool sleep_interruptible(int ms);
  // pooled mode
  void schedule_connect(int delay_ms);
  void connect_once();
  void on_stream_end(const std::string& why, u64 bytes, u64 lost);
  void after_stream_end();
  void mark_failed(const std::string& err, bool connect_error);
  bool pooled_ = true;
  std::shared_ptr<IngestServices> svc_;
  std::shared_ptr<Guard> guard_;
  std::shared_ptr<Handler> handler_;
  std::mutex handler_mu_;
  bool drop_to_key_ = false;  // parse backlog overflowed: skip until the next keyframe
  // Cancellation token of the parse tasks this session posted (checked by each task before it
  // touches the camera) and the strand key they were posted under.
  std::shared_ptr<std::atomic<bool>> parse_live_;
  std::atomic<u64> parse_key_{0};
  std::atomic<bool> lossless_{false};
  Worker& w_;
  int cam_;
  IngestConfig cfg_;
  std::shared_ptr<mux::Archiver> archiver_;
  std::atomic<bool> stop_{false};
  std::thread th_;
  mutable std::mutex mu_;
  SessionState st_;
  // pass-through / archive state (ingest thread only)
  std::unique_ptr<RtmpSender> pub_;
  bool prev_proxy_ = false;
  std::string last_rtmp_err_;
  ParamSets ps_;
  std::vector<AuPtr> gop_;
  i64 gop_start_ms_ = 0;
  bool seen_key_ = false;
};

}  // namespace vep
