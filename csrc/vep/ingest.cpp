// Ingest session / supervisor implementation. See ingest.h.
#include "ingest.h"

#include <cstdlib>
#include <tuple>

#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>

namespace vep {

// Liveness token of the pooled mode: timers and connector tasks enter() before touching the
// session and leave() after; stop() waits for the ones inside and turns later ones away.
struct IngestSession::Guard {
  std::mutex mu;
  std::condition_variable cv;
  bool stopped = false;
  int busy = 0;
  bool enter() {
    std::lock_guard<std::mutex> g(mu);
    if (stopped) return false;
    ++busy;
    return true;
  }
  void leave() {
    std::lock_guard<std::mutex> g(mu);
    --busy;
    cv.notify_all();
  }
  void stop() {
    std::unique_lock<std::mutex> g(mu);
    stopped = true;
    cv.wait(g, [this] { return busy == 0; });
  }
};

// The session's socket on the shared epoll loop.
class IngestSession::Handler : public IoHandler {
 public:
  Handler(IngestSession* s, std::shared_ptr<net::RtspClient> c) : s_(s), c_(std::move(c)) {}
  bool on_readable() override {
    if (!c_->read_available([this](const AuPtr& au) { s_->on_au(au); }, why_)) return false;
    if (s_->backlogged()) {  // lossless mode: hold the socket until the parse strand drains
      paused_.store(true);
      s_->svc_->io.pause_reading(*this);
    }
    return true;
  }
  bool on_tick() override {
    if (paused_.load()) {
      c_->touch_rx();  // held back on purpose: not a stalled camera
      if (s_->drained() && paused_.exchange(false)) {  // (safety net for a missed resume)
        epoll_resume_in_callback();
      }
    }
    return c_->maintain(why_);
  }
  // Parse strand side: the backlog has drained, read again.
  void resume(const std::shared_ptr<Handler>& self) {
    if (paused_.exchange(false)) s_->svc_->io.resume_reading(self);
  }
  void on_closed() override { s_->on_stream_end(why_, c_->bytes(), c_->lost()); }
  const net::RtspClient& client() const { return *c_; }
  bool paused() const { return paused_.load(); }

 private:
  void epoll_resume_in_callback() {
    // on_tick runs with this handler's lock held: re-arm through a task on the connector pool
    std::weak_ptr<IoHandler> wh = self_;
    auto svc = s_->svc_;
    svc->connect.post([svc, wh] {
      if (auto h = wh.lock()) svc->io.resume_reading(h);
    });
  }
  friend class IngestSession;
  std::weak_ptr<IoHandler> self_;
  std::atomic<bool> paused_{false};
  IngestSession* s_;
  std::shared_ptr<net::RtspClient> c_;
  std::string why_;
};

// AUs a camera's parse strand may hold before ingest drops to the next keyframe (~8 s at 30 fps).
constexpr size_t kMaxParseBacklog = 256;
// Lossless mode: the socket is paused above kHighWater queued AUs and resumed at kLowWater.
constexpr size_t kHighWater = 32, kLowWater = 8;

bool IngestSession::backlogged() const {
  const u64 key = parse_key_.load(std::memory_order_relaxed);
  return lossless_.load(std::memory_order_relaxed) && pooled_ && key && svc_->parse.depth(key) >= kHighWater;
}

bool IngestSession::drained() const {
  const u64 key = parse_key_.load(std::memory_order_relaxed);
  return !key || svc_->parse.depth(key) <= kLowWater;
}

IngestSession::IngestSession(Worker& w, int cam, IngestConfig cfg,
                             std::shared_ptr<mux::Archiver> archiver)
    : w_(w), cam_(cam), cfg_(std::move(cfg)), archiver_(std::move(archiver)) {
  lossless_.store(cfg_.lossless);
}

IngestSession::~IngestSession() { stop(); }

void IngestSession::log(bool err, const std::string& s) {
  if (auto c = w_.camera(cam_)) c->logs.add(err, s);
}

void IngestSession::start() {
  stop_ = false;
  const char* th = std::getenv("VEP_INGEST_THREADS");
  pooled_ = !(th && th[0] == '1');
  if (!pooled_) {
    th_ = std::thread([this] {
      name_thread("vep-ingest");
      run();
    });
    return;
  }
  svc_ = w_.ingest_services();  // (the worker's host domain: its GPU's CPUs)
  guard_ = std::make_shared<Guard>();
  parse_live_ = std::make_shared<std::atomic<bool>>(true);
  drop_to_key_ = false;
  {
    std::lock_guard<std::mutex> g(mu_);
    st_.pid = int(::getpid());  // (no thread of its own: the hub process)
  }
  schedule_connect(0);
}

void IngestSession::stop() {
  stop_ = true;
  if (th_.joinable()) th_.join();
  if (guard_) guard_->stop();  // no timer / connector task of this session runs from here on
  std::shared_ptr<Handler> h;
  {
    std::lock_guard<std::mutex> g(handler_mu_);
    h.swap(handler_);
  }
  if (h) {
    svc_->io.remove(h);  // synchronous: no socket callback runs after this
    std::lock_guard<std::mutex> g(mu_);
    st_.bytes += h->client().bytes();
    st_.lost += h->client().lost();
  }
  // No socket callback runs any more, so nothing posts new parse work: cancel what is queued on
  // the camera's strand and wait for the task that may be running. After this the Worker may
  // remove the camera and reuse its slot without a stale task reaching the new camera.
  if (parse_live_) parse_live_->store(false);
  if (const u64 key = parse_key_.exchange(0); key && svc_) svc_->parse.drain(key);
  pub_.reset();
  gop_.clear();
  seen_key_ = false;
  prev_proxy_ = false;
  std::lock_guard<std::mutex> g(mu_);
  if (st_.status != "created") {
    st_.status = "exited";
    st_.running = st_.restarting = false;
    st_.finished_at_ms = now_ms();
  }
}

void IngestSession::schedule_connect(int delay_ms) {
  std::weak_ptr<Guard> wg = guard_;
  svc_->timers.at(mono_us() / 1000 + delay_ms, [this, wg] {
    auto g = wg.lock();
    if (!g || !g->enter()) return;
    try {
      connect_once();
    } catch (...) {
    }
    g->leave();
  });
}

void IngestSession::mark_failed(const std::string& err, bool connect_error) {
  std::lock_guard<std::mutex> g(mu_);
  st_.status = "restarting";
  st_.running = false;
  st_.restarting = true;
  if (connect_error) st_.exit_code = 1;  // rtsp_to_rtmp.py:76-78 os._exit(1)
  st_.error = err;
  st_.finished_at_ms = now_ms();
  st_.restart_count++;
  st_.failing_streak++;
  st_.health = st_.failing_streak >= 3 ? "unhealthy" : "starting";
}

void IngestSession::connect_once() {
  if (stop_.load()) return;
  net::RtspClientOptions opt;
  opt.timeout_ms = cfg_.timeout_ms;
  auto client = std::make_shared<net::RtspClient>(cfg_.rtsp_url, opt);
  net::RtspStreamInfo info;
  try {
    info = client->open();
  } catch (const std::exception& e) {
    log(true, std::string("failed to connect to RTSP camera ") + e.what());
    mark_failed(e.what(), true);
    int streak;
    {
      std::lock_guard<std::mutex> g(mu_);
      streak = st_.failing_streak;
    }
    const int shift = std::min(streak - 1, 5);
    schedule_connect(std::min(cfg_.max_backoff_ms, cfg_.reconnect_delay_ms << shift));
    return;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    st_.status = "running";
    st_.running = true;
    st_.restarting = false;
    st_.dead = false;
    st_.exit_code = 0;
    st_.error.clear();
    st_.started_at_ms = now_ms();
    st_.failing_streak = 0;
    st_.health = "healthy";
    st_.fps = info.framerate;
  }
  ps_ = ParamSets{};
  ps_.codec = info.codec;
  for (auto& ps : info.param_sets) ps_.absorb(ps.data(), ps.size());
  gop_.clear();
  seen_key_ = false;
  prev_proxy_ = false;
  drop_to_key_ = false;
  log(false, "connected to " + cfg_.name + " (" + (info.codec == Codec::kH264 ? "H.264" : "H.265") + ")");
  auto h = std::make_shared<Handler>(this, client);
  h->self_ = h;
  {
    std::lock_guard<std::mutex> g(handler_mu_);
    handler_ = h;
  }
  svc_->io.add(client->fd(), h);
}

// Socket loop thread, inside the handler's callback: record the end, then clean up and schedule
// the reconnect on the connector pool (the RTMP sender join must not stall the loop).
void IngestSession::on_stream_end(const std::string& why, u64 bytes, u64 lost) {
  {
    std::lock_guard<std::mutex> g(mu_);
    st_.bytes += bytes;
    st_.lost += lost;
  }
  if (stop_.load()) return;
  log(false, "rtsp stopped streaming (" + why + ")...waiting for camera to reappear");
  mark_failed(why, false);
  std::weak_ptr<Guard> wg = guard_;
  svc_->connect.post([this, wg] {
    auto g = wg.lock();
    if (!g || !g->enter()) return;
    try {
      after_stream_end();
    } catch (...) {
    }
    g->leave();
  });
}

void IngestSession::after_stream_end() {
  {
    std::lock_guard<std::mutex> g(handler_mu_);
    handler_.reset();
  }
  pub_.reset();
  gop_.clear();
  seen_key_ = false;
  prev_proxy_ = false;
  schedule_connect(cfg_.reconnect_delay_ms);
}

void IngestSession::decode(const std::shared_ptr<Camera>& cam, const AuPtr& au) {
  if (!pooled_) {
    cam->on_access_unit(au);
    return;
  }
  // parse off the socket thread, in order, on the camera's strand of the shared parse pool
  const u64 key = u64(reinterpret_cast<uintptr_t>(cam.get()));
  if (lossless_.load(std::memory_order_relaxed)) {
    // never drop: on_readable pauses the socket above the high-water mark
  } else if (drop_to_key_) {
    if (!au->keyframe) {
      cam->skipped.fetch_add(1, std::memory_order_relaxed);
      return;
    }
    drop_to_key_ = false;
  } else if (svc_->parse.depth(key) >= kMaxParseBacklog) {
    drop_to_key_ = true;
    cam->skipped.fetch_add(1, std::memory_order_relaxed);
    log(true, "parse backlog full: dropping packets until the next keyframe");
    return;
  }
  parse_key_.store(key, std::memory_order_relaxed);
  std::weak_ptr<Handler> wh;  // (always: a socket paused in lossless mode resumes even after
  {                           // set_lossless(false))
    std::lock_guard<std::mutex> g(handler_mu_);
    wh = handler_;
  }
  svc_->parse.post(key, [cam, au, live = parse_live_, wh, svc = svc_, key] {
    if (!live->load(std::memory_order_acquire)) return;  // session stopped: cancelled
    try {
      cam->on_access_unit(au);
      cam->wait_reconstruction();  // (WorkerOptions::backpressure only)
    } catch (const std::exception& e) {
      cam->errors.fetch_add(1);
      cam->logs.add(true, std::string("failed to decode packet: ") + e.what());
    }
    if (auto h = wh.lock())  // lossless: the socket was paused and the backlog has drained
      if (h->paused() && svc->parse.depth(key) <= kLowWater + 1) h->resume(h);
  });
}

SessionState IngestSession::state() const {
  std::lock_guard<std::mutex> g(mu_);
  return st_;
}

bool IngestSession::sleep_interruptible(int ms) {
  for (int t = 0; t < ms && !stop_.load(); t += 20)
    std::this_thread::sleep_for(std::chrono::milliseconds(std::min(20, ms - t)));
  return !stop_.load();
}

void IngestSession::on_au(const AuPtr& au) {
  std::shared_ptr<Camera> cam = w_.camera(cam_);
  if (!cam) return;
  {
    std::lock_guard<std::mutex> g(mu_);
    st_.aus++;
  }
  ps_.absorb(*au);
  // --- archive: previous GOP goes to the archiver on every keyframe (rtsp_to_rtmp.py:97-110)
  if (au->keyframe) {
    if (!gop_.empty() && archiver_ && !cfg_.disk_path.empty() && ps_.complete()) {
      mux::Mp4Info info;
      if (auto ring = cam->ring()) {
        info.width = ring->width();
        info.height = ring->height();
      }
      if (info.width == 0) std::tie(info.width, info.height) = ps_.size();
      info.ps = ps_;
      archiver_->enqueue(cfg_.disk_path, cfg_.name, gop_start_ms_, std::move(gop_), info);
    }
    gop_.clear();
    gop_start_ms_ = now_ms();
    seen_key_ = true;
  }
  if (seen_key_) gop_.push_back(au);

  // --- decode scheduling (lazy / keyframe-only / catch-up) lives in the camera
  decode(cam, au);

  // --- RTMP pass-through (rtsp_to_rtmp.py:127-139, :162-182), sent off this thread
  const bool want = cam->proxy_rtmp.load() && !cfg_.rtmp_url.empty();
  const bool rising = want && !prev_proxy_;
  prev_proxy_ = want;
  if (!want) {
    if (pub_) {
      pub_.reset();  // joins the sender; closes the connection
      log(false, "rtmp publishing stopped");
    }
    return;
  }
  if (!seen_key_) return;
  if (rising || !pub_) {
    pub_ = std::make_unique<RtmpSender>(cfg_.rtmp_url, cfg_.timeout_ms);
    log(false, "rtmp publishing to " + cfg_.rtmp_url);
    pub_->start_gop(ps_, gop_);
  } else if (pub_->needs_keyframe()) {
    if (au->keyframe) pub_->start_gop(ps_, gop_);  // resume after an overflow / error
  } else {
    pub_->push(au);
  }
  std::string err = pub_->error();
  if (err != last_rtmp_err_) {
    if (!err.empty()) log(true, "failed muxing: " + err);
    last_rtmp_err_ = err;
  }
  std::lock_guard<std::mutex> g(mu_);
  st_.rtmp_messages = pub_->messages();
  st_.rtmp_error = err;
}

// ------------------------------------------------------------------------------ RtmpSender

RtmpSender::RtmpSender(std::string url, int timeout_ms, size_t max_bytes)
    : url_(std::move(url)), timeout_ms_(timeout_ms), max_bytes_(max_bytes) {
  th_ = std::thread([this] {
    name_thread("vep-rtmp");
    run();
  });
}

RtmpSender::~RtmpSender() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
    if (cur_) cur_->interrupt();  // a handshake with a server that never answers ends now
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
}

std::string RtmpSender::error() const {
  std::lock_guard<std::mutex> g(mu_);
  return err_;
}

void RtmpSender::drop_all_locked() {
  dropped_.fetch_add(q_.size());
  q_.clear();
  q_bytes_ = 0;
  need_key_.store(true);
}

void RtmpSender::start_gop(const ParamSets& ps, const std::vector<AuPtr>& gop) {
  {
    std::lock_guard<std::mutex> g(mu_);
    drop_all_locked();  // whatever is still queued belongs to the stream being restarted
    if (ps.complete()) q_.push_back(Item{nullptr, ps});
    for (const auto& a : gop) {
      q_.push_back(Item{a, {}});
      q_bytes_ += a->bytes();
    }
    need_key_.store(false);
  }
  cv_.notify_one();
}

void RtmpSender::push(const AuPtr& au) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (need_key_.load()) {
      dropped_.fetch_add(1);
      return;
    }
    if (q_bytes_ + au->bytes() > max_bytes_) {  // the server cannot keep up: resume at a keyframe
      drop_all_locked();
      dropped_.fetch_add(1);
      err_ = "rtmp send queue overflow: dropped to the next keyframe";
      return;
    }
    q_.push_back(Item{au, {}});
    q_bytes_ += au->bytes();
  }
  cv_.notify_one();
}

void RtmpSender::run() {
  std::unique_ptr<mux::RtmpPublisher> pub;
  i64 retry_at = 0;
  for (;;) {
    Item it;
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [this] { return stop_ || !q_.empty(); });
      if (stop_) break;
      it = std::move(q_.front());
      q_.pop_front();
      if (it.au) q_bytes_ -= it.au->bytes();
    }
    try {
      if (!pub || !pub->connected()) {
        if (mono_us() / 1000 < retry_at) {  // still backing off: this AU is lost
          std::lock_guard<std::mutex> g(mu_);
          drop_all_locked();
          dropped_.fetch_add(1);
          continue;
        }
        publish(pub, nullptr);
        auto np = std::make_unique<mux::RtmpPublisher>(url_, timeout_ms_);
        if (!publish(pub, std::move(np))) break;
        pub->connect();
        ts0_ = -1;
      }
      if (!it.au) {
        pub->send_sequence_header(it.ps);
      } else {
        if (ts0_ < 0) ts0_ = it.au->dts;
        pub->send_au(*it.au, u32(std::max<i64>(0, (it.au->dts - ts0_) / 90)));
      }
      msgs_.store(pub->messages());
      std::lock_guard<std::mutex> g(mu_);
      if (err_.rfind("rtmp send queue overflow", 0) != 0) err_.clear();
    } catch (const std::exception& e) {
      publish(pub, nullptr);
      retry_at = mono_us() / 1000 + 2000;
      std::lock_guard<std::mutex> g(mu_);
      err_ = e.what();
      drop_all_locked();  // a new connection must start at a keyframe
    }
  }
  if (pub) pub->close();
  publish(pub, nullptr);
}

bool RtmpSender::publish(std::unique_ptr<mux::RtmpPublisher>& pub, std::unique_ptr<mux::RtmpPublisher> np) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (np && stop_) return false;
    cur_ = np.get();  // the destructor interrupts only a publisher that is still alive
  }
  pub = std::move(np);
  return true;
}

void IngestSession::run() {
  {
    std::lock_guard<std::mutex> g(mu_);
    st_.pid = int(::syscall(SYS_gettid));
  }
  net::RtspClientOptions opt;
  opt.timeout_ms = cfg_.timeout_ms;
  while (!stop_.load()) {
    int delay = cfg_.reconnect_delay_ms;
    try {
      net::RtspClient client(cfg_.rtsp_url, opt);
      net::RtspStreamInfo info = client.open();
      {
        std::lock_guard<std::mutex> g(mu_);
        st_.status = "running";
        st_.running = true;
        st_.restarting = false;
        st_.dead = false;
        st_.exit_code = 0;
        st_.error.clear();
        st_.started_at_ms = now_ms();
        st_.failing_streak = 0;
        st_.health = "healthy";
        st_.fps = info.framerate;
      }
      ps_.codec = info.codec;
      for (auto& ps : info.param_sets) ps_.absorb(ps.data(), ps.size());
      log(false, "connected to " + cfg_.name + " (" +
                     (info.codec == Codec::kH264 ? "H.264" : "H.265") + ")");
      std::string why = client.run([this](const AuPtr& au) { on_au(au); }, stop_);
      {
        std::lock_guard<std::mutex> g(mu_);
        st_.bytes += client.bytes();
        st_.lost += client.lost();
      }
      if (stop_.load()) break;
      log(false, "rtsp stopped streaming (" + why + ")...waiting for camera to reappear");
      std::lock_guard<std::mutex> g(mu_);
      st_.status = "restarting";
      st_.running = false;
      st_.restarting = true;
      st_.finished_at_ms = now_ms();
      st_.restart_count++;
      st_.failing_streak++;
      st_.health = st_.failing_streak >= 3 ? "unhealthy" : "starting";
      st_.error = why;
      delay = cfg_.reconnect_delay_ms;
    } catch (const std::exception& e) {
      log(true, std::string("failed to connect to RTSP camera ") + e.what());
      std::lock_guard<std::mutex> g(mu_);
      st_.status = "restarting";
      st_.running = false;
      st_.restarting = true;
      st_.exit_code = 1;  // rtsp_to_rtmp.py:76-78 os._exit(1)
      st_.error = e.what();
      st_.finished_at_ms = now_ms();
      st_.restart_count++;
      st_.failing_streak++;
      st_.health = st_.failing_streak >= 3 ? "unhealthy" : "starting";
      int shift = std::min(st_.failing_streak - 1, 5);
      delay = std::min(cfg_.max_backoff_ms, cfg_.reconnect_delay_ms << shift);
    }
    gop_.clear();
    seen_key_ = false;
    prev_proxy_ = false;
    pub_.reset();
    if (!sleep_interruptible(delay)) break;
  }
}

}  // namespace vep
