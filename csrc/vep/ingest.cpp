// Ingest session / supervisor implementation. See ingest.h.
#include "ingest.h"

#include <tuple>

#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>

namespace vep {

IngestSession::IngestSession(Worker& w, int cam, IngestConfig cfg,
                             std::shared_ptr<mux::Archiver> archiver)
    : w_(w), cam_(cam), cfg_(std::move(cfg)), archiver_(std::move(archiver)) {}

IngestSession::~IngestSession() { stop(); }

void IngestSession::log(bool err, const std::string& s) {
  if (auto c = w_.camera(cam_)) c->logs.add(err, s);
}

void IngestSession::start() {
  stop_ = false;
  th_ = std::thread([this] { run(); });
}

void IngestSession::stop() {
  stop_ = true;
  if (th_.joinable()) th_.join();
  std::lock_guard<std::mutex> g(mu_);
  if (st_.status != "created") {
    st_.status = "exited";
    st_.running = st_.restarting = false;
    st_.finished_at_ms = now_ms();
  }
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
  cam->on_access_unit(au);

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
  th_ = std::thread([this] { run(); });
}

RtmpSender::~RtmpSender() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
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
        pub = std::make_unique<mux::RtmpPublisher>(url_, timeout_ms_);
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
      pub.reset();
      retry_at = mono_us() / 1000 + 2000;
      std::lock_guard<std::mutex> g(mu_);
      err_ = e.what();
      drop_all_locked();  // a new connection must start at a keyframe
    }
  }
  if (pub) pub->close();
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
