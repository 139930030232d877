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

  // --- RTMP pass-through (rtsp_to_rtmp.py:127-139, :162-182)
  const bool want = cam->proxy_rtmp.load() && !cfg_.rtmp_url.empty();
  const bool rising = want && !prev_proxy_;
  prev_proxy_ = want;
  if (!want) {
    if (pub_) {
      pub_->close();
      pub_.reset();
      pub_ts0_ = -1;
    }
    return;
  }
  if (!seen_key_) return;
  try {
    if (!pub_ || !pub_->connected()) {
      if (mono_us() / 1000 < pub_retry_at_) return;
      pub_ = std::make_unique<mux::RtmpPublisher>(cfg_.rtmp_url, cfg_.timeout_ms);
      pub_->connect();
      log(false, "rtmp publishing to " + cfg_.rtmp_url);
      pub_ts0_ = -1;
    }
    auto ts_ms = [&](const AccessUnit& a) {
      if (pub_ts0_ < 0) pub_ts0_ = a.dts;
      return u32(std::max<i64>(0, (a.dts - pub_ts0_) / 90));
    };
    if (rising || pub_->messages() == 0) {
      // start the stream at a keyframe: sequence header + the whole current GOP
      if (ps_.complete()) pub_->send_sequence_header(ps_);
      for (auto& p : gop_) pub_->send_au(*p, ts_ms(*p));
    } else {
      pub_->send_au(*au, ts_ms(*au));
    }
    std::lock_guard<std::mutex> g(mu_);
    st_.rtmp_messages = pub_->messages();
    st_.rtmp_error.clear();
  } catch (const std::exception& e) {
    log(true, std::string("failed muxing: ") + e.what());
    pub_.reset();
    pub_retry_at_ = mono_us() / 1000 + 2000;
    std::lock_guard<std::mutex> g(mu_);
    st_.rtmp_error = e.what();
  }
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
