// Replay driver implementation. See bench_driver.h.
#include "bench_driver.h"

#include <algorithm>

#include "trace.h"

namespace vep {

ReplayBench::ReplayBench(Worker& w, int ncams, const SynthConfig& base, int cached_frames,
                         int threads, int ring_slots, const std::string& prefix)
    : w_(w), pool_(threads) {
  VEP_CHECK(ncams > 0, "bench needs at least one camera");
  const int gop = std::max(1, base.gop);
  const int nframes = std::max(gop, (cached_frames + gop - 1) / gop * gop);
  aus_.resize(size_t(ncams));
  pos_.assign(size_t(ncams), 0);
  for (int i = 0; i < ncams; ++i)
    cams_.push_back(w_.add_camera(prefix + std::to_string(i), ring_slots));
  pool_.parallel_for(ncams, [&](int i) {
    SynthConfig c = base;
    c.seed = base.seed + u64(i) * 7919u;
    c.idr_phase = base.idr_phase + (i * gop) / ncams;  // unsynchronised cameras
    SynthH264 enc(c);
    auto& v = aus_[size_t(i)];
    v.reserve(size_t(nframes));
    for (int f = 0; f < nframes; ++f) {
      auto au = enc.next();
      au->pin();  // as the RTSP depacketizer does: ingest-side copy into the pinned pool
      stream_bytes_ += au->bytes();
      stream_frames_ += 1;
      v.push_back(au);
    }
  });
  pf_ = std::thread([this] { prefetch_loop(); });
}

ReplayBench::~ReplayBench() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (pf_.joinable()) pf_.join();
}

void ReplayBench::parse_tick(std::vector<DecodeJob>& out) {
  trace::Range tr("vep.parse_tick");
  const int n = int(cams_.size());
  out.clear();
  out.resize(size_t(n));
  std::vector<char> ok(size_t(n), 0);
  // largest-first (LPT) order: a keyframe's parse starts at once instead of trailing the tick
  std::vector<int> order(static_cast<size_t>(n));
  for (int i = 0; i < n; ++i) order[size_t(i)] = i;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    return aus_[size_t(a)][pos_[size_t(a)]]->bytes() > aus_[size_t(b)][pos_[size_t(b)]]->bytes();
  });
  pool_.parallel_for(n, [&](int t) {
    const int i = order[size_t(t)];
    auto& v = aus_[size_t(i)];
    const AuPtr& au = v[pos_[size_t(i)]];
    pos_[size_t(i)] = (pos_[size_t(i)] + 1) % v.size();
    auto c = w_.camera(cams_[size_t(i)]);
    ok[size_t(i)] = c && c->make_job(au, out[size_t(i)]);
  });
  size_t k = 0;
  for (int i = 0; i < n; ++i) {
    if (!ok[size_t(i)]) continue;
    if (size_t(i) != k) out[k] = std::move(out[size_t(i)]);
    ++k;
  }
  out.resize(k);
}

double ReplayBench::parse_only_ms(int ticks) {
  drain();
  std::lock_guard<std::mutex> g(mu_);  // keeps the prefetch thread idle
  std::vector<DecodeJob> jobs;
  const i64 t0 = mono_us();
  for (int t = 0; t < ticks; ++t) parse_tick(jobs);
  return double(mono_us() - t0) / 1000.0 / std::max(1, ticks);
}

void ReplayBench::prefetch_loop() {
  std::vector<DecodeJob> jobs;
  for (;;) {
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [&] { return stop_ || want_; });
      if (stop_) return;
    }
    const i64 t0 = mono_us();
    parse_tick(jobs);
    const i64 t1 = mono_us();
    {
      std::lock_guard<std::mutex> g(mu_);
      parse_us_ += double(t1 - t0);
      ready_.swap(jobs);
      have_ready_ = true;
      want_ = false;
    }
    cv_.notify_all();
  }
}

void ReplayBench::step() {
  std::vector<DecodeJob> jobs;
  {
    std::unique_lock<std::mutex> g(mu_);
    if (!have_ready_ && !want_) {
      want_ = true;
      cv_.notify_all();
    }
    cv_.wait(g, [&] { return have_ready_; });
    jobs.swap(ready_);
    have_ready_ = false;
    want_ = true;  // start parsing tick t+1 while tick t runs on the GPU
  }
  cv_.notify_all();
  for (auto& j : jobs) {
    bytes_ += u64(j.upd.nslots) * kPcmMbBytes;
    for (const auto& p : j.avc) bytes_ += u64(p->coefs.size()) * 2 + p->mbs.size() * sizeof(avc::MbRec);
  }
  const i64 t0 = mono_us();
  const size_t n = jobs.size();
  w_.launch_async(jobs);  // publishes tick t-2; ticks t-1 and t stay in flight
  batch_us_ += double(mono_us() - t0);
  frames_ += n;
}

void ReplayBench::drain() {
  {
    std::unique_lock<std::mutex> g(mu_);
    cv_.wait(g, [&] { return !want_; });
  }
  w_.complete_all();
}

}  // namespace vep
