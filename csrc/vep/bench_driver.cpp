// Replay driver implementation. See bench_driver.h.
#include "bench_driver.h"

#include <algorithm>
#include <chrono>

#include "trace.h"

namespace vep {

ReplayBench::ReplayBench(Worker& w, int ncams, const SynthConfig& base, int cached_frames,
                         int threads, int ring_slots, const std::string& prefix, int window, bool records)
    : w_(w), window_(std::max(1, window)), records_(records) {
  VEP_CHECK(ncams > 0, "bench needs at least one camera");
  const int gop = std::max(1, base.gop);
  const int nframes = std::max(gop, (cached_frames + gop - 1) / gop * gop);
  aus_.resize(size_t(ncams));
  pos_.assign(size_t(ncams), 0);
  for (int i = 0; i < ncams; ++i)
    cams_.push_back(w_.add_camera(prefix + std::to_string(i), ring_slots));
  {
    ThreadPool enc_pool(std::max(1, threads));
    enc_pool.parallel_for(ncams, [&](int i) {
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
  }
  ring_.resize(size_t(window_));
  for (Tick& t : ring_) {
    t.jobs.resize(size_t(ncams));
    t.ok.assign(size_t(ncams), 0);
  }
  cam_tick_.assign(size_t(ncams), 0);
  cam_busy_.assign(size_t(ncams), 0);
  cam_thread_.assign(size_t(ncams), -1);
  if (records_) {  // parse everything now (two cycles, keep the second): no parse threads
    rec_.resize(size_t(ncams));
    rec_pos_.assign(size_t(ncams), 0);
    ThreadPool parse_pool(std::max(1, threads));
    parse_pool.parallel_for(ncams, [&](int i) {
      auto cam = w_.camera(cams_[size_t(i)]);
      const auto& v = aus_[size_t(i)];
      for (int cycle = 0; cycle < 2; ++cycle)
        for (const AuPtr& au : v) {
          DecodeJob job;
          bool ok = false;
          try {
            ok = cam && cam->make_job(au, job);
          } catch (const std::exception&) {
            ok = false;
          }
          if (cycle == 1 && ok) rec_[size_t(i)].push_back(std::move(job));
        }
      VEP_CHECK(!rec_[size_t(i)].empty(), "records replay: no job parsed");
    });
    // one untimed cycle: the IDR of the first replayed cycle outputs the previous cycle's last
    // pictures from the reorder buffer, so those must have been reconstructed once
    size_t longest = 0;
    for (const auto& r : rec_) longest = std::max(longest, r.size());
    for (size_t k = 0; k < longest; ++k) step();
    w_.complete_all();
    frames_ = bytes_ = 0;
    batch_us_ = 0;
    return;
  }
  for (int i = 0; i < std::max(1, threads); ++i) workers_.emplace_back([this, i] {
    name_thread("vep-bparse");
    parse_loop(i);
  });
}

ReplayBench::~ReplayBench() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  work_cv_.notify_all();
  for (auto& t : workers_) t.join();
}

int ReplayBench::pick_locked(int me) const {
  // A camera's decoder state (neighbour state, record pools: a few MB per 1080p camera) stays
  // in the caches of the core that parsed its last picture; taking it on another core costs a
  // cross-core transfer of every line it touches. So: a camera at the oldest tick (the one the
  // launcher waits for) first, preferring this thread's own; then this thread's cameras; then
  // any other, oldest tick first; within equal rank the largest AU first (a keyframe starts at
  // once).
  int best = -1, best_rank = 0;
  for (int c = 0; c < int(cams_.size()); ++c) {
    const size_t k = size_t(c);
    if (cam_busy_[k] || cam_tick_[k] >= consume_ + window_ || cam_tick_[k] >= gate_) continue;
    const bool mine = cam_thread_[k] == me || cam_thread_[k] < 0;
    const int rank = (cam_tick_[k] == consume_ ? 0 : 2) + (mine ? 0 : 1);
    if (best < 0 || rank < best_rank ||
        (rank == best_rank && (cam_tick_[k] < cam_tick_[size_t(best)] ||
                               (cam_tick_[k] == cam_tick_[size_t(best)] &&
                                aus_[k][pos_[k]]->bytes() > aus_[size_t(best)][pos_[size_t(best)]]->bytes())))) {
      best = c;
      best_rank = rank;
    }
  }
  return best;
}

void ReplayBench::parse_loop(int me) {
  std::unique_lock<std::mutex> g(mu_);
  for (;;) {
    int c = -1;
    work_cv_.wait(g, [&] { return stop_ || (c = pick_locked(me)) >= 0; });
    if (stop_) return;
    const i64 t = cam_tick_[size_t(c)];
    cam_busy_[size_t(c)] = 1;
    cam_thread_[size_t(c)] = me;
    auto& v = aus_[size_t(c)];
    const AuPtr au = v[pos_[size_t(c)]];
    pos_[size_t(c)] = (pos_[size_t(c)] + 1) % v.size();
    g.unlock();
    DecodeJob job;
    bool ok = false;
    const auto t0 = std::chrono::steady_clock::now();
    {
      trace::Range tr("vep.parse");
      try {
        auto cam = w_.camera(cams_[size_t(c)]);
        ok = cam && cam->make_job(au, job);
      } catch (const std::exception&) {
        ok = false;  // the camera logs its own decode errors; the frame is dropped
      }
    }
    const auto ns = std::chrono::duration_cast<std::chrono::nanoseconds>(
        std::chrono::steady_clock::now() - t0).count();
    parse_ns_ += u64(ns);
    g.lock();
    Tick& k = ring_[size_t(t % window_)];
    k.jobs[size_t(c)] = std::move(job);
    k.ok[size_t(c)] = ok ? 1 : 0;
    cam_tick_[size_t(c)] = t + 1;
    cam_busy_[size_t(c)] = 0;
    if (++k.done == int(cams_.size()) || gate_ != INT64_MAX) ready_cv_.notify_all();
  }
}

std::vector<DecodeJob> ReplayBench::take(bool timed) {
  std::vector<DecodeJob> out;
  std::unique_lock<std::mutex> g(mu_);
  Tick& k = ring_[size_t(consume_ % window_)];
  const i64 t0 = mono_us();
  ready_cv_.wait(g, [&] { return k.done == int(cams_.size()); });
  if (timed) wait_us_ += double(mono_us() - t0);
  out.reserve(cams_.size());
  for (size_t i = 0; i < cams_.size(); ++i) {
    if (k.ok[i]) out.push_back(std::move(k.jobs[i]));
    else ++parse_fail_;
    k.jobs[i] = DecodeJob{};
    k.ok[i] = 0;
  }
  k.done = 0;
  ++consume_;  // frees the slot for tick consume_ + window_ - 1
  g.unlock();
  work_cv_.notify_all();
  return out;
}

double ReplayBench::parse_only_ms(int ticks) {
  VEP_CHECK(!records_, "parse_only_ms: records mode has no parse");
  drain();
  const i64 t0 = mono_us();
  for (int t = 0; t < ticks; ++t) (void)take(false);
  return double(mono_us() - t0) / 1000.0 / std::max(1, ticks);
}

void ReplayBench::quiesce() {
  if (records_) {
    w_.complete_all();
    return;
  }
  i64 upto;
  {
    std::unique_lock<std::mutex> g(mu_);
    upto = consume_;
    for (size_t c = 0; c < cams_.size(); ++c) upto = std::max(upto, cam_tick_[c] + (cam_busy_[c] ? 1 : 0));
    gate_ = upto;  // no camera starts a tick >= upto; the ones behind catch up to it
  }
  work_cv_.notify_all();
  while (true) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (consume_ >= upto) break;
    }
    std::vector<DecodeJob> jobs = take(false);
    w_.launch_async(jobs);
  }
  {
    std::unique_lock<std::mutex> g(mu_);
    ready_cv_.wait(g, [&] {
      for (size_t c = 0; c < cams_.size(); ++c)
        if (cam_busy_[c]) return false;
      return true;
    });
  }
  w_.complete_all();
}

void ReplayBench::step() {
  if (records_) {  // the next recorded job of every camera (a copy: the records are shared)
    std::vector<DecodeJob> jobs;
    jobs.reserve(rec_.size());
    for (size_t c = 0; c < rec_.size(); ++c) {
      jobs.push_back(rec_[c][rec_pos_[c]]);
      rec_pos_[c] = (rec_pos_[c] + 1) % rec_[c].size();
    }
    for (auto& j : jobs)
      for (const auto& p : j.avc) bytes_ += u64(p->coefs.size()) * 2 + p->mbs.size() * sizeof(avc::MbRec);
    const i64 t0 = mono_us();
    const size_t n = jobs.size();
    w_.launch_async(jobs);
    batch_us_ += double(mono_us() - t0);
    frames_ += n;
    return;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    if (gate_ != INT64_MAX) gate_ = INT64_MAX;  // re-open parsing (after quiesce)
  }
  work_cv_.notify_all();
  std::vector<DecodeJob> jobs = take(true);
  for (auto& j : jobs) {
    bytes_ += u64(j.upd.nslots) * kPcmMbBytes;
    for (const auto& p : j.avc) bytes_ += u64(p->coefs.size()) * 2 + p->mbs.size() * sizeof(avc::MbRec);
  }
  const i64 t0 = mono_us();
  const size_t n = jobs.size();
  w_.launch_async(jobs);  // publishes tick t - stages; the ticks after it stay in flight
  batch_us_ += double(mono_us() - t0);
  frames_ += n;
}

void ReplayBench::drain() { w_.complete_all(); }

}  // namespace vep
