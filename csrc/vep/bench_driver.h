// Replay driver for the headline benchmark: every camera of a worker decodes one access unit
// per step (a "frame tick"). Host MB-layer parsing of tick t+1 is fanned out over a thread pool
// and overlaps the batched GPU launch of tick t (software pipelining across ticks).
//
// The AUs are real H.264 bitstreams from the synthetic camera (synth.h), pre-encoded once per
// camera (a whole number of GOPs) and replayed cyclically; parsing, reconstruction, colour
// conversion, ring publish and letterboxing all run inside every timed step.
#pragma once

#include <condition_variable>
#include <thread>

#include "pool.h"
#include "runtime.h"
#include "synth.h"

namespace vep {

class ReplayBench {
 public:
  ReplayBench(Worker& w, int ncams, const SynthConfig& base, int cached_frames, int threads,
              int ring_slots, const std::string& prefix);
  ~ReplayBench();
  void step();      // blocks until the tick's frames are published
  void drain();     // wait for any prefetch in flight
  // Host parse cost alone: run `ticks` parse ticks (no GPU work, jobs dropped) and return the
  // mean wall ms per tick, split into the parallel parse and the job-vector compaction.
  double parse_only_ms(int ticks);
  u64 frames() const { return frames_; }
  u64 bitstream_bytes() const { return bytes_; }
  // size of the replayed streams (all cameras' cached AUs)
  u64 stream_bytes() const { return stream_bytes_; }
  u64 stream_frames() const { return stream_frames_; }
  double parse_ms() const { return parse_us_ / 1000.0; }
  double batch_ms() const { return batch_us_ / 1000.0; }
  const std::vector<int>& cameras() const { return cams_; }

 private:
  void parse_tick(std::vector<DecodeJob>& out);
  void prefetch_loop();
  Worker& w_;
  std::vector<int> cams_;
  std::vector<std::vector<AuPtr>> aus_;
  std::vector<size_t> pos_;
  ThreadPool pool_;
  std::vector<DecodeJob> ready_;
  bool have_ready_ = false, want_ = false, stop_ = false;
  std::mutex mu_;
  std::condition_variable cv_;
  std::thread pf_;
  u64 frames_ = 0, bytes_ = 0;
  std::atomic<u64> stream_bytes_{0}, stream_frames_{0};
  double parse_us_ = 0, batch_us_ = 0;
};

}  // namespace vep
