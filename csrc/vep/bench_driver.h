// Replay driver for the headline benchmark: every camera of a worker decodes one access unit
// per step (a "frame tick"). Host MB-layer parsing runs continuously on its own threads, each
// camera's frames in order, up to `window` ticks ahead of the tick being launched, so one
// camera's long keyframe parse overlaps the other cameras' next frames instead of stalling a
// per-tick barrier (the live path parses on arrival in the same way).
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
  // records = true: the GPU-side ceiling (bench.py --source records). Every camera's cached
  // access units are parsed up front — two passes over the GOPs, the second one kept, so its
  // jobs carry the steady-state DPB / output bookkeeping of a looped stream — and step()
  // replays those reconstruction jobs (records in pinned memory, gathered over PCIe by the GPU
  // as in the live path) with no host parse in the loop.
  ReplayBench(Worker& w, int ncams, const SynthConfig& base, int cached_frames, int threads,
              int ring_slots, const std::string& prefix, int window = 2, bool records = false);
  ~ReplayBench();
  void step();      // takes the next parsed tick and launches it (publishes tick t - stages)
  void drain();     // publish every launched tick
  // Bring the parse pipeline to rest before a timed region: stop parse threads from starting
  // new ticks, let every camera finish the ticks already started, launch (untimed) every tick
  // parsed so far and drain the GPU. The next step() re-opens parsing, so no tick of the timed
  // region is parsed before it starts.
  void quiesce();
  // jobs whose parse failed (dropped before the GPU); the worker counts its own drops
  u64 parse_failures() const { return parse_fail_; }
  // Host parse throughput alone: consume `ticks` parsed ticks without GPU work (jobs dropped)
  // and return the mean wall ms per tick.
  double parse_only_ms(int ticks);
  u64 frames() const { return frames_; }
  u64 bitstream_bytes() const { return bytes_; }
  // size of the replayed streams (all cameras' cached AUs)
  u64 stream_bytes() const { return stream_bytes_; }
  u64 stream_frames() const { return stream_frames_; }
  // parse work (sum over frames) divided by the parse threads: the parse stage's busy time
  double parse_ms() const { return double(parse_ns_.load()) / 1e6 / double(workers_.size()); }
  double parse_wait_ms() const { return wait_us_ / 1000.0; }  // step() blocked on parsing
  double batch_ms() const { return batch_us_ / 1000.0; }
  const std::vector<int>& cameras() const { return cams_; }

 private:
  struct Tick {
    std::vector<DecodeJob> jobs;
    std::vector<char> ok;
    int done = 0;
  };
  void parse_loop(int me);
  int pick_locked(int me) const;  // a camera allowed to parse its next tick, or -1
  std::vector<DecodeJob> take(bool timed);
  Worker& w_;
  std::vector<int> cams_;
  std::vector<std::vector<AuPtr>> aus_;
  std::vector<size_t> pos_;
  const int window_;
  std::vector<Tick> ring_;      // tick T in slot T % window_
  i64 consume_ = 0;             // next tick step() takes
  i64 gate_ = INT64_MAX;        // parse threads start only ticks < gate_ (quiesce)
  std::vector<i64> cam_tick_;   // next tick each camera parses
  std::vector<char> cam_busy_;
  std::vector<int> cam_thread_;  // parse thread that last parsed each camera (cache affinity)
  bool stop_ = false;
  std::mutex mu_;
  std::condition_variable work_cv_, ready_cv_;
  std::vector<std::thread> workers_;
  u64 frames_ = 0, bytes_ = 0, parse_fail_ = 0;
  std::atomic<u64> stream_bytes_{0}, stream_frames_{0}, parse_ns_{0};
  // records mode: per camera the parsed jobs of one cycle of its GOPs, replayed in order
  bool records_ = false;
  std::vector<std::vector<DecodeJob>> rec_;
  std::vector<size_t> rec_pos_;
  double wait_us_ = 0, batch_us_ = 0;
};

}  // namespace vep
