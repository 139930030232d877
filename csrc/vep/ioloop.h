// Shared ingest machinery: camera sockets are served by a few epoll threads
// instead of one blocking thread per camera, bitstream parsing runs on a separate strand pool
// (per-camera FIFO, one thread at a time per camera), and RTSP handshakes / reconnect back-off run
// on a small connector pool driven by a timer. A stalled or slow camera therefore holds no
// network thread, and the parse budget is a fixed pool instead of 256 competing ingest threads.
//
// Reference behaviour being replaced: one Docker container + Python process per camera
// (python/rtsp_to_rtmp.py:49-187, server/services/rtsp_process_manager.go:50-150).
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "common.h"

namespace vep {

// Host CPUs this process may use: its affinity mask, bounded by a cgroup v2 CPU quota.
int cpu_budget();

// Fixed thread pool running posted tasks in FIFO order.
class TaskQueue {
 public:
  // init (optional) runs first on every pool thread (host domain pinning, hostplan.h)
  explicit TaskQueue(int threads, std::function<void()> init = {});
  ~TaskQueue();
  void post(std::function<void()> fn);

 private:
  void run();
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false;
};

// Per-key serial execution on a shared pool: tasks of one key run in posting order, never two at
// once; different keys run in parallel. A free thread prefers a ready key it ran last (the
// camera's decoder state is still in that core's caches) among the oldest few ready keys.
class StrandPool {
 public:
  explicit StrandPool(int threads, std::function<void()> init = {});
  ~StrandPool();
  // Returns the number of tasks of `key` queued or running after this post.
  size_t post(u64 key, std::function<void()> fn);
  size_t depth(u64 key) const;
  // Block until every task of `key` posted so far has finished.
  void drain(u64 key);
  int threads() const { return int(th_.size()); }

 private:
  struct Strand {
    std::deque<std::function<void()>> q;
    bool running = false;  // a thread owns the strand (running its front task)
  };
  void run(int me);
  std::vector<std::thread> th_;
  mutable std::mutex mu_;
  std::condition_variable cv_, idle_cv_;
  std::map<u64, Strand> strands_;
  std::map<u64, int> owner_;  // thread that last ran each key
  std::deque<u64> ready_;  // keys with queued tasks and no owner
  bool stop_ = false;
};

// One-shot timers executed on a TaskQueue.
class TimerQueue {
 public:
  explicit TimerQueue(TaskQueue& exec, std::function<void()> init = {});
  ~TimerQueue();
  void at(i64 due_ms, std::function<void()> fn);  // mono_us() / 1000 clock

 private:
  void run();
  TaskQueue& exec_;
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::multimap<i64, std::function<void()>> q_;
  bool stop_ = false;
};

// A socket served by the IoLoop. A handler belongs to one loop thread, so its callbacks are
// serialised, and none runs after IoLoop::remove() returned.
class IoHandler {
 public:
  virtual ~IoHandler() = default;
  // Data (or EOF / error) on the socket; false ends the registration (then on_closed()).
  virtual bool on_readable() = 0;
  // About every 200 ms between reads; false ends the registration.
  virtual bool on_tick() = 0;
  // The registration ended because a callback returned false (not called after remove()).
  virtual void on_closed() = 0;

 private:
  friend class IoLoop;
  std::mutex mu_;      // held by the loop thread during a callback and by remove()
  bool gone_ = false;  // removed or closed: no further callbacks
  int fd_ = -1;
  int loop_ = 0;
};

class IoLoop {
 public:
  explicit IoLoop(int threads, std::function<void()> init = {});
  ~IoLoop();
  // The fd must stay open until remove() / on_closed(). on_readable() runs once right away
  // (bytes may already be buffered by a handshake).
  void add(int fd, const std::shared_ptr<IoHandler>& h);
  // Synchronous: when it returns no callback of `h` is running or will run.
  void remove(const std::shared_ptr<IoHandler>& h);
  // Flow control: stop / restart read notifications of `h` (ticks continue). pause_reading()
  // may only be called from inside a callback of `h`; resume_reading() from any other thread.
  void pause_reading(IoHandler& h);
  void resume_reading(const std::shared_ptr<IoHandler>& h);
  int threads() const { return int(loops_.size()); }
  size_t handlers() const;

 private:
  struct Loop {
    int ep = -1;
    int wake = -1;  // eventfd
    std::thread th;
    std::mutex mu;
    std::map<IoHandler*, std::shared_ptr<IoHandler>> live;
    std::vector<std::shared_ptr<IoHandler>> first;  // added: read once right away
  };
  void run(Loop& l);
  void dispatch(Loop& l, const std::shared_ptr<IoHandler>& h, bool readable);
  std::vector<std::unique_ptr<Loop>> loops_;
  std::atomic<bool> stop_{false};
  std::atomic<u32> next_{0};
};

// Ingest services of one host domain (hostplan.h): the GPU worker's socket loops, parse strands,
// intra-picture fan-out pool and connector, every thread pinned to the domain's CPUs. A Worker
// with a host domain owns its services (Worker::ingest_services); acquire() is the process-wide
// default for workers without one (created with the first session, destroyed with the last;
// sizes VEP_IO_THREADS (2), VEP_INGEST_PARSE_THREADS (CPU budget - 2), VEP_CONNECT_THREADS (4)).
struct IngestServices {
  std::unique_ptr<class FanOut> fan;  // the domain's fan-out pool (null: the process-wide one)
  IoLoop io;
  StrandPool parse;
  TaskQueue connect;
  TimerQueue timers;
  int parse_threads = 0, io_threads = 0;
  IngestServices(int io_threads, int parse_threads, int connect_threads);
  explicit IngestServices(const struct HostDomain& d);
  ~IngestServices();
  static std::shared_ptr<IngestServices> acquire();
};

}  // namespace vep
