// Shared ingest machinery. See ioloop.h.
#include "ioloop.h"

#include "fanout.h"
#include "hostplan.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <fcntl.h>
#include <sched.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <unistd.h>

namespace vep {

// ------------------------------------------------------------------------------ TaskQueue

TaskQueue::TaskQueue(int threads, std::function<void()> init) {
  for (int i = 0; i < std::max(1, threads); ++i) th_.emplace_back([this, init] {
    name_thread("vep-task");
    if (init) init();
    run();
  });
}

TaskQueue::~TaskQueue() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
    q_.clear();  // queued tasks are dropped (their owners are gone, see IngestServices)
  }
  cv_.notify_all();
  for (auto& t : th_) t.join();
}

void TaskQueue::post(std::function<void()> fn) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stop_) return;
    q_.push_back(std::move(fn));
  }
  cv_.notify_one();
}

void TaskQueue::run() {
  std::unique_lock<std::mutex> g(mu_);
  for (;;) {
    cv_.wait(g, [this] { return stop_ || !q_.empty(); });
    if (stop_) return;
    std::function<void()> fn = std::move(q_.front());
    q_.pop_front();
    g.unlock();
    try {
      fn();
    } catch (...) {
    }
    g.lock();
  }
}

// ------------------------------------------------------------------------------ StrandPool

StrandPool::StrandPool(int threads, std::function<void()> init) {
  for (int i = 0; i < std::max(1, threads); ++i) th_.emplace_back([this, i, init] {
    name_thread("vep-parse");
    if (init) init();
    run(i);
  });
}

StrandPool::~StrandPool() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : th_) t.join();
}

size_t StrandPool::post(u64 key, std::function<void()> fn) {
  size_t depth;
  {
    std::lock_guard<std::mutex> g(mu_);
    Strand& s = strands_[key];
    s.q.push_back(std::move(fn));
    if (!s.running && s.q.size() == 1) ready_.push_back(key);
    depth = s.q.size() + (s.running ? 1 : 0);
  }
  cv_.notify_one();
  return depth;
}

size_t StrandPool::depth(u64 key) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = strands_.find(key);
  return it == strands_.end() ? 0 : it->second.q.size() + (it->second.running ? 1 : 0);
}

void StrandPool::drain(u64 key) {
  std::unique_lock<std::mutex> g(mu_);
  idle_cv_.wait(g, [&] {
    auto it = strands_.find(key);
    return it == strands_.end() || (it->second.q.empty() && !it->second.running);
  });
}

void StrandPool::run(int me) {
  // ready keys considered for affinity (VEP_STRAND_AFFINITY=0: plain FIFO)
  static const size_t kAffinityScan = [] {
    const char* e = std::getenv("VEP_STRAND_AFFINITY");
    return e && e[0] == '0' ? size_t(0) : size_t(8);
  }();
  std::unique_lock<std::mutex> g(mu_);
  for (;;) {
    cv_.wait(g, [this] { return stop_ || !ready_.empty(); });
    if (stop_) return;
    size_t pick = 0;
    for (size_t i = 0; i < ready_.size() && i < kAffinityScan; ++i) {
      auto o = owner_.find(ready_[i]);
      if (o != owner_.end() && o->second == me) {
        pick = i;
        break;
      }
    }
    const u64 key = ready_[pick];
    ready_.erase(ready_.begin() + std::ptrdiff_t(pick));
    owner_[key] = me;
    Strand& s = strands_[key];
    if (s.q.empty()) continue;
    s.running = true;
    std::function<void()> fn = std::move(s.q.front());
    s.q.pop_front();
    g.unlock();
    try {
      fn();
    } catch (...) {
    }
    g.lock();
    Strand& s2 = strands_[key];
    s2.running = false;
    if (!s2.q.empty()) {
      ready_.push_back(key);
      cv_.notify_one();
    } else {
      strands_.erase(key);
      owner_.erase(key);  // an idle key keeps no affinity (camera addresses get reused)
      idle_cv_.notify_all();
    }
  }
}

// ------------------------------------------------------------------------------ TimerQueue

TimerQueue::TimerQueue(TaskQueue& exec, std::function<void()> init) : exec_(exec) { th_ = std::thread([this, init] {
    name_thread("vep-timer");
    if (init) init();
    run();
  });
}

TimerQueue::~TimerQueue() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  th_.join();
}

void TimerQueue::at(i64 due_ms, std::function<void()> fn) {
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.emplace(due_ms, std::move(fn));
  }
  cv_.notify_all();
}

void TimerQueue::run() {
  std::unique_lock<std::mutex> g(mu_);
  while (!stop_) {
    if (q_.empty()) {
      cv_.wait(g);
      continue;
    }
    const i64 now = mono_us() / 1000;
    auto it = q_.begin();
    if (it->first > now) {
      cv_.wait_for(g, std::chrono::milliseconds(it->first - now));
      continue;
    }
    std::function<void()> fn = std::move(it->second);
    q_.erase(it);
    exec_.post(std::move(fn));
  }
}

// ------------------------------------------------------------------------------ IoLoop

IoLoop::IoLoop(int threads, std::function<void()> init) {
  for (int i = 0; i < std::max(1, threads); ++i) {
    auto l = std::make_unique<Loop>();
    l->ep = ::epoll_create1(EPOLL_CLOEXEC);
    l->wake = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    VEP_CHECK(l->ep >= 0 && l->wake >= 0, "epoll / eventfd creation failed");
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.ptr = nullptr;  // the wake-up fd
    ::epoll_ctl(l->ep, EPOLL_CTL_ADD, l->wake, &ev);
    loops_.push_back(std::move(l));
  }
  for (auto& l : loops_) {
    Loop* lp = l.get();
    l->th = std::thread([this, lp, init] {
      name_thread("vep-io");
      if (init) init();
      run(*lp);
    });
  }
}

IoLoop::~IoLoop() {
  stop_ = true;
  for (auto& l : loops_) {
    const u64 one = 1;
    (void)!::write(l->wake, &one, sizeof(one));
  }
  for (auto& l : loops_) {
    l->th.join();
    ::close(l->ep);
    ::close(l->wake);
  }
}

size_t IoLoop::handlers() const {
  size_t n = 0;
  for (auto& l : loops_) {
    std::lock_guard<std::mutex> g(l->mu);
    n += l->live.size();
  }
  return n;
}

void IoLoop::add(int fd, const std::shared_ptr<IoHandler>& h) {
  const int k = int(next_.fetch_add(1) % u32(loops_.size()));
  Loop& l = *loops_[size_t(k)];
  const int fl = ::fcntl(fd, F_GETFL, 0);
  ::fcntl(fd, F_SETFL, fl | O_NONBLOCK);
  {
    std::lock_guard<std::mutex> hg(h->mu_);
    h->fd_ = fd;
    h->loop_ = k;
    h->gone_ = false;
  }
  {
    std::lock_guard<std::mutex> g(l.mu);
    l.live[h.get()] = h;
  }
  epoll_event ev{};
  ev.events = EPOLLIN | EPOLLRDHUP;
  ev.data.ptr = h.get();
  VEP_CHECK(::epoll_ctl(l.ep, EPOLL_CTL_ADD, fd, &ev) == 0, "epoll_ctl ADD failed");
  // bytes the handshake already buffered: have the loop read once right away
  {
    std::lock_guard<std::mutex> g(l.mu);
    l.first.push_back(h);
  }
  const u64 one = 1;
  (void)!::write(l.wake, &one, sizeof(one));
}

void IoLoop::remove(const std::shared_ptr<IoHandler>& h) {
  if (!h) return;
  int k;
  {
    std::lock_guard<std::mutex> hg(h->mu_);  // waits for a callback in progress
    k = h->loop_;
    if (!h->gone_) {
      h->gone_ = true;
      if (h->fd_ >= 0) ::epoll_ctl(loops_[size_t(k)]->ep, EPOLL_CTL_DEL, h->fd_, nullptr);
    }
  }
  Loop& l = *loops_[size_t(k)];
  std::lock_guard<std::mutex> g(l.mu);
  l.live.erase(h.get());
}

void IoLoop::pause_reading(IoHandler& h) {  // (the loop thread holds h.mu_)
  if (h.gone_ || h.fd_ < 0) return;
  epoll_event ev{};
  ev.events = EPOLLRDHUP;  // still told when the peer goes away
  ev.data.ptr = &h;
  ::epoll_ctl(loops_[size_t(h.loop_)]->ep, EPOLL_CTL_MOD, h.fd_, &ev);
}

void IoLoop::resume_reading(const std::shared_ptr<IoHandler>& h) {
  if (!h) return;
  std::lock_guard<std::mutex> hg(h->mu_);
  if (h->gone_ || h->fd_ < 0) return;  // removed: the fd may already belong to someone else
  epoll_event ev{};
  ev.events = EPOLLIN | EPOLLRDHUP;
  ev.data.ptr = h.get();
  ::epoll_ctl(loops_[size_t(h->loop_)]->ep, EPOLL_CTL_MOD, h->fd_, &ev);
}

void IoLoop::dispatch(Loop& l, const std::shared_ptr<IoHandler>& h, bool readable) {
  bool closed = false;
  {
    std::lock_guard<std::mutex> hg(h->mu_);
    if (h->gone_) return;
    bool ok = false;
    try {
      ok = readable ? h->on_readable() : h->on_tick();
    } catch (...) {
      ok = false;
    }
    if (!ok) {
      h->gone_ = true;
      ::epoll_ctl(l.ep, EPOLL_CTL_DEL, h->fd_, nullptr);
      closed = true;
      try {
        h->on_closed();
      } catch (...) {
      }
    }
  }
  if (closed) {
    std::lock_guard<std::mutex> g(l.mu);
    l.live.erase(h.get());
  }
}

void IoLoop::run(Loop& l) {
  epoll_event evs[64];
  i64 last_tick = mono_us();
  while (!stop_.load()) {
    const int n = ::epoll_wait(l.ep, evs, 64, 100);
    for (int i = 0; i < n; ++i) {
      if (!evs[i].data.ptr) {  // wake-up
        u64 v;
        while (::read(l.wake, &v, sizeof(v)) > 0) {
        }
        continue;
      }
      std::shared_ptr<IoHandler> h;
      {
        std::lock_guard<std::mutex> g(l.mu);
        auto it = l.live.find(static_cast<IoHandler*>(evs[i].data.ptr));
        if (it != l.live.end()) h = it->second;
      }
      if (h) dispatch(l, h, true);
    }
    std::vector<std::shared_ptr<IoHandler>> first;
    {
      std::lock_guard<std::mutex> g(l.mu);
      first.swap(l.first);
    }
    for (auto& h : first) dispatch(l, h, true);
    const i64 now = mono_us();
    if (now - last_tick >= 200'000) {
      last_tick = now;
      std::vector<std::shared_ptr<IoHandler>> all;
      {
        std::lock_guard<std::mutex> g(l.mu);
        for (auto& kv : l.live) all.push_back(kv.second);
      }
      for (auto& h : all) dispatch(l, h, false);
    }
  }
}

// ------------------------------------------------------------------------------ services

static int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::max(1, std::atoi(v)) : dflt;
}

IngestServices::IngestServices(int io_threads, int parse_threads, int connect_threads)
    : io(io_threads), parse(parse_threads), connect(connect_threads), timers(connect),
      parse_threads(std::max(1, parse_threads)), io_threads(std::max(1, io_threads)) {}

// (the fan-out pool helps the parse strands with a picture's slices / tiles / WPP rows: the same
// CPUs, one thread fewer so a strand's own share of the work is not displaced)
IngestServices::IngestServices(const HostDomain& d)
    : fan(std::make_unique<FanOut>(std::max(0, d.parse_threads - 1), domain_thread_init(d, nullptr))),
      io(d.io_threads, domain_thread_init(d, nullptr)),
      parse(d.parse_threads, domain_thread_init(d, fan.get())),
      connect(env_int("VEP_CONNECT_THREADS", 4), domain_thread_init(d, nullptr)),
      timers(connect, domain_thread_init(d, nullptr)),
      parse_threads(std::max(1, d.parse_threads)),
      io_threads(std::max(1, d.io_threads)) {}

IngestServices::~IngestServices() = default;

// Host CPUs this process may use: its affinity mask, bounded by a cgroup v2 CPU quota.
int cpu_budget() {
  int n = 1;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof set, &set) == 0) n = std::max(1, CPU_COUNT(&set));
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char quota[32] = {0};
    long period = 0;
    if (std::fscanf(f, "%31s %ld", quota, &period) == 2 && std::strcmp(quota, "max") != 0 && period > 0)
      n = std::min(n, int(std::max(1L, (std::atol(quota) + period - 1) / period)));
    std::fclose(f);
  }
  return n;
}

std::shared_ptr<IngestServices> IngestServices::acquire() {
  static std::mutex mu;
  static std::weak_ptr<IngestServices> cur;
  std::lock_guard<std::mutex> g(mu);
  if (auto s = cur.lock()) return s;
  // parse strands: the process's CPU budget minus the socket loops and the GPU launcher (no
  // constant cap: a GPU worker with a host domain sizes its own pool, hostplan.h)
  const int parse_default = std::max(2, cpu_budget() - 2);
  auto s = std::make_shared<IngestServices>(env_int("VEP_IO_THREADS", 2),
                                            env_int("VEP_INGEST_PARSE_THREADS", parse_default),
                                            env_int("VEP_CONNECT_THREADS", 4));
  cur = s;
  return s;
}

}  // namespace vep
