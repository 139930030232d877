// See hostprof.h.
#include "hostprof.h"

#include <dlfcn.h>
#include <signal.h>
#include <sys/time.h>
#include <ucontext.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <map>
#include <vector>

#include "common.h"

namespace vep::hostprof {

namespace {

constexpr int kMaxSamples = 1 << 21;
std::vector<uintptr_t> g_samples;  // sized before the handler is installed
std::atomic<int> g_n{0};

void on_prof(int, siginfo_t*, void* uc) {  // async-signal-safe: one atomic add and one store
  const int i = g_n.fetch_add(1, std::memory_order_relaxed);
  if (i < kMaxSamples) g_samples[size_t(i)] = uintptr_t(static_cast<ucontext_t*>(uc)->uc_mcontext.gregs[REG_RIP]);
}

}  // namespace

void start(int interval_us) {
  g_samples.assign(size_t(kMaxSamples), 0);
  g_n.store(0);
  struct sigaction sa {};
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  VEP_CHECK(sigaction(SIGPROF, &sa, nullptr) == 0, "hostprof: sigaction failed");
  const int us = std::max(100, interval_us);
  itimerval it{{0, us}, {0, us}};
  VEP_CHECK(setitimer(ITIMER_PROF, &it, nullptr) == 0, "hostprof: setitimer failed");
}

int stop(const std::string& path) {
  itimerval off{};
  setitimer(ITIMER_PROF, &off, nullptr);
  signal(SIGPROF, SIG_IGN);
  const int n = std::min(g_n.load(), kMaxSamples);
  std::map<uintptr_t, int> hist;
  for (int i = 0; i < n; ++i) ++hist[g_samples[size_t(i)]];
  FILE* f = std::fopen(path.c_str(), "w");
  VEP_CHECK(f, "hostprof: cannot write " + path);
  for (const auto& [a, c] : hist) {
    Dl_info info{};
    if (dladdr(reinterpret_cast<void*>(a), &info) && info.dli_fname) {
      std::fprintf(f, "%d %s 0x%lx %s\n", c, info.dli_fname, (unsigned long)(a - uintptr_t(info.dli_fbase)),
                   info.dli_sname ? info.dli_sname : "?");
    } else {
      std::fprintf(f, "%d ? 0x%lx ?\n", c, (unsigned long)a);
    }
  }
  std::fclose(f);
  g_samples.clear();
  g_samples.shrink_to_fit();
  return n;
}

}  // namespace vep::hostprof
