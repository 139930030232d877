// Poor man's sampling profiler for the host benchmarks (no perf in the image): SIGPROF every
// ms of CPU time records the interrupted instruction address; the histogram goes to
// parse_prof.txt for tools/parse_prof_report.py (llvm-symbolizer, inlined frames). Build the
// profiled binary with -g -no-pie (absolute addresses).
#pragma once
#include <signal.h>
#include <sys/time.h>
#include <ucontext.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <map>

namespace sampler {

constexpr int kMaxSamples = 1 << 20;
inline uintptr_t g_samples[kMaxSamples];
inline std::atomic<int> g_nsamples{0};
inline volatile bool g_on = true;  // samples are recorded only while set (a body may gate phases)

inline void on_prof(int, siginfo_t*, void* uc) {
  if (!g_on) return;
  const int i = g_nsamples.fetch_add(1, std::memory_order_relaxed);
  if (i < kMaxSamples) g_samples[i] = uintptr_t(static_cast<ucontext_t*>(uc)->uc_mcontext.gregs[REG_RIP]);
}

// Runs `body` repeatedly for `seconds` of wall time under the sampler.
template <class F>
void run(double seconds, F&& body) {
  struct sigaction sa {};
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigaction(SIGPROF, &sa, nullptr);
  itimerval it{{0, 1000}, {0, 1000}};
  setitimer(ITIMER_PROF, &it, nullptr);
  const auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < seconds) body();
  itimerval off{};
  setitimer(ITIMER_PROF, &off, nullptr);
  std::map<uintptr_t, int> hist;
  const int n = std::min(g_nsamples.load(), kMaxSamples);
  for (int i = 0; i < n; ++i) ++hist[g_samples[i]];
  FILE* f = std::fopen("parse_prof.txt", "w");
  for (auto& [a, c] : hist) std::fprintf(f, "%d 0x%lx\n", c, (unsigned long)a);
  std::fclose(f);
  std::printf("profile: %d samples -> parse_prof.txt\n", n);
}

}  // namespace sampler
