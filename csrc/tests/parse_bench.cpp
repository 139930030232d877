// Host-only H.264 parse benchmark: encodes a synthetic 1080p stream with the closed-loop encoder
// (High: CABAC IBBP + 8x8; baseline: CAVLC I/P), then times avc::Decoder::parse (entropy layer +
// dequantisation + MB records, no sample reconstruction) over it. Used with gprof
// (`make parse-prof`) to find the parse hot spots that bound the bench.
#include <signal.h>
#include <sys/time.h>
#include <ucontext.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <algorithm>
#include <cstring>

#include "sampler.h"
#include "vep/avc.h"
#include "vep/cabac.h"

using namespace vep;



int main(int argc, char** argv) {
  const bool high = argc < 2 || std::strcmp(argv[1], "baseline") != 0;
  const int frames = argc > 2 ? std::atoi(argv[2]) : 30;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 5;
  std::vector<std::shared_ptr<AccessUnit>> aus;
  if (high) {
    avc::AvcHighConfig c;
    c.width = 1920;
    c.height = 1080;
    c.qp = 25;
    c.noise = 8.0;
    c.temporal_noise = 1.5;
    c.refs = 1;  // the headline bench's streams (bench.py --refs 1, 1080p High, QP 25)
    avc::AvcHighEncoder e(c);
    for (int i = 0; i < frames; ++i) aus.push_back(e.next());
  } else {
    avc::AvcEncConfig c;
    c.width = 1920;
    c.height = 1080;
    c.qp = 27;
    c.noise = 8.0;
    c.temporal_noise = 1.0;
    avc::AvcEncoder e(c);
    for (int i = 0; i < frames; ++i) aus.push_back(e.next());
  }
  size_t bytes = 0;
  for (auto& a : aus) bytes += a->bytes();
  if (const char* p = std::getenv("PROF")) {
    // PROF_TYPE=P / B / I: sample only while pictures of that type are parsed
    const char* pt = std::getenv("PROF_TYPE");
    std::vector<char> types;
    {
      avc::Decoder d;
      for (auto& a : aus) types.push_back(d.parse(*a)->info.pict_type);
    }
    // PROF_CAMS=n: n decoders parse the stream interleaved (cold per-camera state, as the bench's
    // parse pool sees it)
    const int pc = std::getenv("PROF_CAMS") ? std::atoi(std::getenv("PROF_CAMS")) : 1;
    sampler::run(std::atof(p), [&] {
      std::vector<avc::Decoder> ds(static_cast<size_t>(std::max(1, pc)));
      std::vector<avc::PicturePtr> keep(ds.size() * 3);
      for (size_t i = 0; i < aus.size(); ++i)
        for (size_t c = 0; c < ds.size(); ++c) {
          sampler::g_on = !pt || types[i] == pt[0];
          keep[c * 3 + i % 3] = ds[c].parse(*aus[i]);
        }
      sampler::g_on = true;
    });
    return 0;
  }
  double best = 1e30;
  const int passes = std::getenv("PASSES") ? std::atoi(std::getenv("PASSES")) : 5;
  for (int round = 0; round < passes; ++round) {
    avc::Decoder d;
    const auto b0 = std::chrono::steady_clock::now();
    for (auto& a : aus) (void)d.parse(*a);
    best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - b0).count());
  }
  std::printf("best of %d passes: %.3f ms/frame\n", passes, best * 1e3 / frames);
  // several cameras interleaved on one thread (cold decoder state between pictures, as in the
  // bench's parse pool)
  const int ncam = argc > 4 ? std::atoi(argv[4]) : 0;
  if (ncam > 0) {
    double bestm = 1e30;
    for (int round = 0; round < 3; ++round) {
      std::vector<avc::Decoder> decs(static_cast<size_t>(ncam));
      std::vector<avc::PicturePtr> keep(static_cast<size_t>(ncam) * 3);
      const auto b0 = std::chrono::steady_clock::now();
      for (auto& a : aus)
        for (int c = 0; c < ncam; ++c) keep[size_t(c) * 3 + size_t(&a - &aus[0]) % 3] = decs[size_t(c)].parse(*a);
      bestm = std::min(bestm, std::chrono::duration<double>(std::chrono::steady_clock::now() - b0).count());
    }
    std::printf("%d cameras interleaved: %.3f ms/frame\n", ncam, bestm * 1e3 / (frames * ncam));
  }
  // per picture: the minimum over `reps` passes (robust to a noisy host), summed by type
  const auto t0 = std::chrono::steady_clock::now();
  size_t mbs = 0;
  std::vector<double> best_pic(aus.size(), 1e30);
  std::vector<double> bins_pic(aus.size(), 0.0);
  std::vector<int> type_pic(aus.size(), 0);
  u64 kinds[8] = {};
  for (int r = 0; r < reps; ++r) {
    avc::Decoder d;
    for (size_t i = 0; i < aus.size(); ++i) {
      const u64 bins0 = cabac::bins_decoded().load();
      const auto p0 = std::chrono::steady_clock::now();
      auto pic = d.parse(*aus[i]);
      const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - p0).count();
      best_pic[i] = std::min(best_pic[i], dt);
      bins_pic[i] = double(cabac::bins_decoded().load() - bins0);
      type_pic[i] = pic->info.pict_type == 'P' ? 0 : pic->info.pict_type == 'B' ? 1 : 2;
      mbs += size_t(pic->nmbs());
      if (r == 0)
        for (const auto& m : pic->mbs) ++kinds[m.kind & 7];
    }
  }
  double by_type[3] = {0, 0, 0}, bins_type[3] = {0, 0, 0}, sum_best = 0;
  int n_type[3] = {0, 0, 0};
  for (size_t i = 0; i < aus.size(); ++i) {
    by_type[type_pic[i]] += best_pic[i];
    bins_type[type_pic[i]] += bins_pic[i];
    n_type[type_pic[i]] += 1;
    sum_best += best_pic[i];
  }
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::printf("per-picture minimum over %d passes: %.3f ms/frame\n", reps, sum_best * 1e3 / double(aus.size()));
  for (int t = 0; t < 3; ++t)
    if (n_type[t])
      std::printf("  %c: %d pictures, %.3f ms/picture, %.0f bins/picture, %.2f ns/bin\n", "PBI"[t], n_type[t],
                  by_type[t] * 1e3 / n_type[t], bins_type[t] / n_type[t], by_type[t] * 1e9 / bins_type[t]);
  std::printf("  MB kinds (skip inter i4 i16 pcm i8): %llu %llu %llu %llu %llu %llu\n", (unsigned long long)kinds[0],
              (unsigned long long)kinds[1], (unsigned long long)kinds[2], (unsigned long long)kinds[3],
              (unsigned long long)kinds[4], (unsigned long long)kinds[5]);
  std::printf("%s: %d frames x %d, %.1f kB/frame, parse %.3f ms/frame (%.1f ns/MB)\n", high ? "high" : "baseline",
              frames, reps, bytes / 1e3 / frames, s * 1e3 / (frames * reps), s * 1e9 / double(mbs));
  return 0;
}
