// Host parse profile driver (gprof / perf): encodes a 1080p High-profile CABAC IBBP GOP with the
// synthetic camera encoder (the headline bench's stream) and parses it repeatedly with the
// general H.264 decoder — the per-picture host cost that bounds the headline rate.
//   make parse-prof && cd /tmp && /root/repo/build/prof/parse_prof 20 && gprof ...
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "vep/avc.h"
#include "vep/synth.h"

int main(int argc, char** argv) {
  using namespace vep;
  const int reps = argc > 1 ? std::atoi(argv[1]) : 10;
  SynthConfig c;
  c.width = 1920;
  c.height = 1080;
  c.fps = 30;
  c.gop = 30;
  c.compressed = true;
  c.qp = 25;
  c.noise = 8.0;
  c.temporal_noise = 1.5;
  c.profile = "high";
  c.bframes = 2;
  c.cabac = true;
  c.seed = 1;
  SynthH264 enc(c);
  std::vector<std::shared_ptr<AccessUnit>> aus;
  for (int i = 0; i < 30; ++i) aus.push_back(enc.next());
  double best = 1e30;
  for (int r = 0; r < reps; ++r) {
    avc::Decoder dec;
    const auto t0 = std::chrono::steady_clock::now();
    for (const auto& au : aus) dec.parse(*au);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    best = s < best ? s : best;
  }
  std::printf("parse ms/picture (best of %d): %.3f\n", reps, best / 30 * 1e3);
  return 0;
}
