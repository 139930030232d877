// Host benchmark of the general HEVC decoder: encodes a synthetic camera stream once, then
// decodes it several times and reports ms per picture (best pass) and the phase split.
//   hevc_bench [width] [height] [frames] [bframes] [qp] [records]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "sampler.h"
#include "vep/hevc_dec.h"

using namespace vep;

int main(int argc, char** argv) {
  hevc::HevcEncConfig c;
  c.width = argc > 1 ? std::atoi(argv[1]) : 1920;
  c.height = argc > 2 ? std::atoi(argv[2]) : 1080;
  const int frames = argc > 3 ? std::atoi(argv[3]) : 16;
  c.bframes = argc > 4 ? std::atoi(argv[4]) : 2;
  c.qp = argc > 5 ? std::atoi(argv[5]) : 27;
  c.gop = 32;
  c.temporal_noise = 2.0;
  // BENCH=1: the bench's camera streams (bench.py --codec h265: QP 25, texture noise 8, sensor
  // noise 1.5, 8 slices per picture at 4K)
  if (std::getenv("BENCH")) {
    c.qp = argc > 5 ? std::atoi(argv[5]) : 25;
    c.noise = 8.0;
    c.temporal_noise = 1.5;
    c.slices = c.width * c.height >= 3840 * 2160 ? 8 : 1;
  }
  hevc::HevcEncoder enc(c);
  std::vector<std::shared_ptr<AccessUnit>> aus;
  size_t bytes = 0;
  for (int i = 0; i < frames; ++i) {
    aus.push_back(enc.next());
    bytes += aus.back()->bytes();
  }
  const bool records = argc > 6 && std::string(argv[6]) == "records";  // parse only (GPU mode)
  if (const char* p = std::getenv("PROF")) {
    sampler::run(std::atof(p), [&] {
      hevc::Decoder d;
      d.set_gpu_mode(records);
      for (auto& a : aus) {
        d.decode(*a);
        d.take_gpu_pictures();
      }
      d.flush();
    });
    return 0;
  }
  double best = 1e30;
  for (int pass = 0; pass < 5; ++pass) {
    hevc::Decoder d;
    d.set_gpu_mode(records);
    const auto t0 = std::chrono::steady_clock::now();
    for (auto& a : aus) {
      d.decode(*a);
      d.take_gpu_pictures();
    }
    d.flush();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    best = std::min(best, ms);
  }
  std::printf("%dx%d %d frames (%zu bytes/frame): %.2f ms/picture\n", c.width, c.height, frames, bytes / frames,
              best / frames);
  return 0;
}
