// Host-only self test of the general H.264 path: encoder -> bitstream -> decoder -> CPU
// reconstruction must equal the encoder's closed-loop reconstruction, frame by frame.
//   hipcc -std=c++17 -O2 -Icsrc csrc/tests/avc_selftest.cpp csrc/vep/avc*.cpp csrc/vep/h264.cpp
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "../vep/avc.h"

using namespace vep;

static double psnr(const HostSurface& a, const HostSurface& b, int w, int h) {
  double se = 0;
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const double d = double(a.y[size_t(y) * a.coded_w + x]) - b.y[size_t(y) * b.coded_w + x];
      se += d * d;
    }
  const double mse = se / (double(w) * h);
  return mse == 0 ? 99.0 : 10 * std::log10(255.0 * 255.0 / mse);
}

int main(int argc, char** argv) {
  avc::AvcEncConfig c;
  c.width = argc > 1 ? std::atoi(argv[1]) : 176;
  c.height = argc > 2 ? std::atoi(argv[2]) : 144;
  const int frames = argc > 3 ? std::atoi(argv[3]) : 12;
  c.coverage = argc > 4 ? std::atoi(argv[4]) != 0 : true;
  c.refs = argc > 5 ? std::atoi(argv[5]) : 3;
  c.slices = argc > 6 ? std::atoi(argv[6]) : 2;
  c.deblock_idc = argc > 7 ? std::atoi(argv[7]) : 0;
  c.gop = 8;
  c.pcm_rate = 5;
  c.nonref_rate = 20;
  c.alpha_off = 1;
  c.beta_off = -1;
  avc::AvcEncoder enc(c);
  avc::Decoder dec;
  std::vector<HostSurface> slots(17);
  size_t bytes = 0;
  for (int f = 0; f < frames; ++f) {
    auto au = enc.next();
    bytes += au->bytes();
    auto pic = dec.parse(*au);
    for (int s = 0; s < pic->dpb_slots; ++s)
      if (slots[s].coded_w != pic->wmbs * 16) slots[s].alloc(pic->wmbs * 16, pic->hmbs * 16);
    avc::cpu_reconstruct(*pic, slots);
    const HostSurface& got = slots[size_t(pic->target)];
    const HostSurface& want = enc.reconstruction();
    size_t diff = 0;
    for (size_t i = 0; i < got.y.size(); ++i) diff += got.y[i] != want.y[i];
    for (size_t i = 0; i < got.uv.size(); ++i) diff += got.uv[i] != want.uv[i];
    std::printf("frame %d %c bytes=%zu intra=%d inter=%d diff=%zu psnr=%.2f\n", f, pic->info.pict_type,
                au->bytes(), pic->intra_mbs, pic->inter_mbs, diff,
                psnr(got, enc.source(), c.width, c.height));
    if (diff) return 1;
  }
  std::printf("ok %zu bytes\n", bytes);
  return 0;
}
