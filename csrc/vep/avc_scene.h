// Synthetic camera scene shared by the synthetic H.264 encoders (avc_enc.cpp CAVLC Baseline,
// avc_enc_high.cpp Main/High): a static textured background with moving textured objects
// (rectangles / ellipses bouncing off the frame edges) and optional per-frame sensor noise — the
// kind of content a fixed IP camera sends, so motion search, skip, direct and residual decisions
// behave as on real footage. The object motion is known, which seeds the encoders' motion search.
#pragma once

#include <algorithm>
#include <cmath>

#include "codec.h"

namespace vep::avc {

struct Rng {
  u64 s;
  u64 next() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  }
  int uni(int n) { return int(next() % u64(n)); }
  bool chance(int pct) { return uni(100) < pct; }
};

inline u32 hash2(u32 x, u32 y, u32 seed) {
  u32 h = x * 0x8da6b343u ^ y * 0xd8163841u ^ seed * 0xcb1ab31fu;
  h ^= h >> 13;
  h *= 0x5bd1e995u;
  h ^= h >> 15;
  return h;
}

inline u8 sat8(double v) { return u8(v < 0 ? 0 : v > 255 ? 255 : int(v + 0.5)); }

// ---- encoder toolkit shared by the synthetic encoders: 4x4 forward core transform and the
// deadzone quantiser (MF tables of the reference encoder design; intra f = 1/3, inter 1/6)
inline constexpr int kMF[6][3] = {{13107, 5243, 8066}, {11916, 4660, 7490}, {10082, 4194, 6554},
                       {9362, 3647, 5825},  {8192, 3355, 5243},  {7282, 2893, 4559}};

inline int mf_class(int pos) {
  const int i = pos >> 2, j = pos & 3;
  return (!(i & 1) && !(j & 1)) ? 0 : ((i & 1) && (j & 1)) ? 1 : 2;
}

// Forward core transform W = Cf X Cf^T (raster in, raster out).
inline void fwd4x4(const int* x, int* w) {
  int t[16];
  for (int i = 0; i < 4; ++i) {
    const int a = x[i * 4], b = x[i * 4 + 1], c = x[i * 4 + 2], d = x[i * 4 + 3];
    const int s03 = a + d, d03 = a - d, s12 = b + c, d12 = b - c;
    t[i * 4] = s03 + s12;
    t[i * 4 + 1] = 2 * d03 + d12;
    t[i * 4 + 2] = s03 - s12;
    t[i * 4 + 3] = d03 - 2 * d12;
  }
  for (int j = 0; j < 4; ++j) {
    const int a = t[j], b = t[4 + j], c = t[8 + j], d = t[12 + j];
    const int s03 = a + d, d03 = a - d, s12 = b + c, d12 = b - c;
    w[j] = s03 + s12;
    w[4 + j] = 2 * d03 + d12;
    w[8 + j] = s03 - s12;
    w[12 + j] = d03 - 2 * d12;
  }
}

inline int quant(int w, int qp, int cls, bool intra, int extra_shift = 0) {
  const int qbits = 15 + qp / 6 + extra_shift;
  const int f = (1 << qbits) / (intra ? 3 : 6);
  const long long a = (static_cast<long long>(w < 0 ? -w : w) * kMF[qp % 6][cls] + f) >> qbits;
  const int l = int(a > 2047 ? 2047 : a);
  return w < 0 ? -l : l;
}


struct SceneConfig {
  int width, height;  // visible size
  int wpx, hpx;       // coded (MB-aligned) size
  int objects;
  double noise;           // background texture amplitude
  double temporal_noise;  // per-frame sensor noise amplitude
  u64 seed;
};

class Scene {
 public:
  struct Obj {
    double x, y, vx, vy;
    int w, h;
    bool ellipse;
    double p1, p2, p3;
    int by, bu, bv;
  };
  HostSurface bg, src;
  std::vector<Obj> objs;

  void make(const SceneConfig& c, Rng& rng) {
    cfg_ = c;
    const int wpx = c.wpx, hpx = c.hpx;
    bg.alloc(wpx, hpx);
    src.alloc(wpx, hpx);
    const u32 seed = u32(c.seed * 2654435761u);
    for (int y = 0; y < hpx; ++y)
      for (int x = 0; x < wpx; ++x) {
        const double v = 70 + 60 * (0.5 + 0.5 * std::sin(x * 0.011 + y * 0.004 + seed % 7)) +
                         40.0 * y / hpx + c.noise * ((hash2(u32(x), u32(y), seed) & 255) / 128.0 - 1.0);
        bg.y[size_t(y) * wpx + x] = sat8(v);
      }
    for (int y = 0; y < hpx / 2; ++y)
      for (int x = 0; x < wpx / 2; ++x) {
        bg.uv[size_t(y) * wpx + 2 * x] = sat8(128 + 25 * std::sin(x * 0.02 + seed % 5));
        bg.uv[size_t(y) * wpx + 2 * x + 1] = sat8(128 + 25 * std::cos(y * 0.017 + seed % 3));
      }
    const double speeds[] = {0.75, 1.25, 2.0, 2.5, 3.25, 1.0, 4.5};
    for (int i = 0; i < c.objects; ++i) {
      Obj o;
      o.w = std::max(16, c.width / (4 + rng.uni(5)));
      o.h = std::max(16, c.height / (4 + rng.uni(5)));
      o.x = rng.uni(std::max(1, c.width - o.w));
      o.y = rng.uni(std::max(1, c.height - o.h));
      o.vx = speeds[rng.uni(7)] * (rng.uni(2) ? 1 : -1);
      o.vy = speeds[rng.uni(7)] * (rng.uni(2) ? 1 : -1) * 0.5;
      o.ellipse = rng.uni(2);
      o.p1 = 0.05 + rng.uni(100) * 0.003;
      o.p2 = 0.04 + rng.uni(100) * 0.003;
      o.p3 = 0.02 + rng.uni(100) * 0.002;
      o.by = 60 + rng.uni(140);
      o.bu = 90 + rng.uni(80);
      o.bv = 90 + rng.uni(80);
      objs.push_back(o);
    }
  }

  bool inside(const Obj& o, double lx, double ly) const {
    if (lx < 0 || ly < 0 || lx >= o.w || ly >= o.h) return false;
    if (!o.ellipse) return true;
    const double dx = (lx - o.w / 2.0) / (o.w / 2.0), dy = (ly - o.h / 2.0) / (o.h / 2.0);
    return dx * dx + dy * dy <= 1.0;
  }

  void render() {
    const int wpx = cfg_.wpx;
    src.y = bg.y;
    src.uv = bg.uv;
    for (const Obj& o : objs) {
      const int x0 = std::max(0, int(std::floor(o.x))), y0 = std::max(0, int(std::floor(o.y)));
      const int x1 = std::min(cfg_.width, int(std::ceil(o.x + o.w)) + 1);
      const int y1 = std::min(cfg_.height, int(std::ceil(o.y + o.h)) + 1);
      for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) {
          const double lx = x - o.x, ly = y - o.y;
          if (!inside(o, lx, ly)) continue;
          src.y[size_t(y) * wpx + x] =
              sat8(o.by + 50 * std::sin(lx * o.p1) * std::cos(ly * o.p2) + 25 * std::sin((lx + ly) * o.p3));
        }
      for (int y = y0 / 2; y < (y1 + 1) / 2; ++y)
        for (int x = x0 / 2; x < (x1 + 1) / 2; ++x) {
          const double lx = 2 * x - o.x, ly = 2 * y - o.y;
          if (!inside(o, lx, ly)) continue;
          src.uv[size_t(y) * wpx + 2 * x] = sat8(o.bu + 20 * std::sin(lx * o.p2));
          src.uv[size_t(y) * wpx + 2 * x + 1] = sat8(o.bv + 20 * std::cos(ly * o.p1));
        }
    }
  }

  void add_sensor_noise(i64 frame) {
    if (cfg_.temporal_noise <= 0) return;
    const u32 seed = u32(frame * 0x9E3779B1u) ^ u32(cfg_.seed);
    const int amp = int(cfg_.temporal_noise * 2) + 1;
    for (int y = 0; y < cfg_.hpx; ++y)
      for (int x = 0; x < cfg_.wpx; ++x) {
        u8& p = src.y[size_t(y) * cfg_.wpx + x];
        const int n = int(hash2(u32(x), u32(y), seed) % u32(amp)) - amp / 2;
        p = u8(std::min(255, std::max(0, p + n)));
      }
  }

  void advance() {
    for (Obj& o : objs) {
      o.x += o.vx;
      o.y += o.vy;
      if (o.x < -o.w / 2.0 || o.x + o.w / 2.0 > cfg_.width) o.vx = -o.vx;
      if (o.y < -o.h / 2.0 || o.y + o.h / 2.0 > cfg_.height) o.vy = -o.vy;
    }
  }

 private:
  SceneConfig cfg_{};
};

}  // namespace vep::avc
