// Host emulation of avc_hbd_kernel's per-MB functions (gpu_avc_hbd.hip: intra prediction + loop
// filter of High 10 / 4:2:2 pictures) under AddressSanitizer: every MB of real pictures (the
// synthetic High encoder's coverage streams, parsed by avc::Decoder) runs lane by lane in the
// kernel's diagonal order against exactly-sized buffers, so an access outside the picture, the
// records, the bS array or the residual slots is reported by ASan instead of faulting a GPU.
// (Sample values are not checked here: lanes run one after another, so a lane may read a tile
// cell another lane writes later. Bit-exactness is the GPU tests' job.)
//
//   hipcc -std=c++17 -O1 -g -Xarch_host -fsanitize=address -fno-gpu-sanitize --offload-host-only -Icsrc \
//     csrc/tests/hbd_emu.cpp csrc/vep/{avc_enc_high,avc_mb,avc_cabac,avc_cavlc,avc,h264,codec,
//     fanout,hostmem,hostplan,hevc,ioloop}.cpp -o build/hbd_emu -lpthread
#include <algorithm>
#include <cstdio>
#include <vector>

#include "../vep/avc.h"
#include "../vep/synth.h"
#define VEP_HBD_EMU 1
#include "../vep/gpu_avc_hbd.hip"

using namespace vep;
using vep::gpu::AvcDbkInfo;
using vep::gpu::AvcDesc;

// avc_bs_kernel's derivation (gpu_avc.hip), for the filter pass's bS
static void bs_info(const avc::Picture& pic, int cf, std::vector<AvcDbkInfo>& out) {
  const int W = pic.wmbs;
  out.assign(size_t(pic.nmbs()), AvcDbkInfo{});
  static const i16 kZero[64] = {};
  for (int mb = 0; mb < pic.nmbs(); ++mb) {
    const avc::MbRec& q = pic.mbs[size_t(mb)];
    AvcDbkInfo info{};
    const int x = mb % W, row = mb / W;
    if (!(q.dbk & 1)) {
      const avc::MbRec& lm = x > 0 ? pic.mbs[size_t(mb - 1)] : q;
      const avc::MbRec& tm = row > 0 ? pic.mbs[size_t(mb - W)] : q;
      const bool left = x > 0 && !((q.dbk & 2) && lm.slice != q.slice);
      const bool top = row > 0 && !((q.dbk & 2) && tm.slice != q.slice);
      auto mvs = [&](const avc::MbRec& r) { return avc::is_intra(r.kind) ? kZero : &pic.mvs[size_t(r.mv)]; };
      const bool t8 = (q.flags & avc::kMbT8x8) != 0;
      for (int dir = 0; dir < 2; ++dir)
        for (int e = 0; e < 4; ++e) {
          if (e == 0 && !(dir == 0 ? left : top)) continue;
          if ((e & 1) && t8 && !(cf == 2 && dir == 1)) continue;
          const avc::MbRec& p = e > 0 ? q : (dir == 0 ? lm : tm);
          for (int sg = 0; sg < 4; ++sg) {
            const int bq = dir == 0 ? sg * 4 + e : e * 4 + sg;
            const int bp = e > 0 ? (dir == 0 ? bq - 1 : bq - 4) : (dir == 0 ? bq + 3 : bq + 12);
            const int bs = avc::boundary_strength(p, bp, mvs(p), q, bq, mvs(q), e == 0, false, dir == 0);
            const int i = dir * 16 + e * 4 + sg;
            info.bs[i >> 3] |= u32(bs) << (4 * (i & 7));
          }
        }
      info.any = (info.bs[0] | info.bs[1] | info.bs[2] | info.bs[3]) ? 1 : 0;
      const avc::MbRec* ps[3] = {&lm, &tm, &q};
      for (int k = 0; k < 3; ++k) {
        const avc::EdgeParams ep[3] = {
            avc::edge_params(ps[k]->qp - pic.qp_bias, q.qp - pic.qp_bias, q.alpha_off, q.beta_off),
            avc::edge_params(ps[k]->qpc - pic.qpc_bias, q.qpc - pic.qpc_bias, q.alpha_off, q.beta_off),
            avc::edge_params(ps[k]->qpc2 - pic.qpc_bias, q.qpc2 - pic.qpc_bias, q.alpha_off, q.beta_off)};
        for (int c = 0; c < 3; ++c) {
          info.alpha[c * 3 + k] = u8(ep[c].alpha);
          info.beta[c * 3 + k] = u8(ep[c].beta);
          for (int j = 0; j < 3; ++j) info.tc0[c * 3 + k][j] = u8(ep[c].tc0[j]);
        }
      }
    }
    out[size_t(mb)] = info;
  }
}

template <class P, int CF>
static int run_picture(const avc::Picture& pic, bool half = false) {
  const int W = pic.wmbs, H = pic.hmbs, ch = CF == 2 ? 16 : 8;
  const size_t ny = size_t(W) * 16 * H * 16, nuv = size_t(W) * 16 * H * ch;
  const int slots = pic.dpb_slots;
  // exactly-sized buffers (ASan redzones at both ends)
  std::vector<P> y(ny * size_t(slots), P(64)), uv(nuv * size_t(slots), P(512));
  std::vector<i16> res(size_t(pic.intra_res) * gpu::kAvcResSamples + 1, 0);
  std::vector<AvcDbkInfo> dbk;
  bs_info(pic, CF, dbk);
  std::vector<avc::MbRec> mbs(pic.mbs.begin(), pic.mbs.end());
  u32 err = 0;
  AvcDesc d{};
  d.mbs = mbs.data();
  d.y = reinterpret_cast<u8*>(y.data());
  d.uv = reinterpret_cast<u8*>(uv.data());
  d.slot_y = ny * sizeof(P);
  d.slot_uv = nuv * sizeof(P);
  d.wmbs = W;
  d.hmbs = H;
  d.target = pic.target;
  d.constrained = pic.constrained_intra ? 1 : 0;
  d.err = &err;
  d.dbk = dbk.data();
  d.res = res.data();
  d.bd = pic.bd;
  d.qp_bias = pic.qp_bias;
  d.qpc_bias = pic.qpc_bias;
  d.cf = pic.cf;
  d.ncoef = u32(pic.coefs.size());
  d.nres = u32(pic.intra_res);
  d.intra_mbs = pic.intra_mbs;
  d.deblock = pic.deblock ? 1 : 0;
  gpu::HbdWave L{};
  const int steps = W + 2 * (H - 1);
  for (int pass = 0; pass < 2; ++pass)
    for (int t = 0; t < steps; ++t) {
      const int ylo = std::max(0, (t - W + 2) >> 1), yhi = std::min(H - 1, t >> 1);
      for (int yy = ylo; yy <= yhi; ++yy) {
        const int mb = yy * W + t - 2 * yy;
        for (int lane = 0; lane < 64; ++lane) {
          if (pass == 0) gpu::intra_mb<P, CF>(d, L, mb, lane);
          else if (half) gpu::deblock_mb<P, CF, 32>(d, L.db, mb, lane & 31, true);
          else gpu::deblock_mb<P, CF>(d, L.db, mb, lane);
        }
      }
    }
  return int(err);
}

// filter_samples_u (the GPU loop filter's one-stream form) against filter_samples, random lines
static int check_filter_u() {
  u64 st = 88172645463325252ull;
  auto rnd = [&](int n) {
    st ^= st << 13, st ^= st >> 7, st ^= st << 17;
    return int(st % u64(n));
  };
  int bad = 0;
  for (int it = 0; it < 2000000; ++it) {
    const int bd = 8 + rnd(3), maxv = (1 << bd) - 1, bs = 1 + rnd(4), chroma = rnd(2);
    const int base = rnd(maxv + 1), spread = 1 + rnd(40 << (bd - 8));
    int p[4], q[4], p2[4], q2[4];
    for (int k = 0; k < 4; ++k) {
      p[k] = p2[k] = std::min(maxv, std::max(0, base + rnd(2 * spread + 1) - spread));
      q[k] = q2[k] = std::min(maxv, std::max(0, base + rnd(2 * spread + 1) - spread));
    }
    const int ia = rnd(52), sh = bd - 8;
    const int alpha = avc::kAlpha[ia] << sh, beta = avc::kBeta[rnd(52)] << sh, tc0 = avc::kTc0[ia][rnd(3)] << sh;
    const bool a = avc::filter_samples(p, q, bs, alpha, beta, tc0, chroma, bd);
    const bool b = avc::filter_samples_u(p2, q2, bs, alpha, beta, tc0, chroma, bd);
    for (int k = 0; k < 4; ++k) bad += a != b || p[k] != p2[k] || q[k] != q2[k];
  }
  return bad;
}

int main() {
  int worst = 0, pics = 0;
  const int fbad = check_filter_u();
  std::printf("filter_samples_u vs filter_samples: %d mismatches\n", fbad);
  if (fbad) return 1;
  for (int variant = 0; variant < 3; ++variant)
    for (int seed = 1; seed <= 3; ++seed) {
      avc::AvcHighConfig c;
      c.width = 176;
      c.height = 144;
      c.gop = 8;
      c.bframes = 2;
      c.coverage = true;
      c.seed = u64(seed);
      c.slices = seed;
      c.deblock_idc = seed == 3 ? 2 : 0;
      c.bit_depth = variant == 1 ? 8 : 10;
      c.chroma_format = variant == 0 ? 1 : 2;
      avc::AvcHighEncoder enc(c);
      avc::Decoder dec;
      for (int i = 0; i < 12; ++i) {
        auto au = enc.next();
        auto pic = dec.parse(*au, 0, nullptr);
        int e;
        if (variant == 0) e = run_picture<u16, 1>(*pic) | run_picture<u16, 1>(*pic, true);
        else if (variant == 1) e = run_picture<u8, 2>(*pic) | run_picture<u8, 2>(*pic, true);
        else e = run_picture<u16, 2>(*pic) | run_picture<u16, 2>(*pic, true);
        ++pics;
        if (e) std::printf("variant %d seed %d picture %d: bound-check bits 0x%x\n", variant, seed, i, e);
        worst |= e;
      }
    }
  // the GPU tests' camera streams (tests/test_avc_422.py, test_avc_high10.py: SynthConfig)
  struct Cam { int bd, cf, bframes, slices, dbk; bool cabac, wp; };
  const Cam cams[] = {{8, 2, 2, 2, 0, true, false}, {8, 2, 1, 1, 0, false, true}, {10, 2, 2, 3, 2, true, false},
                      {10, 1, 2, 2, 0, true, false}, {9, 1, 2, 3, 2, true, false}};
  for (const Cam& k : cams) {
    SynthConfig sc;
    sc.width = 176;
    sc.height = 144;
    sc.gop = 8;
    sc.codec = Codec::kH264;
    sc.compressed = true;
    sc.profile = "high";
    sc.coverage = true;
    sc.bframes = k.bframes;
    sc.slices = k.slices;
    sc.deblock_idc = k.dbk;
    sc.cabac = k.cabac;
    sc.weighted_p = k.wp;
    sc.weighted_b = k.wp ? 1 : 0;
    sc.bit_depth = k.bd;
    sc.chroma_format = k.cf;
    SynthH264 s(sc);
    avc::Decoder dec;
    for (int i = 0; i < 14; ++i) {
      auto au = s.next();
      {
        auto pic = dec.parse(*au, 0, nullptr);
        if (!pic) continue;
        int e;
        if (k.cf != 2) e = run_picture<u16, 1>(*pic) | run_picture<u16, 1>(*pic, true);
        else if (k.bd == 8) e = run_picture<u8, 2>(*pic) | run_picture<u8, 2>(*pic, true);
        else e = run_picture<u16, 2>(*pic) | run_picture<u16, 2>(*pic, true);
        ++pics;
        if (e) std::printf("camera bd %d cf %d picture %d: bound-check bits 0x%x\n", k.bd, k.cf, i, e);
        worst |= e;
      }
    }
  }
  std::printf("hbd_emu: %d pictures, bound-check bits 0x%x\n", pics, worst);
  return 0;
}
