// Test hooks of the HEVC reconstruction primitives (`_vep.hevc_recon`): the CPU reference
// (hevc_recon.h) and the per-sample functions the gfx950 kernels run (hevc_kern.h), for the
// independent spec oracle (tests/spec_oracle_hevc.py, tests/test_spec_oracle_hevc.py).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "bind_ext.h"
#include "vep/hevc_kern.h"
#include "vep/hevc_recon.h"

namespace py = pybind11;
using namespace vep;

void bind_hevc(py::module_& m) {
  auto h = m.def_submodule("hevc_recon", "HEVC reconstruction primitives (hevc_recon.h, hevc_kern.h)");
  // CPU reference inverse transform: scaled coefficients (raster n x n) -> residual
  // (bd: the sample bit depth, 8 or Main10's 9..10; sample planes of bd > 8 are passed as the
  // bytes of little-endian uint16 arrays)
  h.def("itx", [](const std::vector<int>& d, int log2, bool dst, bool tskip, int bd) {
    const int n = 1 << log2;
    VEP_CHECK(int(d.size()) == n * n && log2 >= 2 && log2 <= 5, "itx: n x n coefficients, log2 2..5");
    std::vector<i32> in(d.begin(), d.end()), out(size_t(n) * n);
    hevc::inverse_transform(in.data(), log2, dst, tskip, out.data(), bd);
    return std::vector<int>(out.begin(), out.end());
  }, py::arg("d"), py::arg("log2"), py::arg("dst"), py::arg("tskip"), py::arg("bd") = 8);
  // Kernel form: hk_itx_col / hk_itx_row (the coefficients must fit int16, as the records)
  h.def("itx_kern", [](const std::vector<int>& d, int log2, bool dst, int bd) {
    const int n = 1 << log2;
    VEP_CHECK(int(d.size()) == n * n && log2 >= 2 && log2 <= 5, "itx_kern: n x n coefficients");
    std::vector<i16> q(d.size());
    int mx = 0, my = 0;
    for (size_t k = 0; k < d.size(); ++k) {
      q[k] = i16(std::clamp(d[k], -32768, 32767));
      if (q[k]) mx = std::max(mx, int(k) % n), my = std::max(my, int(k) / n);
    }
    std::vector<int> g(size_t(n) * n), r(size_t(n) * n);
    for (int y = 0; y < n; ++y)
      for (int x = 0; x <= mx; ++x) g[size_t(y) * n + x] = hevc::hk_itx_col(q.data(), log2, dst, y, x, my);
    for (int y = 0; y < n; ++y)
      for (int x = 0; x < n; ++x) r[size_t(y) * n + x] = hevc::hk_itx_row(g.data() + size_t(y) * n, log2, dst, x, mx, bd);
    return r;
  }, py::arg("d"), py::arg("log2"), py::arg("dst"), py::arg("bd") = 8);
  h.def("dequant", [](int level, int qp, int log2, int m, int bd) { return hevc::dequant_level(level, qp, log2, m, bd); },
        py::arg("level"), py::arg("qp"), py::arg("log2"), py::arg("m") = 16, py::arg("bd") = 8);
  // CPU reference intra: references as the spec's p[x][-1] (x = -1 .. 2n-1) and p[-1][y]
  // (y = 0 .. 2n-1), already substituted; filtering (§8.4.4.2.3) then prediction.
  h.def("intra", [](std::vector<int> top, std::vector<int> left, int log2, int mode, bool luma, bool strong, int bd) {
    const int n = 1 << log2;
    VEP_CHECK(int(top.size()) == 2 * n + 1 && int(left.size()) == 2 * n, "intra: 2n + 1 top, 2n left samples");
    if (luma) hevc::filter_intra_refs(top.data(), left.data(), log2, mode, strong, bd);
    std::vector<u16> out(size_t(n) * n);
    hevc::intra_predict(top.data(), left.data(), log2, mode, luma, out.data(), n, true, bd);
    return std::vector<int>(out.begin(), out.end());
  }, py::arg("top"), py::arg("left"), py::arg("log2"), py::arg("mode"), py::arg("luma"), py::arg("strong"), py::arg("bd") = 8);
  // Kernel form: hk_prepare_refs (gather + substitution + filtering from a plane with an
  // availability mask) and hk_intra_sample. `plane` is a W x H luma plane (step 1).
  h.def("intra_kern", [](const std::string& plane, int W, int x0, int y0, int log2, bool luma, u64 avail, int mode,
                         bool strong, int bd) {
    const int n = 1 << log2;
    int top[129], left[128];
    if (bd > 8) {
      std::vector<u16> p(plane.size() / 2);
      std::memcpy(p.data(), plane.data(), p.size() * 2);
      hevc::hk_prepare_refs(p.data(), W, 1, x0, y0, log2, luma, avail, mode, strong, top, left, bd);
    } else {
      std::vector<u8> p(plane.begin(), plane.end());
      hevc::hk_prepare_refs(p.data(), W, 1, x0, y0, log2, luma, avail, mode, strong, top, left);
    }
    std::vector<int> out(size_t(n) * n);
    for (int y = 0; y < n; ++y)
      for (int x = 0; x < n; ++x) out[size_t(y) * n + x] = hevc::hk_intra_sample(top, left, log2, mode, luma, x, y, bd);
    return out;
  }, py::arg("plane"), py::arg("W"), py::arg("x0"), py::arg("y0"), py::arg("log2"), py::arg("luma"), py::arg("avail"),
     py::arg("mode"), py::arg("strong"), py::arg("bd") = 8);
  h.def("luma_mc", [](const std::string& plane, int W, int H, int xi, int yi, int fx, int fy, int bd) {
    if (bd > 8) return hevc::hk_luma_mc(reinterpret_cast<const u16*>(plane.data()), W, W, H, xi, yi, fx, fy, bd);
    return hevc::hk_luma_mc(reinterpret_cast<const u8*>(plane.data()), W, W, H, xi, yi, fx, fy);
  }, py::arg("plane"), py::arg("W"), py::arg("H"), py::arg("xi"), py::arg("yi"), py::arg("fx"), py::arg("fy"),
     py::arg("bd") = 8);
  // `uv`: interleaved Cb / Cr of a (W x H chroma) plane, stride 2 W
  h.def("chroma_mc", [](const std::string& uv, int W, int H, int c, int xi, int yi, int fx, int fy, int bd) {
    if (bd > 8) return hevc::hk_chroma_mc(reinterpret_cast<const u16*>(uv.data()), 2 * W, W, H, c, xi, yi, fx, fy, bd);
    return hevc::hk_chroma_mc(reinterpret_cast<const u8*>(uv.data()), 2 * W, W, H, c, xi, yi, fx, fy);
  }, py::arg("uv"), py::arg("W"), py::arg("H"), py::arg("c"), py::arg("xi"), py::arg("yi"), py::arg("fx"),
     py::arg("fy"), py::arg("bd") = 8);
  h.def("weight", [](int p0, int p1, bool bi, int bd) { return hevc::hk_weight(p0, p1, bi, bd); },
        py::arg("p0"), py::arg("p1"), py::arg("bi"), py::arg("bd") = 8);
  h.def("weight_explicit", [](int w0, int o0, int w1, int o1, int log2wd, int p0, int p1, bool bi, int l, int bd) {
    hevc::GpuWp e{};
    e.w[0][0] = i16(w0), e.o[0][0] = i16(o0), e.w[1][0] = i16(w1), e.o[1][0] = i16(o1);
    e.shift[0] = u8(log2wd);
    return hevc::hk_weight_explicit(e, 0, p0, p1, bi, l, bd);
  }, py::arg("w0"), py::arg("o0"), py::arg("w1"), py::arg("o1"), py::arg("log2wd"), py::arg("p0"), py::arg("p1"),
     py::arg("bi"), py::arg("l"), py::arg("bd") = 8);
  // One 4-line luma edge segment: lines[k] = p3 p2 p1 p0 q0 q1 q2 q3 (k = 0..3)
  h.def("deblock_luma", [](std::vector<std::vector<int>> lines, int bs, int qpl, int beta_offset, int tc_offset,
                           bool nfp, bool nfq, int bd) {
    u16 buf[4][8];
    for (int k = 0; k < 4; ++k)
      for (int i = 0; i < 8; ++i) buf[k][i] = u16(lines[size_t(k)][size_t(i)]);
    hevc::HkLumaEdgeT<u16> e{&buf[0][4], 8, 1};
    hevc::hk_deblock_luma(e, bs, qpl, beta_offset, tc_offset, nfp, nfq, bd);
    std::vector<std::vector<int>> out(4, std::vector<int>(8));
    for (int k = 0; k < 4; ++k)
      for (int i = 0; i < 8; ++i) out[size_t(k)][size_t(i)] = buf[k][i];
    return out;
  }, py::arg("lines"), py::arg("bs"), py::arg("qpl"), py::arg("beta_offset"), py::arg("tc_offset"), py::arg("nfp"),
     py::arg("nfq"), py::arg("bd") = 8);
  // Two chroma lines: lines[k] = p1 p0 q0 q1
  h.def("deblock_chroma", [](std::vector<std::vector<int>> lines, int qpp, int qpq, int cqp_offset, int tc_offset,
                             int bd) {
    u16 buf[2][4];
    for (int k = 0; k < 2; ++k)
      for (int i = 0; i < 4; ++i) buf[k][i] = u16(lines[size_t(k)][size_t(i)]);
    hevc::hk_deblock_chroma(&buf[0][2], 4, 1, qpp, qpq, cqp_offset, tc_offset, false, false, bd);
    std::vector<std::vector<int>> out(2, std::vector<int>(4));
    for (int k = 0; k < 2; ++k)
      for (int i = 0; i < 4; ++i) out[size_t(k)][size_t(i)] = buf[k][i];
    return out;
  }, py::arg("lines"), py::arg("qpp"), py::arg("qpq"), py::arg("cqp_offset"), py::arg("tc_offset"), py::arg("bd") = 8);
  // SAO of the centre of a 3 x 3 neighbourhood (all neighbours usable)
  h.def("sao", [](std::vector<int> nb9, int type, int band, int eo, std::vector<int> off, int bd) {
    u16 p[9];
    for (int i = 0; i < 9; ++i) p[i] = u16(nb9[size_t(i)]);
    hevc::GpuSao sp{};
    sp.type[0] = u8(type);
    sp.band[0] = u8(band);
    sp.eo[0] = u8(eo);
    for (int i = 0; i < 4; ++i) sp.off[0][i] = static_cast<signed char>(off[size_t(i)]);
    return hevc::hk_sao_sample(p, 3, 1, sp, 0, 1, 1, [](int, int) { return true; }, bd);
  }, py::arg("nb9"), py::arg("type"), py::arg("band"), py::arg("eo"), py::arg("off"), py::arg("bd") = 8);
}
