"""The HEVC reconstruction primitives against the independent spec oracle
(tests/spec_oracle_hevc.py, written from the H.265 text), on randomised inputs. Both C++ forms
are checked: the CPU reference decoder's (hevc_recon.cpp) and the per-sample functions the
gfx950 kernels run (hevc_kern.h, through `_vep.hevc_recon` hooks): inverse DCT 4..32 / DST 4x4 /
transform skip, scaling with flat and custom matrices, all 35 intra modes with reference
substitution for random availability and (strong) reference filtering, every luma quarter- and
chroma eighth-sample position incl. picture-edge clamping, default and explicit weighted
prediction, the luma / chroma deblocking decisions and filters across the QP / offset ranges,
and SAO band / edge offsets. So the encoder, the CPU decoder and the GPU kernels no longer share
a single point of truth."""
import random

import pytest

import spec_oracle_hevc as so

from video_edge_ai_proxy_amd import _vep as v

rc = v.hevc_recon


def test_matrix_rows_match_spec_listing():
    # rows quoted in the spec's transMatrix listing (§8.6.4.2)
    assert so.TRANS32[0] == [64] * 32
    assert so.TRANS32[1][:16] == [90, 90, 88, 85, 82, 78, 73, 67, 61, 54, 46, 38, 31, 22, 13, 4]
    assert so.TRANS32[2][:8] == [90, 87, 80, 70, 57, 43, 25, 9]
    assert so.TRANS32[4][:4] == [89, 75, 50, 18]
    assert so.TRANS32[8][:4] == [83, 36, -36, -83]
    assert so.TRANS32[16][:4] == [64, -64, -64, 64]
    assert [so.TRANS32[8 * j][:4] for j in range(4)] == [[64, 64, 64, 64], [83, 36, -36, -83], [64, -64, -64, 64],
                                                          [36, -83, 83, -36]]


@pytest.mark.parametrize("log2", [2, 3, 4, 5])
def test_inverse_transform(log2):
    rnd = random.Random(100 + log2)
    n = 1 << log2
    for it in range(40 if log2 < 5 else 12):
        density = rnd.choice([0.05, 0.3, 1.0])
        d = [[rnd.randint(-3000, 3000) if rnd.random() < density else 0 for _ in range(n)] for _ in range(n)]
        if it == 0:
            d = [[32767 if (x + y) % 3 == 0 else -32768 for x in range(n)] for y in range(n)]  # clipping
        for dst in ([False, True] if log2 == 2 else [False]):
            want = sum(so.inverse_transform(d, log2, dst), [])
            flat = sum(d, [])
            assert rc.itx(flat, log2, dst, False) == want, (log2, dst, it)
            assert rc.itx_kern(flat, log2, dst) == want, (log2, dst, it)
    d = [[rnd.randint(-500, 500) for _ in range(4)] for _ in range(4)]
    assert rc.itx(sum(d, []), 2, False, True) == sum(so.inverse_transform(d, 2, tskip=True), [])


def test_scaling_with_matrices():
    rnd = random.Random(7)
    for _ in range(3000):
        level, qp, log2, m = rnd.randint(-5000, 5000), rnd.randint(0, 51), rnd.randint(2, 5), rnd.randint(1, 255)
        assert rc.dequant(level, qp, log2, m) == so.scale_level(level, qp, log2, m), (level, qp, log2, m)
    assert rc.dequant(100, 30, 3) == so.scale_level(100, 30, 3, 16)


def _plane(rnd, w, h, smooth):
    if smooth:
        base = rnd.randint(40, 200)
        return [[max(0, min(255, base + (x * 3 + y * 2) // 4 + rnd.randint(-3, 3))) for x in range(w)] for y in range(h)]
    return [[rnd.randint(0, 255) for _ in range(w)] for _ in range(h)]


@pytest.mark.parametrize("log2", [2, 3, 4, 5])
def test_intra_all_modes_kernel_and_reference(log2):
    rnd = random.Random(200 + log2)
    n = 1 << log2
    x0 = y0 = 64
    W = H = 192
    for it in range(6 if log2 == 5 else 10):
        plane = _plane(rnd, W, H, smooth=it % 2 == 0)
        raw = bytes(sum(plane, []))
        mask = rnd.getrandbits(33) if it % 3 else (1 << 33) - 1
        if it == 4:
            mask = 0  # nothing available: 128
        units = 2 * n // 4
        p, avail = {}, {}
        avail[(-1, -1)] = bool(mask & 1)
        p[(-1, -1)] = plane[y0 - 1][x0 - 1]
        for y in range(2 * n):
            avail[(-1, y)] = bool((mask >> (1 + y // 4)) & 1) and y // 4 < units
            p[(-1, y)] = plane[y0 + y][x0 - 1]
        for x in range(2 * n):
            avail[(x, -1)] = bool((mask >> (17 + x // 4)) & 1) and x // 4 < units
            p[(x, -1)] = plane[y0 - 1][x0 + x]
        for mode in range(35):
            for strong in (False, True):
                want = so.intra(p, avail, n, mode, 0, strong)
                got = rc.intra_kern(raw, W, x0, y0, log2, True, mask, mode, strong)
                assert got == sum(want, []), (log2, it, mode, strong)
                # CPU reference (substituted references in, filtering + prediction inside)
                sp = so.substitute(p, avail, n)
                top = [sp[(-1, -1)]] + [sp[(x, -1)] for x in range(2 * n)]
                left = [sp[(-1, y)] for y in range(2 * n)]
                assert rc.intra(top, left, log2, mode, True, strong) == sum(want, []), (log2, it, mode, strong)
            if log2 <= 4:  # chroma (4:2:0 chroma blocks are at most 16x16): availability in 2-sample units
                cav = dict(avail)
                for y in range(2 * n):
                    cav[(-1, y)] = bool((mask >> (1 + y // 2)) & 1) and y // 2 < 16
                for x in range(2 * n):
                    cav[(x, -1)] = bool((mask >> (17 + x // 2)) & 1) and x // 2 < 16
                want_c = so.intra(p, cav, n, mode, 1, False)
                assert rc.intra_kern(raw, W, x0, y0, log2, False, mask, mode, False) == sum(want_c, []), (log2, mode)
                want_c = so.intra(p, avail, n, mode, 1, False)
                sp = so.substitute(p, avail, n)
                top = [sp[(-1, -1)]] + [sp[(x, -1)] for x in range(2 * n)]
                left = [sp[(-1, y)] for y in range(2 * n)]
                assert rc.intra(top, left, log2, mode, False, False) == sum(want_c, []), (log2, it, mode)


def test_inter_luma_all_fractions_with_clamping():
    rnd = random.Random(11)
    W, H = 24, 20
    plane = _plane(rnd, W, H, smooth=False)
    raw = bytes(sum(plane, []))
    for fy in range(4):
        for fx in range(4):
            for _ in range(25):
                xi, yi = rnd.randint(-12, W + 8), rnd.randint(-12, H + 8)
                assert rc.luma_mc(raw, W, H, xi, yi, fx, fy) == so.luma_sample(plane, xi, yi, fx, fy), (xi, yi, fx, fy)


def test_inter_chroma_all_fractions_with_clamping():
    rnd = random.Random(12)
    W, H = 12, 10
    cb, cr = _plane(rnd, W, H, False), _plane(rnd, W, H, False)
    raw = bytes(v for y in range(H) for x in range(W) for v in (cb[y][x], cr[y][x]))
    for fy in range(8):
        for fx in range(8):
            for _ in range(8):
                xi, yi = rnd.randint(-6, W + 4), rnd.randint(-6, H + 4)
                for c, ref in ((0, cb), (1, cr)):
                    assert rc.chroma_mc(raw, W, H, c, xi, yi, fx, fy) == so.chroma_sample(ref, xi, yi, fx, fy)


def test_weighted_prediction_default_and_explicit():
    rnd = random.Random(13)
    for _ in range(4000):
        p0, p1 = rnd.randint(-10000, 26000), rnd.randint(-10000, 26000)
        assert rc.weight(p0, 0, False) == so.default_weighted(p0)
        assert rc.weight(p0, p1, True) == so.default_weighted(p0, p1)
        denom = rnd.randint(0, 7)
        log2wd = denom + 14 - so.BIT_DEPTH
        w0, w1 = (1 << denom) + rnd.randint(-128, 127), (1 << denom) + rnd.randint(-128, 127)
        o0, o1 = rnd.randint(-128, 127), rnd.randint(-128, 127)
        assert rc.weight_explicit(w0, o0, w1, o1, log2wd, p0, 0, False, 0) == so.explicit_weighted(log2wd, w0, o0, p0)
        assert rc.weight_explicit(w0, o0, w1, o1, log2wd, p1, 0, False, 1) == so.explicit_weighted(log2wd, w1, o1, p1)
        assert rc.weight_explicit(w0, o0, w1, o1, log2wd, p0, p1, True, 0) == \
            so.explicit_weighted(log2wd, w0, o0, p0, w1, o1, p1)


def _edge_lines(rnd):
    kind = rnd.random()
    lines = []
    base, step = rnd.randint(20, 230), rnd.randint(-30, 30)
    for _ in range(4):
        if kind < 0.6:  # smooth sides with a step: the filters engage
            g = rnd.randint(-2, 2)
            left = [base + g * i + rnd.randint(-1, 1) for i in range(4)]
            right = [base + step + g * i + rnd.randint(-1, 1) for i in range(4)]
            ln = left + right
        else:
            ln = [rnd.randint(0, 255) for _ in range(8)]
        lines.append([max(0, min(255, s)) for s in ln])
    return lines


def test_deblocking_luma():
    rnd = random.Random(14)
    changed = 0
    for _ in range(6000):
        lines = _edge_lines(rnd)
        bs, qpl = rnd.randint(1, 2), rnd.randint(0, 51)
        bo, to = 2 * rnd.randint(-6, 6), 2 * rnd.randint(-6, 6)
        nfp, nfq = rnd.random() < 0.1, rnd.random() < 0.1
        want = so.deblock_luma(lines, bs, qpl, bo, to, nfp, nfq)
        assert rc.deblock_luma(lines, bs, qpl, bo, to, nfp, nfq) == want, (lines, bs, qpl, bo, to)
        changed += want != lines
    assert changed > 1000  # the random edges exercise the filters, not only the skip decision


def test_deblocking_chroma_full_offset_range():
    rnd = random.Random(15)
    for _ in range(6000):
        lines = [[rnd.randint(0, 255) for _ in range(4)] for _ in range(2)]
        if rnd.random() < 0.7:  # small step across the edge
            b = rnd.randint(10, 240)
            lines = [[b, b + rnd.randint(-2, 2), b + rnd.randint(-20, 20), b + rnd.randint(-20, 20)] for _ in range(2)]
            lines = [[max(0, min(255, s)) for s in ln] for ln in lines]
        qpp, qpq = rnd.randint(0, 51), rnd.randint(0, 51)
        cqp, to = rnd.randint(-12, 12), 2 * rnd.randint(-6, 6)
        assert rc.deblock_chroma(lines, qpp, qpq, cqp, to) == so.deblock_chroma(lines, qpp, qpq, cqp, to), \
            (lines, qpp, qpq, cqp, to)


def test_sao_band_and_edge():
    rnd = random.Random(16)
    for _ in range(6000):
        nb = [[rnd.randint(0, 255) for _ in range(3)] for _ in range(3)]
        if rnd.random() < 0.5:
            c = nb[1][1]
            nb = [[max(0, min(255, c + rnd.randint(-2, 2))) for _ in range(3)] for _ in range(3)]
        t = rnd.randint(1, 2)
        band, eo = rnd.randint(0, 31), rnd.randint(0, 3)
        if t == 1:
            off = [rnd.randint(-7, 7) for _ in range(4)]
        else:
            off = [rnd.randint(0, 7), rnd.randint(0, 7), -rnd.randint(0, 7), -rnd.randint(0, 7)]
        flat = sum(nb, [])
        assert rc.sao(flat, t, band, eo, off) == so.sao_sample(nb, t, band, eo, off), (nb, t, band, eo, off)
