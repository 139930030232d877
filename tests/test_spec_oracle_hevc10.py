"""HEVC Main10: the reconstruction primitives at bit depth 10 against the spec oracle
(tests/spec_oracle_hevc.py with set_bit_depth(10)): both C++ forms — the CPU reference decoder's
(hevc_recon.cpp) and the per-sample functions the gfx950 kernels run on u16 planes
(hevc_kern.h) — for the inverse transforms (bdShift 20 - 10), scaling (bdShift 10 + log2 - 5),
all 35 intra modes with the 10-bit substitution value (512) and strong-smoothing threshold
(1 << 5), the 8-tap / 4-tap interpolation with shift1 = 2 and full samples << 4, default and
explicit weighting (shift 4 / 5), deblocking with beta / tC scaled by 4, and SAO bands of 32
values with offsets up to 31."""
import random

import pytest

import spec_oracle_hevc as so

from video_edge_ai_proxy_amd import _vep as v

rc = v.hevc_recon
BD = 10
MAXV = (1 << BD) - 1


@pytest.fixture(autouse=True)
def ten_bit():
    prev = so.set_bit_depth(BD)
    yield
    so.set_bit_depth(prev)


def u16_bytes(rows):
    return b"".join(int(x).to_bytes(2, "little") for r in rows for x in r)


@pytest.mark.parametrize("log2", [2, 3, 4, 5])
def test_inverse_transform_10bit(log2):
    rnd = random.Random(300 + log2)
    n = 1 << log2
    for it in range(20 if log2 < 5 else 6):
        density = rnd.choice([0.05, 0.3, 1.0])
        d = [[rnd.randint(-12000, 12000) if rnd.random() < density else 0 for _ in range(n)] for _ in range(n)]
        for dst in ([False, True] if log2 == 2 else [False]):
            want = sum(so.inverse_transform(d, log2, dst), [])
            flat = sum(d, [])
            assert rc.itx(flat, log2, dst, False, BD) == want, (log2, dst, it)
            assert rc.itx_kern(flat, log2, dst, BD) == want, (log2, dst, it)
    d = [[rnd.randint(-2000, 2000) for _ in range(4)] for _ in range(4)]
    assert rc.itx(sum(d, []), 2, False, True, BD) == sum(so.inverse_transform(d, 2, tskip=True), [])


def test_scaling_10bit_including_qp_bd_offset():
    rnd = random.Random(17)
    for _ in range(3000):  # Qp' = QpY + 12 reaches 63
        level, qp, log2, m = rnd.randint(-5000, 5000), rnd.randint(0, 63), rnd.randint(2, 5), rnd.randint(1, 255)
        assert rc.dequant(level, qp, log2, m, BD) == so.scale_level(level, qp, log2, m), (level, qp, log2, m)


@pytest.mark.parametrize("log2", [2, 3, 4, 5])
def test_intra_all_modes_10bit(log2):
    rnd = random.Random(400 + log2)
    n = 1 << log2
    x0 = y0 = 64
    W = H = 192
    for it in range(4 if log2 == 5 else 6):
        if it % 2 == 0:
            base = rnd.randint(160, 800)
            plane = [[max(0, min(MAXV, base + (x * 3 + y * 2) // 2 + rnd.randint(-6, 6))) for x in range(W)]
                     for y in range(H)]
        else:
            plane = [[rnd.randint(0, MAXV) for _ in range(W)] for _ in range(H)]
        raw = u16_bytes(plane)
        mask = rnd.getrandbits(33) if it % 3 else (1 << 33) - 1
        if it == 4:
            mask = 0  # nothing available: 1 << (BitDepth - 1) = 512
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
                want = sum(so.intra(p, avail, n, mode, 0, strong), [])
                assert rc.intra_kern(raw, W, x0, y0, log2, True, mask, mode, strong, BD) == want, (log2, it, mode)
                sp = so.substitute(p, avail, n)
                top = [sp[(-1, -1)]] + [sp[(x, -1)] for x in range(2 * n)]
                left = [sp[(-1, y)] for y in range(2 * n)]
                assert rc.intra(top, left, log2, mode, True, strong, BD) == want, (log2, it, mode, strong)


def test_intra_strong_smoothing_threshold_scales_with_bit_depth():
    # flat-ish 32x32 references whose second difference is 20: below 1 << (10 - 5) = 32 (strong
    # smoothing at 10 bits) but not below 8 (it would not be at 8 bits)
    n = 32
    top = [400] + [400 + (10 if x == n - 1 else 0) for x in range(2 * n)]
    left = [400 + (10 if y == n - 1 else 0) for y in range(2 * n)]
    p = {(-1, -1): top[0]}
    for x in range(2 * n):
        p[(x, -1)] = top[x + 1]
    for y in range(2 * n):
        p[(-1, y)] = left[y]
    want = sum(so.predict(so.filter_refs(p, n, 18, 0, True), n, 18, 0), [])
    assert rc.intra(top, left, 5, 18, True, True, BD) == want


def test_inter_10bit_all_fractions():
    rnd = random.Random(19)
    W, H = 24, 20
    plane = [[rnd.randint(0, MAXV) for _ in range(W)] for _ in range(H)]
    raw = u16_bytes(plane)
    for fy in range(4):
        for fx in range(4):
            for _ in range(12):
                xi, yi = rnd.randint(-12, W + 8), rnd.randint(-12, H + 8)
                assert rc.luma_mc(raw, W, H, xi, yi, fx, fy, BD) == so.luma_sample(plane, xi, yi, fx, fy)
    Wc, Hc = 12, 10
    cb = [[rnd.randint(0, MAXV) for _ in range(Wc)] for _ in range(Hc)]
    cr = [[rnd.randint(0, MAXV) for _ in range(Wc)] for _ in range(Hc)]
    rawc = b"".join(int(val).to_bytes(2, "little") for y in range(Hc) for x in range(Wc) for val in (cb[y][x], cr[y][x]))
    for fy in range(8):
        for fx in range(8):
            for _ in range(4):
                xi, yi = rnd.randint(-6, Wc + 4), rnd.randint(-6, Hc + 4)
                for c, ref in ((0, cb), (1, cr)):
                    assert rc.chroma_mc(rawc, Wc, Hc, c, xi, yi, fx, fy, BD) == so.chroma_sample(ref, xi, yi, fx, fy)


def test_weighting_10bit():
    rnd = random.Random(20)
    for _ in range(3000):
        p0, p1 = rnd.randint(-10000, 26000), rnd.randint(-10000, 26000)
        assert rc.weight(p0, 0, False, BD) == so.default_weighted(p0)
        assert rc.weight(p0, p1, True, BD) == so.default_weighted(p0, p1)
        denom = rnd.randint(0, 7)
        log2wd = denom + 14 - BD
        w0, w1 = (1 << denom) + rnd.randint(-128, 127), (1 << denom) + rnd.randint(-128, 127)
        o0, o1 = rnd.randint(-128, 127) * 4, rnd.randint(-128, 127) * 4  # offsets << (BitDepth - 8)
        assert rc.weight_explicit(w0, o0, w1, o1, log2wd, p0, 0, False, 0, BD) == so.explicit_weighted(log2wd, w0, o0, p0)
        assert rc.weight_explicit(w0, o0, w1, o1, log2wd, p0, p1, True, 0, BD) == \
            so.explicit_weighted(log2wd, w0, o0, p0, w1, o1, p1)


def test_deblocking_10bit():
    rnd = random.Random(21)
    changed = 0
    for _ in range(4000):
        base, step = rnd.randint(80, 920), rnd.randint(-120, 120)
        lines = []
        for _ in range(4):
            if rnd.random() < 0.6:
                g = rnd.randint(-8, 8)
                ln = [base + g * i + rnd.randint(-4, 4) for i in range(4)] + \
                     [base + step + g * i + rnd.randint(-4, 4) for i in range(4)]
            else:
                ln = [rnd.randint(0, MAXV) for _ in range(8)]
            lines.append([max(0, min(MAXV, s)) for s in ln])
        bs, qpl = rnd.randint(1, 2), rnd.randint(-12, 51)  # QpY below 0 (QpBdOffsetY 12)
        bo, to = 2 * rnd.randint(-6, 6), 2 * rnd.randint(-6, 6)
        nfp, nfq = rnd.random() < 0.1, rnd.random() < 0.1
        want = so.deblock_luma(lines, bs, qpl, bo, to, nfp, nfq)
        assert rc.deblock_luma(lines, bs, qpl, bo, to, nfp, nfq, BD) == want
        changed += want != lines
        cl = [[max(0, min(MAXV, base + rnd.randint(-60, 60))) for _ in range(4)] for _ in range(2)]
        qpp, qpq, cqp = rnd.randint(-12, 51), rnd.randint(-12, 51), rnd.randint(-12, 12)
        assert rc.deblock_chroma(cl, qpp, qpq, cqp, to, BD) == so.deblock_chroma(cl, qpp, qpq, cqp, to)
    assert changed > 600


def test_sao_10bit_bands_and_offsets():
    rnd = random.Random(22)
    for _ in range(4000):
        nb = [[rnd.randint(0, MAXV) for _ in range(3)] for _ in range(3)]
        if rnd.random() < 0.5:
            c = nb[1][1]
            nb = [[max(0, min(MAXV, c + rnd.randint(-3, 3))) for _ in range(3)] for _ in range(3)]
        t = rnd.randint(1, 2)
        band, eo = rnd.randint(0, 31), rnd.randint(0, 3)
        if t == 1:
            off = [rnd.randint(-31, 31) for _ in range(4)]
        else:
            off = [rnd.randint(0, 31), rnd.randint(0, 31), -rnd.randint(0, 31), -rnd.randint(0, 31)]
        assert rc.sao(sum(nb, []), t, band, eo, off, BD) == so.sao_sample(nb, t, band, eo, off), (nb, t, band, eo, off)
