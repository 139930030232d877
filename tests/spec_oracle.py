"""Independent H.264 reconstruction oracle, written from the text of ITU-T H.264 (2016) — not
from avc_recon.h — in plain Python, one equation at a time, so that the CPU decoder, the gfx950
kernels and the synthetic encoders (which all share avc_recon.h) no longer have a single point
of truth. Clause numbers refer to the standard.

Sample arrays follow the standard's notation: ``top[x + 1] = p[x, -1]`` (x = -1 ..), ``left[y] =
p[-1, y]``; predictions are returned row-major ``pred[y][x]``.
"""
from __future__ import annotations


def clip3(lo, hi, v):
    return lo if v < lo else hi if v > hi else v


def clip1(v, bd=8):
    """Clip1Y / Clip1C (5-3 / 5-4) at sample bit depth bd (High 10: 9 or 10)."""
    return clip3(0, (1 << bd) - 1, v)


# ------------------------------------------------------------------ 8.5.12.2 / 8.5.13.2
def inverse_4x4(d):
    """d: 4x4 scaled coefficients (list of rows) -> residual r (list of rows)."""
    f = [[0] * 4 for _ in range(4)]
    for i in range(4):  # each (horizontal) row
        e0 = d[i][0] + d[i][2]
        e1 = d[i][0] - d[i][2]
        e2 = (d[i][1] >> 1) - d[i][3]
        e3 = d[i][1] + (d[i][3] >> 1)
        f[i] = [e0 + e3, e1 + e2, e1 - e2, e0 - e3]
    h = [[0] * 4 for _ in range(4)]
    for j in range(4):  # each (vertical) column
        g0 = f[0][j] + f[2][j]
        g1 = f[0][j] - f[2][j]
        g2 = (f[1][j] >> 1) - f[3][j]
        g3 = f[1][j] + (f[3][j] >> 1)
        h[0][j], h[1][j], h[2][j], h[3][j] = g0 + g3, g1 + g2, g1 - g2, g0 - g3
    return [[(h[i][j] + 32) >> 6 for j in range(4)] for i in range(4)]


def _idct8_pass(v):
    e0 = v[0] + v[4]
    e1 = -v[3] + v[5] - v[7] - (v[7] >> 1)
    e2 = v[0] - v[4]
    e3 = v[1] + v[7] - v[3] - (v[3] >> 1)
    e4 = (v[2] >> 1) - v[6]
    e5 = -v[1] + v[7] + v[5] + (v[5] >> 1)
    e6 = v[2] + (v[6] >> 1)
    e7 = v[3] + v[5] + v[1] + (v[1] >> 1)
    f0 = e0 + e6
    f1 = e1 + (e7 >> 2)
    f2 = e2 + e4
    f3 = e3 + (e5 >> 2)
    f4 = e2 - e4
    f5 = (e3 >> 2) - e5
    f6 = e0 - e6
    f7 = e7 - (e1 >> 2)
    return [f0 + f7, f2 + f5, f4 + f3, f6 + f1, f6 - f1, f4 - f3, f2 - f5, f0 - f7]


def inverse_8x8(d):
    g = [_idct8_pass(row) for row in d]
    m = [[0] * 8 for _ in range(8)]
    for j in range(8):
        col = _idct8_pass([g[i][j] for i in range(8)])
        for i in range(8):
            m[i][j] = col[i]
    return [[(m[i][j] + 32) >> 6 for j in range(8)] for i in range(8)]


# 8.5.9 (flat weight matrices): LevelScale4x4 = 16 * normAdjust4x4
_V4 = [[10, 16, 13], [11, 18, 14], [13, 20, 16], [14, 23, 18], [16, 25, 20], [18, 29, 23]]


def dequant_4x4(c, qp, i, j):
    m = qp % 6
    v = _V4[m][0] if (i % 2 == 0 and j % 2 == 0) else _V4[m][1] if (i % 2 == 1 and j % 2 == 1) else _V4[m][2]
    ls = 16 * v
    if qp >= 24:
        return (c * ls) << (qp // 6 - 4)
    return (c * ls + 2 ** (3 - qp // 6)) >> (4 - qp // 6)


# ------------------------------------------------------------------ 8.3.1.2 Intra_4x4
def intra_4x4(top, left, has_top, has_left, mode, bd=8):
    """top = p[-1..7, -1] (top-right substituted), left = p[-1, 0..3]."""
    def P(x, y):
        return top[x + 1] if y == -1 else left[y]

    out = [[0] * 4 for _ in range(4)]
    for y in range(4):
        for x in range(4):
            if mode == 0:
                v = P(x, -1)
            elif mode == 1:
                v = P(-1, y)
            elif mode == 2:
                st = sum(P(k, -1) for k in range(4))
                sl = sum(P(-1, k) for k in range(4))
                if has_top and has_left:
                    v = (st + sl + 4) >> 3
                elif has_left:
                    v = (sl + 2) >> 2
                elif has_top:
                    v = (st + 2) >> 2
                else:
                    v = 1 << (bd - 1)  # (8-51 etc.: 1 << (BitDepth - 1))
            elif mode == 3:
                if x == 3 and y == 3:
                    v = (P(6, -1) + 3 * P(7, -1) + 2) >> 2
                else:
                    v = (P(x + y, -1) + 2 * P(x + y + 1, -1) + P(x + y + 2, -1) + 2) >> 2
            elif mode == 4:
                if x > y:
                    v = (P(x - y - 2, -1) + 2 * P(x - y - 1, -1) + P(x - y, -1) + 2) >> 2
                elif x < y:
                    v = (P(-1, y - x - 2) + 2 * P(-1, y - x - 1) + P(-1, y - x) + 2) >> 2
                else:
                    v = (P(0, -1) + 2 * P(-1, -1) + P(-1, 0) + 2) >> 2
            elif mode == 5:
                z = 2 * x - y
                if z >= 0 and z % 2 == 0:
                    v = (P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 1) >> 1
                elif z >= 0:
                    v = (P(x - (y >> 1) - 2, -1) + 2 * P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 2) >> 2
                elif z == -1:
                    v = (P(-1, 0) + 2 * P(-1, -1) + P(0, -1) + 2) >> 2
                else:
                    v = (P(-1, y - 1) + 2 * P(-1, y - 2) + P(-1, y - 3) + 2) >> 2
            elif mode == 6:
                z = 2 * y - x
                if z >= 0 and z % 2 == 0:
                    v = (P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 1) >> 1
                elif z >= 0:
                    v = (P(-1, y - (x >> 1) - 2) + 2 * P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 2) >> 2
                elif z == -1:
                    v = (P(-1, 0) + 2 * P(-1, -1) + P(0, -1) + 2) >> 2
                else:
                    v = (P(x - 1, -1) + 2 * P(x - 2, -1) + P(x - 3, -1) + 2) >> 2
            elif mode == 7:
                if y % 2 == 0:
                    v = (P(x + (y >> 1), -1) + P(x + (y >> 1) + 1, -1) + 1) >> 1
                else:
                    v = (P(x + (y >> 1), -1) + 2 * P(x + (y >> 1) + 1, -1) + P(x + (y >> 1) + 2, -1) + 2) >> 2
            else:
                z = x + 2 * y
                if z in (0, 2, 4):
                    v = (P(-1, y + (x >> 1)) + P(-1, y + (x >> 1) + 1) + 1) >> 1
                elif z in (1, 3):
                    v = (P(-1, y + (x >> 1)) + 2 * P(-1, y + (x >> 1) + 1) + P(-1, y + (x >> 1) + 2) + 2) >> 2
                elif z == 5:
                    v = (P(-1, 2) + 3 * P(-1, 3) + 2) >> 2
                else:
                    v = P(-1, 3)
            out[y][x] = v
    return out


# ------------------------------------------------------------------ 8.3.2.2 Intra_8x8
def filter_8x8_refs(top, left, has_top, has_left, has_tl):
    """8.3.2.2.1: top = p[-1..15, -1], left = p[-1, 0..7] -> (top', left') in the same layout
    (unavailable samples are returned as None)."""
    t = [None] * 17
    lf = [None] * 8
    if has_top:
        for x in range(16):
            if x == 0:
                t[1] = (top[0] + 2 * top[1] + top[2] + 2) >> 2 if has_tl else (3 * top[1] + top[2] + 2) >> 2
            elif x == 15:
                t[16] = (top[15] + 3 * top[16] + 2) >> 2
            else:
                t[x + 1] = (top[x] + 2 * top[x + 1] + top[x + 2] + 2) >> 2
    if has_tl:
        if not has_top or not has_left:
            if has_top:
                t[0] = (3 * top[0] + top[1] + 2) >> 2
            elif has_left:
                t[0] = (3 * top[0] + left[0] + 2) >> 2
            else:
                t[0] = top[0]
        else:
            t[0] = (top[1] + 2 * top[0] + left[0] + 2) >> 2
    if has_left:
        for y in range(8):
            if y == 0:
                lf[0] = (top[0] + 2 * left[0] + left[1] + 2) >> 2 if has_tl else (3 * left[0] + left[1] + 2) >> 2
            elif y == 7:
                lf[7] = (left[6] + 3 * left[7] + 2) >> 2
            else:
                lf[y] = (left[y - 1] + 2 * left[y] + left[y + 1] + 2) >> 2
    return t, lf


def intra_8x8(top, left, has_top, has_left, has_tl, mode, bd=8):
    t, lf = filter_8x8_refs(top, left, has_top, has_left, has_tl)

    def P(x, y):
        return t[x + 1] if y == -1 else lf[y]

    out = [[0] * 8 for _ in range(8)]
    for y in range(8):
        for x in range(8):
            if mode == 0:
                v = P(x, -1)
            elif mode == 1:
                v = P(-1, y)
            elif mode == 2:
                if has_top and has_left:
                    v = (sum(P(k, -1) for k in range(8)) + sum(P(-1, k) for k in range(8)) + 8) >> 4
                elif has_left:
                    v = (sum(P(-1, k) for k in range(8)) + 4) >> 3
                elif has_top:
                    v = (sum(P(k, -1) for k in range(8)) + 4) >> 3
                else:
                    v = 1 << (bd - 1)  # (8-51 etc.: 1 << (BitDepth - 1))
            elif mode == 3:
                if x == 7 and y == 7:
                    v = (P(14, -1) + 3 * P(15, -1) + 2) >> 2
                else:
                    v = (P(x + y, -1) + 2 * P(x + y + 1, -1) + P(x + y + 2, -1) + 2) >> 2
            elif mode == 4:
                if x > y:
                    v = (P(x - y - 2, -1) + 2 * P(x - y - 1, -1) + P(x - y, -1) + 2) >> 2
                elif x < y:
                    v = (P(-1, y - x - 2) + 2 * P(-1, y - x - 1) + P(-1, y - x) + 2) >> 2
                else:
                    v = (P(0, -1) + 2 * P(-1, -1) + P(-1, 0) + 2) >> 2
            elif mode == 5:
                z = 2 * x - y
                if z >= 0 and z % 2 == 0:
                    v = (P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 1) >> 1
                elif z >= 0:
                    v = (P(x - (y >> 1) - 2, -1) + 2 * P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 2) >> 2
                elif z == -1:
                    v = (P(-1, 0) + 2 * P(-1, -1) + P(0, -1) + 2) >> 2
                else:
                    v = (P(-1, y - 2 * x - 1) + 2 * P(-1, y - 2 * x - 2) + P(-1, y - 2 * x - 3) + 2) >> 2
            elif mode == 6:
                z = 2 * y - x
                if z >= 0 and z % 2 == 0:
                    v = (P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 1) >> 1
                elif z >= 0:
                    v = (P(-1, y - (x >> 1) - 2) + 2 * P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 2) >> 2
                elif z == -1:
                    v = (P(-1, 0) + 2 * P(-1, -1) + P(0, -1) + 2) >> 2
                else:
                    v = (P(x - 2 * y - 1, -1) + 2 * P(x - 2 * y - 2, -1) + P(x - 2 * y - 3, -1) + 2) >> 2
            elif mode == 7:
                if y % 2 == 0:
                    v = (P(x + (y >> 1), -1) + P(x + (y >> 1) + 1, -1) + 1) >> 1
                else:
                    v = (P(x + (y >> 1), -1) + 2 * P(x + (y >> 1) + 1, -1) + P(x + (y >> 1) + 2, -1) + 2) >> 2
            else:
                z = x + 2 * y
                if z < 13 and z % 2 == 0:
                    v = (P(-1, y + (x >> 1)) + P(-1, y + (x >> 1) + 1) + 1) >> 1
                elif z < 13:
                    v = (P(-1, y + (x >> 1)) + 2 * P(-1, y + (x >> 1) + 1) + P(-1, y + (x >> 1) + 2) + 2) >> 2
                elif z == 13:
                    v = (P(-1, 6) + 3 * P(-1, 7) + 2) >> 2
                else:
                    v = P(-1, 7)
            out[y][x] = v
    return out


# ------------------------------------------------------------------ 8.3.3 Intra_16x16
def intra_16x16(top, left, has_top, has_left, mode, bd=8):
    """top = p[-1..15, -1], left = p[-1, 0..15]."""
    def P(x, y):
        return top[x + 1] if y == -1 else left[y]

    out = [[0] * 16 for _ in range(16)]
    if mode == 3:
        H = sum((k + 1) * (P(8 + k, -1) - P(6 - k, -1)) for k in range(8))
        V = sum((k + 1) * (P(-1, 8 + k) - (P(-1, 6 - k) if 6 - k >= 0 else top[0])) for k in range(8))  # p[-1,-1]
        a = 16 * (P(-1, 15) + P(15, -1))
        b = (5 * H + 32) >> 6
        c = (5 * V + 32) >> 6
    for y in range(16):
        for x in range(16):
            if mode == 0:
                v = P(x, -1)
            elif mode == 1:
                v = P(-1, y)
            elif mode == 2:
                st = sum(P(k, -1) for k in range(16))
                sl = sum(P(-1, k) for k in range(16))
                if has_top and has_left:
                    v = (st + sl + 16) >> 5
                elif has_left:
                    v = (sl + 8) >> 4
                elif has_top:
                    v = (st + 8) >> 4
                else:
                    v = 1 << (bd - 1)  # (8-51 etc.: 1 << (BitDepth - 1))
            else:
                v = clip1((a + b * (x - 7) + c * (y - 7) + 16) >> 5, bd)
            out[y][x] = v
    return out


# ------------------------------------------------------------------ 8.3.4 chroma (4:2:0)
def intra_chroma(top, left, has_top, has_left, mode, bd=8, cf=1):
    """top = p[-1..7, -1], left = p[-1, 0..MbHeightC-1]; mode: 0 DC, 1 horizontal, 2 vertical,
    3 plane. cf = chroma_format_idc (2: 4:2:2, MbHeightC 16; 8.3.4 with xCF = 0, yCF = 4)."""
    def P(x, y):
        return top[x + 1] if y == -1 else left[y]

    hc = 16 if cf == 2 else 8
    ycf = 4 if cf == 2 else 0
    out = [[0] * 8 for _ in range(hc)]
    if mode == 3:
        H = sum((k + 1) * (P(4 + k, -1) - P(2 - k, -1)) for k in range(4))
        V = sum((k + 1) * (P(-1, 4 + ycf + k) - P(-1, 2 + ycf - k)) for k in range(4 + ycf))  # P(-1,-1) = top[0]
        a = 16 * (P(-1, hc - 1) + P(7, -1))
        b = (34 * H + 32) >> 6
        c = ((34 - 29 * (cf != 1)) * V + 32) >> 6
    for y in range(hc):
        for x in range(8):
            if mode == 0:
                xo, yo = (x // 4) * 4, (y // 4) * 4
                st = sum(P(xo + k, -1) for k in range(4))
                sl = sum(P(-1, yo + k) for k in range(4))
                if (xo == 0 and yo == 0) or (xo > 0 and yo > 0):  # (8.3.4.1-3: chroma4x4BlkIdx rules)
                    v = (st + sl + 4) >> 3 if has_top and has_left else (sl + 2) >> 2 if has_left else \
                        (st + 2) >> 2 if has_top else 1 << (bd - 1)
                elif xo > 0:
                    v = (st + 2) >> 2 if has_top else (sl + 2) >> 2 if has_left else 1 << (bd - 1)
                else:
                    v = (sl + 2) >> 2 if has_left else (st + 2) >> 2 if has_top else 1 << (bd - 1)
            elif mode == 1:
                v = P(-1, y)
            elif mode == 2:
                v = P(x, -1)
            else:
                v = clip1((a + b * (x - 3) + c * (y - 3 - ycf) + 16) >> 5, bd)
            out[y][x] = v
    return out


# ------------------------------------------------------------------ 8.5.11 4:2:2 chroma DC
CHROMA422_DC_C = [[0, 2], [1, 5], [3, 6], [4, 7]]  # c[i][j] = chromaList[CHROMA422_DC_C[i][j]] (8-330)


def chroma422_dc(levels, qpdc, ls):
    """levels: the 8 chroma DC levels in parsing order; qpdc = QP'C + 3; ls = LevelScale4x4(qpdc %
    6, 0, 0). Returns dcC[i][j] (4 rows x 2 columns of 4x4 chroma blocks)."""
    c = [[levels[CHROMA422_DC_C[i][j]] for j in range(2)] for i in range(4)]
    A = [[1, 1, 1, 1], [1, 1, -1, -1], [1, -1, -1, 1], [1, -1, 1, -1]]
    B = [[1, 1], [1, -1]]
    ac = [[sum(A[i][k] * c[k][j] for k in range(4)) for j in range(2)] for i in range(4)]
    f = [[sum(ac[i][k] * B[k][j] for k in range(2)) for j in range(2)] for i in range(4)]
    if qpdc >= 36:
        return [[(f[i][j] * ls) << (qpdc // 6 - 6) for j in range(2)] for i in range(4)]
    return [[(f[i][j] * ls + 2 ** (5 - qpdc // 6)) >> (6 - qpdc // 6) for j in range(2)] for i in range(4)]


# ------------------------------------------------------------------ 8.4.2.2 interpolation
def luma_sample(plane, xi, yi, fx, fy, bd=8):
    """8.4.2.2.1: plane = 2-D list/array of rows; (xi, yi) integer luma position, (fx, fy)
    quarter-sample fraction; reference positions are clamped into the picture."""
    h, w = len(plane), len(plane[0])

    def G(x, y):
        return int(plane[clip3(0, h - 1, y)][clip3(0, w - 1, x)])

    def tap(a, b, c, d, e, f):
        return a - 5 * b + 20 * c + 20 * d - 5 * e + f

    def b1(x, y):  # horizontal half-sample intermediate between (x, y) and (x + 1, y)
        return tap(G(x - 2, y), G(x - 1, y), G(x, y), G(x + 1, y), G(x + 2, y), G(x + 3, y))

    def h1(x, y):  # vertical half-sample intermediate between (x, y) and (x, y + 1)
        return tap(G(x, y - 2), G(x, y - 1), G(x, y), G(x, y + 1), G(x, y + 2), G(x, y + 3))

    x, y = xi, yi
    Gs = G(x, y)
    b = clip1((b1(x, y) + 16) >> 5, bd)
    hh = clip1((h1(x, y) + 16) >> 5, bd)
    s = clip1((b1(x, y + 1) + 16) >> 5, bd)
    m = clip1((h1(x + 1, y) + 16) >> 5, bd)
    j1 = tap(b1(x, y - 2), b1(x, y - 1), b1(x, y), b1(x, y + 1), b1(x, y + 2), b1(x, y + 3))
    j = clip1((j1 + 512) >> 10, bd)
    table = {
        (0, 0): Gs,
        (0, 1): (Gs + hh + 1) >> 1,             # d
        (0, 2): hh,                             # h
        (0, 3): (G(x, y + 1) + hh + 1) >> 1,    # n
        (1, 0): (Gs + b + 1) >> 1,              # a
        (1, 1): (b + hh + 1) >> 1,              # e
        (1, 2): (hh + j + 1) >> 1,              # i
        (1, 3): (hh + s + 1) >> 1,              # p
        (2, 0): b,                              # b
        (2, 1): (b + j + 1) >> 1,               # f
        (2, 2): j,                              # j
        (2, 3): (j + s + 1) >> 1,               # q
        (3, 0): (G(x + 1, y) + b + 1) >> 1,     # c
        (3, 1): (b + m + 1) >> 1,               # g
        (3, 2): (j + m + 1) >> 1,               # k
        (3, 3): (m + s + 1) >> 1,               # r
    }
    return table[(fx, fy)]


def chroma_sample(plane, xi, yi, fx, fy):
    """8.4.2.2.2: one chroma component (2-D rows), eighth-sample fraction."""
    h, w = len(plane), len(plane[0])

    def S(x, y):
        return int(plane[clip3(0, h - 1, y)][clip3(0, w - 1, x)])

    A, B, C, D = S(xi, yi), S(xi + 1, yi), S(xi, yi + 1), S(xi + 1, yi + 1)
    return ((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C + fx * fy * D + 32) >> 6


# ------------------------------------------------------------------ 8.7.2 deblocking
ALPHA = [0] * 16 + [4, 4, 5, 6, 7, 8, 9, 10, 12, 13, 15, 17, 20, 22, 25, 28, 32, 36, 40, 45, 50, 56, 63, 71,
                    80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255]
BETA = [0] * 16 + [2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 14,
                   14, 15, 15, 16, 16, 17, 17, 18, 18]
TC0 = [[0, 0, 0]] * 17 + [
    [0, 0, 1], [0, 0, 1], [0, 0, 1], [0, 0, 1], [0, 1, 1], [0, 1, 1], [1, 1, 1], [1, 1, 1], [1, 1, 1],
    [1, 1, 1], [1, 1, 2], [1, 1, 2], [1, 1, 2], [1, 1, 2], [1, 2, 3], [1, 2, 3], [2, 2, 3], [2, 2, 4],
    [2, 3, 4], [2, 3, 4], [3, 3, 5], [3, 4, 6], [3, 4, 6], [4, 5, 7], [4, 5, 8], [4, 6, 9], [5, 7, 10],
    [6, 8, 11], [6, 8, 13], [7, 10, 14], [8, 11, 16], [9, 12, 18], [10, 13, 20], [11, 15, 23], [13, 17, 25]]


def edge_thresholds(qp_p, qp_q, off_a, off_b, bd=8):
    """8-324..8-328: alpha = alpha' * (1 << (BitDepth - 8)), beta and tC0 likewise; qp_p / qp_q
    are QPY / QPC (negative above 8 bits), indexA / indexB clipped to 0..51."""
    qav = (qp_p + qp_q + 1) >> 1
    ia = clip3(0, 51, qav + off_a)
    ib = clip3(0, 51, qav + off_b)
    sc = 1 << (bd - 8)
    return ALPHA[ia] * sc, BETA[ib] * sc, [t * sc for t in TC0[ia]]


def filter_line(p, q, bs, alpha, beta, tc0, chroma, bd=8):
    """8.7.2.3 (bS < 4) / 8.7.2.4 (bS = 4) on one line: p = [p0..p3], q = [q0..q3]."""
    p, q = list(p), list(q)
    p0, p1, p2, p3 = p
    q0, q1, q2, q3 = q
    if not (bs > 0 and abs(p0 - q0) < alpha and abs(p1 - p0) < beta and abs(q1 - q0) < beta):
        return p, q
    ap = abs(p2 - p0)
    aq = abs(q2 - q0)
    if bs < 4:
        tc = tc0 + 1 if chroma else tc0 + (1 if ap < beta else 0) + (1 if aq < beta else 0)
        delta = clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3)
        p[0] = clip1(p0 + delta, bd)
        q[0] = clip1(q0 - delta, bd)
        if not chroma:
            if ap < beta:
                p[1] = p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1)
            if aq < beta:
                q[1] = q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1)
        return p, q
    strong = abs(p0 - q0) < ((alpha >> 2) + 2)
    if not chroma and ap < beta and strong:
        p[0] = (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3
        p[1] = (p2 + p1 + p0 + q0 + 2) >> 2
        p[2] = (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3
    else:
        p[0] = (2 * p1 + p0 + q1 + 2) >> 2
    if not chroma and aq < beta and strong:
        q[0] = (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3
        q[1] = (p0 + q0 + q1 + q2 + 2) >> 2
        q[2] = (2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3
    else:
        q[0] = (2 * q1 + q0 + p1 + 2) >> 2
    return p, q


# ------------------------------------------------------------------ 8.5.8 / Table 8-15
QPC_TABLE = {30: 29, 31: 30, 32: 31, 33: 32, 34: 32, 35: 33, 36: 34, 37: 34, 38: 35, 39: 35, 40: 36, 41: 36,
             42: 37, 43: 37, 44: 37, 45: 38, 46: 38, 47: 38, 48: 39, 49: 39, 50: 39, 51: 39}


def chroma_qp(qpy, offset, bd_c=8):
    """QPC from QPY: qPI = Clip3(-QpBdOffsetC, 51, QPY + qPOffset) (8-313), Table 8-15."""
    qpi = clip3(-6 * (bd_c - 8), 51, qpy + offset)
    return qpi if qpi < 30 else QPC_TABLE[qpi]


def mb_qp(prev_qpy, mb_qp_delta, bd=8):
    """QPY of a macroblock (7-37): ((QPY,PRED + mb_qp_delta + 52 + 2 * QpBdOffsetY) %
    (52 + QpBdOffsetY)) - QpBdOffsetY."""
    off = 6 * (bd - 8)
    return ((prev_qpy + mb_qp_delta + 52 + 2 * off) % (52 + off)) - off
