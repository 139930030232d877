"""Independent H.265 (ITU-T H.265 v3, 04/2015) reconstruction oracle for the tests, written from
the specification text in plain Python — not from csrc/vep/hevc_recon.* or hevc_kern.h, which
the decoder, the gfx950 kernels and the closed-loop encoder share. tests/test_spec_oracle_hevc.py
cross-checks both C++ implementations against it on randomised inputs.

Conventions: 2-D arrays are indexed [y][x]; BitDepth 8 unless set_bit_depth() chose 9..10
(Main10).
"""
from __future__ import annotations

import math

BIT_DEPTH = 8
MAX_VAL = (1 << BIT_DEPTH) - 1


def set_bit_depth(bd):
    """Switch the oracle to BitDepthY = BitDepthC = bd (8 .. 10: Main / Main10); returns the
    previous value. Every formula reads the module-level values at call time."""
    global BIT_DEPTH, MAX_VAL, SHIFT1, SHIFT3
    prev = BIT_DEPTH
    BIT_DEPTH, MAX_VAL = bd, (1 << bd) - 1
    SHIFT1, SHIFT3 = min(4, bd - 8), max(2, 14 - bd)
    return prev


def clip3(lo, hi, v):
    return lo if v < lo else hi if v > hi else v


def clip1(v):
    return clip3(0, MAX_VAL, v)


def sign(v):
    return (v > 0) - (v < 0)


# ----------------------------------------------------------------------------- transforms (8.6.4)
# The spec lists transMatrix (32 x 32) explicitly; its entries are the integers below for the
# angles m * pi / 64 (m = 0 .. 32) with the sign of cos(pi * k * (2 n + 1) / 64), row k, column n.
_COS_INT = [64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
            61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9, 4, 0]


def trans_matrix_32():
    mat = []
    for k in range(32):
        row = []
        for n in range(32):
            a = (k * (2 * n + 1)) % 128  # angle in units of pi / 64, one period
            c = math.cos(math.pi * a / 64)
            m = a if a <= 64 else 128 - a  # |cos| symmetric about pi
            if m > 32:
                m = 64 - m
            row.append(int(math.copysign(_COS_INT[m], c)) if abs(c) > 1e-9 else 0)
        mat.append(row)
    return mat


TRANS32 = trans_matrix_32()
DST4 = [[29, 55, 74, 84], [74, 74, 0, -74], [84, -29, -74, 55], [55, -84, 74, -29]]


def _basis(n, dst):
    if dst:
        return DST4
    step = 32 // n
    return [TRANS32[j * step][:n] for j in range(n)]


def transform_1d(x, n, dst):
    """y[i] = sum_j transMatrix[j][i] * x[j] (eq. 8-318 / 8-319)."""
    b = _basis(n, dst)
    return [sum(b[j][i] * x[j] for j in range(n)) for i in range(n)]


def inverse_transform(d, log2, dst=False, tskip=False):
    """Scaled coefficients d[y][x] -> residual r[y][x] (§8.6.4.1 / .2, 8-bit)."""
    n = 1 << log2
    bd_shift = 20 - BIT_DEPTH
    if tskip:  # §8.6.4.2 (v1): r = d << 7
        return [[(d[y][x] << 7) + (1 << (bd_shift - 1)) >> bd_shift for x in range(n)] for y in range(n)]
    coeff_min, coeff_max = -(1 << 15), (1 << 15) - 1
    # 1. vertical: each column
    e = [[0] * n for _ in range(n)]
    for x in range(n):
        col = transform_1d([d[y][x] for y in range(n)], n, dst)
        for y in range(n):
            e[y][x] = col[y]
    g = [[clip3(coeff_min, coeff_max, (e[y][x] + 64) >> 7) for x in range(n)] for y in range(n)]
    # 2. horizontal: each row
    r = []
    for y in range(n):
        row = transform_1d(g[y], n, dst)
        r.append([(v + (1 << (bd_shift - 1))) >> bd_shift for v in row])
    return r


LEVEL_SCALE = [40, 45, 51, 57, 64, 72]


def scale_level(level, qp, log2, m=16):
    """§8.6.3: TransCoeffLevel -> d (clipped to 16 bit)."""
    bd_shift = BIT_DEPTH + log2 - 5
    v = ((level * m * LEVEL_SCALE[qp % 6]) << (qp // 6)) + (1 << (bd_shift - 1))
    return clip3(-(1 << 15), (1 << 15) - 1, v >> bd_shift)


# ----------------------------------------------------------------------------- intra (8.4.4.2)
INTRA_PRED_ANGLE = {m: a for m, a in zip(range(2, 35), [32, 26, 21, 17, 13, 9, 5, 2, 0, -2, -5, -9, -13, -17, -21, -26,
                                                         -32, -26, -21, -17, -13, -9, -5, -2, 0, 2, 5, 9, 13, 17, 21,
                                                         26, 32])}
INV_ANGLE = {m: a for m, a in zip(range(11, 26), [-4096, -1638, -910, -630, -482, -390, -315, -256, -315, -390, -482,
                                                   -630, -910, -1638, -4096])}


def substitute(p, avail, n):
    """§8.4.4.2.2. p, avail: dicts keyed by (x, y) for x = -1, y = -1 .. 2n-1 and y = -1,
    x = 0 .. 2n-1. Unavailable samples are replaced by the search order of the clause."""
    order = [(-1, y) for y in range(2 * n - 1, -2, -1)] + [(x, -1) for x in range(0, 2 * n)]
    if not any(avail[k] for k in order):
        return {k: 1 << (BIT_DEPTH - 1) for k in order}
    out = dict(p)
    if not avail[order[0]]:
        for k in order[1:]:
            if avail[k]:
                out[order[0]] = p[k]
                break
    for i in range(1, len(order)):
        if not avail[order[i]]:
            out[order[i]] = out[order[i - 1]]
    return out


def filter_refs(p, n, mode, c_idx, strong_enabled):
    """§8.4.4.2.3 (applied to luma for 4:2:0)."""
    if c_idx != 0 or mode == 1 or n == 4:
        return p
    min_dist = min(abs(mode - 26), abs(mode - 10))
    thres = {8: 7, 16: 1, 32: 0}[n]
    if not min_dist > thres:
        return p
    tl = p[(-1, -1)]
    bi_int = (strong_enabled and c_idx == 0 and n == 32
              and abs(tl + p[(2 * n - 1, -1)] - 2 * p[(n - 1, -1)]) < (1 << (BIT_DEPTH - 5))
              and abs(tl + p[(-1, 2 * n - 1)] - 2 * p[(-1, n - 1)]) < (1 << (BIT_DEPTH - 5)))
    f = {(-1, -1): tl}
    if bi_int:
        for y in range(63):
            f[(-1, y)] = ((63 - y) * tl + (y + 1) * p[(-1, 63)] + 32) >> 6
        f[(-1, 63)] = p[(-1, 63)]
        for x in range(63):
            f[(x, -1)] = ((63 - x) * tl + (x + 1) * p[(63, -1)] + 32) >> 6
        f[(63, -1)] = p[(63, -1)]
    else:
        f[(-1, -1)] = (p[(-1, 0)] + 2 * tl + p[(0, -1)] + 2) >> 2
        for y in range(2 * n - 1):
            f[(-1, y)] = (p[(-1, y + 1)] + 2 * p[(-1, y)] + p[(-1, y - 1)] + 2) >> 2
        f[(-1, 2 * n - 1)] = p[(-1, 2 * n - 1)]
        for x in range(2 * n - 1):
            f[(x, -1)] = (p[(x - 1, -1)] + 2 * p[(x, -1)] + p[(x + 1, -1)] + 2) >> 2
        f[(2 * n - 1, -1)] = p[(2 * n - 1, -1)]
    return f


def predict(p, n, mode, c_idx):
    """§8.4.4.2.4-6 -> pred[y][x] from the (filtered) references p[(x, y)]."""
    log2 = n.bit_length() - 1
    pred = [[0] * n for _ in range(n)]
    if mode == 0:  # planar
        for y in range(n):
            for x in range(n):
                pred[y][x] = ((n - 1 - x) * p[(-1, y)] + (x + 1) * p[(n, -1)] + (n - 1 - y) * p[(x, -1)]
                              + (y + 1) * p[(-1, n)] + n) >> (log2 + 1)
        return pred
    if mode == 1:  # DC
        dc = (sum(p[(x, -1)] for x in range(n)) + sum(p[(-1, y)] for y in range(n)) + n) >> (log2 + 1)
        for y in range(n):
            for x in range(n):
                pred[y][x] = dc
        if c_idx == 0 and n < 32:
            pred[0][0] = (p[(-1, 0)] + 2 * dc + p[(0, -1)] + 2) >> 2
            for x in range(1, n):
                pred[0][x] = (p[(x, -1)] + 3 * dc + 2) >> 2
            for y in range(1, n):
                pred[y][0] = (p[(-1, y)] + 3 * dc + 2) >> 2
        return pred
    angle = INTRA_PRED_ANGLE[mode]
    ref = {}
    if mode >= 18:
        for x in range(n + 1):
            ref[x] = p[(-1 + x, -1)]
        if angle < 0:
            if (n * angle) >> 5 < -1:
                for x in range((n * angle) >> 5, 0):
                    ref[x] = p[(-1, -1 + ((x * INV_ANGLE[mode] + 128) >> 8))]
        else:
            for x in range(n + 1, 2 * n + 1):
                ref[x] = p[(-1 + x, -1)]
        for y in range(n):
            i_idx, i_fact = ((y + 1) * angle) >> 5, ((y + 1) * angle) & 31
            for x in range(n):
                if i_fact:
                    pred[y][x] = ((32 - i_fact) * ref[x + i_idx + 1] + i_fact * ref[x + i_idx + 2] + 16) >> 5
                else:
                    pred[y][x] = ref[x + i_idx + 1]
        if mode == 26 and c_idx == 0 and n < 32:
            for y in range(n):
                pred[y][0] = clip1(p[(0, -1)] + ((p[(-1, y)] - p[(-1, -1)]) >> 1))
    else:
        for x in range(n + 1):
            ref[x] = p[(-1, -1 + x)]
        if angle < 0:
            if (n * angle) >> 5 < -1:
                for x in range((n * angle) >> 5, 0):
                    ref[x] = p[(-1 + ((x * INV_ANGLE[mode] + 128) >> 8), -1)]
        else:
            for x in range(n + 1, 2 * n + 1):
                ref[x] = p[(-1, -1 + x)]
        for x in range(n):
            i_idx, i_fact = ((x + 1) * angle) >> 5, ((x + 1) * angle) & 31
            for y in range(n):
                if i_fact:
                    pred[y][x] = ((32 - i_fact) * ref[y + i_idx + 1] + i_fact * ref[y + i_idx + 2] + 16) >> 5
                else:
                    pred[y][x] = ref[y + i_idx + 1]
        if mode == 10 and c_idx == 0 and n < 32:
            for x in range(n):
                pred[0][x] = clip1(p[(-1, 0)] + ((p[(x, -1)] - p[(-1, -1)]) >> 1))
    return pred


def intra(p, avail, n, mode, c_idx, strong_enabled):
    p = substitute(p, avail, n)
    p = filter_refs(p, n, mode, c_idx, strong_enabled)
    return predict(p, n, mode, c_idx)


# ----------------------------------------------------------------------------- inter (8.5.3.3)
FL = {1: [-1, 4, -10, 58, 17, -5, 1, 0], 2: [-1, 4, -11, 40, 40, -11, 4, -1], 3: [0, 1, -5, 17, 58, -10, 4, -1]}
FC = {1: [-2, 58, 10, -2], 2: [-4, 54, 16, -2], 3: [-6, 46, 28, -4], 4: [-4, 36, 36, -4], 5: [-4, 28, 46, -6],
      6: [-2, 16, 54, -4], 7: [-2, 10, 58, -2]}
SHIFT1, SHIFT2, SHIFT3 = min(4, BIT_DEPTH - 8), 6, max(2, 14 - BIT_DEPTH)


def luma_sample(ref, x_int, y_int, x_frac, y_frac):
    """§8.5.3.3.3.1: ref[y][x] picture with clamped coordinates -> predSampleLX (14 bit)."""
    h, w = len(ref), len(ref[0])

    def at(x, y):
        return ref[clip3(0, h - 1, y)][clip3(0, w - 1, x)]

    if x_frac == 0 and y_frac == 0:
        return at(x_int, y_int) << SHIFT3
    if y_frac == 0:
        return sum(FL[x_frac][i] * at(x_int + i - 3, y_int) for i in range(8)) >> SHIFT1
    if x_frac == 0:
        return sum(FL[y_frac][i] * at(x_int, y_int + i - 3) for i in range(8)) >> SHIFT1
    temp = [sum(FL[x_frac][i] * at(x_int + i - 3, y_int + n - 3) for i in range(8)) >> SHIFT1 for n in range(8)]
    return sum(FL[y_frac][i] * temp[i] for i in range(8)) >> SHIFT2


def chroma_sample(ref, x_int, y_int, x_frac, y_frac):
    """§8.5.3.3.3.2 (eighth-sample chroma)."""
    h, w = len(ref), len(ref[0])

    def at(x, y):
        return ref[clip3(0, h - 1, y)][clip3(0, w - 1, x)]

    if x_frac == 0 and y_frac == 0:
        return at(x_int, y_int) << SHIFT3
    if y_frac == 0:
        return sum(FC[x_frac][i] * at(x_int + i - 1, y_int) for i in range(4)) >> SHIFT1
    if x_frac == 0:
        return sum(FC[y_frac][i] * at(x_int, y_int + i - 1) for i in range(4)) >> SHIFT1
    temp = [sum(FC[x_frac][i] * at(x_int + i - 1, y_int + n - 1) for i in range(4)) >> SHIFT1 for n in range(4)]
    return sum(FC[y_frac][i] * temp[i] for i in range(4)) >> SHIFT2


def default_weighted(p0, p1=None):
    """§8.5.3.3.4.2."""
    shift1, shift2 = 14 - BIT_DEPTH, 15 - BIT_DEPTH
    if p1 is None:
        return clip1((p0 + (1 << (shift1 - 1))) >> shift1)
    return clip1((p0 + p1 + (1 << (shift2 - 1))) >> shift2)


def explicit_weighted(log2wd, w0, o0, p0, w1=None, o1=None, p1=None):
    """§8.5.3.3.4.3 (offsets already scaled to the bit depth)."""
    if p1 is None:
        if log2wd >= 1:
            return clip1(((p0 * w0 + (1 << (log2wd - 1))) >> log2wd) + o0)
        return clip1(p0 * w0 + o0)
    return clip1((p0 * w0 + p1 * w1 + ((o0 + o1 + 1) << log2wd)) >> (log2wd + 1))


# ----------------------------------------------------------------------------- deblocking (8.7.2)
BETA_PRIME = [0] * 16 + [6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 28, 30, 32, 34, 36, 38, 40, 42,
                         44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64]
TC_PRIME = ([0] * 18 + [1] * 9 + [2] * 4 + [3] * 4 + [4] * 3
            + [5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24])
assert len(BETA_PRIME) == 52 and len(TC_PRIME) == 54


def qpc_420(qpi):
    """Table 8-10 (ChromaArrayType 1)."""
    if qpi < 30:
        return qpi
    if qpi > 43:
        return qpi - 6
    return [29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37][qpi - 30]


def deblock_luma(lines, bs, qpl, beta_offset, tc_offset, nfp=False, nfq=False):
    """One 4-line edge segment; lines[k] = [p3, p2, p1, p0, q0, q1, q2, q3]. beta_offset /
    tc_offset are slice_*_offset_div2 * 2. Returns the filtered lines (§8.7.2.5.3, .6, .7)."""
    beta = BETA_PRIME[clip3(0, 51, qpl + beta_offset)] * (1 << (BIT_DEPTH - 8))
    tc = TC_PRIME[clip3(0, 53, qpl + 2 * (bs - 1) + tc_offset)] * (1 << (BIT_DEPTH - 8))
    P = [[ln[3 - i] for i in range(4)] for ln in lines]   # P[k][i] = p_i,k
    Q = [[ln[4 + i] for i in range(4)] for ln in lines]   # Q[k][i] = q_i,k
    dp0 = abs(P[0][2] - 2 * P[0][1] + P[0][0])
    dp3 = abs(P[3][2] - 2 * P[3][1] + P[3][0])
    dq0 = abs(Q[0][2] - 2 * Q[0][1] + Q[0][0])
    dq3 = abs(Q[3][2] - 2 * Q[3][1] + Q[3][0])
    dpq0, dpq3 = dp0 + dq0, dp3 + dq3
    dp, dq = dp0 + dp3, dq0 + dq3
    d = dpq0 + dpq3
    out = [list(ln) for ln in lines]
    if not d < beta:
        return out

    def dsam(k, dpq):
        return (dpq < (beta >> 2) and abs(P[k][3] - P[k][0]) + abs(Q[k][0] - Q[k][3]) < (beta >> 3)
                and abs(P[k][0] - Q[k][0]) < ((5 * tc + 1) >> 1))

    d_e = 2 if dsam(0, 2 * dpq0) and dsam(3, 2 * dpq3) else 1
    d_ep = dp < ((beta + (beta >> 1)) >> 3)
    d_eq = dq < ((beta + (beta >> 1)) >> 3)
    for k in range(4):
        p0, p1, p2, p3 = P[k]
        q0, q1, q2, q3 = Q[k]
        np_, nq = {}, {}
        if d_e == 2:
            np_[0] = clip3(p0 - 2 * tc, p0 + 2 * tc, (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3)
            np_[1] = clip3(p1 - 2 * tc, p1 + 2 * tc, (p2 + p1 + p0 + q0 + 2) >> 2)
            np_[2] = clip3(p2 - 2 * tc, p2 + 2 * tc, (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3)
            nq[0] = clip3(q0 - 2 * tc, q0 + 2 * tc, (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3)
            nq[1] = clip3(q1 - 2 * tc, q1 + 2 * tc, (p0 + q0 + q1 + q2 + 2) >> 2)
            nq[2] = clip3(q2 - 2 * tc, q2 + 2 * tc, (p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3)
        else:
            delta = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4
            if abs(delta) < tc * 10:
                delta = clip3(-tc, tc, delta)
                np_[0] = clip1(p0 + delta)
                nq[0] = clip1(q0 - delta)
                if d_ep:
                    np_[1] = clip1(p1 + clip3(-(tc >> 1), tc >> 1, (((p2 + p0 + 1) >> 1) - p1 + delta) >> 1))
                if d_eq:
                    nq[1] = clip1(q1 + clip3(-(tc >> 1), tc >> 1, (((q2 + q0 + 1) >> 1) - q1 - delta) >> 1))
        if not nfp:
            for i, v in np_.items():
                out[k][3 - i] = v
        if not nfq:
            for i, v in nq.items():
                out[k][4 + i] = v
    return out


def deblock_chroma(lines, qpp, qpq, c_qp_pic_offset, tc_offset):
    """§8.7.2.5.5 (bS 2 edges); lines[k] = [p1, p0, q0, q1]."""
    qpi = ((qpq + qpp + 1) >> 1) + c_qp_pic_offset
    tc = TC_PRIME[clip3(0, 53, qpc_420(qpi) + 2 + tc_offset)] * (1 << (BIT_DEPTH - 8))
    out = []
    for p1, p0, q0, q1 in lines:
        delta = clip3(-tc, tc, ((((q0 - p0) << 2) + p1 - q1 + 4) >> 3))
        out.append([p1, clip1(p0 + delta), clip1(q0 - delta), q1])
    return out


# ----------------------------------------------------------------------------- SAO (8.7.3)
SAO_EO_OFFSETS = [((-1, 0), (1, 0)), ((0, -1), (0, 1)), ((-1, -1), (1, 1)), ((1, -1), (-1, 1))]


def sao_sample(nb, sao_type, band_position, eo_class, offset_val):
    """Centre of a 3 x 3 neighbourhood nb[y][x]; offset_val = SaoOffsetVal[1..4]."""
    v = nb[1][1]
    val = [0] + list(offset_val)
    if sao_type == 1:  # band offset
        band_table = [0] * 32
        for k in range(4):
            band_table[(k + band_position) & 31] = k + 1
        return clip1(v + val[band_table[v >> (BIT_DEPTH - 5)]])
    edge_idx = 2
    for dx, dy in SAO_EO_OFFSETS[eo_class]:
        edge_idx += sign(v - nb[1 + dy][1 + dx])
    if edge_idx in (0, 1, 2):
        edge_idx = 0 if edge_idx == 2 else edge_idx + 1
    return clip1(v + val[edge_idx])
