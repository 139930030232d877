"""H.264 High 10 arithmetic of avc_recon.h (shared by the CPU decoder, the gfx950 kernels and the
synthetic encoder) against the independent spec oracle (tests/spec_oracle.py, written from the
H.264 text, at sample bit depth bd) on randomised 9 / 10-bit inputs: every intra prediction
mode (1 << (bd - 1) DC defaults, Clip1 at the depth in the plane modes), luma quarter-sample and
chroma eighth-sample interpolation on u16 planes, the scaled deblocking thresholds with
QPs below 0, the edge filters at the depth, and Table 8-15 with QpBdOffsetC.

This pins the depth-dependent pieces independently of the closed encoder / decoder loop
(tests/test_avc_high10.py); High 10 slice-data syntax parity stays unpinned (no third-party
High 10 stream in the image)."""
import random

import numpy as np
import pytest

import spec_oracle as so


@pytest.fixture(scope="module")
def rc(native):
    return native.recon


AVAIL = [(t, l) for t in (False, True) for l in (False, True)]
DEPTHS = (9, 10)


@pytest.mark.parametrize("bd", DEPTHS)
def test_intra_4x4_and_8x8_at_depth(rc, bd):
    rnd = random.Random(10 + bd)
    mx = (1 << bd) - 1
    for _ in range(30):
        top4 = [rnd.randint(0, mx) for _ in range(9)]
        left4 = [rnd.randint(0, mx) for _ in range(4)]
        top8 = [rnd.randint(0, mx) for _ in range(17)]
        left8 = [rnd.randint(0, mx) for _ in range(8)]
        for has_top, has_left in AVAIL:
            for mode in range(9):
                needs_top = mode in (0, 3, 4, 5, 6, 7)
                needs_left = mode in (1, 4, 5, 6, 8)
                if (needs_top and not has_top) or (needs_left and not has_left):
                    continue
                assert rc.intra4x4(top4, left4, has_top, has_left, mode, bd) == \
                    sum(so.intra_4x4(top4, left4, has_top, has_left, mode, bd), []), (bd, mode)
                for has_tl in ((False, True) if has_top and has_left else (False,)):
                    if mode in (4, 5, 6) and not has_tl:
                        continue
                    assert rc.intra8x8(top8, left8, has_top, has_left, has_tl, mode, bd) == \
                        sum(so.intra_8x8(top8, left8, has_top, has_left, has_tl, mode, bd), []), (bd, mode)


@pytest.mark.parametrize("bd", DEPTHS)
def test_intra_16x16_and_chroma_at_depth(rc, bd):
    rnd = random.Random(20 + bd)
    mx = (1 << bd) - 1
    for _ in range(30):
        # extremes too: the plane modes must clip at the depth, not at 255
        top = [rnd.choice((0, mx, rnd.randint(0, mx))) for _ in range(17)]
        left = [rnd.choice((0, mx, rnd.randint(0, mx))) for _ in range(16)]
        ctop = [rnd.randint(0, mx) for _ in range(9)]
        cleft = [rnd.randint(0, mx) for _ in range(8)]
        for has_top, has_left in AVAIL:
            for mode in range(4):
                if not ((mode == 0 and not has_top) or (mode == 1 and not has_left) or
                        (mode == 3 and not (has_top and has_left))):
                    assert rc.intra16x16(top, left, has_top, has_left, mode, bd) == \
                        sum(so.intra_16x16(top, left, has_top, has_left, mode, bd), []), (bd, mode)
                if not ((mode == 2 and not has_top) or (mode == 1 and not has_left) or
                        (mode == 3 and not (has_top and has_left))):
                    assert rc.intra_chroma(ctop, cleft, has_top, has_left, mode, bd) == \
                        sum(so.intra_chroma(ctop, cleft, has_top, has_left, mode, bd), []), (bd, mode)
    # no neighbours: DC is 1 << (bd - 1)
    assert set(rc.intra16x16([0] * 17, [0] * 16, False, False, 2, bd)) == {1 << (bd - 1)}


@pytest.mark.parametrize("bd", DEPTHS)
def test_interpolation_on_u16_planes(rc, bd):
    rng = np.random.default_rng(30 + bd)
    plane = rng.integers(0, 1 << bd, size=(24, 40), dtype=np.uint16)
    plane[3:6, 5:9] = (1 << bd) - 1  # saturated patches: the 6-tap clips at the depth
    plane[10:12, 20:26] = 0
    rows = plane.tolist()
    for _ in range(150):
        xi, yi = int(rng.integers(-6, 46)), int(rng.integers(-6, 30))
        for fx in range(4):
            for fy in range(4):
                assert rc.luma_qpel16(plane, xi, yi, fx, fy, bd) == so.luma_sample(rows, xi, yi, fx, fy, bd)
    uv = rng.integers(0, 1 << bd, size=(12, 40), dtype=np.uint16)
    comp = [uv[:, 0::2].tolist(), uv[:, 1::2].tolist()]
    for _ in range(60):
        xi, yi = int(rng.integers(-3, 23)), int(rng.integers(-3, 15))
        for c in (0, 1):
            for fx in range(8):
                for fy in range(8):
                    assert rc.chroma_epel16(uv, c, xi, yi, fx, fy) == so.chroma_sample(comp[c], xi, yi, fx, fy)


@pytest.mark.parametrize("bd", DEPTHS)
def test_deblocking_at_depth(rc, bd):
    off = 6 * (bd - 8)
    for qp_p in range(-off, 52, 4):
        for qp_q in range(-off, 52, 7):
            for oa, ob in ((0, 0), (-12, 6), (12, -12)):
                a, b, t = rc.edge_params(qp_p, qp_q, oa, ob, bd)
                assert (a, b, list(t)) == so.edge_thresholds(qp_p, qp_q, oa, ob, bd)
    rnd = random.Random(40 + bd)
    mx = (1 << bd) - 1
    for _ in range(3000):
        base = rnd.randint(8, mx - 8)
        spread = rnd.choice((4, 16, 60, 200))
        p = [max(0, min(mx, base + rnd.randint(-spread, spread))) for _ in range(4)]
        q = [max(0, min(mx, base + rnd.randint(-spread, spread) + rnd.choice((0, 0, 30, -30)))) for _ in range(4)]
        qp = rnd.randint(-off, 51)
        alpha, beta, tc0s = so.edge_thresholds(qp, qp, 0, 0, bd)
        bs = rnd.randint(1, 4)
        tc0 = tc0s[bs - 1] if bs < 4 else 0
        chroma = rnd.random() < 0.3
        want = so.filter_line(p, q, bs, alpha, beta, tc0, chroma, bd)
        got = rc.filter_line(p, q, bs, alpha, beta, tc0, chroma, bd)
        assert (list(got[0]), list(got[1])) == want
        # the GPU High 10 / 4:2:2 loop filter's one-stream luma / chroma form
        got = rc.filter_line(p, q, bs, alpha, beta, tc0, chroma, bd, True)
        assert (list(got[0]), list(got[1])) == want


def test_chroma_qp_and_qp_wrap(rc):
    for bd in (8, 9, 10):
        off = 6 * (bd - 8)
        for qpy in range(-off, 52):
            for o in range(-12, 13):
                assert rc.chroma_qp_bd(qpy, o, off) == so.chroma_qp(qpy, o, bd)
        # 7-37: the QP range wraps at -QpBdOffsetY / 51 (the decoder's MbLayer formula)
        assert so.mb_qp(51, 1, bd) == -off
        assert so.mb_qp(-off, -1, bd) == 51
