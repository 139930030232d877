"""avc_recon.h (the reconstruction code the CPU decoder, the gfx950 kernels and both synthetic
encoders share) against the independent spec oracle (tests/spec_oracle.py, written from the
H.264 text), on randomised inputs: inverse transforms, dequantisation, every intra prediction
mode with every neighbour-availability combination, all 16 luma quarter-sample and all 64
chroma eighth-sample positions (including picture-edge clamping), the deblocking thresholds
and the luma / chroma edge filters for every bS."""
import random

import numpy as np
import pytest

import spec_oracle as so


@pytest.fixture(scope="module")
def rc(native):
    return native.recon


def test_inverse_transforms(rc):
    rnd = random.Random(1)
    for _ in range(400):
        d4 = [[rnd.randint(-2048, 2047) if rnd.random() < 0.5 else 0 for _ in range(4)] for _ in range(4)]
        assert rc.idct4(sum(d4, [])) == sum(so.inverse_4x4(d4), [])
        d8 = [[rnd.randint(-4096, 4095) if rnd.random() < 0.3 else 0 for _ in range(8)] for _ in range(8)]
        assert rc.idct8(sum(d8, [])) == sum(so.inverse_8x8(d8), [])


def test_dequant_4x4(rc):
    for qp in range(52):
        for i in range(4):
            for j in range(4):
                for c in (-37, -1, 1, 5, 200):
                    assert rc.dequant4(c, qp, i, j) == so.dequant_4x4(c, qp, i, j), (qp, i, j, c)


AVAIL = [(t, l) for t in (False, True) for l in (False, True)]


def test_intra_4x4_all_modes(rc):
    rnd = random.Random(2)
    for _ in range(60):
        top = [rnd.randint(0, 255) for _ in range(9)]
        left = [rnd.randint(0, 255) for _ in range(4)]
        for has_top, has_left in AVAIL:
            for mode in range(9):
                needs_top = mode in (0, 3, 4, 5, 6, 7)
                needs_left = mode in (1, 4, 5, 6, 8)
                if (needs_top and not has_top) or (needs_left and not has_left):
                    continue  # not allowed by the standard with these neighbours
                got = rc.intra4x4(top, left, has_top, has_left, mode)
                assert got == sum(so.intra_4x4(top, left, has_top, has_left, mode), []), (mode, has_top, has_left)


def test_intra_8x8_all_modes_with_reference_filtering(rc):
    rnd = random.Random(3)
    for _ in range(40):
        top = [rnd.randint(0, 255) for _ in range(17)]
        left = [rnd.randint(0, 255) for _ in range(8)]
        for has_top, has_left in AVAIL:
            for has_tl in ((False, True) if has_top and has_left else (False,)):
                for mode in range(9):
                    needs_top = mode in (0, 3, 4, 5, 6, 7)
                    needs_left = mode in (1, 4, 5, 6, 8)
                    if (needs_top and not has_top) or (needs_left and not has_left):
                        continue
                    if mode in (4, 5, 6) and not has_tl:
                        continue
                    got = rc.intra8x8(top, left, has_top, has_left, has_tl, mode)
                    want = so.intra_8x8(top, left, has_top, has_left, has_tl, mode)
                    assert got == sum(want, []), (mode, has_top, has_left, has_tl)


def test_intra_16x16_and_chroma(rc):
    rnd = random.Random(4)
    for _ in range(40):
        top = [rnd.randint(0, 255) for _ in range(17)]
        left = [rnd.randint(0, 255) for _ in range(16)]
        ctop = [rnd.randint(0, 255) for _ in range(9)]
        cleft = [rnd.randint(0, 255) for _ in range(8)]
        for has_top, has_left in AVAIL:
            for mode in range(4):
                ok16 = not ((mode == 0 and not has_top) or (mode == 1 and not has_left) or
                            (mode == 3 and not (has_top and has_left)))
                if ok16:
                    assert rc.intra16x16(top, left, has_top, has_left, mode) == \
                        sum(so.intra_16x16(top, left, has_top, has_left, mode), []), (mode, has_top, has_left)
                okc = not ((mode == 2 and not has_top) or (mode == 1 and not has_left) or
                           (mode == 3 and not (has_top and has_left)))
                if okc:
                    assert rc.intra_chroma(ctop, cleft, has_top, has_left, mode) == \
                        sum(so.intra_chroma(ctop, cleft, has_top, has_left, mode), []), (mode, has_top, has_left)


def test_luma_quarter_sample_interpolation(rc):
    rng = np.random.default_rng(5)
    plane = rng.integers(0, 256, size=(24, 40), dtype=np.uint8)
    rows = plane.tolist()
    for _ in range(300):
        xi, yi = int(rng.integers(-6, 46)), int(rng.integers(-6, 30))  # includes edge clamping
        for fx in range(4):
            for fy in range(4):
                assert rc.luma_qpel(plane, xi, yi, fx, fy) == so.luma_sample(rows, xi, yi, fx, fy), (xi, yi, fx, fy)


def test_chroma_eighth_sample_interpolation(rc):
    rng = np.random.default_rng(6)
    uv = rng.integers(0, 256, size=(12, 2 * 20), dtype=np.uint8)  # interleaved Cb/Cr
    comp = [uv[:, 0::2].tolist(), uv[:, 1::2].tolist()]
    for _ in range(120):
        xi, yi = int(rng.integers(-3, 23)), int(rng.integers(-3, 15))
        for c in (0, 1):
            for fx in range(8):
                for fy in range(8):
                    assert rc.chroma_epel(uv, c, xi, yi, fx, fy) == so.chroma_sample(comp[c], xi, yi, fx, fy)


def test_deblocking_thresholds(rc):
    for qp_p in range(0, 52, 3):
        for qp_q in range(0, 52, 5):
            for off_a, off_b in ((0, 0), (-12, 6), (12, -12), (4, 4)):
                alpha, beta, tc0 = rc.edge_params(qp_p, qp_q, off_a, off_b)
                assert (alpha, beta, list(tc0)) == (lambda a, b, t: (a, b, list(t)))(
                    *so.edge_thresholds(qp_p, qp_q, off_a, off_b))


def test_deblocking_edge_filters(rc):
    rnd = random.Random(7)
    for _ in range(4000):
        base = rnd.randint(10, 245)
        spread = rnd.choice((2, 6, 20, 60))
        p = [clip(base + rnd.randint(-spread, spread)) for _ in range(4)]
        q = [clip(base + rnd.randint(-spread, spread) + rnd.choice((0, 0, 8, -8))) for _ in range(4)]
        qp = rnd.randint(16, 51)
        alpha, beta, tc0s = so.edge_thresholds(qp, qp, 0, 0)
        bs = rnd.randint(1, 4)
        tc0 = tc0s[bs - 1] if bs < 4 else 0
        chroma = rnd.random() < 0.3
        got = rc.filter_line(p, q, bs, alpha, beta, tc0, chroma)
        want = so.filter_line(p, q, bs, alpha, beta, tc0, chroma)
        assert (list(got[0]), list(got[1])) == want, (p, q, bs, alpha, beta, tc0, chroma)


def clip(v):
    return max(0, min(255, v))


def test_intra_8x8_tap_forms(native):
    """The GPU kernel's branch-free Intra_8x8 form (one tap word per filtered reference and per
    (mode, x, y) sample) equals the direct formulas (intra8x8_filter_at / intra8x8_pred_g, which
    test_intra_8x8_all_modes_with_reference_filtering checks against the spec oracle) on random
    and extreme samples, every mode but DC and every availability combination."""
    assert native.avc_intra8x8_tap_check(1, 3000) == 0
    assert native.avc_intra8x8_tap_check(12345, 3000) == 0


@pytest.mark.parametrize("seed", [1, 7, 2024])
def test_sparse_coefficient_records(native, seed):
    """Sparse coefficient records (mask word per 16 coefficients, then the non-zero values) give
    back the dense blocks exactly: H.264 through store_mb -> expand_coefs (4x4 and 8x8
    transforms, any coded pattern, int16 extremes, every density from empty to full) and H.265
    through hk_sparse_store -> hk_sparse_expand for 4x4..32x32 TBs with unordered positions.
    The GPU kernels expand the same words (expand_coefs_wave / tu_wave), and the bit-exact
    decode tests cover them end to end."""
    assert tuple(native.sparse_coef_fuzz(seed, 2000)) == (0, 0)
