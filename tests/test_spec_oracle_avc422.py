"""H.264 4:2:2 arithmetic of avc_recon.h (shared by the CPU decoder, the gfx950 kernels and the
synthetic encoder) against the independent spec oracle (tests/spec_oracle.py): 8x16 intra chroma
prediction (the chroma4x4BlkIdx DC rules for the blocks below the first row, the plane mode with
yCF = 4 and the 5 / 64 vertical gradient weight) at 8 and 10 bits, and the 2x4 chroma DC (the
4:2:2 chroma DC scan, the 4x4 x 2x2 transform and the qP,DC = QP'C + 3 scaling) over the whole QP
range. The closed encoder / decoder loop is tests/test_avc_422.py."""
import random

import pytest

import spec_oracle as so

AVAIL = [(t, l) for t in (False, True) for l in (False, True)]
NORM00 = [10, 11, 13, 14, 16, 18]  # normAdjust4x4(m, 0, 0)


@pytest.mark.parametrize("bd", [8, 10])
def test_intra_chroma_8x16(native, bd):
    rc = native.recon
    rnd = random.Random(50 + bd)
    mx = (1 << bd) - 1
    for _ in range(40):
        top = [rnd.choice((0, mx, rnd.randint(0, mx))) for _ in range(9)]
        left = [rnd.choice((0, mx, rnd.randint(0, mx))) for _ in range(16)]
        for has_top, has_left in AVAIL:
            for mode in range(4):
                if (mode == 2 and not has_top) or (mode == 1 and not has_left) or \
                        (mode == 3 and not (has_top and has_left)):
                    continue
                got = rc.intra_chroma(top, left, has_top, has_left, mode, bd, 2)
                want = so.intra_chroma(top, left, has_top, has_left, mode, bd, cf=2)
                assert got == sum(want, []), (bd, mode, has_top, has_left)


def test_chroma422_dc(native):
    rc = native.recon
    rnd = random.Random(60)
    for qpc in range(0, 52 + 12):  # QP'C (High 10 up to 63)
        qpdc = qpc + 3
        ls = 16 * NORM00[qpdc % 6]  # flat scaling list
        for _ in range(8):
            lv = [rnd.choice((0, 0, 1, -1, rnd.randint(-40, 40))) for _ in range(8)]
            got = rc.chroma422_dc(lv, qpdc, ls)
            want = so.chroma422_dc(lv, qpdc, ls)
            assert got == [want[i][j] for i in range(4) for j in range(2)], (qpc, lv)


def test_cavlc_chroma422_dc_tables_round_trip(native):
    """nC = -2 coeff_token (Table 9-5) and the 2x4 total_zeros (Table 9-9b): every TotalCoeff /
    TrailingOnes / total_zeros / run combination of an 8-coefficient block writes and reads back
    (the decoder's tables are single-lookup decode tables built from the same code lists, so a
    code collision or a wrong length would break the round trip)."""
    rnd = random.Random(70)
    seen = set()
    for _ in range(4000):
        n = rnd.randint(0, 8)
        pos = sorted(rnd.sample(range(8), n))
        c = [0] * 8
        for p in pos:
            c[p] = rnd.choice((1, -1, 1, -1, rnd.randint(-60, 60) or 2))
        out, total = native.cavlc_roundtrip(-2, 8, c)
        assert list(out) == c and total == sum(1 for v in c if v), c
        nz = [v for v in c if v]
        t1 = 0
        for v in reversed(nz):
            if abs(v) == 1 and t1 < 3:
                t1 += 1
            else:
                break
        seen.add((len(nz), t1, (max(pos) + 1 - n) if n else 0))
    assert len({(t, o) for t, o, _ in seen}) == 30  # every coeff_token of the table
