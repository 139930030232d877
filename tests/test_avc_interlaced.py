"""Interlaced H.264 streams (SPS frame_mbs_only_flag 0). Frame pictures of an interlaced stream
(mb_adaptive_frame_field_flag 0) consist of frame macroblocks and decode like progressive ones;
their POC is min(top, bottom) with delta_pic_order_cnt_bottom (§8.2.1), the crop unit is 4 rows.
The Main / High encoder emits such streams (`interlaced`): CABAC and CAVLC, I / P / B, direct and
weighted prediction round-trip bit-exactly. Field pictures (PAFF) and MBAFF frames are reported
as UnsupportedStream (CABAC field decoding needs the field-coded context tables, ctxIdx
277..398 / 436..459, which no source in this image holds: parity unpinned)."""
import numpy as np
import pytest

from conftest import high_encoder, roundtrip


@pytest.mark.parametrize("kw", [dict(bframes=2), dict(bframes=1, cabac=False), dict(bframes=2, coverage=True),
                                dict(bframes=3, direct_spatial=False, weighted_b=2, slices=2)],
                         ids=["cabac-ibbp", "cavlc-ibp", "coverage", "temporal-implicit-slices"])
def test_interlaced_sps_frame_pictures_bit_exact(native, kw):
    enc = high_encoder(native, 176, 144, gop=10, seed=3, interlaced=True, **kw)
    rec, got, dec, aus = roundtrip(native, enc, 14)
    assert set(got) == set(rec)
    for pts in rec:
        assert np.array_equal(rec[pts][0], got[pts][0]) and np.array_equal(rec[pts][1], got[pts][1]), pts
    sps = enc.sps_nal  # frame_mbs_only_flag 0 in the SPS (parsed back by the decoder: 176x160 coded)
    assert dec.info["coded_height"] == 160 and dec.info["height"] == 144


def _set_field_pic_flag(nal):
    """Flip field_pic_flag of an IDR slice NAL (first_mb_in_slice, slice_type, pps_id as ue(v),
    frame_num as u(16)): the bit after them."""
    bits = "".join(f"{b:08b}" for b in nal[1:9])
    pos = 0
    for _ in range(3):  # three ue(v)
        z = 0
        while bits[pos] == "0":
            z += 1
            pos += 1
        pos += z + 1
    pos += 16  # frame_num (log2_max_frame_num 16)
    assert bits[pos] == "0"
    byte, bit = 1 + pos // 8, 7 - pos % 8
    out = bytearray(nal)
    out[byte] |= 1 << bit
    return bytes(out)


def test_field_pictures_are_rejected_as_unsupported(native):
    enc = high_encoder(native, 176, 144, gop=10, seed=3, interlaced=True, bframes=0)
    au = enc.next()
    nals = [(_set_field_pic_flag(bytes(n)) if (n[0] & 0x1F) == 5 else n) for n in au.nals()]
    au2 = native.AccessUnit.from_nals(nals, au.pts, au.dts, au.keyframe)
    with pytest.raises(native.UnsupportedStream, match="field pictures"):
        native.CpuDecoder().decode(au2)
