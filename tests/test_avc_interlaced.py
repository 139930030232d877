"""Interlaced H.264 streams (SPS frame_mbs_only_flag 0). Frame pictures of an interlaced stream
(mb_adaptive_frame_field_flag 0) consist of frame macroblocks and decode like progressive ones;
their POC is min(top, bottom) with delta_pic_order_cnt_bottom (§8.2.1), the crop unit is 4 rows.
The Main / High encoder emits such streams (`interlaced`): CABAC and CAVLC, I / P / B, direct and
weighted prediction round-trip bit-exactly. Field pictures (PAFF) are covered in
test_avc_paff.py; MBAFF frames are reported as UnsupportedStream (test_codec_cpu.py)."""
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
