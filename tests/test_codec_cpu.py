"""Bitstream, synthetic encoder and native subset decoder (CPU)."""
import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from conftest import synth


@given(st.lists(st.integers(0, 2**31 - 2), max_size=40), st.lists(st.integers(-2**30, 2**30), max_size=40))
@settings(max_examples=200, deadline=None)
def test_exp_golomb_roundtrip(native, ue, se):
    u, s, at_stop = native.bitwriter_roundtrip(ue, se)
    assert u == ue and s == se and at_stop


@given(st.binary(max_size=300))
@settings(max_examples=300, deadline=None)
def test_emulation_prevention_roundtrip(native, raw):
    esc = native.rbsp_to_ebsp(raw)
    # no start-code emulation survives escaping
    for i in range(len(esc) - 2):
        assert not (esc[i] == 0 and esc[i + 1] == 0 and esc[i + 2] <= 2)
    assert native.ebsp_to_rbsp(esc) == raw
    assert len(native.find_epb(esc)) == len(esc) - len(raw)


def test_split_annexb(native):
    stream = b"\x00\x00\x00\x01\x67\x42" + b"\x00\x00\x01\x68\xce" + b"\x00\x00\x01\x65\x88\x00"
    assert native.split_annexb(stream) == [b"\x67\x42", b"\x68\xce", b"\x65\x88"]


def test_sps_fields(native):
    enc = synth(native, 1920, 1080, fps=25)
    s = native.parse_sps(enc.sps_nal)
    assert (s["width"], s["height"]) == (1920, 1080)
    assert (s["coded_width"], s["coded_height"]) == (1920, 1088)
    assert s["fps"] == 25.0 and s["profile_idc"] == 66 and s["poc_type"] == 2


@pytest.mark.parametrize("w,h,slices,motion", [(640, 480, 1, 0.05), (1920, 1080, 3, 0.1), (176, 144, 9, 0.3), (64, 48, 1, 0.0)])
def test_decoder_reconstructs_encoder_picture(native, w, h, slices, motion):
    enc = synth(native, w, h, gop=7, motion=motion, slices=slices)
    dec = native.CpuDecoder()
    for i in range(16):
        au = enc.next()
        assert au.keyframe == (i % 7 == 0)
        bgr = dec.decode(au)
        y, uv = enc.picture()
        y2, uv2 = dec.surface()
        assert np.array_equal(y, y2) and np.array_equal(uv, uv2), i
        assert bgr.shape == (h, w, 3)
        info = dec.info
        assert info["pict_type"] == ("I" if i % 7 == 0 else "P")
        if i % 7:
            assert info["coded_mbs"] < (w // 16) * ((h + 15) // 16) or motion > 0.2


def test_p_frames_are_mostly_skip(native):
    enc = synth(native, 1920, 1080, gop=30, motion=0.05)
    idr = enc.next()
    p = enc.next()
    assert p.size < idr.size / 8


def test_emulation_prevention_in_stream(native):
    enc = synth(native, 320, 240, gop=3, zero=True)
    dec = native.CpuDecoder()
    seen = 0
    for _ in range(5):
        au = enc.next()
        seen += sum(len(native.find_epb(n)) for n in au.nals())
        dec.decode(au)
        y, uv = enc.picture()
        assert np.array_equal(dec.surface()[0], y)
    assert seen > 0


def _sps_interlaced():
    """An SPS RBSP (with NAL header) for an interlaced (field-coded) 64x64 Main-profile stream."""
    bits = []

    def u(n, v):
        bits.extend((v >> (n - 1 - i)) & 1 for i in range(n))

    def ue(v):
        x = v + 1
        n = x.bit_length()
        u(n - 1, 0)
        u(n, x)

    u(8, 0x67)
    u(8, 77), u(8, 0), u(8, 40)
    ue(0)           # sps_id
    ue(0)           # log2_max_frame_num - 4
    ue(2)           # pic_order_cnt_type
    ue(1)           # max_num_ref_frames
    u(1, 0)         # gaps
    ue(3), ue(1)    # 4 MBs wide, 2 map units (64x64 frame)
    u(1, 0)         # frame_mbs_only_flag = 0 -> interlaced
    u(1, 1)         # mb_adaptive_frame_field_flag = 1 -> MBAFF frames
    u(1, 1)         # direct_8x8_inference
    u(1, 0), u(1, 0)  # no crop, no VUI
    u(1, 1)
    while len(bits) % 8:
        bits.append(0)
    return bytes(int("".join(map(str, bits[i:i + 8])), 2) for i in range(0, len(bits), 8))


def test_unsupported_stream_is_reported(native):
    # MBAFF (interlaced frames with field / frame MB pairs) is outside the native decoder: it must
    # refuse loudly (VCN backend's job). (Interlaced streams of frame pictures decode:
    # tests/test_avc_interlaced.py.)
    enc = synth(native, 64, 48)
    au = enc.next()
    nals = au.nals()
    bad = native.AccessUnit.from_nals([_sps_interlaced(), nals[1], nals[2]], keyframe=True)
    with pytest.raises(native.UnsupportedStream):
        native.CpuDecoder().decode(bad)


def test_bt601_reference_matches_numpy(native):
    enc = synth(native, 96, 64, gop=1)
    au = enc.next()
    bgr = native.CpuDecoder().decode(au)
    y, uv = enc.picture()
    Y = y[:64, :96].astype(np.int64)
    U = uv[np.arange(64)[:, None] // 2, (np.arange(96)[None, :] // 2) * 2].astype(np.int64)
    V = uv[np.arange(64)[:, None] // 2, (np.arange(96)[None, :] // 2) * 2 + 1].astype(np.int64)
    c = (Y - 16) * 76309 + 32768
    r = np.clip((c + 104597 * (V - 128)) >> 16, 0, 255)
    g = np.clip((c - 25675 * (U - 128) - 53279 * (V - 128)) >> 16, 0, 255)
    b = np.clip((c + 132201 * (U - 128)) >> 16, 0, 255)
    assert np.array_equal(bgr, np.stack([b, g, r], -1).astype(np.uint8))
    # sanity vs float BT.601 matrix within 1 LSB
    rf = 1.164383 * (Y - 16) + 1.596027 * (V - 128)
    assert np.abs(np.clip(np.round(rf), 0, 255) - r).max() <= 1


@pytest.mark.parametrize("codec", ["h264", "h265"])
def test_ingest_scan_matches_parser_scan(native, codec):
    """AccessUnit.pin() records emulation-prevention bytes at ingest (fused into the pinned copy,
    or scan-only without a GPU); parsing with the recorded positions must decode identically to
    parsing with the parser's own scan."""
    enc = synth(native, 320, 240, gop=3, zero=True, codec=codec)
    a, b = native.CpuDecoder(), native.CpuDecoder()
    for _ in range(5):
        au = enc.next()
        want = a.decode(au)
        au.pin()
        assert np.array_equal(b.decode(au), want)
        assert np.array_equal(b.surface()[0], enc.picture()[0])
