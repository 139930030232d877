"""Native H.265 subset codec (CPU): CABAC engine, parameter sets, PCM/skip coding-tree walk,
RTSP (RFC 7798) delivery, hvcC / enhanced-RTMP muxing.

Parity note: no external HEVC decoder exists in this image (no FFmpeg / PyAV / rocDecode), so
conformance of the synthetic bitstreams to third-party decoders is *parity unpinned*; these tests
pin the encoder/decoder pair against each other and against the encoder's ground-truth picture,
and the CABAC engine against a random-bin round trip.
"""
import struct

import numpy as np
import pytest

from conftest import synth


@pytest.mark.parametrize("seed,qp", [(1, 26), (2, 0), (3, 51), (4, 37)])
def test_cabac_engine_roundtrip(native, seed, qp):
    ok, nbytes = native.cabac_roundtrip(seed, 20000, qp)
    assert ok and nbytes > 0


def test_hevc_parameter_sets(native):
    enc = synth(native, 1920, 1080, codec="h265")
    sps = native.parse_hevc_sps(enc.sps_nal)
    assert (sps["width"], sps["height"]) == (1920, 1080)
    assert (sps["coded_width"], sps["coded_height"]) == (1920, 1088)
    assert sps["profile_idc"] == 1 and sps["ctb_size"] == 16 and sps["pcm"]
    assert sps["fps"] == 30.0
    # NAL header types: VPS 32, SPS 33, PPS 34
    assert [(n[0] >> 1) & 0x3f for n in (enc.vps_nal, enc.sps_nal, enc.pps_nal)] == [32, 33, 34]
    au = enc.next()
    types = [(n[0] >> 1) & 0x3f for n in au.nals()]
    assert types[:3] == [32, 33, 34] and types[3] == 19  # IDR_W_RADL
    assert au.codec == 1 and au.keyframe
    p = enc.next()
    assert [(n[0] >> 1) & 0x3f for n in p.nals()] == [1]  # TRAIL_R


@pytest.mark.parametrize("w,h,slices,merge", [(640, 480, 1, 1), (352, 288, 3, 5), (1920, 1080, 2, 2),
                                              (3840, 2160, 1, 1)])
def test_hevc_decoder_reconstructs_encoder_picture(native, w, h, slices, merge):
    enc = synth(native, w, h, gop=4, motion=0.1, slices=slices, codec="h265", merge_cands=merge)
    dec = native.CpuDecoder()
    for i in range(6):  # crosses an IDR
        au = enc.next()
        out = dec.decode(au)
        y, uv = enc.picture()
        yd, uvd = dec.surface()
        assert np.array_equal(y, yd) and np.array_equal(uv, uvd), i
        assert out.shape == (h, w, 3)
        info = dec.info
        assert info["pict_type"] == ("I" if i % 4 == 0 else "P")
        assert info["idr"] == (i % 4 == 0)
    # P pictures code only the moving object's CTBs
    assert 0 < dec.coded_mbs < (w // 16) * (h // 16) // 2


def test_hevc_emulation_prevention(native):
    enc = synth(native, 320, 240, gop=3, zero=True, codec="h265")
    dec = native.CpuDecoder()
    saw = False
    for _ in range(4):
        au = enc.next()
        saw |= any(native.find_epb(n) for n in au.nals())
        dec.decode(au)
        assert np.array_equal(enc.picture()[0], dec.surface()[0])
    assert saw


def test_hevc_and_h264_outputs_agree(native):
    """Same synthetic pictures through both codecs decode to identical BGR frames."""
    a = synth(native, 640, 360, gop=5, seed=9)
    b = synth(native, 640, 360, gop=5, seed=9, codec="h265")
    da, db = native.CpuDecoder(), native.CpuDecoder()
    for _ in range(7):
        assert np.array_equal(da.decode(a.next()), db.decode(b.next()))


def test_hevc_unsupported_is_reported(native):
    enc = synth(native, 320, 240, codec="h265")
    au = enc.next()
    nals = au.nals()
    bad = bytearray(nals[3])
    for i in range(4, len(bad)):  # wreck the CABAC payload after the slice header
        bad[i] = 0x00 if i % 3 else 0x01
    dec = native.CpuDecoder()
    with pytest.raises((native.UnsupportedStream, native.NativeError)):
        dec.decode(native.AccessUnit.from_nals(nals[:3] + [bytes(bad)], keyframe=True, codec=1))


def test_rtsp_serves_hevc(native):
    srv = native.RtspServer("127.0.0.1", 0)
    cfg = native.SynthConfig()
    cfg.width, cfg.height, cfg.gop, cfg.seed, cfg.codec = 320, 240, 6, 3, "h265"
    srv.add_stream("/hevc", cfg, realtime=False, cached_frames=12)
    srv.start()
    try:
        c = native.RtspClient(f"rtsp://127.0.0.1:{srv.port}/hevc", 3000)
        info = c.open()
        assert info["codec"] == "h265" and len(info["param_sets"]) == 3
        aus, _ = c.read(12, 10.0)
        c.close()
    finally:
        srv.stop()
    assert len(aus) == 12 and aus[0].keyframe and aus[0].codec == 1
    ref = synth(native, 320, 240, gop=6, seed=3, codec="h265")
    dec = native.CpuDecoder()
    for au in aus:
        ref.next()
        dec.decode(au)
        assert np.array_equal(dec.surface()[0], ref.picture()[0])


def test_hvcc_record_and_mp4(native):
    enc = synth(native, 320, 240, gop=5, codec="h265")
    rec = native.hvcc_record(enc.vps_nal, enc.sps_nal, enc.pps_nal)
    assert rec[0] == 1 and rec[1] & 0x1f == 1            # version, Main profile
    assert rec[12] == 123                                 # level 4.1
    assert rec[21] & 3 == 3                               # lengthSizeMinusOne
    assert rec[22] == 3                                   # VPS, SPS, PPS arrays
    off, types = 23, []
    for _ in range(3):
        types.append(rec[off] & 0x3f)
        n = struct.unpack(">H", rec[off + 3:off + 5])[0]
        off += 5 + n
    assert types == [32, 33, 34] and off == len(rec)
    aus = [enc.next() for _ in range(5)]
    mp4 = native.build_mp4(aus, 320, 240, enc.sps_nal, enc.pps_nal, vps=enc.vps_nal, codec=1)
    assert b"hvc1" in mp4 and b"hvcC" in mp4 and b"avcC" not in mp4
    assert mp4[8:12] == b"isom"


def test_enhanced_rtmp_hevc(native):
    enc = synth(native, 320, 240, gop=4, codec="h265")
    seq = native.flv_sequence_header(enc.sps_nal, enc.pps_nal, vps=enc.vps_nal, codec=1)
    assert seq[0] == 0x90 and seq[1:5] == b"hvc1"          # ExHeader | key | SequenceStart
    key = native.flv_video_body(enc.next())
    assert key[0] == 0x93 and key[1:5] == b"hvc1"          # key | CodedFramesX
    inter = native.flv_video_body(enc.next())
    assert inter[0] == 0xA3
    n = struct.unpack(">I", inter[5:9])[0]
    assert n + 9 == len(inter) and (inter[9] >> 1) & 0x3f == 1
    sink = native.RtmpSink()
    sink.start()
    try:
        pub = native.RtmpPublisher(f"rtmp://127.0.0.1:{sink.port}/live/hevckey", 3000)
        pub.connect()
        pub.send_sequence_header(enc.sps_nal, enc.pps_nal, vps=enc.vps_nal, codec=1)
        for i in range(4):
            pub.send_au(enc.next(), 33 * i)
        import time
        deadline = time.time() + 5
        while sink.video_messages < 4 and time.time() < deadline:
            time.sleep(0.02)
        pub.close()
    finally:
        sink.stop()
    assert sink.sequence_headers == 1 and sink.video_messages == 4 and sink.hevc_messages == 5
    assert sink.stream_key == "hevckey"
