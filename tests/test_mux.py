"""MP4 segments, FLV tags and RTMP publish -> sink round trip (CPU)."""
import struct
import time

import pytest

from conftest import synth


def boxes(buf, off=0, end=None):
    """Minimal ISO-BMFF walker: list of (type, payload_offset, size)."""
    end = len(buf) if end is None else end
    out = []
    while off + 8 <= end:
        size, typ = struct.unpack(">I4s", buf[off:off + 8])
        out.append((typ.decode(), off + 8, size))
        off += size
    return out


def find(buf, path):
    off, end = 0, len(buf)
    for name in path:
        for typ, p, size in boxes(buf, off, end):
            if typ == name:
                skip = {"stsd": 8, "avc1": 78}.get(name, 0)
                off, end = p + skip, p - 8 + size
                break
        else:
            raise KeyError(name)
    return off, end


def test_mp4_segment_structure(native):
    enc = synth(native, 320, 240, gop=10)
    aus = [enc.next() for _ in range(10)]
    for i, a in enumerate(aus):
        a.duration = 3000
    mp4 = native.build_mp4(aus, 320, 240, enc.sps_nal, enc.pps_nal)
    top = [t for t, _, _ in boxes(mp4)]
    assert top == ["ftyp", "moov", "mdat"]
    o, e = find(mp4, ["moov", "trak", "mdia", "minf", "stbl", "stsz"])
    _, _, count = struct.unpack(">III", mp4[o:o + 12])
    sizes = struct.unpack(f">{count}I", mp4[o + 12:o + 12 + 4 * count])
    assert count == 10
    o, e = find(mp4, ["moov", "trak", "mdia", "minf", "stbl", "stco"])
    chunk_off = struct.unpack(">I", mp4[o + 8:o + 12])[0]
    # the first sample is the IDR in AVCC form: 4-byte length + slice NAL (SPS/PPS stripped)
    n0 = struct.unpack(">I", mp4[chunk_off:chunk_off + 4])[0]
    assert mp4[chunk_off + 4] & 0x1f == 5 and n0 + 4 == sizes[0]
    assert sum(sizes) == len(mp4) - chunk_off
    o, e = find(mp4, ["moov", "trak", "mdia", "minf", "stbl", "stss"])
    assert struct.unpack(">II", mp4[o + 4:o + 12]) == (1, 1)
    o, e = find(mp4, ["moov", "trak", "mdia", "mdhd"])
    ts, dur = struct.unpack(">II", mp4[o + 12:o + 20])
    assert (ts, dur) == (90000, 30000)
    o, e = find(mp4, ["moov", "trak", "mdia", "minf", "stbl", "stsd", "avc1", "avcC"])
    assert mp4[o] == 1 and mp4[o + 1] == 66  # configurationVersion, profile baseline
    assert native.segment_duration_ms(aus) == 333
    for a in aus:
        a.duration = 0  # no durations -> DTS span (archive.py:58-73)
    assert native.segment_duration_ms(aus) == 300


def test_flv_tags(native):
    enc = synth(native, 64, 48, gop=2)
    idr, p = enc.next(), enc.next()
    hdr = native.flv_file_header()
    assert hdr[:3] == b"FLV" and len(hdr) == 13
    seq = native.flv_sequence_header(enc.sps_nal, enc.pps_nal)
    assert seq[:2] == b"\x17\x00" and seq[5] == 1
    body = native.flv_video_body(idr)
    assert body[:2] == b"\x17\x01"
    nal_len = struct.unpack(">I", body[5:9])[0]
    assert body[9] & 0x1f == 5 and nal_len == len(body) - 9
    assert native.flv_video_body(p)[0] == 0x27
    tag = native.flv_tag(9, 0x01020304, body)
    assert tag[0] == 9 and tag[4:8] == b"\x02\x03\x04\x01"  # 24-bit ts + extended byte
    assert struct.unpack(">I", tag[-4:])[0] == len(body) + 11


def test_rtmp_publish_roundtrip(native):
    sink = native.RtmpSink("127.0.0.1", 0)
    sink.start()
    try:
        pub = native.RtmpPublisher(f"rtmp://127.0.0.1:{sink.port}/live/mykey", 3000)
        pub.connect()
        enc = synth(native, 160, 120, gop=5)
        pub.send_sequence_header(enc.sps_nal, enc.pps_nal)
        sent = []
        for i in range(12):
            au = enc.next()
            pub.send_au(au, i * 33)
            sent.append(native.flv_video_body(au))
        t0 = time.time()
        while sink.video_messages < 12 and time.time() - t0 < 5:
            time.sleep(0.02)
        assert sink.stream_key == "mykey" and sink.sequence_headers == 1
        assert sink.video_messages == 12 and sink.keyframes == 3
        assert sink.video_bodies()[1:] == sent  # chunked (4096 B) and reassembled byte-exact
        pub.close()
    finally:
        sink.stop()


def test_rtmp_connect_failure(native):
    with pytest.raises(native.NativeError):
        native.RtmpPublisher("rtmp://127.0.0.1:1/live/x", 500).connect()
    with pytest.raises(native.NativeError):
        native.RtmpPublisher("rtmp://127.0.0.1/onlyapp", 500)
