"""RTP packetization, RTSP client/server (synthetic camera farm), fault injection (CPU)."""
import time

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from conftest import synth


def _rtp_stream(native, nals, codec, mtu, ts=1000, seq0=100):
    pkts = []
    seq = seq0
    for i, n in enumerate(nals):
        parts = native.packetize_nal(n, codec, mtu)
        for j, p in enumerate(parts):
            last = i == len(nals) - 1 and j == len(parts) - 1
            pkts.append(native.rtp_packet(p, seq & 0xFFFF, ts, last))
            seq += 1
    return pkts


@given(st.lists(st.binary(min_size=1, max_size=5000), min_size=1, max_size=6), st.integers(64, 1500))
@settings(max_examples=60, deadline=None)
def test_h264_packetize_roundtrip(native, bodies, mtu):
    nals = [bytes([0x41]) + b for b in bodies]  # non-IDR slice NALs
    d = native.Depacketizer(0)
    aus = []
    for p in _rtp_stream(native, nals, 0, mtu):
        aus += d.push(p)
    assert len(aus) == 1
    assert aus[0].nals() == nals and not aus[0].corrupt


@given(st.lists(st.binary(min_size=1, max_size=5000), min_size=1, max_size=6), st.integers(64, 1500))
@settings(max_examples=60, deadline=None)
def test_h265_packetize_roundtrip(native, bodies, mtu):
    nals = [bytes([19 << 1, 1]) + b for b in bodies]  # IDR_W_RADL NALs
    d = native.Depacketizer(1)
    aus = []
    for p in _rtp_stream(native, nals, 1, mtu):
        aus += d.push(p)
    assert len(aus) == 1 and aus[0].keyframe
    assert aus[0].nals() == nals


def test_aggregation_and_loss(native):
    sps, pps, idr = b"\x67\x42\x00\x1f", b"\x68\xce\x3c\x80", b"\x65" + bytes(range(1, 200)) * 20
    d = native.Depacketizer(0)
    stap = native.aggregate_nals([sps, pps], 0)
    pk = [native.rtp_packet(stap, 1, 90)]
    frags = native.packetize_nal(idr, 0, 500)
    pk += [native.rtp_packet(f, 2 + i, 90, i == len(frags) - 1) for i, f in enumerate(frags)]
    aus = []
    for p in pk:
        aus += d.push(p)
    assert len(aus) == 1 and aus[0].keyframe and aus[0].nals() == [sps, pps, idr]
    # drop the middle fragment of the next AU -> AU flagged corrupt, damaged NAL dropped
    pk2 = [native.rtp_packet(f, 2 + len(frags) + i, 180, i == len(frags) - 1) for i, f in enumerate(frags)]
    del pk2[1]
    aus = []
    for p in pk2:
        aus += d.push(p)
    assert len(aus) == 0 or aus[0].corrupt
    assert d.lost == 1


def test_url_and_base64(native):
    u = native.parse_url("rtsp://admin:pa:ss@10.0.0.5:8554/live/ch1")
    assert (u["user"], u["password"], u["host"], u["port"], u["path"]) == ("admin", "pa:ss", "10.0.0.5", 8554, "/live/ch1")
    assert native.parse_url("rtmp://h/app/key")["port"] == 1935
    for s in [b"", b"a", b"ab", b"abc", bytes(range(256))]:
        assert native.base64_decode(native.base64_encode(s)) == s


@pytest.fixture
def farm(native):
    srv = native.RtspServer("127.0.0.1", 0)
    cfg = native.SynthConfig()
    cfg.width, cfg.height, cfg.gop, cfg.seed = 320, 240, 8, 5
    srv.add_stream("/cam0", cfg, realtime=False, cached_frames=16)
    srv.add_stream("/secure", cfg, realtime=False, cached_frames=8, user="u", password="p")
    srv.start()
    yield srv, cfg
    srv.stop()


def test_rtsp_client_receives_decodable_stream(native, farm):
    srv, cfg = farm
    c = native.RtspClient(f"rtsp://127.0.0.1:{srv.port}/cam0", 3000)
    info = c.open()
    assert info["codec"] == "h264" and len(info["param_sets"]) == 2
    aus, why = c.read(20, 10.0)
    c.close()
    assert len(aus) == 20 and why == "stopped"
    assert aus[0].keyframe
    ref = synth(native, 320, 240, gop=8, seed=5)
    dec = native.CpuDecoder()
    for i, au in enumerate(aus):
        want = ref.next()
        if i >= 16:
            break  # cached loop restarts; pictures repeat
        got = dec.decode(au)
        assert np.array_equal(got, native.CpuDecoder().decode(want) if want.keyframe else got)
        y, _ = ref.picture()
        assert np.array_equal(dec.surface()[0], y), i
    assert aus[1].pts - aus[0].pts == 3000


def test_rtsp_basic_auth(native, farm):
    srv, _ = farm
    with pytest.raises(native.NativeError):
        native.RtspClient(f"rtsp://127.0.0.1:{srv.port}/secure", 2000).open()
    c = native.RtspClient(f"rtsp://u:p@127.0.0.1:{srv.port}/secure", 2000)
    c.open()
    aus, _ = c.read(3, 5.0)
    assert len(aus) == 3


def test_rtsp_unknown_path_and_refused_port(native, farm):
    srv, _ = farm
    with pytest.raises(native.NativeError):
        native.RtspClient(f"rtsp://127.0.0.1:{srv.port}/nope", 2000).open()
    with pytest.raises(native.NativeError):
        native.RtspClient("rtsp://127.0.0.1:1/x", 1000).open()


def test_fault_drop_connection_ends_stream(native, farm):
    srv, _ = farm
    c = native.RtspClient(f"rtsp://127.0.0.1:{srv.port}/cam0", 2000)
    c.open()
    aus, _ = c.read(4, 5.0)
    srv.inject("/cam0", native.Fault.DROP_CONNECTION)
    aus2, why = c.read(10**6, 5.0)
    assert why in ("eof", "recv error")
