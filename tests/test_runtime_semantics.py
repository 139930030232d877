"""Lazy decode / keyframe-only / GOP catch-up / idle cutoff / frame ring (CPU backend).

Reference semantics: python/rtsp_to_rtmp.py:94-160 and python/read_image.py:47-133."""
import time

import numpy as np
import pytest

from conftest import synth


@pytest.fixture
def live(native):
    w = native.Worker(device=-1)
    w.start()
    yield w
    w.stop()


def _now():
    return int(time.time() * 1000)


def test_no_query_no_decode(native, live):
    cam = live.add_camera("idle", 2)
    enc = synth(native, 64, 48, gop=4)
    for _ in range(6):
        assert live.submit_au(cam, enc.next()) is False
    live.flush()
    st = live.stats(cam)
    assert st["packets"] == 6 and st["decoded"] == 0 and st["published"] == 0


def test_packets_before_first_keyframe_are_skipped(native, live):
    cam = live.add_camera("late", 2)
    enc = synth(native, 64, 48, gop=4)
    aus = [enc.next() for _ in range(8)]
    live.set_last_query(cam, _now())
    for au in aus[1:4]:  # joined mid-GOP: P frames without their IDR
        assert live.submit_au(cam, au) is False
    assert live.stats(cam)["skipped"] == 3
    assert live.submit_au(cam, aus[4])  # next IDR starts decoding
    live.flush()
    assert live.stats(cam)["decoded"] == 1


def test_catch_up_reconstructs_current_frame(native, live):
    """P frames that arrived while nobody was watching are folded into one GPU update when a
    query arrives; the published picture equals a full sequential decode."""
    cam = live.add_camera("catchup", 2)
    enc = synth(native, 128, 96, gop=20, motion=0.2)
    ref = native.CpuDecoder()
    for _ in range(7):  # IDR + 6 P, no viewer
        au = enc.next()
        want = ref.decode(au)
        live.submit_au(cam, au)
    live.flush()
    assert live.stats(cam)["decoded"] == 0
    live.set_last_query(cam, _now())
    au = enc.next()
    want = ref.decode(au)
    assert live.submit_au(cam, au)
    live.flush()
    meta, got = live.read_latest(cam, 0)
    assert np.array_equal(got, want)
    assert meta["packet"] == 7 and meta["frame_type"] == "P" and meta["keyframe"] == 1
    assert live.stats(cam)["decoded"] == 1


def test_keyframe_only_mode(native, live):
    cam = live.add_camera("kf", 2)
    live.set_keyframe_only(cam, True)
    live.set_last_query(cam, _now())
    enc = synth(native, 64, 48, gop=5)
    types = []
    for i in range(15):
        live.submit_au(cam, enc.next())
        live.flush()
        r = live.read_latest(cam, 0)
        if r:
            types.append(r[0]["frame_type"])
    assert live.stats(cam)["decoded"] == 3  # the three IDRs only
    assert set(types) == {"I"}


def test_idle_cutoff(native, live):
    cam = live.add_camera("cut", 2)
    enc = synth(native, 64, 48, gop=3)
    live.set_last_query(cam, _now() - 11_000)  # last viewer left 11 s ago
    for _ in range(3):
        assert live.submit_au(cam, enc.next()) is False
    live.set_idle_cutoff_ms(cam, 60_000)
    assert live.submit_au(cam, enc.next())


def test_ring_cursor_semantics(native):
    w = native.Worker(device=-1)
    cam = w.add_camera("ring", 3)
    enc = synth(native, 64, 48, gop=10)
    w.decode_now(cam, enc.next())
    m1, _ = w.read_latest(cam, 0)
    assert w.read_latest(cam, m1["seq"]) is None  # nothing newer than the cursor
    assert w.wait_frame(cam, m1["seq"], 50) is False
    w.decode_now(cam, enc.next())
    assert w.wait_frame(cam, m1["seq"], 50) is True
    m2, _ = w.read_latest(cam, m1["seq"])
    assert m2["seq"] == m1["seq"] + 1 and m2["pts"] == 3000
    assert w.published(cam) == 2


def test_cpu_worker_nv12_consumer_matches_reference(native):
    import torch

    from video_edge_ai_proxy_amd import ops

    S = 64
    w = native.Worker(device=-1, letterbox_size=S, max_cameras=1, letterbox_format=1)
    buf = torch.zeros((1, S * S * 3 // 2), dtype=torch.uint8)
    w.set_consumer_buffers(buf.data_ptr(), 0, 1)
    cam = w.add_camera("c", 2)
    enc = synth(native, 96, 64, gop=4)
    ref = native.CpuDecoder()
    au = enc.next()
    ref.decode(au)
    w.decode_now(cam, au)
    yh, uvh = ref.surface()
    want = ops.letterbox_nv12_reference(torch.from_numpy(yh), torch.from_numpy(uvh), S, 96, 64)
    assert (buf[0].int() - want.int()).abs().max().item() <= 1


def corrupt_inner_pcm_header(native, au, records_from_end=100):
    """Same length, but one I_PCM MB header deep inside the slice is wrong: only the worker's
    speculative-header check can see it (the host walk does not read those bytes)."""
    nals = au.nals()
    sl = bytearray(nals[-1])
    pos = len(sl) - 1 - 386 * records_from_end
    assert sl[pos] == 0x0D and sl[pos + 1] == 0x00
    sl[pos] = 0x0E
    return native.AccessUnit.from_nals(nals[:-1] + [bytes(sl)], pts=au.pts, dts=au.dts,
                                       keyframe=True)


def run_speculation_check(native, device):
    wk = native.Worker(device=device)
    cam = wk.add_camera("spec", 3)
    enc = synth(native, 640, 480, gop=3, motion=0.2)
    ref = native.CpuDecoder()
    aus = [enc.next() for _ in range(7)]  # I P P I P P I
    wk.decode_now(cam, aus[0])
    wk.decode_now(cam, aus[1])
    assert wk.published(cam) == 2
    bad = corrupt_inner_pcm_header(native, aus[3])
    wk.decode_now(cam, bad)
    wk.decode_now(cam, aus[4])  # reference is garbage: suppressed until the next keyframe
    wk.decode_now(cam, aus[5])
    assert wk.published(cam) == 2 and wk.stats(cam)["errors"] == 1
    assert "I_PCM header check failed" in wk.logs(cam, True)
    wk.decode_now(cam, aus[6])
    assert wk.published(cam) == 3
    for a in aus:
        want = ref.decode(a)
    _, got = wk.read_latest(cam, 0)
    assert np.array_equal(got, want)


def test_speculative_keyframe_walk_is_verified_cpu(native):
    run_speculation_check(native, -1)
