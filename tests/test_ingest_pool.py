"""Shared ingest machinery (csrc/vep/ioloop.h): many camera sessions are served by a fixed epoll
loop + parse strand pool + connector pool instead of one blocking thread per camera; the
threaded round-1 mode stays selectable (VEP_INGEST_THREADS=1). Reference behaviour being
replaced: one container + Python process per camera (python/rtsp_to_rtmp.py:49-187)."""
import os
import time

import pytest


def threads():
    return len(os.listdir("/proc/self/task"))


def farm(native, n, fps=30):
    srv = native.RtspServer("127.0.0.1", 0)
    for i in range(n):
        c = native.SynthConfig()
        c.width, c.height, c.gop, c.fps, c.seed = 160, 96, 10, fps, 100 + i
        srv.add_stream(f"/c{i}", c, realtime=True, cached_frames=20)
    srv.start()
    return srv


def run_sessions(native, n, seconds=2.0):
    srv = farm(native, n)
    w = native.Worker(device=-1)
    w.start()
    cams = [w.add_camera(f"c{i}", 4) for i in range(n)]
    base = threads()
    sess = []
    for i, cam in enumerate(cams):
        w.set_last_query(cam, int(time.time() * 1000))
        s = native.IngestSession(w, cam, f"c{i}", f"rtsp://127.0.0.1:{srv.port}/c{i}")
        s.start()
        sess.append(s)
    end = time.time() + seconds
    while time.time() < end:
        for cam in cams:
            w.set_last_query(cam, int(time.time() * 1000))
        time.sleep(0.1)
    grown = threads() - base
    decoded = [w.stats(cam)["decoded"] for cam in cams]
    states = [s.state()["status"] for s in sess]
    for s in sess:
        s.stop()
    w.stop()
    srv.stop()
    return grown, decoded, states


def test_pooled_ingest_uses_fixed_threads_threaded_mode_one_per_camera(native, monkeypatch):
    # (the loopback farm itself runs one server thread per connection: n in both runs)
    n = 24
    grown, decoded, states = run_sessions(native, n)
    assert all(st == "running" for st in states), states
    assert all(d > 5 for d in decoded), decoded
    monkeypatch.setenv("VEP_INGEST_THREADS", "1")
    grown_threaded, decoded_t, states_t = run_sessions(native, n)
    assert all(st == "running" for st in states_t)
    assert all(d > 5 for d in decoded_t), decoded_t
    assert grown_threaded >= 2 * n            # server + one ingest thread per camera
    assert grown <= n + 14, (grown, grown_threaded)  # server + the shared pools only


def test_pooled_session_restarts_after_server_loss(native):
    srv = farm(native, 1)
    w = native.Worker(device=-1)
    w.start()
    cam = w.add_camera("c0", 4)
    s = native.IngestSession(w, cam, "c0", f"rtsp://127.0.0.1:{srv.port}/c0")
    s.start()
    time.sleep(1.0)
    assert s.state()["status"] == "running"
    port = srv.port
    srv.stop()
    t = time.time()
    while time.time() - t < 8 and s.state()["status"] == "running":
        time.sleep(0.1)
    st = s.state()
    assert st["status"] == "restarting" and st["restart_count"] >= 1
    s.stop()
    assert s.state()["status"] == "exited"
    w.stop()


def test_stop_cancels_parse_backlog_before_slot_reuse(native, monkeypatch):
    # One parse thread and an unthrottled 640x480 compressed camera: the camera's parse strand
    # holds a backlog when the session stops. stop() must cancel/drain it, so after the slot is
    # removed and reused by a new camera, no stale access unit of the old stream reaches it
    # (ingest.cpp stop() left queued strand tasks running against the reused index).
    monkeypatch.setenv("VEP_INGEST_PARSE_THREADS", "1")
    srv = native.RtspServer("127.0.0.1", 0)
    c = native.SynthConfig()
    c.width, c.height, c.gop, c.seed = 640, 480, 30, 7
    c.compressed = True
    srv.add_stream("/fast", c, realtime=False, cached_frames=30)
    srv.start()
    w = native.Worker(device=-1)
    w.start()
    try:
        for _ in range(3):
            cam = w.add_camera("old", 2)
            w.set_last_query(cam, int(time.time() * 1000))
            s = native.IngestSession(w, cam, "old", f"rtsp://127.0.0.1:{srv.port}/fast")
            s.start()
            t = time.time()
            while time.time() - t < 10 and w.stats(cam)["decoded"] < 3:
                time.sleep(0.02)
            assert w.stats(cam)["decoded"] >= 3
            s.stop()
            w.remove_camera(cam)
            new = w.add_camera("new", 2)
            assert new == cam  # the slot is reused
            w.set_last_query(new, int(time.time() * 1000))
            time.sleep(0.5)
            st = w.stats(new)
            assert st["decoded"] == 0 and st["published"] == 0 and st["packets"] == 0, st
            w.remove_camera(new)
    finally:
        w.stop()
        srv.stop()
