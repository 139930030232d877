"""Isolated hub (engine/isolated.py): one supervised worker process per GPU. A native fault
(here: SIGKILL of one worker process) takes down only that worker's cameras; the supervisor
starts a fresh process and re-adds them, while the other worker's cameras keep serving.
Reference: per-camera containers with restart: always
(server/services/rtsp_process_manager.go:70-81)."""
import os
import signal
import time

import pytest

from video_edge_ai_proxy_amd.config import Config


def farm(native, n):
    srv = native.RtspServer("127.0.0.1", 0)
    for i in range(n):
        c = native.SynthConfig()
        c.width, c.height, c.gop, c.fps, c.seed = 160, 96, 10, 30, 7 + i
        srv.add_stream(f"/c{i}", c, realtime=True, cached_frames=20)
    srv.start()
    return srv


def wait_frames(hub, name, timeout=20.0, after=0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        hub.touch(name)
        try:
            r = hub.latest_frame_bytes(name, after, 200)
        except RuntimeError:
            r = None
        if r:
            return r
        time.sleep(0.05)
    return None


def test_isolated_hub_restarts_a_dead_worker_process(native, tmp_path):
    from video_edge_ai_proxy_amd.engine.isolated import ProcessHub

    srv = farm(native, 2)
    cfg = Config()
    cfg.data_dir = str(tmp_path)
    cfg.gpu.isolation = "process"
    hub = ProcessHub(cfg, devices=[-1, -1], supervise_interval_s=0.2)
    try:
        for i in range(2):
            hub.start_camera(f"c{i}", f"rtsp://127.0.0.1:{srv.port}/c{i}")
        assert {hub.handle("c0").worker_index, hub.handle("c1").worker_index} == {0, 1}
        for n in ("c0", "c1"):
            r = wait_frames(hub, n)
            assert r is not None, n
            seq, frame, meta = r
            assert len(frame) > 160 * 96 * 3
        st = hub.state("c0")
        victim = st["worker_pid"]
        other = hub.state("c1")["worker_pid"]
        assert victim != other and victim != os.getpid()
        os.kill(victim, signal.SIGKILL)  # a native fault in that worker process
        deadline = time.time() + 60
        while time.time() < deadline and hub.child_restarts[hub.handle("c0").worker_index] == 0:
            # the other worker's camera keeps serving meanwhile
            assert wait_frames(hub, "c1", timeout=5) is not None
            time.sleep(0.1)
        wi = hub.handle("c0").worker_index
        assert hub.child_restarts[wi] == 1
        assert hub.state("c0")["worker_pid"] != victim
        assert wait_frames(hub, "c0", timeout=30) is not None  # re-added on the fresh process
        assert hub.state("c1")["worker_pid"] == other
        assert hub.workers[wi].frames >= 1
    finally:
        hub.shutdown()
        srv.stop()
