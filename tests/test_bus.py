"""Frame bus (csrc/vep/bus.h) and the serving processes that read it (server/frontend.py).

The bus replaces the reference's Redis frame stream (python/read_image.py:121 XADD,
server/grpcapi/grpc_api.go:186-231 XREAD): an owner process publishes its cameras' frames on
demand into shared memory, any process reads them. Checked here on the CPU backend: frames equal
the in-process VideoFrame encoding, a reader in another process gets the same bytes, one DMA
serves every reader of a frame, camera removal / owner shutdown wake waiting readers, and
``serving.frontends`` processes bound with SO_REUSEPORT serve VideoLatestImage from the bus while
forwarding the other RPCs to the main process (and are restarted when one dies)."""
import json
import os
import signal
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

from conftest import synth
from video_edge_ai_proxy_amd.models import StreamProcess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _owner(native, tag, n=4):
    w = native.Worker(device=-1)
    w.start()
    o = native.BusOwner(tag, 0, n)
    o.attach(w)
    return w, o


def test_bus_roundtrip_matches_in_process_encoding(native):
    from video_edge_ai_proxy_amd.proto import pb

    tag = f"t{os.getpid()}a"
    w, o = _owner(native, tag)
    try:
        cam = w.add_camera("camA", 3)
        o.add(cam, "camA")
        r = native.BusReader(tag)
        assert r.has("camA") and r.names() == ["camA"] and not r.has("nope")
        assert r.frame("camA", 0, 30, 0) is None  # nothing decoded yet: times out
        enc, ref = synth(native, 320, 240, gop=5), native.CpuDecoder()
        for k in range(3):
            au = enc.next()
            want = ref.decode(au)
            got = {}
            th = threading.Thread(target=lambda: got.setdefault("f", r.frame("camA", k, 3000, 0)))
            th.start()  # waiting reader: woken by the publish hook -> pump -> futex
            time.sleep(0.05)
            w.decode_now(cam, au)
            th.join()
            seq, data = got["f"]
            assert seq == k + 1
            seq2, same, _ = w.video_frame(cam, 0, "camA")  # the in-process serving path
            assert seq2 == seq and data == same
            vf = pb.VideoFrame.FromString(data)
            assert (vf.width, vf.height, vf.device_id) == (320, 240, "camA")
            assert np.array_equal(np.frombuffer(vf.data, np.uint8).reshape(240, 320, 3), want)
        # a caller that holds the newest frame's bytes is told so instead of copying them again
        assert r.frame("camA", 0, 100, 0, 3) == (3, None)
        assert r.frame("camA", 3, 30, 0) is None  # nothing newer
        assert o.published == 3  # one DMA per frame, however many readers
        # demand reaches the camera's control atomics (the lazy decoder's last_query / mode)
        r.touch("camA", 1)
        time.sleep(0.1)
        assert w.keyframe_only(cam) and w.last_query(cam) > 0
        o.remove(cam)
        assert not r.has("camA") and r.frame("camA", 0, 30, 0) is None
    finally:
        o.stop()
        w.stop()


def test_bus_reader_in_another_process(native, tmp_path):
    """A reader process (no worker, no GPU) gets the owner's frames: the same bytes."""
    tag = f"t{os.getpid()}b"
    w, o = _owner(native, tag)
    code = f"""
import sys, json, hashlib
sys.path.insert(0, {ROOT!r})
from video_edge_ai_proxy_amd import native
r = native.BusReader({tag!r})
print("ready", flush=True)
seen = []
after = 0
while len(seen) < 3:
    f = r.frame("cam", after, 5000, 0)
    if f is None:
        break
    after = f[0]
    seen.append([f[0], hashlib.sha1(f[1]).hexdigest()])
print(json.dumps(seen), flush=True)
"""
    try:
        cam = w.add_camera("cam", 3)
        o.add(cam, "cam")
        p = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True)
        assert p.stdout.readline().strip() == "ready"
        enc = synth(native, 160, 96, gop=4)
        want = {}
        import hashlib

        for _ in range(3):
            time.sleep(0.3)
            w.decode_now(cam, enc.next())
            seq, data, _ = w.video_frame(cam, 0, "cam")
            want[seq] = hashlib.sha1(data).hexdigest()
        out = p.stdout.readline()
        p.wait(timeout=60)
        seen = json.loads(out)
        assert [s for s, _ in seen] == [1, 2, 3]
        assert all(want[s] == h for s, h in seen)
    finally:
        o.stop()
        w.stop()


def test_bus_owner_stop_wakes_readers_and_cleans_up(native):
    tag = f"t{os.getpid()}c"
    w, o = _owner(native, tag)
    cam = w.add_camera("cam", 2)
    o.add(cam, "cam")
    r = native.BusReader(tag)
    res = {}
    th = threading.Thread(target=lambda: res.setdefault("f", r.frame("cam", 0, 10000, 0)))
    t0 = time.time()
    th.start()
    time.sleep(0.1)
    o.stop()
    th.join(timeout=5)
    assert res["f"] is None and time.time() - t0 < 3
    path = o.path
    del o
    w.stop()
    assert not os.path.exists(path)
    assert native.bus_remove_segments(os.getpid()) == 0


def _frontend_app(tmp_path, n):
    from video_edge_ai_proxy_amd.config import Config
    from video_edge_ai_proxy_amd.server.app import build_app

    cfg = Config()
    cfg.data_dir = str(tmp_path / "data")
    cfg.gpu.devices = [-1]
    cfg.serving.frontends = n
    cfg.serving.threads = 32
    return build_app(cfg, host="127.0.0.1", rest_port=0, grpc_port=0, start_rest=False)


def _frames(cli, name, n, timeout=30.0):
    import grpc

    got, deadline = [], time.time() + timeout
    while len(got) < n and time.time() < deadline:
        try:
            vf = cli.latest_frame(name, timeout=10)
        except grpc.RpcError as e:  # (a restarted serving process is not listening yet)
            assert e.code() == grpc.StatusCode.UNAVAILABLE, e
            time.sleep(0.2)
            continue
        if vf is not None and vf.width:
            got.append(vf)
    return got


def test_serving_processes_serve_frames_and_forward_control(native, tmp_path):
    import grpc

    from video_edge_ai_proxy_amd.proto import pb
    from video_edge_ai_proxy_amd.server.grpc_server import ImageClient

    srv = native.RtspServer("127.0.0.1", 0)
    c = native.SynthConfig()
    c.width, c.height, c.gop, c.fps, c.seed = 160, 96, 10, 30, 3
    srv.add_stream("/cam", c, realtime=True, cached_frames=20)
    srv.start()
    app = _frontend_app(tmp_path, 2)
    try:
        assert app.frontends is not None and app.grpc_port != app.grpc_server.bound_port
        app.pm.start(StreamProcess(name="cam1", rtsp_endpoint=f"rtsp://127.0.0.1:{srv.port}/cam"))
        cli = ImageClient(f"127.0.0.1:{app.grpc_port}")
        vfs = _frames(cli, "cam1", 3)
        assert len(vfs) == 3 and all((v.width, v.height) == (160, 96) for v in vfs)
        assert vfs[0].shape.dim[2].size == 3 and vfs[0].device_id == "cam1"
        # the cursor is per connection: consecutive requests get newer frames
        assert vfs[0].pts != vfs[1].pts != vfs[2].pts
        # unknown camera: an empty frame (after the reference's waits), not an error
        empty = cli.latest_frame("nope", timeout=20)
        assert empty is not None and not empty.width
        # forwarded RPCs: ListStreams and a validation error from Annotate
        names = [m.name for m in cli.ListStreams(pb.ListStreamRequest(), timeout=20)]
        assert names == ["cam1"]
        with pytest.raises(grpc.RpcError) as e:
            cli.Annotate(pb.AnnotateRequest(device_name="cam1"), timeout=20)
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        # /metrics sees the serving processes' frames
        time.sleep(1.5)
        assert app.frontends.frames_served() >= 3
        cli.close()
    finally:
        app.stop()
        srv.stop()


def test_serving_process_restart(native, tmp_path):
    """A serving process that dies is restarted by the supervisor; clients reconnect."""
    import psutil

    from video_edge_ai_proxy_amd.server.grpc_server import ImageClient

    srv = native.RtspServer("127.0.0.1", 0)
    c = native.SynthConfig()
    c.width, c.height, c.gop, c.fps, c.seed = 160, 96, 10, 30, 5
    srv.add_stream("/cam", c, realtime=True, cached_frames=20)
    srv.start()
    app = _frontend_app(tmp_path, 1)
    try:
        app.pm.start(StreamProcess(name="cam1", rtsp_endpoint=f"rtsp://127.0.0.1:{srv.port}/cam"))
        cli = ImageClient(f"127.0.0.1:{app.grpc_port}")
        assert len(_frames(cli, "cam1", 2)) == 2
        sup = psutil.Process(app.frontends.p.pid)
        kids = sup.children()
        assert len(kids) == 1
        os.kill(kids[0].pid, signal.SIGKILL)
        deadline = time.time() + 60
        while time.time() < deadline:
            now = [k.pid for k in sup.children()]
            if now and now[0] != kids[0].pid:
                break
            time.sleep(0.2)
        assert sup.children() and sup.children()[0].pid != kids[0].pid
        assert len(_frames(cli, "cam1", 2, timeout=60)) == 2
        cli.close()
    finally:
        app.stop()
        srv.stop()


def test_bus_reader_unmaps_data_of_removed_cameras_and_dead_owners(native):
    """A reader's data-segment mappings do not outlive the camera (removed / re-registered) or
    its owner process (killed): an unlinked /dev/shm file keeps its pages while mapped."""
    tag = f"t{os.getpid()}m"
    w, o = _owner(native, tag)
    r = native.BusReader(tag)
    try:
        cam = w.add_camera("camM", 3)
        o.add(cam, "camM")
        w.decode_now(cam, synth(native, 160, 96, gop=4).next())
        assert r.frame("camM", 0, 3000, 0) is not None
        assert r.mapped_data_segments() == 1
        o.remove(cam)
        assert r.mapped_data_segments() == 0
    finally:
        o.stop()
        w.stop()
    # an owner in another process, killed while the reader holds its camera's data mapped
    tag2 = f"t{os.getpid()}n"
    code = f"""
import sys, time
sys.path.insert(0, {ROOT!r})
sys.path.insert(0, {os.path.join(ROOT, 'tests')!r})
from video_edge_ai_proxy_amd import native
from conftest import synth
w = native.Worker(device=-1)
w.start()
o = native.BusOwner({tag2!r}, 0, 4)
o.attach(w)
cam = w.add_camera("camK", 3)
o.add(cam, "camK")
w.decode_now(cam, synth(native, 160, 96, gop=4).next())
print("ready", flush=True)
time.sleep(60)
"""
    p = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True)
    try:
        assert p.stdout.readline().strip() == "ready"
        r2 = native.BusReader(tag2)
        assert r2.frame("camK", 0, 5000, 0) is not None
        assert r2.mapped_data_segments() == 1
        p.kill()
        p.wait(timeout=30)
        assert r2.mapped_data_segments() == 0
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()
        native.bus_remove_segments(p.pid)
