"""End-to-end (CPU backend): synthetic RTSP camera farm -> native ingest -> lazy decode ->
gRPC VideoLatestImage / ListStreams / Proxy / Storage / Annotate, REST API, archive, cron."""
import base64
import hashlib
import hmac
import http.server
import json
import os
import threading
import time

import numpy as np
import pytest

from conftest import synth


class FakeCloud:
    """Records signed requests (annotation POSTs, storage PUTs) like the cloud API would."""

    def __init__(self, status=200):
        self.requests = []
        self.status = status
        outer = self

        class H(http.server.BaseHTTPRequestHandler):
            def _handle(self):
                n = int(self.headers.get("Content-Length", 0))
                body = self.rfile.read(n)
                outer.requests.append((self.command, self.path, dict(self.headers), body))
                self.send_response(outer.status)
                self.end_headers()
                self.wfile.write(b"{}")

            do_POST = do_PUT = _handle

            def log_message(self, *a):
                pass

        self.srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.port = self.srv.server_address[1]
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def close(self):
        self.srv.shutdown()


@pytest.fixture
def farm(native):
    srv = native.RtspServer("127.0.0.1", 0)
    cfg = native.SynthConfig()
    cfg.width, cfg.height, cfg.gop, cfg.fps, cfg.seed = 320, 240, 10, 30, 11
    srv.add_stream("/cam", cfg, realtime=True, cached_frames=20)
    srv.start()
    yield srv
    srv.stop()


@pytest.fixture
def hubapp(tmp_path, native):
    from video_edge_ai_proxy_amd.config import Config
    from video_edge_ai_proxy_amd.server.app import build_app

    cloud = FakeCloud()
    cfg = Config()
    cfg.data_dir = str(tmp_path / "data")
    cfg.annotation.endpoint = f"http://127.0.0.1:{cloud.port}/api/v1/annotate"
    cfg.annotation.poll_duration_ms = 50
    cfg.api.endpoint = f"http://127.0.0.1:{cloud.port}"
    cfg.buffer.on_disk = True
    cfg.buffer.on_disk_folder = str(tmp_path / "archive")
    cfg.gpu.devices = [-1]
    app = build_app(cfg, host="127.0.0.1", rest_port=0, grpc_port=0)
    app.cloud = cloud
    yield app
    app.stop()
    cloud.close()


def _rest(app):
    from fastapi.testclient import TestClient

    from video_edge_ai_proxy_amd.server.rest import create_app

    return TestClient(create_app(app.pm, app.settings, app.metrics))


def test_end_to_end_serving(native, farm, hubapp):
    from video_edge_ai_proxy_amd.proto import pb
    from video_edge_ai_proxy_amd.server.grpc_server import ImageClient

    rest = _rest(hubapp)
    url = f"rtsp://127.0.0.1:{farm.port}/cam"
    r = rest.post("/api/v1/process", json={"name": "front_door", "rtsp_endpoint": url})
    assert r.status_code == 200, r.text
    assert rest.post("/api/v1/process", json={"name": "front_door", "rtsp_endpoint": url}).status_code == 409
    assert rest.post("/api/v1/process", json={"name": "x"}).status_code == 400
    assert rest.post("/api/v1/process", content=b"{not json").status_code == 400

    cli = ImageClient(f"127.0.0.1:{hubapp.grpc_port}")
    # first request wakes the lazy decoder; frames follow within a GOP
    deadline = time.time() + 15
    vf = None
    while time.time() < deadline:
        vf = cli.latest_frame("front_door")
        if vf is not None and vf.width:
            break
        time.sleep(0.1)
    assert vf is not None and vf.width == 320 and vf.height == 240
    assert [(d.size, d.name) for d in vf.shape.dim] == [(240, "0"), (320, "1"), (3, "2")]
    assert len(vf.data) == 320 * 240 * 3 and vf.frame_type in ("I", "P")
    assert vf.device_id == "front_door" and abs(vf.time_base - 1 / 90000) < 1e-12
    # pixels are a faithful decode of the camera's stream: check against the CPU oracle
    img = np.frombuffer(vf.data, np.uint8).reshape(240, 320, 3)
    ref = synth(native, 320, 240, gop=10, seed=11)
    dec = native.CpuDecoder()
    pics = [dec.decode(ref.next()) for _ in range(20)]
    assert any(np.array_equal(img, p) for p in pics)
    # next request on the same channel returns a *newer* frame (per-client cursor)
    vf2 = cli.latest_frame("front_door")
    assert vf2.pts != vf.pts or vf2.keyframe != vf.keyframe
    # keyframe-only mode serves I frames (frames decoded before the switch may still be served
    # first: bounded by a frame count, not a wall-clock window, so a loaded host cannot fail it)
    kfs = []
    for _ in range(10):
        kfs.append(cli.latest_frame("front_door", key_frame_only=True))
        if kfs[-1].frame_type == "I":
            break
    assert kfs[-1].frame_type == "I" and kfs[-1].is_keyframe, [k.frame_type for k in kfs]
    kf2 = cli.latest_frame("front_door", key_frame_only=True)
    assert kf2.frame_type == "I" and kf2.is_keyframe
    # unknown device -> empty VideoFrame (reference behaviour)
    assert cli.latest_frame("nope").width == 0

    streams = list(cli.ListStreams(pb.ListStreamRequest()))
    assert [s.name for s in streams] == ["front_door"]
    assert streams[0].running and streams[0].status == "running" and streams[0].pid > 0

    info = rest.get("/api/v1/process/front_door").json()
    assert info["state"]["Running"] and info["status"] == "running"
    assert "connected" in base64.b64decode(info["logs"]["stdout"]).decode()
    assert rest.get("/api/v1/processlist").json()[0]["name"] == "front_door"
    assert rest.get("/api/v1/process/none").status_code == 400
    m = rest.get("/metrics").text
    assert "vep_decoded_frames_total" in m and 'camera="front_door"' in m
    assert "vep_decode_latency_seconds_bucket" in m and "vep_pinned_pool_bytes" in m
    h = rest.get("/healthz").json()
    assert h["decoder_backends"] == ["native"]
    hp = h["host_plane"]  # the worker's host domain: its CPUs and its live parse strands
    assert len(hp) == 1 and hp[0]["cpulist"] and hp[0]["parse_threads"] >= 1
    assert hp[0]["ingest_parse_threads"] == hp[0]["parse_threads"] and hp[0]["cameras"] == 1

    # per-GOP archive on disk: <dir>/<device>/<start_ms>_<dur_ms>.mp4
    t0 = time.time()
    while hubapp.hub.archiver.written == 0 and time.time() - t0 < 30:
        time.sleep(0.1)
    p = hubapp.hub.archiver.last_path
    assert p and os.path.exists(p) and os.path.basename(os.path.dirname(p)) == "front_door"
    start, dur = os.path.basename(p)[:-4].split("_")
    # RTP packets carry no durations -> DTS span of the GOP (archive.py:58-73): 9 x 1/30 s
    assert int(dur) == 300

    assert rest.delete("/api/v1/process/front_door").status_code == 200
    assert rest.delete("/api/v1/process/front_door").status_code == 409
    assert list(cli.ListStreams(pb.ListStreamRequest())) == []
    cli.close()


def test_settings_annotate_storage_proxy(native, farm, hubapp):
    import grpc

    from video_edge_ai_proxy_amd.proto import pb
    from video_edge_ai_proxy_amd.server.grpc_server import ImageClient

    rest = _rest(hubapp)
    cli = ImageClient(f"127.0.0.1:{hubapp.grpc_port}")
    now = int(time.time() * 1000)
    # Annotate without an edge key -> INVALID_ARGUMENT
    with pytest.raises(grpc.RpcError) as e:
        cli.Annotate(pb.AnnotateRequest(device_name="d", type="t", start_timestamp=now))
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    assert rest.post("/api/v1/settings", json={"name": "default", "edge_key": "K", "edge_secret": "S"}).status_code == 202
    s = rest.get("/api/v1/settings").json()
    assert s["edge_key"] == "K" and s["created"] > 0
    with pytest.raises(grpc.RpcError) as e:
        cli.Annotate(pb.AnnotateRequest(device_name="d", type="t", start_timestamp=now - 8 * 86400 * 1000))
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    resp = cli.Annotate(pb.AnnotateRequest(device_name="cam1", type="moving", start_timestamp=now,
                                           confidence=0.9, object_bouding_box=pb.BoudingBox(top=1, left=2, width=3, height=4)))
    assert resp.device_name == "cam1" and resp.type == "moving"
    t0 = time.time()
    while not hubapp.cloud.requests and time.time() - t0 < 5:
        time.sleep(0.05)
    method, path, headers, body = hubapp.cloud.requests[0]
    assert method == "POST" and path == "/api/v1/annotate"
    doc = json.loads(body)
    assert doc["data"][0]["device_name"] == "cam1" and doc["data"][0]["object_bounding_box"]["width"] == 3
    md5 = hashlib.md5(body).hexdigest()
    assert headers["Content-MD5"] == md5
    mac = base64.b64encode(hmac.new(b"S", (headers["X-Chrys-Date"] + md5).encode(), hashlib.sha256).digest()).decode()
    assert headers["X-ChrysEdge-Auth"] == "K:" + mac

    # proxy / storage need an RTMP endpoint
    sink = native.RtmpSink("127.0.0.1", 0)
    sink.start()
    url = f"rtsp://127.0.0.1:{farm.port}/cam"
    assert rest.post("/api/v1/process", json={"name": "norm", "rtsp_endpoint": url}).status_code == 200
    with pytest.raises(grpc.RpcError) as e:
        cli.Proxy(pb.ProxyRequest(device_id="norm", passthrough=True))
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    with pytest.raises(grpc.RpcError) as e:
        cli.Storage(pb.StorageRequest(device_id="norm", start=True))
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    rtmp = f"rtmp://127.0.0.1:{sink.port}/live/streamkey42"
    assert rest.post("/api/v1/process", json={"name": "cloudcam", "rtsp_endpoint": url, "rtmp_endpoint": rtmp}).status_code == 200
    # RTMP pass-through starts on start (rtmp given) at a keyframe
    t0 = time.time()
    while sink.video_messages < 15 and time.time() - t0 < 10:
        time.sleep(0.05)
    assert sink.sequence_headers >= 1 and sink.video_messages >= 15 and sink.keyframes >= 1
    assert sink.stream_key == "streamkey42"
    assert sink.video_bodies()[1][0] == 0x17  # first NALU message is a keyframe
    r = cli.Proxy(pb.ProxyRequest(device_id="cloudcam", passthrough=False))
    assert r.passthrough is False
    assert rest.get("/api/v1/process/cloudcam").json()["rtmp_stream_status"]["streaming"] is False
    r = cli.Storage(pb.StorageRequest(device_id="cloudcam", start=True))
    assert r.start
    put = [q for q in hubapp.cloud.requests if q[0] == "PUT"][0]
    assert put[1] == "/api/v1/edge/storage/streamkey42" and json.loads(put[3]) == {"enable": True}
    assert rest.get("/api/v1/process/cloudcam").json()["rtmp_stream_status"]["storing"] is True
    hubapp.cloud.status = 403
    with pytest.raises(grpc.RpcError) as e:
        cli.Storage(pb.StorageRequest(device_id="cloudcam", start=False))
    assert e.value.code() == grpc.StatusCode.PERMISSION_DENIED
    sink.stop()
    cli.close()


def test_supervisor_reconnects_after_fault(native, farm, hubapp):
    rest = _rest(hubapp)
    url = f"rtsp://127.0.0.1:{farm.port}/cam"
    assert rest.post("/api/v1/process", json={"name": "flaky", "rtsp_endpoint": url}).status_code == 200
    t0 = time.time()
    while not hubapp.hub.state("flaky")["running"] and time.time() - t0 < 5:
        time.sleep(0.05)
    farm.inject("/cam", native.Fault.DROP_CONNECTION)
    t0 = time.time()
    seen_restart = False
    while time.time() - t0 < 8:
        st = hubapp.hub.state("flaky")
        seen_restart |= st["restart_count"] >= 1
        if seen_restart and st["running"]:
            break
        time.sleep(0.05)
    st = hubapp.hub.state("flaky")
    assert seen_restart and st["running"]
    # unreachable camera -> restarting with a growing failing streak
    assert rest.post("/api/v1/process", json={"name": "dead_cam", "rtsp_endpoint": "rtsp://127.0.0.1:1/x"}).status_code == 200
    time.sleep(1.5)
    info = rest.get("/api/v1/process/dead_cam").json()
    assert info["state"]["Restarting"] and info["state"]["ExitCode"] == 1
    assert info["state"]["Health"]["FailingStreak"] >= 1


def test_registry_restore(native, farm, tmp_path):
    from video_edge_ai_proxy_amd.config import Config
    from video_edge_ai_proxy_amd.server.app import build_app

    cfg = Config()
    cfg.data_dir = str(tmp_path / "d")
    cfg.gpu.devices = [-1]
    a = build_app(cfg, host="127.0.0.1", rest_port=0, grpc_port=0, start_rest=False)
    from video_edge_ai_proxy_amd.models import StreamProcess

    a.pm.start(StreamProcess(name="keepme", rtsp_endpoint=f"rtsp://127.0.0.1:{farm.port}/cam"))
    a.stop()
    b = build_app(cfg, host="127.0.0.1", rest_port=0, grpc_port=0, start_rest=False)
    try:
        assert b.hub.has("keepme")
    finally:
        b.stop()


def test_hevc_camera_end_to_end(native, hubapp):
    """H.265 RTSP camera -> hub -> gRPC frame, hvc1 MP4 archive and enhanced-RTMP pass-through."""
    from video_edge_ai_proxy_amd.server.grpc_server import ImageClient

    srv = native.RtspServer("127.0.0.1", 0)
    cfg = native.SynthConfig()
    cfg.width, cfg.height, cfg.gop, cfg.fps, cfg.seed, cfg.codec = 320, 240, 10, 30, 21, "h265"
    srv.add_stream("/hevc", cfg, realtime=True, cached_frames=20)
    srv.start()
    sink = native.RtmpSink("127.0.0.1", 0)
    sink.start()
    rest = _rest(hubapp)
    cli = ImageClient(f"127.0.0.1:{hubapp.grpc_port}")
    try:
        r = rest.post("/api/v1/process", json={
            "name": "hevc_cam", "rtsp_endpoint": f"rtsp://127.0.0.1:{srv.port}/hevc",
            "rtmp_endpoint": f"rtmp://127.0.0.1:{sink.port}/live/hevc42"})
        assert r.status_code == 200, r.text
        deadline, vf = time.time() + 15, None
        while time.time() < deadline:
            vf = cli.latest_frame("hevc_cam")
            if vf is not None and vf.width:
                break
            time.sleep(0.1)
        assert vf is not None and (vf.width, vf.height) == (320, 240)
        img = np.frombuffer(vf.data, np.uint8).reshape(240, 320, 3)
        ref = synth(native, 320, 240, gop=10, seed=21, codec="h265")
        dec = native.CpuDecoder()
        assert any(np.array_equal(img, dec.decode(ref.next())) for _ in range(20))
        t0 = time.time()
        while (sink.video_messages < 12 or hubapp.hub.archiver.written == 0) and time.time() - t0 < 10:
            time.sleep(0.05)
        assert sink.sequence_headers >= 1 and sink.hevc_messages >= 12 and sink.keyframes >= 1
        p = hubapp.hub.archiver.last_path
        with open(p, "rb") as f:
            mp4 = f.read()
        assert b"hvc1" in mp4 and b"hvcC" in mp4
    finally:
        cli.close()
        sink.stop()
        srv.stop()
