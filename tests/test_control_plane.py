"""Control plane units: proto wire format, config, registry, settings, signing, annotation
queue, cron, models (CPU)."""
import base64
import hashlib
import hmac
import json
import os
import time

import pytest


# ------------------------------------------------------------------------------- proto
def test_proto_golden_encodings():
    from video_edge_ai_proxy_amd.proto import SERVICE, pb

    assert pb.VideoFrame(width=640).SerializeToString() == b"\x08\x80\x05"
    assert pb.VideoFrameRequest(key_frame_only=True, device_id="c").SerializeToString() == b"\x08\x01\x12\x01c"
    assert pb.ProxyRequest(device_id="a", passthrough=True).SerializeToString() == b"\x0a\x01a\x10\x01"
    assert pb.StorageRequest(device_id="a", start=True).SerializeToString() == b"\x0a\x01a\x10\x01"
    # field 10 time_base is a fixed64 double, field 11 shape is a nested message of Dim(2)
    vf = pb.VideoFrame(time_base=0.5)
    assert vf.SerializeToString() == b"\x51" + (0.5).hex().encode() * 0 + bytes.fromhex("000000000000e03f")
    d = pb.ShapeProto(dim=[pb.ShapeProto_Dim(size=3, name="2")])
    assert d.SerializeToString() == b"\x12\x05\x08\x03\x12\x012"
    ls = pb.ListStream(name="x", pid=7, running=True)
    assert ls.SerializeToString() == b"\x0a\x01x\x38\x07\x40\x01"
    ar = pb.AnnotateRequest(custom_meta_5="z", offset_packet_id=1)
    assert ar.SerializeToString() == b"\xc0\x01\x01\xea\x01\x01z"
    assert SERVICE.full_name == "chrys.cloud.videostreaming.v1beta1.Image"
    ms = {m.name: (m.client_streaming, m.server_streaming) for m in SERVICE.methods}
    assert ms == {"VideoLatestImage": (True, True), "ListStreams": (False, True),
                  "Annotate": (False, False), "Proxy": (False, False), "Storage": (False, False)}


def test_native_videoframe_encoding_matches_protobuf(native):
    """The hand-encoded VideoFrame from the native serving path parses to the same fields."""
    from conftest import synth
    from video_edge_ai_proxy_amd.proto import pb

    w = native.Worker(device=-1)
    cam = w.add_camera("golden", 2)
    enc = synth(native, 96, 64, gop=4)
    for _ in range(3):
        w.decode_now(cam, enc.next())
    seq, raw, meta = w.video_frame(cam, 0, "golden")
    vf = pb.VideoFrame.FromString(raw)
    assert (vf.width, vf.height, vf.frame_type, vf.device_id) == (96, 64, "P", "golden")
    assert vf.pts == meta["pts"] == 2 * 3000 and vf.packet == 2 and vf.keyframe == 1
    assert [(d.size, d.name) for d in vf.shape.dim] == [(64, "0"), (96, "1"), (3, "2")]
    _, img = w.read_latest(cam, 0)
    assert vf.data == img.tobytes()
    ref = pb.VideoFrame(width=vf.width, height=vf.height, data=vf.data, timestamp=vf.timestamp,
                        is_keyframe=vf.is_keyframe, pts=vf.pts, dts=vf.dts, frame_type=vf.frame_type,
                        is_corrupt=vf.is_corrupt, time_base=vf.time_base, shape=vf.shape,
                        device_id=vf.device_id, packet=vf.packet, keyframe=vf.keyframe)
    assert ref.SerializeToString() == raw  # canonical field order, byte-identical


def test_proto_parser_rejects_unsupported():
    from video_edge_ai_proxy_amd.proto import parse_proto

    fd, svcs = parse_proto('syntax = "proto3"; package a.b; message M { repeated int64 x = 1; M y = 2; }')
    assert fd.message_type[0].field[1].type_name == ".a.b.M" and not svcs
    with pytest.raises(NotImplementedError):
        parse_proto('syntax = "proto3"; package a; message M { enum E { A = 0; } }')


# ------------------------------------------------------------------------------ config
def test_config_defaults_and_yaml(tmp_path):
    from video_edge_ai_proxy_amd.config import load_config, parse_duration

    c = load_config(data_dir=str(tmp_path))
    assert c.annotation.max_batch_size == 299 and c.annotation.poll_duration_ms == 300
    assert c.annotation.unacked_limit == 1000 and c.buffer.in_memory == 1
    assert c.buffer.on_disk_schedule == "@every 5m" and c.buffer.on_disk_clean_older_than == "30s"
    assert c.api.endpoint == "https://api.chryscloud.com" and c.port == 8080
    (tmp_path / "conf.yaml").write_text(
        "version: 0.0.3\nmode: release\nredis:\n  connection: redis:6379\n"
        "annotation:\n  endpoint: http://x/annotate\n  max_batch_size: 10\n"
        "buffer:\n  n_memory: 5\n  on_disk: true\n  on_disk_folder: /tmp/a\n  on_disk_schedule: \"@every 5s\"\n"
        "gpu:\n  devices: [0, 1]\n  letterbox_size: 640\n")
    c = load_config(data_dir=str(tmp_path))
    assert c.annotation.endpoint == "http://x/annotate" and c.annotation.max_batch_size == 10
    assert c.buffer.in_memory == 5 and c.buffer.on_disk and c.ring_slots == 5
    assert c.gpu.devices == [0, 1] and c.gpu.letterbox_size == 640
    assert parse_duration("1h30m") == 5400 and parse_duration("250ms") == 0.25
    with pytest.raises(ValueError):
        parse_duration("5 minutes")


# ------------------------------------------------------------------------- storage/models
def test_storage_prefix_scan(tmp_path):
    """Reference server/services/storage_test.go: put/get round-trip and a 10-key prefix scan."""
    from video_edge_ai_proxy_amd.services.storage import KeyNotFound, Storage

    s = Storage(str(tmp_path / "kv.db"))
    s.put("/test/", "a", b"1")
    assert s.get("/test/", "a") == b"1"
    for i in range(10):
        s.put("/prefix/", f"k{i}", str(i).encode())
    s.put("/prefiy/", "x", b"no")
    assert len(s.list("/prefix/")) == 10
    s.delete("/prefix/", "k0")
    assert len(s.list("/prefix/")) == 9
    with pytest.raises(KeyNotFound):
        s.get("/prefix/", "k0")


def test_stream_process_json_roundtrip():
    from video_edge_ai_proxy_amd.models import ContainerState, DockerLogs, StreamProcess

    sp = StreamProcess(name="cam", rtsp_endpoint="rtsp://x")
    assert sp.to_json() == {"name": "cam", "rtsp_endpoint": "rtsp://x"}
    sp.state = ContainerState.from_session({"status": "running", "running": True, "pid": 5,
                                            "started_at_ms": 1, "failing_streak": 2})
    sp.logs = DockerLogs.from_text("hello\n", "")
    j = json.loads(json.dumps(sp.to_json()))
    assert j["state"]["Running"] and j["state"]["Pid"] == 5 and j["state"]["Health"]["FailingStreak"] == 2
    assert j["state"]["StartedAt"].startswith("1970-01-01T00:00:00.001")
    assert base64.b64decode(j["logs"]["stdout"]) == b"hello\n"
    back = StreamProcess.from_json(j)
    assert back.state.Pid == 5 and back.state.Health.FailingStreak == 2
    with pytest.raises(ValueError):
        StreamProcess.from_json({"name": 5})


def test_settings_manager(tmp_path):
    from video_edge_ai_proxy_amd.models import Settings
    from video_edge_ai_proxy_amd.services.settings import MissingEdgeCredentials, SettingsManager
    from video_edge_ai_proxy_amd.services.storage import Storage

    sm = SettingsManager(Storage(str(tmp_path / "s.db")))
    assert sm.get().name == "default" and sm.get().edge_key == ""
    with pytest.raises(MissingEdgeCredentials):
        sm.current_edge_key_and_secret()
    s = sm.overwrite(Settings(edge_key="k", edge_secret="s"))
    assert s.created > 0 and s.modified >= s.created
    assert sm.current_edge_key_and_secret() == ("k", "s")
    sm2 = SettingsManager(sm.storage)
    assert sm2.current_edge_key_and_secret() == ("k", "s")


def test_edge_signature_known_vector():
    from video_edge_ai_proxy_amd.services.edge import sign

    body = b'{"data":[]}'
    h = sign(body, "KEY", "SECRET", ts_ms=1600000000000)
    md5 = hashlib.md5(body).hexdigest()
    assert h["Content-MD5"] == md5
    mac = base64.b64encode(hmac.new(b"SECRET", b"1600000000000" + md5.encode(), hashlib.sha256).digest()).decode()
    assert h["X-ChrysEdge-Auth"] == "KEY:" + mac and h["X-Chrys-Date"] == "1600000000000"


def test_parse_rtmp_key():
    from video_edge_ai_proxy_amd.utils import parse_rtmp_key

    assert parse_rtmp_key("rtmp://rtmp.chryscloud.com:1935/live/abc123") == "abc123"
    with pytest.raises(ValueError):
        parse_rtmp_key("http://x/y")
    with pytest.raises(ValueError):
        parse_rtmp_key("rtmp://host/")


# ---------------------------------------------------------------------- annotation queue
def test_annotation_queue_batches_ack_reject_requeue(tmp_path):
    from video_edge_ai_proxy_amd.services.annotation import REJECTED, AnnotationQueue

    q = AnnotationQueue(str(tmp_path / "q.db"))
    for i in range(700):
        assert q.publish(f"m{i}".encode())
    seen = []

    def consumer(b):
        seen.append(len(b))
        if len(seen) == 1:
            b.reject()
        else:
            b.ack()

    assert q.poll_once(consumer, unacked_limit=1000, max_batch=299) == 299
    assert q.counts()[REJECTED] == 299
    assert q.poll_once(consumer, max_batch=299) == 299
    assert q.poll_once(consumer, max_batch=299) == 102
    assert q.poll_once(consumer) == 0
    assert q.return_all_rejected() == 299
    assert q.poll_once(consumer, max_batch=299) == 299
    assert q.counts() == {"ready": 0, "unacked": 0, "rejected": 0}
    # unacked limit bounds the batch
    for i in range(10):
        q.publish(b"x")
    q.take(8)  # 8 outstanding deliveries
    assert q.poll_once(lambda b: b.ack(), unacked_limit=10, max_batch=299) == 2
    q.close()
    # crash recovery: unacked deliveries return to ready
    q2 = AnnotationQueue(str(tmp_path / "q.db"))
    assert q2.counts()["ready"] == 8
    q2.close()


def test_annotation_consumer_maps_and_rejects(tmp_path):
    from video_edge_ai_proxy_amd.proto import pb
    from video_edge_ai_proxy_amd.services.annotation import (AnnotationConsumer, AnnotationQueue,
                                                             request_to_annotation)

    req = pb.AnnotateRequest(device_name="d", type="entry", start_timestamp=5, confidence=0.5,
                             mask=[pb.Coordinate(x=1, y=2)], object_signature=[0.1, 0.2],
                             location=pb.Location(lat=1.5, lon=2.5), object_coordinate=pb.Coordinate(z=3))
    a = request_to_annotation(req)
    assert a["event_type"] == "entry" and a["object_mask"] == [{"x": 1, "y": 2, "z": 0}]
    assert a["location"] == {"lat": 1.5, "lon": 2.5} and a["object_signature"] == [0.1, 0.2]
    assert a["object_coordinate"]["z"] == 3

    class Settings:
        def current_edge_key_and_secret(self):
            return "k", "s"

    class Edge:
        def __init__(self):
            self.calls = []
            self.fail = True

        def call_api_with_body(self, method, url, body, k, s):
            self.calls.append(body)
            if self.fail:
                raise RuntimeError("network down")

    edge = Edge()
    q = AnnotationQueue(str(tmp_path / "a.db"))
    q.publish(req.SerializeToString())
    q.publish(b"\xff\xff garbage")
    c = AnnotationConsumer(Settings(), edge, "http://cloud/annotate")
    q.poll_once(c)
    assert q.counts()["rejected"] == 2 and c.failed_batches == 1
    edge.fail = False
    q.return_all_rejected()
    q.poll_once(c)
    assert q.counts() == {"ready": 0, "unacked": 0, "rejected": 0}
    assert len(edge.calls[-1]["data"]) == 1 and c.sent == 1
    q.close()


# ------------------------------------------------------------------------------- cron
def test_cron_schedule_and_cleanup(tmp_path):
    from video_edge_ai_proxy_amd.services.cron import CleanupJob, Schedule, cleanup_mp4

    s = Schedule("@every 5m")
    assert s.next_after(100.0) == 400.0
    t = time.mktime((2024, 1, 1, 0, 0, 30, 0, 0, 0)) - time.timezone
    nxt = Schedule("*/15 * * * *").next_after(t)
    assert (nxt - t) == 14 * 60 + 30
    assert Schedule("@hourly").next_after(t) - t == 3600 - 30
    with pytest.raises(ValueError):
        Schedule("* * *")
    d = tmp_path / "arch" / "cam"
    d.mkdir(parents=True)
    old, new, other = d / "1_2.mp4", d / "3_4.mp4", d / "x.txt"
    for p in (old, new, other):
        p.write_bytes(b"x")
    os.utime(old, (time.time() - 100, time.time() - 100))
    os.utime(other, (time.time() - 100, time.time() - 100))
    assert cleanup_mp4(str(tmp_path / "arch"), 30) == [str(old)]
    assert new.exists() and other.exists()
    job = CleanupJob(str(tmp_path / "arch"), "@every 200ms", "0s").start()
    time.sleep(0.6)
    job.stop()
    assert not new.exists() and job.runs >= 1


def test_auto_serving_processes():
    """serving.frontends -2: one serving process per GPU on multi-GPU nodes; on one GPU two when
    8 CPUs remain beyond the GPU's 16-CPU decode share, else the main process serves."""
    from video_edge_ai_proxy_amd.server.app import auto_frontends

    assert auto_frontends(8, 256) == 8 and auto_frontends(2, 8) == 2
    assert auto_frontends(1, 16) == 0 and auto_frontends(1, 23) == 0
    assert auto_frontends(1, 24) == 2 and auto_frontends(1, 64) == 2
