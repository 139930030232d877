"""``python -m video_edge_ai_proxy_amd <command>`` — daemon, synthetic camera farm, clients.

  serve     hub daemon: REST :8080 + gRPC :50001 (server/main.go analog)
  camera    single-camera hub (python/rtsp_to_rtmp.py flags: --rtsp --rtmp --device_id
            --memory_buffer --disk_path)
  farm      synthetic RTSP camera farm (H.264 I_PCM/P_Skip streams) for tests and benchmarks
  list | frame | annotate | storage | proxy   gRPC clients (examples/*.py analogs)
"""
from __future__ import annotations

import argparse
import os
import sys
import time


def _addr(a):
    return f"{a.host}:{a.grpc_port}"


def cmd_serve(a):
    from .config import load_config
    from .server.app import run_forever
    from .utils import setup_logging

    setup_logging(a.log_level)
    cfg = load_config(a.config, data_dir=a.data_dir)
    if a.port is not None:
        cfg.port = a.port
    if a.grpc_port is not None:
        cfg.grpc_port = a.grpc_port
    if a.isolate:
        cfg.gpu.isolation = "process"
    devices = [int(x) for x in a.devices.split(",")] if a.devices else None
    run_forever(cfg, host=a.bind, devices=devices)


def cmd_camera(a):
    from .config import load_config
    from .models import StreamProcess
    from .server.app import build_app
    from .utils import setup_logging

    setup_logging(a.log_level)
    cfg = load_config(None, data_dir=a.data_dir)
    cfg.buffer.in_memory = a.memory_buffer
    if a.disk_path:
        cfg.buffer.on_disk = True
        cfg.buffer.on_disk_folder = a.disk_path
    app = build_app(cfg, host=a.bind, rest_port=a.port, grpc_port=a.grpc_port, restore=False)
    app.pm.start(StreamProcess(name=a.device_id, rtsp_endpoint=a.rtsp, rtmp_endpoint=a.rtmp or ""))
    print(f"camera {a.device_id}: gRPC :{app.grpc_port} REST :{app.rest_port}", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        app.stop()


def cmd_farm(a):
    from . import native

    srv = native.RtspServer(a.bind, a.port)
    for i in range(a.cams):
        c = native.SynthConfig()
        c.width, c.height, c.fps, c.gop, c.motion = a.width, a.height, a.fps, a.gop, a.motion
        c.seed = 1 + i
        c.codec = a.codec
        c.idr_phase = (i * a.gop) // max(1, a.cams)
        srv.add_stream(f"/cam{i}", c, realtime=not a.unpaced, cached_frames=a.cached_frames)
    srv.start()
    for i in range(a.cams):
        print(f"rtsp://{a.bind}:{srv.port}/cam{i}", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        srv.stop()


def cmd_list(a):
    from .proto import pb
    from .server.grpc_server import ImageClient

    cli = ImageClient(_addr(a))
    for s in cli.ListStreams(pb.ListStreamRequest()):
        print(s)


def cmd_frame(a):
    import numpy as np

    from .server.grpc_server import ImageClient

    cli = ImageClient(_addr(a))
    for _ in range(a.count):
        vf = cli.latest_frame(a.device, a.keyframe)
        print("is keyframe:", vf.is_keyframe, "frame type:", vf.frame_type,
              "shape:", [d.size for d in vf.shape.dim], "pts:", vf.pts)
        if a.out and vf.width:
            img = np.frombuffer(vf.data, np.uint8).reshape(vf.height, vf.width, 3)
            with open(a.out, "wb") as f:
                f.write(f"P6 {vf.width} {vf.height} 255\n".encode() + img[:, :, ::-1].tobytes())


def cmd_annotate(a):
    from .proto import pb
    from .server.grpc_server import ImageClient

    cli = ImageClient(_addr(a))
    now = int(time.time() * 1000)
    req = pb.AnnotateRequest(device_name=a.device, type=a.type, start_timestamp=now,
                             end_timestamp=now + 1000, object_type="person", confidence=0.9,
                             object_bouding_box=pb.BoudingBox(top=10, left=10, width=100, height=200),
                             ml_model="synthetic", ml_model_version="1")
    print(cli.Annotate(req))


def _bool(s):
    return str(s).lower() in ("1", "true", "yes", "on", "y", "t")


def cmd_storage(a):
    from .proto import pb
    from .server.grpc_server import ImageClient

    print(ImageClient(_addr(a)).Storage(pb.StorageRequest(device_id=a.device, start=_bool(a.on))))


def cmd_proxy(a):
    from .proto import pb
    from .server.grpc_server import ImageClient

    print(ImageClient(_addr(a)).Proxy(pb.ProxyRequest(device_id=a.device, passthrough=_bool(a.on))))


def cmd_bench(a, rest):
    """``vep bench ...`` = the repo's bench.py (headline benchmark) with the same flags."""
    import subprocess

    bench = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
    if not os.path.exists(bench):
        raise SystemExit("bench.py not found next to the package")
    raise SystemExit(subprocess.call([sys.executable, bench, *rest]))


def main(argv=None):
    ap = argparse.ArgumentParser(prog="vep", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)

    s = sub.add_parser("serve")
    s.add_argument("--config", default=None)
    s.add_argument("--data-dir", default=os.environ.get("VEP_DATA_DIR", "/data/chrysalis"))
    s.add_argument("--bind", default="0.0.0.0")
    s.add_argument("--port", type=int, default=None)
    s.add_argument("--grpc-port", type=int, default=None)
    s.add_argument("--devices", default="", help="comma-separated GPU ids; -1 = CPU backend")
    s.add_argument("--log-level", default="info")
    s.add_argument("--isolate", action="store_true",
                   help="one supervised worker process per GPU (gpu.isolation: process): a native "
                        "fault restarts that GPU's process, the other cameras keep running")
    s.set_defaults(fn=cmd_serve)

    c = sub.add_parser("camera")
    c.add_argument("--rtsp", required=True)
    c.add_argument("--rtmp", default=None)
    c.add_argument("--device_id", required=True)
    c.add_argument("--memory_buffer", type=int, default=1)
    c.add_argument("--disk_path", default=None)
    c.add_argument("--data-dir", default="/tmp/vep-camera")
    c.add_argument("--bind", default="0.0.0.0")
    c.add_argument("--port", type=int, default=8080)
    c.add_argument("--grpc-port", type=int, default=50001)
    c.add_argument("--log-level", default="info")
    c.set_defaults(fn=cmd_camera)

    f = sub.add_parser("farm")
    f.add_argument("--cams", type=int, default=4)
    f.add_argument("--width", type=int, default=640)
    f.add_argument("--height", type=int, default=480)
    f.add_argument("--fps", type=int, default=30)
    f.add_argument("--gop", type=int, default=30)
    f.add_argument("--motion", type=float, default=0.05)
    f.add_argument("--codec", choices=["h264", "h265"], default="h264")
    f.add_argument("--bind", default="127.0.0.1")
    f.add_argument("--port", type=int, default=8554)
    f.add_argument("--unpaced", action="store_true")
    f.add_argument("--cached-frames", type=int, default=60)
    f.set_defaults(fn=cmd_farm)

    for name, fn in (("list", cmd_list), ("frame", cmd_frame), ("annotate", cmd_annotate),
                     ("storage", cmd_storage), ("proxy", cmd_proxy)):
        p = sub.add_parser(name)
        p.add_argument("--host", default="127.0.0.1")
        p.add_argument("--grpc-port", type=int, default=50001)
        if name != "list":
            p.add_argument("--device", required=True)
        if name == "frame":
            p.add_argument("--keyframe", action="store_true")
            p.add_argument("--count", type=int, default=1)
            p.add_argument("--out", default=None, help="write the last frame as PPM")
        if name == "annotate":
            p.add_argument("--type", required=True)
        if name in ("storage", "proxy"):
            p.add_argument("--on", required=True)
        p.set_defaults(fn=fn)

    b = sub.add_parser("bench", help="run bench.py (flags passed through, e.g. --codec h265)")
    b.set_defaults(fn=None)

    a, rest = ap.parse_known_args(argv)
    if a.cmd == "bench":
        cmd_bench(a, rest)
    if rest:
        ap.error(f"unrecognized arguments: {' '.join(rest)}")
    a.fn(a)


if __name__ == "__main__":
    main(sys.argv[1:])
