"""Serving processes: node-scale ``VideoLatestImage`` without a front-end hop.

Reference parity: the Go gRPC server serves every ``VideoLatestImage`` stream on its own goroutine
straight from Redis, with no interpreter lock on the path (server/grpcapi/grpc_api.go:133-235,
server/main.go:142-154). One Python grpcio process cannot do that for a whole node (one GIL for
every client of every GPU), so ``serving.frontends: K`` runs K serving processes:

* every one binds the public gRPC port with ``SO_REUSEPORT``; the kernel spreads client
  connections over them;
* ``VideoLatestImage`` is answered from the node's frame bus (csrc/vep/bus.h): the process maps
  every owner's control segment, marks the camera's demand (the lazy decoder's last_query /
  keyframe-only), waits on the camera's futex word and copies the frame the owner's pump DMA'd
  into shared memory straight into the reply — no connection to the decoding process, no GPU
  context here, and one DMA per frame for every client of a camera in every serving process;
* the other RPCs (``ListStreams``, ``Annotate``, ``Proxy``, ``Storage``) need the registry and
  the annotation queue, so they are forwarded as raw bytes to the main process's control port.

A supervisor process (``--supervise K``) starts the K serving processes and restarts any that
dies; the daemon starts the supervisor before it touches a GPU, because a process holding a GPU
context must not start programs.

    python -m video_edge_ai_proxy_amd.server.frontend --bus TAG --listen 0.0.0.0:50001 \\
        --control 127.0.0.1:PORT [--threads 256] [--supervise K]

prints ``ready <port>`` once listening and exits when its stdin closes.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import select
import subprocess
import sys
import threading
import time
from typing import Optional

log = logging.getLogger("vep.frontend")

_PKG_PARENT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FORWARDED = {"ListStreams": "unary_stream", "Annotate": "unary_unary", "Proxy": "unary_unary",
             "Storage": "unary_unary"}


def _env() -> dict:
    env = dict(os.environ)
    env["PYTHONPATH"] = _PKG_PARENT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    # serving processes never use a GPU: hide it so nothing in them can initialise one
    env["HIP_VISIBLE_DEVICES"] = ""
    env["CUDA_VISIBLE_DEVICES"] = ""
    env.pop("GPU_MAX_HW_QUEUES", None)
    return env


def make_forwarding_handler(svc, control: str):
    """VideoLatestImage from the bus (``svc``: ImageService with a BusFrames source); every other
    method forwarded byte-for-byte to the main process at ``control``."""
    import grpc

    from ..proto import SERVICE, pb
    from .grpc_server import FRAME_CHANNEL_OPTS, _identity

    chan = grpc.insecure_channel(control, options=FRAME_CHANNEL_OPTS)

    def fwd(method: str, kind: str):
        path = SERVICE.path(method)
        if kind == "unary_unary":
            call = chan.unary_unary(path)

            def h(req: bytes, context):
                try:
                    return call(req, timeout=30)
                except grpc.RpcError as e:
                    context.abort(e.code(), e.details() or "")
            return grpc.unary_unary_rpc_method_handler(h)
        call = chan.unary_stream(path)

        def hs(req: bytes, context):
            try:
                yield from call(req, timeout=30)
            except grpc.RpcError as e:
                context.abort(e.code(), e.details() or "")
        return grpc.unary_stream_rpc_method_handler(hs)

    handlers = {m: fwd(m, k) for m, k in FORWARDED.items()}
    handlers["VideoLatestImage"] = grpc.stream_stream_rpc_method_handler(
        svc.VideoLatestImage, request_deserializer=pb.VideoFrameRequest.FromString, response_serializer=_identity)
    return grpc.method_handlers_generic_handler(SERVICE.full_name, handlers), chan


class NativeForwarder:
    """The native endpoint's callback for the non-frame methods: forwards the request bytes to the
    main process's grpcio server (``control``) and returns (status, message, [responses])."""

    def __init__(self, control: str):
        import grpc

        from ..proto import SERVICE
        from .grpc_server import FRAME_CHANNEL_OPTS

        self.grpc = grpc
        self.chan = grpc.insecure_channel(control, options=FRAME_CHANNEL_OPTS)
        self.calls = {m: (self.chan.unary_unary(SERVICE.path(m)) if k == "unary_unary"
                          else self.chan.unary_stream(SERVICE.path(m))) for m, k in FORWARDED.items()}

    def __call__(self, method: str, req: bytes, peer: str):
        call = self.calls.get(method)
        if call is None:
            return 12, f"unknown method {method}", []
        try:
            if FORWARDED[method] == "unary_unary":
                return 0, "", [call(req, timeout=30)]
            return 0, "", list(call(req, timeout=30))
        except self.grpc.RpcError as e:
            return e.code().value[0], e.details() or "", []

    def close(self):
        self.chan.close()


def run_frontend(tag: str, listen: str, control: str, threads: int, native: bool = False, io_threads: int = 2) -> int:
    from .grpc_server import BusFrames, ImageService, serve

    if native:  # C++ HTTP/2 endpoint: frames from the bus without Python; the rest forwarded
        from .._native import native as _n

        host, port = listen.rsplit(":", 1)
        fwd = NativeForwarder(control)
        nsrv = _n.RpcServer(host, int(port), tag, io_threads=io_threads, wait_threads=threads, handler=fwd,
                            reuseport=True)
        print(f"ready {nsrv.port}", flush=True)
        stats_path = os.environ.get("VEP_FRONTEND_STATS")

        def report_native():
            while True:
                time.sleep(1.0)
                if stats_path:
                    try:
                        with open(f"{stats_path}.{os.getpid()}.tmp", "w") as f:
                            json.dump({"pid": os.getpid(), "frames_served": nsrv.stats()["frames_served"]}, f)
                        os.replace(f"{stats_path}.{os.getpid()}.tmp", f"{stats_path}.{os.getpid()}")
                    except OSError:
                        pass

        threading.Thread(target=report_native, daemon=True).start()
        try:
            sys.stdin.read()
        except Exception:  # noqa: BLE001
            pass
        nsrv.stop()
        fwd.close()
        return 0
    svc = ImageService(None, bus=BusFrames(tag))
    handler, chan = make_forwarding_handler(svc, control)
    server = serve(svc, listen, workers=threads, reuseport=True, handler=handler, tune_malloc=True)
    print(f"ready {server.bound_port}", flush=True)
    stats_path = os.environ.get("VEP_FRONTEND_STATS")

    def report():  # served-frame counters for the supervisor (metrics / benches)
        while True:
            time.sleep(1.0)
            if stats_path:
                try:
                    with open(f"{stats_path}.{os.getpid()}.tmp", "w") as f:
                        json.dump({"pid": os.getpid(), "frames_served": svc.frames_served}, f)
                    os.replace(f"{stats_path}.{os.getpid()}.tmp", f"{stats_path}.{os.getpid()}")
                except OSError:
                    pass

    threading.Thread(target=report, daemon=True).start()
    try:
        sys.stdin.read()  # until the supervisor closes the pipe (or dies)
    except Exception:  # noqa: BLE001
        pass
    server.stop(grace=1).wait(3)
    chan.close()
    return 0


class _Proc:
    """One serving process (started by the supervisor)."""

    def __init__(self, args: list[str], start_timeout_s: float = 120.0):
        self.p = subprocess.Popen([sys.executable, "-u", "-m", "video_edge_ai_proxy_amd.server.frontend", *args],
                                  stdin=subprocess.PIPE, stdout=subprocess.PIPE, env=_env())
        self.port = _read_ready(self.p, start_timeout_s)

    def alive(self) -> bool:
        return self.p.poll() is None

    def close(self, timeout_s: float = 5.0) -> None:
        try:
            self.p.stdin.close()
        except Exception:  # noqa: BLE001
            pass
        try:
            self.p.wait(timeout=timeout_s)
        except subprocess.TimeoutExpired:
            self.p.kill()
            self.p.wait()


def _read_ready(p: subprocess.Popen, timeout_s: float) -> int:
    line = b""
    deadline = time.time() + timeout_s
    while not line.endswith(b"\n"):
        if p.poll() is not None:
            raise RuntimeError(f"serving process exited during start (code {p.returncode})")
        r, _, _ = select.select([p.stdout], [], [], 0.5)
        if r:
            ch = os.read(p.stdout.fileno(), 1)
            if not ch:
                raise RuntimeError("serving process closed its output")
            line += ch
        if time.time() > deadline:
            p.kill()
            raise RuntimeError("serving process did not start in time")
    parts = line.decode().split()
    if len(parts) != 2 or parts[0] != "ready":
        raise RuntimeError(f"serving process: unexpected start line {line!r}")
    return int(parts[1])


def run_supervisor(k: int, child_args: list[str]) -> int:
    procs = [_Proc(child_args) for _ in range(k)]
    print(f"ready {procs[0].port}", flush=True)
    stop = threading.Event()
    restarts = [0] * k

    def supervise():
        while not stop.wait(0.5):
            for i, pr in enumerate(procs):
                if stop.is_set() or pr.alive():
                    continue
                log.error("serving process %d (pid %d) exited with %s: restarting", i, pr.p.pid, pr.p.returncode)
                try:
                    procs[i] = _Proc(child_args)
                    restarts[i] += 1
                except Exception as e:  # noqa: BLE001 — retried at the next pass
                    log.error("restart of serving process %d failed: %s", i, e)

    th = threading.Thread(target=supervise, daemon=True)
    th.start()
    try:
        sys.stdin.read()
    except Exception:  # noqa: BLE001
        pass
    stop.set()
    th.join(timeout=5)
    for pr in procs:
        pr.close()
    return 0


class FrontendPool:
    """The daemon's handle on the serving processes: starts the supervisor (call before this
    process touches a GPU) and stops it."""

    def __init__(self, n: int, tag: str, listen: str, control: str, threads: int = 256,
                 start_timeout_s: float = 180.0, stats_path: Optional[str] = None, native: bool = False,
                 io_threads: int = 2):
        args = ["--bus", tag, "--listen", listen, "--control", control, "--threads", str(threads),
                "--io-threads", str(io_threads)] + (["--native"] if native else [])
        env = _env()
        if stats_path:
            env["VEP_FRONTEND_STATS"] = stats_path
        self.n, self.stats_path = n, stats_path
        self.p = subprocess.Popen([sys.executable, "-u", "-m", "video_edge_ai_proxy_amd.server.frontend",
                                   "--supervise", str(n), *args], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                  env=env)
        try:
            self.port = _read_ready(self.p, start_timeout_s)
        except Exception:
            self.close()
            raise

    def frames_served(self) -> int:
        """Frames served by every serving process (their last 1 s reports)."""
        if not self.stats_path:
            return 0
        d, base = os.path.split(self.stats_path)
        n = 0
        for f in os.listdir(d or "."):
            if f.startswith(base + ".") and not f.endswith(".tmp"):
                try:
                    with open(os.path.join(d, f)) as fh:
                        n += int(json.load(fh)["frames_served"])
                except (OSError, ValueError, KeyError):
                    pass
        return n

    def close(self, timeout_s: float = 15.0) -> None:
        try:
            self.p.stdin.close()
        except Exception:  # noqa: BLE001
            pass
        try:
            self.p.wait(timeout=timeout_s)
        except subprocess.TimeoutExpired:
            self.p.kill()
            self.p.wait()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--bus", required=True, help="frame-bus tag of the hub instance")
    ap.add_argument("--listen", required=True)
    ap.add_argument("--control", required=True, help="main process's gRPC address (non-frame RPCs)")
    ap.add_argument("--threads", type=int, default=256)
    ap.add_argument("--supervise", type=int, default=0, help="start and supervise this many serving processes")
    ap.add_argument("--native", action="store_true", help="VideoLatestImage on the native HTTP/2 endpoint")
    ap.add_argument("--io-threads", type=int, default=2)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s frontend[%(process)d] %(name)s: %(message)s")
    if a.supervise > 0:
        return run_supervisor(a.supervise, ["--bus", a.bus, "--listen", a.listen, "--control", a.control,
                                            "--threads", str(a.threads), "--io-threads", str(a.io_threads)] +
                              (["--native"] if a.native else []))
    return run_frontend(a.bus, a.listen, a.control, a.threads, a.native, a.io_threads)


if __name__ == "__main__":
    sys.exit(main())
