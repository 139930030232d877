"""Client-observed ``VideoLatestImage`` latency for bench.py, through the production gRPC path:
by default the native HTTP/2 endpoint ``vep serve`` runs (csrc/vep/rpcsrv.h: the worker's frame
bus -> one shared copy per frame -> writev), or (``native=False``) the grpcio ImageService
(native ring D2H into the response bytes -> grpcio). Client decode in separate processes.

The server runs in the bench (GPU) process; the clients run in separate processes
(:class:`~vep_bench.latency_clients.ClientPool`, started before the bench
touches the GPU), so their receive/parse work never holds the server's GIL. Definitions:
  * ``next`` (headline): N concurrent clients, one connected channel and camera each, issuing
    back-to-back requests while the cameras stream live at their frame rate: request sent -> the
    camera's next frame received and parsed (includes waiting for it, up to one frame interval).
  * ``serve``: one request per pre-connected channel: the newest frame already in the HBM ring.
"""
from __future__ import annotations

import statistics
import threading
import time
from contextlib import contextmanager

from video_edge_ai_proxy_amd.utils import now_ms
from video_edge_ai_proxy_amd.server.grpc_server import ImageService, serve


class _WorkerHub:
    """Hub facade over a bare native Worker (bench cameras are not in a registry)."""

    def __init__(self, worker, cams):
        self.w = worker
        self.map = {f"cam{c}": c for c in cams}

    def has(self, name):
        return name in self.map

    def touch(self, name, keyframe_only=None):
        c = self.map[name]
        if keyframe_only is not None:
            self.w.set_keyframe_only(c, bool(keyframe_only))
        self.w.set_last_query(c, now_ms())

    def latest_frame_bytes(self, name, after=0, wait_ms=0):
        c = self.map[name]
        pub = self.w.published(c)
        if pub < after:
            after = 0
        if wait_ms > 0 and pub <= after:
            self.w.wait_frame(c, after, wait_ms)
        return self.w.video_frame(c, after, name)


class _PM:
    def __init__(self, hub):
        self.hub = hub


class _NativeSvc:
    """The counters measure() reads, from the native endpoint."""

    def __init__(self, srv):
        self.srv = srv
        self.latencies_ms = _Lat(srv)

    @property
    def frames_served(self):
        return self.srv.stats()["frames_served"]


class _Lat(list):
    def __init__(self, srv):
        super().__init__()
        self.srv = srv

    def clear(self):
        self.srv.take_latencies()

    def __iter__(self):
        return iter(self.srv.take_latencies())


@contextmanager
def serving(worker, cams, workers: int = 64, native: bool = True):
    """gRPC server (this process) over the worker's cameras: yields (target, camera names, svc).
    native: the worker's cameras go on a frame bus and the native endpoint serves them (the
    production default); else the grpcio ImageService reads the worker's rings."""
    hub = _WorkerHub(worker, cams)
    if native:
        import os

        from video_edge_ai_proxy_amd import native as vep

        tag = f"bl{os.getpid()}"
        owner = vep.BusOwner(tag, 0, max(cams) + 1)
        owner.attach(worker)
        for name, c in hub.map.items():
            owner.add(c, name)
        srv = vep.RpcServer("127.0.0.1", 0, tag, wait_threads=workers, reuseport=False)
        try:
            yield f"127.0.0.1:{srv.port}", list(hub.map), _NativeSvc(srv)
        finally:
            srv.stop()
            owner.stop()
        return
    svc = ImageService(_PM(hub))
    server = serve(svc, "127.0.0.1:0", workers=workers, tune_malloc=True)  # (a serving-only process)
    try:
        yield f"127.0.0.1:{server.bound_port}", list(hub.map), svc
    finally:
        server.stop(0)


@contextmanager
def ticking(tick, fps: float):
    """Replay mode: call ``tick()`` (decode one frame per camera) at ``fps`` in the background."""
    stop = threading.Event()

    def run():
        nxt = time.perf_counter()
        while not stop.is_set():
            tick()
            nxt += 1.0 / fps
            time.sleep(max(0.0, nxt - time.perf_counter()))

    th = None
    if tick is not None:
        th = threading.Thread(target=run, daemon=True)
        th.start()
    try:
        yield
    finally:
        stop.set()
        if th is not None:
            th.join(timeout=10)


def measure(pool, worker, cams, duration_s: float = 3.0, serve_samples: int = 100, native: bool = True):
    """Runs the ``serve`` then the ``next`` measurement on the out-of-process ``pool``.
    Returns {"serve": [ms...], "next": [ms...], "frames_served": n, "server_ms": [...]}."""
    with serving(worker, cams, workers=max(16, 2 * pool.clients), native=native) as (target, names, svc):
        serve_ms = pool.run(target, names, mode="serve", samples=serve_samples, procs=1) if serve_samples else []
        svc.latencies_ms.clear()
        n0 = svc.frames_served
        next_ms = pool.run(target, names, mode="next", duration_s=duration_s)
        server_ms = list(svc.latencies_ms)
        return {"serve": serve_ms, "next": next_ms, "frames_served": svc.frames_served - n0,
                "server_ms": server_ms}


def summarize(xs):
    if not xs:
        return None, None
    s = sorted(xs)
    return statistics.median(s), s[max(0, int(len(s) * 0.99) - 1)]
