"""Client-observed ``VideoLatestImage`` latency for bench.py, through the production gRPC path
(ImageService -> native ring D2H -> pre-encoded VideoFrame -> grpcio -> client decode).

Two definitions are measured while the cameras keep decoding at their real frame rate:
  * ``serve``: a new channel per request — the server answers with the newest frame already
    in the HBM ring (request sent -> VideoFrame fully received and parsed).
  * ``next_frame``: one channel, back-to-back requests (the reference example clients'
    pattern): each answer must be a frame newer than the previous one, so the time includes
    waiting for the camera's next decoded frame (bounded by the frame interval).
"""
from __future__ import annotations

import statistics
import threading
import time

from ..utils import now_ms
from .grpc_server import ImageClient, ImageService, serve


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
        if wait_ms > 0 and self.w.published(c) <= after:
            self.w.wait_frame(c, after, wait_ms)
        return self.w.video_frame(c, after, name)


class _PM:
    def __init__(self, hub):
        self.hub = hub


def grpc_latency(worker, cams, samples: int, tick=None, fps: float = 30.0):
    """Returns (serve_ms list, next_frame_ms list). ``tick()`` decodes one frame per camera."""
    hub = _WorkerHub(worker, cams)
    svc = ImageService(_PM(hub))
    server = serve(svc, "127.0.0.1:0", workers=16)
    stop = threading.Event()

    def ticker():
        nxt = time.perf_counter()
        while not stop.is_set():
            if tick is not None:
                tick()
            nxt += 1.0 / fps
            time.sleep(max(0.0, nxt - time.perf_counter()))

    th = threading.Thread(target=ticker, daemon=True)
    th.start()
    target = f"127.0.0.1:{server.bound_port}"
    names = list(hub.map)
    serve_ms, next_ms = [], []
    try:
        import grpc

        time.sleep(0.2)
        # connected channels prepared up front: the timed span is request -> frame received
        clients = [ImageClient(target) for _ in range(samples)]
        for c in clients:
            grpc.channel_ready_future(c.channel).result(timeout=10)
        for i, cli in enumerate(clients):
            t0 = time.perf_counter()
            vf = cli.latest_frame(names[i % len(names)])
            t1 = time.perf_counter()
            if vf is not None and vf.width:
                serve_ms.append((t1 - t0) * 1e3)
        for c in clients:
            c.close()
        cli = ImageClient(target)
        name = names[0]
        cli.latest_frame(name)
        for _ in range(max(10, samples // 2)):
            t0 = time.perf_counter()
            vf = cli.latest_frame(name)
            t1 = time.perf_counter()
            if vf is not None and vf.width:
                next_ms.append((t1 - t0) * 1e3)
        cli.close()
    finally:
        stop.set()
        th.join(timeout=5)
        server.stop(0)
    return serve_ms, next_ms


def grpc_concurrent_latency(worker, cams, clients: int, duration_s: float = 3.0, tick=None,
                            fps: float = 30.0):
    """``clients`` concurrent gRPC clients, each on its own connected channel and camera
    (round-robin), issuing back-to-back VideoLatestImage requests for ``duration_s`` — the
    reference clients' pattern, all at once. Each answer is a frame newer than the client's
    previous one, so a sample is request sent -> the camera's next frame received and parsed.
    ``tick()`` (replay mode) decodes one frame per camera at ``fps``; None when the cameras decode
    live (RTSP farm). Returns the per-request latencies in ms."""
    import grpc

    hub = _WorkerHub(worker, cams)
    svc = ImageService(_PM(hub))
    server = serve(svc, "127.0.0.1:0", workers=max(16, 2 * clients))
    stop = threading.Event()
    ticker_th = None
    if tick is not None:
        def ticker():
            nxt = time.perf_counter()
            while not stop.is_set():
                tick()
                nxt += 1.0 / fps
                time.sleep(max(0.0, nxt - time.perf_counter()))

        ticker_th = threading.Thread(target=ticker, daemon=True)
        ticker_th.start()
    target = f"127.0.0.1:{server.bound_port}"
    names = list(hub.map)
    lat: list[list[float]] = [[] for _ in range(clients)]
    go = threading.Event()

    def client(k):
        cli = ImageClient(target)
        try:
            grpc.channel_ready_future(cli.channel).result(timeout=10)
            name = names[k % len(names)]
            cli.latest_frame(name)  # cursor at the current frame
            go.wait()
            end = time.perf_counter() + duration_s
            while time.perf_counter() < end:
                t0 = time.perf_counter()
                vf = cli.latest_frame(name)
                t1 = time.perf_counter()
                if vf is not None and vf.width:
                    lat[k].append((t1 - t0) * 1e3)
        finally:
            cli.close()

    threads = [threading.Thread(target=client, args=(k,), daemon=True) for k in range(clients)]
    try:
        for t in threads:
            t.start()
        time.sleep(0.5)
        go.set()
        for t in threads:
            t.join(timeout=duration_s + 30)
    finally:
        stop.set()
        if ticker_th is not None:
            ticker_th.join(timeout=5)
        server.stop(0)
    return [x for xs in lat for x in xs]


def grpc_latency_samples(worker, cams, samples, tick=None):
    serve_ms, _ = grpc_latency(worker, cams, samples, tick)
    return serve_ms


def summarize(xs):
    if not xs:
        return None, None
    s = sorted(xs)
    return statistics.median(s), s[max(0, int(len(s) * 0.99) - 1)]
