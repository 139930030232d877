#!/usr/bin/env python3
"""Serving benchmark: VideoLatestImage at node scale (aggregate frames/s served, client latency).

Live cameras (an in-process loopback RTSP farm paced at --fps, the production IngestSession +
lazy decoder + gfx950 worker) publish into their HBM rings and onto the frame bus; then, for every
(serving mode, client count) pair, --duration seconds of back-to-back VideoLatestImage requests
from out-of-process clients (ClientPool: several clients per camera when clients > cameras):

  * ``frontends=0``: the round-3 path, one grpcio server inside the decoding process (each request
    D2H-copies its frame through the worker's pinned serve pool);
  * ``frontends=K``: K serving processes bound to one port with SO_REUSEPORT, reading the frame bus
    (server/frontend.py): one DMA per frame for all of a camera's clients, no GPU context and no
    connection to the decoding process;
  * ``native:K`` (--modes): the same with the native HTTP/2 endpoint (csrc/vep/rpcsrv.h) in the
    serving processes instead of grpcio; ``native:0`` runs it inside the decoding process (the
    default ``vep serve`` path on one GPU), reading that process's own frame bus.

Reported per pair: p50 / p99 client latency (request sent -> next frame received and parsed),
aggregate frames/s served, and the CPU the machine, the serving processes and the clients used.
Every process is started before this one touches the GPU.

    python tools/bench_serving.py --cams 32 --clients 32,128,256 --frontends 0,1,2,4
    python tools/bench_serving.py --cams 32 --clients 128,256 --modes native:0,native:2,grpcio:2
    python tools/bench_serving.py --codec h265 --width 3840 --height 2160 --cams 8 --clients 8,32
    python tools/bench_serving.py --cpu --width 320 --height 240 ...   (CPU backend rehearsal)

Reference: server/grpcapi/grpc_api.go:133-235 (one goroutine per stream, frames from Redis).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def ints(s: str) -> list[int]:
    return [int(x) for x in s.split(",") if x.strip()]


def cpu_of(pids) -> float:
    import psutil

    t = 0.0
    for pid in pids:
        try:
            p = psutil.Process(pid)
            for q in [p] + p.children(recursive=True):
                c = q.cpu_times()
                t += c.user + c.system
        except psutil.Error:
            pass
    return t


def hist_sum(w, cams):
    tot, bounds = None, None
    for c in cams:
        st = w.stats(c)
        h = st["latency_hist"]
        bounds = st["latency_bounds_ms"]
        tot = list(h) if tot is None else [a + b for a, b in zip(tot, h)]
    return tot, bounds


def hist_pct(h0, h1, q):
    """Upper bound (ms) of the histogram bucket holding quantile q of the samples between two
    snapshots (None: no samples; inf: the overflow bucket)."""
    (a, bounds), (b, _) = h0, h1
    d = [y - x for x, y in zip(a, b)]
    n = sum(d)
    if n <= 0:
        return None
    acc = 0
    for i, v in enumerate(d):
        acc += v
        if acc >= q * n:
            return bounds[i] if i < len(bounds) else float("inf")
    return None


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--cams", type=int, default=32)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--fps", type=int, default=30)
    ap.add_argument("--gop", type=int, default=30)
    ap.add_argument("--codec", choices=["h264", "h265"], default="h264")
    ap.add_argument("--slices", type=int, default=1, help="slices per picture (H.265 4K: 8, parsed in parallel)")
    ap.add_argument("--clients", default="32,128")
    ap.add_argument("--frontends", default="0,1,4", help="serving processes per trial (0 = in-process server)")
    ap.add_argument("--modes", default="", help="serving modes 'kind:K' (kind grpcio | native); overrides --frontends")
    ap.add_argument("--client-threads", type=int, default=8, help="client threads per client process")
    ap.add_argument("--serve-threads", type=int, default=256)
    ap.add_argument("--duration", type=float, default=4.0)
    ap.add_argument("--cpu", action="store_true", help="CPU backend (no GPU)")
    ap.add_argument("--out", default="", help="also append the JSON lines to this file")
    ap.add_argument("--client", choices=["grpcio", "native"], default="grpcio",
                    help="load generator: grpcio clients (Python, parse every VideoFrame) or the native "
                         "HTTP/2 clients (csrc/vep/h2load.h: count and discard the frame bytes)")
    a = ap.parse_args()

    from video_edge_ai_proxy_amd.server.frontend import FrontendPool
    from vep_bench.latency_clients import ClientPool

    clients = ints(a.clients)
    modes = ([(m.split(":")[0], int(m.split(":")[1])) for m in a.modes.split(",") if m.strip()] if a.modes
             else [("grpcio", k) for k in ints(a.frontends)])
    tag = f"sb{os.getpid()}"
    # every process first: this one initialises the GPU below
    t = a.client_threads
    pool = ClientPool(max(1, -(-max(clients) // t)), t)
    fpools = {(kind, k): FrontendPool(k, tag, f"127.0.0.1:{free_port()}", f"127.0.0.1:{free_port()}", a.serve_threads,
                                      native=kind == "native")
              for kind, k in modes if k > 0}

    import psutil
    import torch

    from video_edge_ai_proxy_amd import native as vep
    from vep_bench.bench_latency import serving, summarize

    use_gpu = (not a.cpu) and torch.cuda.is_available()
    dev = 0 if use_gpu else -1
    w = vep.Worker(device=dev, max_cameras=a.cams)
    w.start()
    srv = vep.RtspServer("127.0.0.1", 0)
    for i in range(a.cams):
        c = vep.SynthConfig()
        c.width, c.height, c.fps, c.gop, c.codec = a.width, a.height, a.fps, a.gop, a.codec
        c.seed = 11 + i * 7919
        c.compressed = True
        c.qp, c.noise, c.temporal_noise, c.profile, c.bframes = 25, 8.0, 1.5, "high", 2
        c.idr_phase = (i * a.gop) // a.cams
        c.slices = a.slices
        srv.add_stream(f"/cam{i}", c, realtime=True, cached_frames=a.gop)
    srv.start()
    owner = vep.BusOwner(tag, 0, a.cams)
    owner.attach(w)
    cams, sess = [], []
    now = int(time.time() * 1000)
    for i in range(a.cams):
        cam = w.add_camera(f"cam{i}", 3)
        owner.add(cam, f"cam{i}")
        w.set_last_query(cam, now)
        s = vep.IngestSession(w, cam, f"cam{i}", f"rtsp://127.0.0.1:{srv.port}/cam{i}")
        s.start()
        cams.append(cam)
        sess.append(s)
    deadline = time.time() + 120
    while time.time() < deadline and min(w.published(c) for c in cams) < 3:
        for c in cams:
            w.set_last_query(c, int(time.time() * 1000))
        time.sleep(0.1)
    names = [f"cam{i}" for i in range(a.cams)]
    out = []
    base = {"cams": a.cams, "resolution": f"{a.width}x{a.height}", "codec": a.codec, "fps": a.fps, "slices": a.slices,
            "backend": "gfx950" if use_gpu else "cpu", "frame_bytes": a.width * a.height * 3,
            "cpus": psutil.cpu_count(), "client_threads_per_process": t}
    nsrv = None
    try:
        for kind, k in modes:
            for m in clients:
                procs = max(1, -(-m // t))
                if k == 0 and kind == "native":
                    ctx, svc = None, None
                    if nsrv is None:
                        nsrv = vep.RpcServer("127.0.0.1", 0, tag, wait_threads=max(64, 2 * m), reuseport=False)
                    target = f"127.0.0.1:{nsrv.port}"
                    srv_pids = [os.getpid()]
                elif k == 0:
                    ctx = serving(w, cams, workers=max(64, 2 * m))
                    target, _, svc = ctx.__enter__()
                    srv_pids = [os.getpid()]
                else:
                    ctx, svc = None, None
                    target = f"127.0.0.1:{fpools[(kind, k)].port}"
                    srv_pids = [fpools[(kind, k)].p.pid]
                try:
                    cmode = "native" if a.client == "native" else "next"
                    pool.run(target, names, mode=cmode, duration_s=1.0, procs=procs)  # connect + warm
                    pub0, dma0 = owner.published, owner.dma_bytes
                    c0 = psutil.cpu_times()
                    s0 = cpu_of(srv_pids)
                    k0 = cpu_of([p.pid for p in pool._p[:procs]])
                    f0 = sum(w.published(c) for c in cams)
                    h0 = hist_sum(w, cams)
                    t0 = time.perf_counter()
                    lat = pool.run(target, names, mode=cmode, duration_s=a.duration, procs=procs)
                    el = time.perf_counter() - t0
                    c1 = psutil.cpu_times()
                    s1 = cpu_of(srv_pids)
                    k1 = cpu_of([p.pid for p in pool._p[:procs]])
                    f1 = sum(w.published(c) for c in cams)
                    h1 = hist_sum(w, cams)
                finally:
                    if ctx is not None:
                        ctx.__exit__(None, None, None)
                busy = (c1.user + c1.system) - (c0.user + c0.system)
                p50, p99 = summarize(lat)
                served = len(lat) / a.duration
                r = dict(base, serving=kind, frontends=k, clients=m, client_procs=procs, client_impl=a.client,
                         p50_ms=round(p50, 2) if p50 else None, p99_ms=round(p99, 2) if p99 else None,
                         samples=len(lat), frames_served_per_s=round(served, 1),
                         served_gbytes_per_s=round(served * a.width * a.height * 3 / 1e9, 2),
                         decoded_frames_per_s=round((f1 - f0) / el, 1),
                         # packet arrival -> frame published (the worker's per-camera histogram)
                         publish_latency_ms_p50=hist_pct(h0, h1, 0.5), publish_latency_ms_p99=hist_pct(h0, h1, 0.99),
                         bus_dma_frames=(owner.published - pub0) if (k > 0 or kind == "native") else None,
                         bus_dma_gbytes_per_s=(round((owner.dma_bytes - dma0) / el / 1e9, 2)
                                               if (k > 0 or kind == "native") else None),
                         machine_cpu_busy=round(busy / el, 2),
                         serving_cpu=round((s1 - s0) / el, 2), client_cpu=round((k1 - k0) / el, 2),
                         # serving CPU seconds per GB served (k > 0: the serving processes alone)
                         serving_cpu_s_per_gb=(round((s1 - s0) / el / (served * a.width * a.height * 3 / 1e9), 3)
                                               if k > 0 and served > 0 else None),
                         latency_definition=("client-side: request sent -> the camera's next VideoFrame "
                                             + ("received and parsed" if a.client == "grpcio" else
                                                "received (all DATA bytes, then the trailers; native HTTP/2 "
                                                "client, bytes counted and discarded)")
                                             + " (back-to-back requests, includes waiting for the frame, up "
                                               "to one frame interval)"))
                if nsrv is not None and k == 0 and kind == "native":
                    r["native_stats"] = nsrv.stats()
                print(json.dumps(r), flush=True)
                out.append(r)
    finally:
        if nsrv is not None:
            nsrv.stop()
        for s in sess:
            s.stop()
        owner.stop()
        srv.stop()
        w.stop()
        pool.close()
        for p in fpools.values():
            p.close()
    if a.out:
        with open(a.out, "a") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
