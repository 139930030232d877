"""Node-scale serving rehearsal: aggregate VideoLatestImage frames/s as decoding worker processes
(one per GPU on a node) and serving processes are added.

The production daemon (``build_app``) runs with ``gpu.isolation: process`` over N worker
processes (``--devices``: -1 = the CPU backend, so N = 8 rehearses an 8-GPU node on a host without
8 GPUs) and ``serving.frontends`` serving processes (-1 = one per worker) reading the workers'
frame buses. A loopback RTSP farm feeds ``--cams-per-worker`` cameras to each worker; clients in
separate processes (several per camera when clients > cameras) issue back-to-back
VideoLatestImage requests for --duration seconds. For each N of ``--workers`` it prints one JSON
line: aggregate frames served per second, client p50 / p99, decoded frames per second and the CPU
the machine used.

    python -m vep_bench.serving_node --workers 1,2,4,8 --cams-per-worker 4 --clients-per-cam 2

Reference: server/grpcapi/grpc_api.go:133-235 (one goroutine per client stream),
server/main.go:142-154.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time


def ints(s: str) -> list[int]:
    return [int(x) for x in s.split(",") if x.strip()]


def _settle(hub, names, n_frames=3, timeout=90.0) -> bool:
    deadline = time.time() + timeout
    seen = set()
    while time.time() < deadline and len(seen) < len(names):
        for n in names:
            hub.touch(n)
            try:
                r = hub.latest_frame_bytes(n, 0, 50)
            except RuntimeError:
                r = None
            if r and r[0] >= n_frames:
                seen.add(n)
        time.sleep(0.05)
    return len(seen) == len(names)


def trial(a, n_workers: int, pool) -> dict:
    import psutil

    from video_edge_ai_proxy_amd._native import native
    from video_edge_ai_proxy_amd.config import Config
    from video_edge_ai_proxy_amd.server.app import build_app
    from vep_bench.bench_latency import summarize

    cams = n_workers * a.cams_per_worker
    names = [f"c{i}" for i in range(cams)]
    srv = native.RtspServer("127.0.0.1", 0)
    for i, n in enumerate(names):
        c = native.SynthConfig()
        c.width, c.height, c.gop, c.fps, c.seed = a.width, a.height, 30, a.fps, 11 + i
        srv.add_stream(f"/{n}", c, realtime=True, cached_frames=30)
    srv.start()
    tmp = tempfile.TemporaryDirectory(prefix="vep-node-")
    cfg = Config()
    cfg.data_dir = tmp.name
    cfg.gpu.isolation = "process"
    cfg.gpu.max_cameras_per_gpu = max(4, a.cams_per_worker)
    cfg.serving.frontends = a.frontends if a.frontends >= 0 else n_workers
    cfg.serving.threads = a.serve_threads
    devices = [a.device] * n_workers if a.device < 0 else list(range(n_workers))
    app = build_app(cfg, host="127.0.0.1", grpc_port=0, devices=devices, start_rest=False, restore=False)
    out = {"workers": n_workers, "frontends": cfg.serving.frontends, "cams": cams,
           "resolution": f"{a.width}x{a.height}", "fps": a.fps, "backend": "cpu" if a.device < 0 else "gfx950",
           "host_cpus": psutil.cpu_count()}
    try:
        for n in names:
            app.hub.start_camera(n, f"rtsp://127.0.0.1:{srv.port}/{n}")
        out["settled"] = _settle(app.hub, names)
        target = f"127.0.0.1:{app.grpc_port}"
        clients = names * a.clients_per_cam
        procs = max(1, -(-len(clients) // pool.threads))
        procs = min(procs, pool.procs)
        pool.run(target, clients, mode="next", duration_s=1.0, procs=procs)  # connect + warm
        c0 = psutil.cpu_times()
        d0 = sum(app.hub.state(n).get("published", 0) for n in names)
        t0 = time.perf_counter()
        lat = pool.run(target, clients, mode="next", duration_s=a.duration, procs=procs)
        el = time.perf_counter() - t0
        d1 = sum(app.hub.state(n).get("published", 0) for n in names)
        c1 = psutil.cpu_times()
        p50, p99 = summarize(lat)
        out.update(clients=len(clients), client_procs=procs, samples=len(lat),
                   frames_served_per_s=round(len(lat) / a.duration, 1),
                   # each client asks for every new frame of its camera: clients x fps is the demand
                   frames_offered_per_s=len(clients) * a.fps,
                   served_fraction=round(len(lat) / a.duration / (len(clients) * a.fps), 3),
                   served_mbytes_per_s=round(len(lat) / a.duration * a.width * a.height * 3 / 1e6, 1),
                   p50_ms=round(p50, 2) if p50 else None, p99_ms=round(p99, 2) if p99 else None,
                   decoded_frames_per_s=round((d1 - d0) / el, 1),
                   machine_cpu_busy=round(((c1.user + c1.system) - (c0.user + c0.system)) / el, 2))
    finally:
        app.stop()
        srv.stop()
        tmp.cleanup()
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--workers", default="1,2,4,8", help="worker processes per trial")
    ap.add_argument("--device", type=int, default=-1, help="-1: CPU backend workers; 0: worker k on GPU k")
    ap.add_argument("--cams-per-worker", type=int, default=4)
    ap.add_argument("--clients-per-cam", type=int, default=2)
    ap.add_argument("--frontends", type=int, default=-1, help="serving processes (-1: one per worker)")
    ap.add_argument("--serve-threads", type=int, default=256)
    ap.add_argument("--client-threads", type=int, default=8)
    ap.add_argument("--width", type=int, default=320)
    ap.add_argument("--height", type=int, default=240)
    ap.add_argument("--fps", type=int, default=30)
    ap.add_argument("--duration", type=float, default=4.0)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)

    from vep_bench.latency_clients import ClientPool

    ws = ints(a.workers)
    most = max(ws) * a.cams_per_worker * a.clients_per_cam
    pool = ClientPool(max(1, -(-most // a.client_threads)), a.client_threads)  # before any GPU use
    rows = []
    try:
        for n in ws:
            r = trial(a, n, pool)
            print(json.dumps(r), flush=True)
            rows.append(r)
    finally:
        pool.close()
    if a.out:
        with open(a.out, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    return 0 if all(r.get("settled") for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
