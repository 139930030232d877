"""End-to-end check of the process-isolated hub on real devices (``gpu.isolation: process``).

Run it as its own program (``python -m vep_bench.isolated_check --devices 0``):
this process is the front-end and never touches a GPU; the worker processes it supervises do.
It starts a loopback RTSP farm, one supervised worker process per device, and checks:

* frames served through the frame bus (the worker's page-locked shared-memory segments on GPUs:
  ``pinned``) equal the ring's latest frame, with the serving latency of back-to-back
  ``latest_frame_bytes`` requests;
* ``consumer_batch()`` — an all-gather across the worker processes' group (RCCL on GPUs) — matches
  the fp32 letterbox reference of every camera's latest frame; then ``--gathers`` steady-state
  gathers are timed (group formation excluded);
* with ``--kill``: a SIGKILLed worker is restarted, its cameras re-added, the group re-formed and
  the gather works again.

Prints one JSON line; exit status 0 when every check passed.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import sys
import tempfile
import time


def _settle(hub, names, n_frames=3, timeout=60.0):
    deadline = time.time() + timeout
    seen = {}
    while time.time() < deadline and len(seen) < len(names):
        for n in names:
            hub.touch(n)
            try:
                r = hub.latest_frame_bytes(n, 0, 100)
            except RuntimeError:
                r = None
            if r and r[0] >= n_frames:
                seen[n] = r[0]
        time.sleep(0.05)
    return len(seen) == len(names)


def _rows_match(hub, batch, names, size) -> float:
    import numpy as np
    import torch

    from video_edge_ai_proxy_amd.ops import letterbox_reference

    worst = 0.0
    for row, n in zip(batch, names):
        _, img = hub.latest_frame(n, 0)
        ref, _ = letterbox_reference(torch.from_numpy(np.ascontiguousarray(img)), size)
        worst = max(worst, float((row.int() - ref.int()).abs().max().item()))
    return worst


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--devices", default="0", help="comma-separated device ids (-1: CPU backend)")
    ap.add_argument("--cams", type=int, default=4)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--letterbox", type=int, default=640)
    ap.add_argument("--samples", type=int, default=60)
    ap.add_argument("--kill", action="store_true")
    ap.add_argument("--gathers", type=int, default=20, help="steady-state consumer gathers to time")
    a = ap.parse_args(argv)

    from video_edge_ai_proxy_amd._native import native
    from video_edge_ai_proxy_amd.config import Config
    from video_edge_ai_proxy_amd.engine.isolated import ProcessHub

    devices = [int(x) for x in a.devices.split(",")]
    srv = native.RtspServer("127.0.0.1", 0)
    for i in range(a.cams):
        c = native.SynthConfig()
        c.width, c.height, c.gop, c.fps, c.seed = a.width, a.height, 30, 30, 11 + i
        srv.add_stream(f"/c{i}", c, realtime=True, cached_frames=30)
    srv.start()
    tmp = tempfile.TemporaryDirectory(prefix="vep-iso-")
    cfg = Config()
    cfg.data_dir = tmp.name
    cfg.gpu.isolation = "process"
    cfg.gpu.letterbox_size = a.letterbox
    cfg.gpu.max_cameras_per_gpu = max(4, a.cams)
    cfg.gpu.idle_cutoff_ms = 400
    out = {"devices": devices, "cams": a.cams, "width": a.width, "height": a.height, "ok": False}
    hub = ProcessHub(cfg, devices=devices, supervise_interval_s=0.5)
    try:
        names = [f"c{i}" for i in range(a.cams)]
        for n in names:
            hub.start_camera(n, f"rtsp://127.0.0.1:{srv.port}/{n}")
        out["settled"] = _settle(hub, names)
        # serving through shared memory: back-to-back requests for the next frame
        lat = []
        seq = 0
        nbytes = 0
        t_all = time.perf_counter()
        for _ in range(a.samples):
            hub.touch(names[0])
            t0 = time.perf_counter()
            r = hub.latest_frame_bytes(names[0], seq, 200)
            if r is None:
                continue
            lat.append((time.perf_counter() - t0) * 1e3)
            out["shm_pinned"] = bool(r[2].get("shm_pinned"))
            seq = r[0]
            nbytes += len(r[1])
        wall = time.perf_counter() - t_all
        lat.sort()
        out["serve_samples"] = len(lat)
        out["serve_p50_ms"] = round(lat[len(lat) // 2], 3) if lat else None
        out["served_MBps"] = round(nbytes / wall / 1e6, 1)
        # the same VideoFrame bytes as the ring's latest frame
        import numpy as np

        from video_edge_ai_proxy_amd.proto import pb

        time.sleep(1.0)  # > idle cutoff: decoding pauses, the latest frames stay put
        seq, frame, _ = hub.latest_frame_bytes(names[0], 0, 0)
        vf = pb.VideoFrame()
        vf.ParseFromString(frame)
        _, img = hub.latest_frame(names[0], 0)
        out["frame_equal"] = bool(np.array_equal(np.frombuffer(vf.data, np.uint8).reshape(img.shape), img))
        t0 = time.perf_counter()
        batch, order = hub.consumer_batch(names=names)
        out["first_gather_ms"] = round((time.perf_counter() - t0) * 1e3, 2)  # (includes group formation)
        for _ in range(a.gathers):  # steady state: the group exists
            hub.consumer_batch(names=names, to_host=False)
        ms = sorted(hub.gather_ms[-a.gathers:]) if a.gathers else []
        out["steady_gathers"] = len(ms)
        out["steady_gather_ms_p50"] = round(ms[len(ms) // 2], 3) if ms else None
        out["steady_gather_ms_max"] = round(ms[-1], 3) if ms else None
        out["gather_definition"] = ("per call, max over ranks: snapshot of the consumer rows + the header and "
                                    "row all-gathers (RCCL on GPUs) + stream sync; group formation excluded")
        out["batch_shape"] = list(batch.shape)
        out["batch_max_abs_err"] = _rows_match(hub, batch, order, a.letterbox)
        out["group"] = [c.call("group_info") for c in hub._children]
        ok = out["settled"] and out["frame_equal"] and out["batch_max_abs_err"] <= 1 and len(lat) > 0
        if a.kill:
            victim = hub.state(names[0])["worker_pid"]
            wi = hub.handle(names[0]).worker_index
            os.kill(victim, signal.SIGKILL)
            deadline = time.time() + 120
            while time.time() < deadline and hub.child_restarts[wi] == 0:
                time.sleep(0.2)
            out["restarted"] = hub.child_restarts[wi] == 1
            out["resettled"] = _settle(hub, names)
            time.sleep(1.0)
            batch, order = hub.consumer_batch(names=names)
            out["batch_after_restart_max_abs_err"] = _rows_match(hub, batch, order, a.letterbox)
            out["group_epoch"] = hub._group_epoch
            ok = ok and out["restarted"] and out["resettled"] and out["batch_after_restart_max_abs_err"] <= 1
        out["ok"] = bool(ok)
    finally:
        hub.shutdown()
        srv.stop()
        tmp.cleanup()
    print(json.dumps(out), flush=True)
    return 0 if out["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
