"""Per-GPU host data plane rehearsal: aggregate decoded pictures/s of the production daemon as
GPU workers are added, each with its own host domain (hostplan.h).

``vep serve``'s app (``build_app``, thread isolation: one process, one native Worker per GPU) runs
on the CPU backend with N workers standing in for N GPUs. Each worker's host domain is pinned to
its own slice of ``--worker-cpus`` (``gpu.host_cpus``: the NUMA-local CPUs a GPU would have on a
node), and a loopback RTSP camera farm in a separate process (pinned to ``--farm-cpus``, as is
this process's Python) serves ``--cams-per-worker`` cameras per worker, unthrottled
(``--fps 0``: every camera sends as fast as the sockets take it, so decoded pictures/s is the
node's decode capacity) or paced (``--fps F``: an offered rate, e.g. BASELINE config 5 scaled to
the container). Unthrottled cameras are ingested losslessly (a camera whose parse backlog is deep
has its socket paused: TCP back-pressure on the farm), paced ones with the production lossy
ingest. Clients keep every camera's demand alive (the lazy decoder's last_query). For
each N of ``--workers`` one JSON line: decoded pictures/s (whole daemon and per worker), the
offered rate when paced, and each worker's CPU list and parse threads as ``/healthz`` reports them.

    python -m vep_bench.host_plane --workers 1,2,3,4,6,8 --worker-cpus 0-5 --cpus-per-worker 1 --farm-cpus 6-7

Reference: one container per camera, each with its own CPU share
(server/services/rtsp_process_manager.go:70-81,106-115).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

FARM = r"""
import sys, time, json
sys.path.insert(0, {root!r})
from video_edge_ai_proxy_amd._native import native
a = json.loads({args!r})
srv = native.RtspServer("127.0.0.1", 0)
for i in range(a["cams"]):
    c = native.SynthConfig()
    c.width, c.height, c.gop, c.fps, c.seed = a["width"], a["height"], a["gop"], max(1, a["fps"]), 101 + i * 7919
    c.codec, c.compressed = a["codec"], True
    c.bframes, c.slices = a["bframes"], a["slices"]
    c.idr_phase = (i * a["gop"]) // max(1, a["cams"])
    srv.add_stream("/c%d" % i, c, realtime=a["fps"] > 0, cached_frames=a["gop"])
srv.start()
print(srv.port, flush=True)
sys.stdin.read()  # until the parent closes the pipe
srv.stop()
"""


def cpus_of(s: str) -> list[int]:
    from video_edge_ai_proxy_amd._native import native

    return native.parse_cpulist(s)


def thread_cpu() -> dict:
    tick = os.sysconf("SC_CLK_TCK")
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/comm") as f:
                name = f.read().strip()
            with open(f"/proc/self/task/{tid}/stat") as f:
                st = f.read().rsplit(")", 1)[1].split()
        except OSError:
            continue
        name = name if name.startswith("vep-") else "other"
        out[name] = out.get(name, 0.0) + (int(st[11]) + int(st[12])) / tick
    return out


def trial(a, n: int) -> dict:
    from video_edge_ai_proxy_amd._native import native
    from video_edge_ai_proxy_amd.config import Config
    from video_edge_ai_proxy_amd.server.app import build_app

    wc = cpus_of(a.worker_cpus)
    cams = n * a.cams_per_worker
    farm_args = dict(cams=cams, width=a.width, height=a.height, gop=a.gop, fps=a.fps, codec=a.codec,
                     bframes=a.bframes, slices=a.slices)
    farm = subprocess.Popen([sys.executable, "-c", FARM.format(root=ROOT, args=json.dumps(farm_args))],
                            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True,
                            preexec_fn=lambda: os.sched_setaffinity(0, cpus_of(a.farm_cpus)))
    port = int(farm.stdout.readline())
    tmp = tempfile.TemporaryDirectory(prefix="vep-hostplane-")
    cfg = Config()
    cfg.data_dir = tmp.name
    cfg.gpu.isolation = "thread"
    cfg.gpu.max_cameras_per_gpu = max(4, a.cams_per_worker)
    # each worker's domain: --cpus-per-worker CPUs of the worker CPUs (a GPU's NUMA-local CPUs on a
    # node), in order; past the last CPU the workers wrap around and share (0: split them evenly)
    k = a.cpus_per_worker
    if k > 0:
        cfg.gpu.host_cpus = [native.format_cpulist(sorted({wc[(j * k + i) % len(wc)] for i in range(k)}))
                             for j in range(n)]
    else:
        cfg.gpu.host_cpus = [native.format_cpulist(wc[j * len(wc) // n:(j + 1) * len(wc) // n]) if len(wc) >= n
                             else native.format_cpulist(wc) for j in range(n)]
    os.sched_setaffinity(0, a.all_cpus)  # (the plan intersects each list with this thread's mask)
    app = build_app(cfg, host="127.0.0.1", grpc_port=0, devices=[-1] * n, start_rest=False, restore=False)
    hub = app.hub
    os.sched_setaffinity(0, cpus_of(a.farm_cpus))  # this thread (Python) off the workers' CPUs
    names = [f"c{i}" for i in range(cams)]
    out = {"workers": n, "cams": cams, "codec": a.codec, "resolution": f"{a.width}x{a.height}",
           "farm": f"{a.fps} fps per camera" if a.fps > 0 else "unthrottled", "worker_cpus": a.worker_cpus,
           "farm_cpus": a.farm_cpus}
    try:
        for nm in names:
            h = hub.start_camera(nm, f"rtsp://127.0.0.1:{port}/{nm}")
            if a.fps <= 0:  # capacity: the unthrottled farm is back-pressured (paused sockets), not shed
                h.session.set_lossless(True)
        deadline = time.time() + 60
        while time.time() < deadline:  # every camera decoding
            for nm in names:
                hub.touch(nm)
            if all(hub.state(nm).get("decoded", 0) > 0 for nm in names):
                break
            time.sleep(0.2)
        time.sleep(a.settle)
        p0 = [w.pictures for w in hub.workers]
        sk0 = sum(hub.state(nm).get("skipped", 0) for nm in names)
        c0, t0 = thread_cpu(), time.perf_counter()
        while time.perf_counter() - t0 < a.duration:
            for nm in names:
                hub.touch(nm)
            time.sleep(0.25)
        el = time.perf_counter() - t0
        c1 = thread_cpu()
        per = [(w.pictures - p) / el for w, p in zip(hub.workers, p0)]
        out["decoded_pictures_per_s"] = round(sum(per), 1)
        out["per_worker_pictures_per_s"] = [round(x, 1) for x in per]
        if a.fps > 0:
            out["offered_pictures_per_s"] = cams * a.fps
            out["kept_up"] = sum(per) >= 0.97 * cams * a.fps
        out["access_units_skipped"] = sum(hub.state(nm).get("skipped", 0) for nm in names) - sk0
        out["cpu_cores_by_thread"] = {k: round((c1.get(k, 0) - c0.get(k, 0)) / el, 2) for k in c1
                                      if c1.get(k, 0) - c0.get(k, 0) > 0.01 * el}
        out["host_plane"] = [{k: d[k] for k in ("cpulist", "parse_threads", "ingest_parse_threads", "cameras", "source")}
                             for d in hub.host_plane()]
    finally:
        app.stop()
        farm.stdin.close()
        farm.wait(timeout=30)
        tmp.cleanup()
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--workers", default="1,2,3,6,8")
    ap.add_argument("--cams-per-worker", type=int, default=8)
    ap.add_argument("--codec", choices=["h264", "h265"], default="h264")
    ap.add_argument("--width", type=int, default=320)
    ap.add_argument("--height", type=int, default=192)
    ap.add_argument("--gop", type=int, default=30)
    ap.add_argument("--bframes", type=int, default=2)
    ap.add_argument("--slices", type=int, default=1)
    ap.add_argument("--fps", type=int, default=0, help="0 = unthrottled farm (capacity)")
    ap.add_argument("--worker-cpus", default="0-5")
    ap.add_argument("--cpus-per-worker", type=int, default=1,
                    help="CPUs each worker's host domain gets (a GPU's local CPUs); 0 = split --worker-cpus")
    ap.add_argument("--farm-cpus", default="6-7")
    ap.add_argument("--settle", type=float, default=2.0)
    ap.add_argument("--duration", type=float, default=6.0)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    sys.path.insert(0, ROOT)
    a.all_cpus = sorted(os.sched_getaffinity(0))
    for n in [int(x) for x in a.workers.split(",") if x]:
        r = trial(a, n)
        line = json.dumps(r)
        print(line, flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
