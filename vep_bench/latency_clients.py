"""Out-of-process gRPC latency clients for bench.py and load tests.

The clients of a frame server must not share its process: receiving and parsing a 6.2 MB 1080p
``VideoFrame`` costs the Python gRPC client ~10 ms of CPU, and in the server's process that work
would hold the server's GIL. :class:`ClientPool` therefore runs the clients in fresh interpreter
processes (``python -m vep_bench.latency_clients``), started with
``subprocess`` *before* the parent initialises the GPU (a process that holds a GPU context must
not be the one that starts other programs), each running several client threads.

A job is one JSON line on a worker's stdin; the worker answers with one JSON line of latencies.
Two modes, both measured client-side (request sent -> ``VideoFrame`` received and parsed):
Every client has its own TCP connection (grpc-core would otherwise share one connection among
the channels of a process, and the server's per-connection cursors and HTTP/2 streams with it).
  * ``next``: each client owns one connected channel and camera and issues back-to-back
    ``VideoLatestImage`` requests (the reference example clients' pattern,
    examples/opencv_display.py:43-45); every answer is a frame newer than the client's previous
    one, so a sample includes waiting for the camera's next decoded frame.
  * ``serve``: one request per pre-connected channel (a new peer, so the server's cursor is
    empty): the newest frame already in the ring.

Reference: server/grpcapi/grpc_api.go:133-235 (the handler being measured).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import threading
import time

_PKG_PARENT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# glibc would mmap (and page-fault) every freshly allocated multi-MB frame buffer; keep them in
# the heap so they are reused (see native.tune_malloc_for_frames for the server side)
MALLOC_ENV = {"MALLOC_MMAP_THRESHOLD_": str(64 << 20), "MALLOC_TRIM_THRESHOLD_": str(256 << 20),
              "MALLOC_TOP_PAD_": str(64 << 20)}


class ClientPool:
    """``procs`` client processes with ``threads`` client threads each (clients = procs x threads)."""

    def __init__(self, procs: int, threads: int, start_timeout_s: float = 120.0):
        self.procs, self.threads = procs, threads
        env = dict(os.environ, **MALLOC_ENV)
        env["PYTHONPATH"] = _PKG_PARENT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        env.pop("GPU_MAX_HW_QUEUES", None)
        # the clients never use the GPU: hide it so nothing in them can initialise it
        env["HIP_VISIBLE_DEVICES"] = ""
        env["CUDA_VISIBLE_DEVICES"] = ""
        self._p = [subprocess.Popen([sys.executable, "-u", "-m", "vep_bench.latency_clients",
                                     "--threads", str(threads)], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                    env=env, text=True) for _ in range(procs)]
        deadline = time.time() + start_timeout_s
        for p in self._p:
            line = p.stdout.readline()
            if line.strip() != "ready":
                self.close()
                raise RuntimeError(f"latency client process failed to start ({line!r})")
            if time.time() > deadline:
                self.close()
                raise RuntimeError("latency client processes did not start in time")

    @property
    def clients(self) -> int:
        return self.procs * self.threads

    def run(self, target: str, names: list[str], mode: str = "next", duration_s: float = 3.0,
            samples: int = 0, key_frame_only: bool = False, procs: int = 0) -> list[float]:
        """Run one job on every process (or the first ``procs``): client k (of procs x threads)
        asks for camera ``names[k % len(names)]``. Returns every latency sample (ms).
        ``mode="native"``: the ``next`` pattern with the native load generator (``native.h2_load``,
        csrc/vep/h2load.h) instead of grpcio clients: each process runs its clients as raw HTTP/2
        connections on two epoll threads, counting and discarding the frame bytes."""
        use = self._p[:procs] if procs > 0 else self._p
        start_at = time.time() + 1.0 + 0.05 * len(use)  # all processes connect first
        for i, p in enumerate(use):
            mine = [names[(i * self.threads + t) % len(names)] for t in range(self.threads)]
            job = {"target": target, "names": mine, "mode": mode, "duration": duration_s,
                   "samples": samples, "start_at": start_at, "key_frame_only": key_frame_only}
            p.stdin.write(json.dumps(job) + "\n")
            p.stdin.flush()
        out: list[float] = []
        errors = []
        for p in use:
            line = p.stdout.readline()
            if not line:
                raise RuntimeError("latency client process exited")
            r = json.loads(line)
            out += r["lat"]
            errors += r.get("errors", [])
        if errors and not out:
            raise RuntimeError(f"every latency client failed: {errors[:3]}")
        return out

    def close(self) -> None:
        for p in self._p:
            try:
                p.stdin.close()
            except Exception:  # noqa: BLE001
                pass
        for p in self._p:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _client_next(target, name, key_frame_only, start_at, duration, lat, errors):
    import grpc

    from video_edge_ai_proxy_amd.server.grpc_server import ImageClient

    cli = ImageClient(target, own_connection=True)  # (a camera viewer: its own TCP connection)
    try:
        grpc.channel_ready_future(cli.channel).result(timeout=20)
        cli.latest_frame(name, key_frame_only)  # the server-side cursor sits at the current frame
        time.sleep(max(0.0, start_at - time.time()))
        end = time.perf_counter() + duration
        while time.perf_counter() < end:
            t0 = time.perf_counter()
            vf = cli.latest_frame(name, key_frame_only)
            t1 = time.perf_counter()
            if vf is not None and vf.width:
                lat.append((t1 - t0) * 1e3)
    except Exception as e:  # noqa: BLE001 — reported to the parent
        errors.append(f"{type(e).__name__}: {e}")
    finally:
        cli.close()


def _client_serve(target, names, key_frame_only, samples, lat, errors):
    import grpc

    from video_edge_ai_proxy_amd.server.grpc_server import ImageClient

    clis = [ImageClient(target, own_connection=True) for _ in range(samples)]
    try:
        for c in clis:
            grpc.channel_ready_future(c.channel).result(timeout=20)
        for i, c in enumerate(clis):
            t0 = time.perf_counter()
            vf = c.latest_frame(names[i % len(names)], key_frame_only)
            t1 = time.perf_counter()
            if vf is not None and vf.width:
                lat.append((t1 - t0) * 1e3)
    except Exception as e:  # noqa: BLE001
        errors.append(f"{type(e).__name__}: {e}")
    finally:
        for c in clis:
            c.close()


def main(argv=None) -> int:
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=4)
    a = ap.parse_args(argv)
    import grpc  # noqa: F401 — imported once up front (the first import is slow on a fresh box)

    from video_edge_ai_proxy_amd.server import grpc_server  # noqa: F401

    print("ready", flush=True)
    for line in sys.stdin:
        job = json.loads(line)
        lat: list[float] = []
        errors: list[str] = []
        if job["mode"] == "serve":
            _client_serve(job["target"], job["names"], job["key_frame_only"], max(1, job["samples"]), lat, errors)
        elif job["mode"] == "native":
            from video_edge_ai_proxy_amd import native

            host, port = job["target"].rsplit(":", 1)
            names = job["names"][:a.threads]
            r = native.h2_load(host, int(port), names, clients=len(names), threads=min(2, len(names)),
                               start_at=job["start_at"], duration_s=job["duration"],
                               key_frame_only=job["key_frame_only"])
            lat = list(r["lat_ms"])
            if r["errors"]:
                errors.append(f"h2_load: {r['errors']} errors ({r['first_error']})")
        else:
            ths = [threading.Thread(target=_client_next, args=(job["target"], n, job["key_frame_only"],
                                                               job["start_at"], job["duration"], lat, errors),
                                    daemon=True) for n in job["names"][:a.threads]]
            for t in ths:
                t.start()
            for t in ths:
                t.join(timeout=job["duration"] + 60)
        print(json.dumps({"lat": lat, "errors": errors}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
