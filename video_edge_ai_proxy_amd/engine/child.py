"""One per-GPU worker process of the isolated hub (``gpu.isolation: process``, see isolated.py).

Runs an in-process :class:`~video_edge_ai_proxy_amd.engine.hub.Hub` for one device and serves its
methods over authenticated local connections (``multiprocessing.connection``), one thread per
connection. The parent hub supervises the process: a native fault here (a crash in a camera's
bitstream parse or a GPU error) ends this process only, and the parent starts a fresh one and
re-adds its cameras — the reference's per-camera ``restart: always`` container
(server/services/rtsp_process_manager.go:70-81) at per-GPU granularity.

Usage (by the parent only): ``python -m video_edge_ai_proxy_amd.engine.child --device D
--config JSON`` with the connection key in ``VEP_CHILD_KEY``; prints ``{"port": P}`` once ready
and exits when its stdin closes (the parent is gone).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import threading
from multiprocessing.connection import Listener

# methods of Hub a parent may call
EXPORTED = {"start_camera", "stop_camera", "state", "logs", "touch", "set_proxy", "proxy",
            "latest_frame_bytes", "latest_frame", "wait_decoded", "has"}


def _serve(hub, conn, lock_stop: threading.Event) -> None:
    while not lock_stop.is_set():
        try:
            req = conn.recv()
        except (EOFError, OSError):
            return
        method, args, kwargs = req
        try:
            if method == "ping":
                res = os.getpid()
            elif method == "worker_stats":
                w = hub.workers[0]
                res = {"batches": w.batches, "frames": w.frames, "gpu_ms_total": w.gpu_ms_total,
                       "direct_reads": bool(w.direct_reads), "decoder": str(w.decoder)}
            elif method == "start_camera":
                h = hub.start_camera(*args, **kwargs)
                res = {"cam": h.cam}
            elif method in EXPORTED:
                res = getattr(hub, method)(*args, **kwargs)
            else:
                raise AttributeError(f"no such method {method!r}")
            conn.send(("ok", res))
        except Exception as e:  # noqa: BLE001 — the error travels back to the caller
            try:
                conn.send(("err", type(e).__name__, str(e)))
            except (OSError, EOFError):
                return


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", type=int, required=True)
    ap.add_argument("--config", required=True, help="Config as JSON")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format=f"%(asctime)s child[{a.device}] %(name)s: %(message)s")
    from ..config import Config, _merge
    from .hub import Hub

    cfg = _merge(Config(), json.loads(a.config))
    hub = Hub(cfg, devices=[a.device])
    key = bytes.fromhex(os.environ["VEP_CHILD_KEY"])
    listener = Listener(("127.0.0.1", 0), authkey=key)
    stop = threading.Event()

    def accept_loop():
        while not stop.is_set():
            try:
                conn = listener.accept()
            except Exception:  # noqa: BLE001 — listener closed or a bad handshake
                if stop.is_set():
                    return
                continue
            threading.Thread(target=_serve, args=(hub, conn, stop), daemon=True).start()

    threading.Thread(target=accept_loop, daemon=True, name="vep-child-accept").start()
    print(json.dumps({"port": listener.address[1], "pid": os.getpid()}), flush=True)
    try:
        sys.stdin.read()  # returns when the parent closes the pipe (or dies)
    except Exception:  # noqa: BLE001
        pass
    stop.set()
    try:
        listener.close()
    except Exception:  # noqa: BLE001
        pass
    hub.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
