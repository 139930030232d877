"""One per-GPU worker process of the isolated hub (``gpu.isolation: process``, see isolated.py).

Runs an in-process :class:`~video_edge_ai_proxy_amd.engine.hub.Hub` for one device and serves its
methods over authenticated local connections (``multiprocessing.connection``), one thread per
connection. The parent hub supervises the process: a native fault here (a crash in a camera's
bitstream parse or a GPU error) ends this process only, and the parent starts a fresh one and
re-adds its cameras — the reference's per-camera ``restart: always`` container
(server/services/rtsp_process_manager.go:70-81) at per-GPU granularity.

Frames leave through the node's frame bus (csrc/vep/bus.h): the Hub of this process publishes
its cameras under ``cfg.bus_tag`` with owner index ``--owner``, and readers (the parent, the serving
processes) take frames from shared memory without calling this process. A gathered consumer batch
still leaves through the connection's page-locked segment (engine/shm.py).

The worker processes of one hub are the ranks of a ``torch.distributed`` group (RCCL over xGMI
on GPUs, gloo on the CPU backend), formed by the parent on demand and re-formed with a fresh
rendezvous after a restart. ``consumer_gather`` all-gathers every rank's letterboxed consumer
rows, so every GPU holds the node-wide batch (handed to ``gpu.consumer_hook`` if configured); one
rank also DMAs it into shared memory for the front-end's ``consumer_batch()``.

Usage (by the parent only): ``python -m video_edge_ai_proxy_amd.engine.child --device D
--config JSON`` with the connection key in ``VEP_CHILD_KEY``; prints ``{"port": P}`` once ready
and exits when its stdin closes (the parent is gone).
"""
from __future__ import annotations

import argparse
import importlib
import json
import logging
import os
import sys
import threading
from datetime import timedelta
from multiprocessing.connection import Listener

from .shm import ShmSlot, remove_segments

log = logging.getLogger("vep.child")

# methods of Hub a parent may call
EXPORTED = {"start_camera", "stop_camera", "state", "logs", "touch", "set_proxy", "proxy", "host_plane",
            "latest_frame_bytes", "latest_frame", "wait_decoded", "has"}


class RankGroup:
    """This process's membership in the hub's process group and the gathered node batch."""

    def __init__(self, hub, device: int, hook: str = ""):
        self.hub, self.device = hub, device
        self.epoch, self.rank, self.world, self.backend = -1, 0, 1, ""
        self.batch = None  # (tensor on this rank's device, names) of the last gather
        self.hook = None
        if hook:
            mod, _, fn = hook.partition(":")
            self.hook = getattr(importlib.import_module(mod), fn)
        self.gathers = 0
        self.gather_ms: list[float] = []  # per gather, this rank: snapshot + collectives

    def abort(self) -> dict:
        """Abort this rank's communicator (a collective pending on it fails at once): the parent
        does this before re-forming the group, instead of waiting for the collective's timeout."""
        import torch.distributed as dist
        from torch.distributed import distributed_c10d as c10d

        if dist.is_initialized():
            try:
                c10d._abort_process_group()
            except Exception:  # noqa: BLE001 — fall back to a plain teardown
                dist.destroy_process_group()
        self.epoch = -1
        return {"aborted": True}

    def form(self, epoch: int, port: int, rank: int, world: int, timeout_s: float = 60.0,
             backend: str = "") -> dict:
        import torch
        import torch.distributed as dist

        if dist.is_initialized():
            self.abort()
        backend = backend or ("nccl" if self.device >= 0 else "gloo")
        if self.device >= 0:
            torch.cuda.set_device(self.device)
        dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                                timeout=timedelta(seconds=timeout_s))
        self.epoch, self.rank, self.world, self.backend = epoch, rank, world, backend
        return {"rank": rank, "world": world, "backend": backend}

    def _local_rows(self, names: list, k: int, src):
        """This rank's k rows: a consistent snapshot of the worker's live consumer rows
        (Worker.snapshot_consumer, ordered on the current stream), zero rows for cameras it no
        longer has. Returns (rows, missing)."""
        import torch

        hub = self.hub
        local = torch.zeros((k, *src.shape[1:]), dtype=src.dtype, device=src.device)
        missing, rows, at = [], [], []
        for j, n in enumerate(names):
            try:
                rows.append(hub.handle(n).cam)
                at.append(j)
            except KeyError:
                missing.append(n)
        if rows:
            snap = hub.snapshot(0, max(rows) + 1)
            local[torch.tensor(at, device=src.device)] = snap.index_select(0, torch.tensor(rows, device=src.device))
        return local, missing

    def gather(self, epoch: int, names: list, k: int, order: list, perm: list, slot=None) -> dict:
        """All-gather ``k`` consumer rows per rank (this rank's ``names``, zero-padded); reorder
        the node batch by ``perm`` into the caller's camera ``order``.

        Every rank of the group enters both collectives whatever went wrong locally (a missing
        camera or a failed snapshot reads as zero rows and sets this rank's error flag), so one bad
        request never leaves the other ranks waiting; a small header collective carries every
        rank's (epoch, error) so all ranks agree on whether the batch is whole. A rank that is not
        in group `epoch` at all (restarted meanwhile) cannot join it: it fails at once, and the
        parent aborts the survivors' communicators before re-forming."""
        import time

        import torch
        import torch.distributed as dist

        if epoch != self.epoch:
            raise RuntimeError(f"gather for group epoch {epoch}, this rank is in {self.epoch}")
        t0 = time.perf_counter()
        src = self.hub.consumer[0]
        err = ""
        try:
            local, missing = self._local_rows(names, k, src)
        except Exception as e:  # noqa: BLE001 — still join the collectives, with zero rows
            err = f"{type(e).__name__}: {e}"
            local = torch.zeros((k, *src.shape[1:]), dtype=src.dtype, device=src.device)
            missing = list(names)
        cdev = src.device if self.backend == "nccl" or not src.is_cuda else torch.device("cpu")
        hdr = torch.tensor([epoch, 1 if err else 0], dtype=torch.int64, device=cdev)
        hdrs = torch.empty((self.world * 2,), dtype=torch.int64, device=cdev)
        dist.all_gather_into_tensor(hdrs, hdr)
        out = torch.empty((self.world * k, *src.shape[1:]), dtype=src.dtype, device=cdev)
        dist.all_gather_into_tensor(out, local.to(cdev))
        batch = out.index_select(0, torch.tensor(perm, dtype=torch.long, device=out.device))
        hs = hdrs.view(self.world, 2).tolist()
        if src.is_cuda:
            torch.cuda.current_stream(src.device).synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        self.gather_ms.append(ms)
        if len(self.gather_ms) > 4096:
            del self.gather_ms[:2048]
        rank_errors = [r for r, (e, f) in enumerate(hs) if f or e != epoch]
        self.gathers += 1
        if not rank_errors:
            self.batch = (batch, list(order))
            if self.hook is not None:
                self.hook(batch, list(order), self.rank)
        res = {"rank": self.rank, "missing": missing, "shape": list(batch.shape), "error": err,
               "rank_errors": rank_errors, "gather_ms": ms}
        if slot is not None:
            nbytes = batch.numel() * batch.element_size()
            slot.ensure(max(nbytes, 1))
            host = torch.frombuffer(slot.view(nbytes), dtype=torch.uint8) if nbytes else None
            if host is not None:
                host.copy_(batch.reshape(-1).view(torch.uint8))  # one D2H into the (page-locked) segment
            res.update(segment=slot.name, nbytes=nbytes)
        return res


def _serve(hub, group: RankGroup, conn, stop: threading.Event) -> None:
    slot = ShmSlot(hub.workers[0])
    try:
        while not stop.is_set():
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
                elif method == "group_form":
                    res = group.form(*args, **kwargs)
                elif method == "group_abort":
                    res = group.abort()
                elif method == "consumer_gather":
                    to_host = kwargs.pop("to_host", False)
                    res = group.gather(*args, slot=slot if to_host else None, **kwargs)
                elif method == "group_info":
                    res = {"epoch": group.epoch, "rank": group.rank, "world": group.world, "gathers": group.gathers,
                           "backend": group.backend, "gather_ms": list(group.gather_ms[-256:])}
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
    finally:
        slot.close()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", type=int, required=True)
    ap.add_argument("--config", required=True, help="Config as JSON")
    ap.add_argument("--owner", type=int, default=0, help="frame-bus owner index of this worker")
    ap.add_argument("--plan-devices", default="",
                    help="devices of every worker process of the node, comma-separated (this one is "
                         "entry --owner): each child takes its part of the node's host data plane")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format=f"%(asctime)s child[{a.device}] %(name)s: %(message)s")
    from ..config import Config, _merge
    from .hub import Hub

    cfg = _merge(Config(), json.loads(a.config))
    from .._native import native

    # this child's host domain: the plan over every worker process of the node (deterministic,
    # so the children agree without talking), the whole process pinned to its CPUs
    plan_devices = [int(x) for x in a.plan_devices.split(",") if x != ""] or [a.device]
    idx = a.owner if a.owner < len(plan_devices) else 0
    explicit = [str(c) for c in (cfg.gpu.host_cpus or [])]
    dom = native.plan_host_domains(plan_devices, explicit)[idx]
    dom["device"] = a.device
    if dom["cpus"]:
        try:
            os.sched_setaffinity(0, dom["cpus"])
        except OSError:
            pass
    hub = Hub(cfg, devices=[a.device], bus_owner=a.owner, host_domains=[dom])
    group = RankGroup(hub, a.device, cfg.gpu.consumer_hook)
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
            threading.Thread(target=_serve, args=(hub, group, conn, stop), daemon=True).start()

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
    remove_segments(os.getpid())  # (serving threads are daemons: they do not unwind)
    try:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
