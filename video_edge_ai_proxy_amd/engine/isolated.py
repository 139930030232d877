"""Isolated hub: one supervised worker process per GPU (``gpu.isolation: process``).

The in-process :class:`Hub` runs every camera of the node in one process, so a native fault in
any camera's bitstream parse or a GPU error takes all cameras down. ``ProcessHub`` keeps the same
interface for the servers and services but places each GPU's cameras in a child process
(``engine/child.py``, started as a fresh interpreter, never by exec from a GPU process) and
supervises them: when a child dies, its cameras report ``restarting``, a fresh child is started
for the device and the cameras are re-added with their pass-through state — the reference's
per-camera ``restart: always`` containers (server/services/rtsp_process_manager.go:70-81,
:106-115) at per-GPU granularity, without one process per camera.

The supervising process never initialises the GPU itself (devices are counted through
``torch.cuda.device_count()``, which does not): starting a child from a process that holds a GPU
context is what the children are for, not something the parent may do. The GPU tests therefore
do not drive this class (their pytest process holds a context); tests/test_isolated_hub.py does,
with CPU-backend children.

Control calls travel over authenticated local connections (a small pool per child). Frames do
not: every child publishes its cameras on the node's frame bus (csrc/vep/bus.h, tag
``cfg.bus_tag``), and ``latest_frame_bytes`` / ``touch`` read and mark it directly — the child's
pump DMAs a camera's newest frame into shared memory once for every reader (this process, the
serving processes of ``serving.frontends``), with no call to the child on the frame path.

The children are the ranks of one ``torch.distributed`` group (RCCL over xGMI between GPUs, gloo
for CPU-backend children). The parent forms it on demand — a fresh TCP rendezvous on 127.0.0.1
per epoch, re-formed after any child restart, since a collective group cannot re-admit a rank —
and ``consumer_batch()`` drives one all-gather of the letterboxed consumer rows across all
ranks: every GPU then holds the node-wide batch (for ``gpu.consumer_hook`` consumers in the
children) and one rank DMAs it into shared memory for the caller here.
"""
from __future__ import annotations

import dataclasses
import json
import logging
import os
import queue
import secrets
import select
import subprocess
import sys
import threading
import time
import socket
from concurrent.futures import ThreadPoolExecutor
from multiprocessing.connection import Client
from typing import Optional

from ..config import Config
from .hub import CameraExists, CameraHandle, CameraNotFound, new_bus_tag, place_camera
from .shm import ShmReader, remove_segments

log = logging.getLogger("vep.isolated")

_PKG_PARENT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class WorkerRestarting(RuntimeError):
    """The camera's worker process died and is being restarted."""


_ERRORS = {"CameraNotFound": CameraNotFound, "CameraExists": CameraExists, "KeyError": KeyError,
           "ValueError": ValueError}


class _Child:
    def __init__(self, device: int, cfg_json: str, nconn: int = 4, start_timeout_s: float = 180.0,
                 owner: int = 0, first_start: bool = True, plan_devices: Optional[list[int]] = None):
        self.device = device
        key = secrets.token_bytes(16)
        env = dict(os.environ, VEP_CHILD_KEY=key.hex())
        if not first_start:  # injected faults (VEP_FAULT_CAMERA) hit the first process only
            env.pop("VEP_FAULT_CAMERA", None)
        env["PYTHONPATH"] = _PKG_PARENT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        self.proc = subprocess.Popen(
            [sys.executable, "-m", "video_edge_ai_proxy_amd.engine.child", "--device", str(device),
             "--config", cfg_json, "--owner", str(owner),
             "--plan-devices=" + ",".join(str(d) for d in (plan_devices or [device]))],
            stdin=subprocess.PIPE, stdout=subprocess.PIPE, env=env)
        line = b""
        deadline = time.time() + start_timeout_s
        while not line.endswith(b"\n"):
            if self.proc.poll() is not None:
                raise RuntimeError(f"worker process for device {device} exited during start "
                                   f"(code {self.proc.returncode})")
            r, _, _ = select.select([self.proc.stdout], [], [], 0.5)
            if r:
                ch = os.read(self.proc.stdout.fileno(), 1)
                if not ch:
                    raise RuntimeError(f"worker process for device {device} closed its output")
                line += ch
            if time.time() > deadline:
                self.proc.kill()
                raise RuntimeError(f"worker process for device {device} did not start in time")
        hello = json.loads(line)
        self.pid = int(hello["pid"])
        self.port = int(hello["port"])
        self.free: queue.Queue = queue.Queue()
        for _ in range(nconn):  # (connection, reader of its shared-memory segment)
            self.free.put((Client(("127.0.0.1", self.port), authkey=key), ShmReader()))
        # collectives (group_form / consumer_gather) travel on a connection of their own: a
        # collective stuck on a dead peer holds only it, and the parent can still reach this
        # child over the pool above to abort it (group_abort) before re-forming the group
        self.gconn = (Client(("127.0.0.1", self.port), authkey=key), ShmReader())
        self.glock = threading.Lock()
        threading.Thread(target=self._drain, daemon=True).start()  # stray stdout never blocks it

    def _drain(self) -> None:
        try:
            while self.proc.stdout.read(4096):
                pass
        except Exception:  # noqa: BLE001
            pass

    def alive(self) -> bool:
        return self.proc.poll() is None

    def call(self, method: str, *args, read=None, **kwargs):
        """Run ``method`` in the child. ``read(result, shm_reader)`` post-processes the result
        while this connection (and so its shared-memory segment) is still held."""
        if not self.alive():
            raise WorkerRestarting(f"worker process for device {self.device} is restarting")
        conn, shm = self.free.get(timeout=60)
        try:
            conn.send((method, args, kwargs))
            r = conn.recv()
            if r[0] == "ok" and read is not None:
                r = ("ok", read(r[1], shm))
        except (EOFError, OSError) as e:
            shm.close()
            raise WorkerRestarting(f"worker process for device {self.device} died: {e}") from e
        except BaseException:
            self.free.put((conn, shm))
            raise
        self.free.put((conn, shm))
        if r[0] == "ok":
            return r[1]
        raise _ERRORS.get(r[1], RuntimeError)(r[2])

    def call_group(self, method: str, *args, read=None, **kwargs):
        """A collective call on the dedicated connection. Fails at once (no queueing behind it)
        when this child's previous collective has not returned."""
        if not self.alive():
            raise WorkerRestarting(f"worker process for device {self.device} is restarting")
        if not self.glock.acquire(blocking=False):
            raise RuntimeError(f"worker process for device {self.device}: previous collective still pending")
        conn, shm = self.gconn
        try:
            conn.send((method, args, kwargs))
            r = conn.recv()
            if r[0] == "ok" and read is not None:
                r = ("ok", read(r[1], shm))
        except (EOFError, OSError) as e:
            raise WorkerRestarting(f"worker process for device {self.device} died: {e}") from e
        finally:
            self.glock.release()
        if r[0] == "ok":
            return r[1]
        raise _ERRORS.get(r[1], RuntimeError)(r[2])

    def group_pending(self) -> bool:
        return self.glock.locked()

    def close_pipes(self) -> None:
        while True:  # unmap the shared-memory segments and drop the connections
            try:
                conn, shm = self.free.get_nowait()
            except (queue.Empty, AttributeError):
                break
            shm.close()
            try:
                conn.close()
            except Exception:  # noqa: BLE001
                pass
        try:
            self.gconn[1].close()
            self.gconn[0].close()
        except Exception:  # noqa: BLE001
            pass
        for f in (self.proc.stdin, self.proc.stdout):
            try:
                if f is not None:
                    f.close()
            except Exception:  # noqa: BLE001
                pass

    def close(self, timeout_s: float = 20.0) -> None:
        try:
            self.proc.stdin.close()  # the child shuts its hub down and exits
        except Exception:  # noqa: BLE001
            pass
        try:
            self.proc.wait(timeout=timeout_s)
        except subprocess.TimeoutExpired:
            self.proc.kill()
            self.proc.wait()
        self.close_pipes()
        remove_segments(self.pid)
        _remove_bus_segments(self.pid)


def _remove_bus_segments(pid: int) -> None:
    from .._native import native

    native.bus_remove_segments(pid)


class _WorkerView:
    """Worker statistics of one child (what /metrics and /health read from hub.workers)."""

    def __init__(self, hub: "ProcessHub", index: int):
        self._hub, self._i = hub, index

    def _stats(self) -> dict:
        try:
            return self._hub._child(self._i).call("worker_stats")
        except Exception:  # noqa: BLE001 — a restarting child reports zeros
            return {"batches": 0, "frames": 0, "gpu_ms_total": 0.0, "direct_reads": False,
                    "decoder": self._hub.cfg.gpu.decoder}

    @property
    def batches(self):
        return self._stats()["batches"]

    @property
    def frames(self):
        return self._stats()["frames"]

    @property
    def gpu_ms_total(self):
        return self._stats()["gpu_ms_total"]

    @property
    def direct_reads(self):
        return self._stats()["direct_reads"]

    @property
    def decoder(self):
        return self._stats()["decoder"]


class ProcessHub:
    def __init__(self, cfg: Config, devices: Optional[list[int]] = None, supervise_interval_s: float = 0.5):
        self.cfg = cfg
        if devices is None:
            devices = list(cfg.gpu.devices) if cfg.gpu.devices else _count_gpus()
        # one child per (GPU, camera group): gpu.workers_per_gpu children share each device
        k = max(1, int(getattr(cfg.gpu, "workers_per_gpu", 1)))
        self.devices = [d for d in (devices or [-1]) for _ in range(k)]
        if not cfg.bus_tag:  # the children publish their frames on the node's frame bus
            cfg.bus_tag = new_bus_tag()
        self._cfg_json = json.dumps(dataclasses.asdict(cfg))
        from .._native import native

        self.bus = native.BusReader(cfg.bus_tag)
        with ThreadPoolExecutor(max_workers=len(self.devices)) as ex:  # start them side by side
            futs = [ex.submit(_Child, d, self._cfg_json, owner=i, plan_devices=self.devices)
                    for i, d in enumerate(self.devices)]
        errs = [f.exception() for f in futs]
        started = [f.result() for f, e in zip(futs, errs) if e is None]
        if any(e is not None for e in errs):
            for c in started:
                c.close(timeout_s=5.0)
            raise next(e for e in errs if e is not None)
        self._children = started
        self.workers = [_WorkerView(self, i) for i in range(len(self.devices))]
        self.cameras: dict[str, CameraHandle] = {}
        self._specs: dict[str, dict] = {}
        self._proxy: dict[str, bool] = {}
        self.child_restarts = [0] * len(self.devices)
        self._lock = threading.RLock()
        # the children's torch.distributed group: formed on demand, re-formed after a restart
        self._group_epoch = 0
        self._group_ok = False
        self._group_lock = threading.Lock()
        self._gather_lock = threading.Lock()
        # (2 x ranks: a gather's calls and the next form's can both be outstanding; a call into a
        # child whose collective is still pending fails fast instead of waiting for a thread)
        self._pool = ThreadPoolExecutor(max_workers=max(2, 2 * len(self.devices)), thread_name_prefix="vep-group")
        self.group_timeout_s = 60.0
        self.gather_ms: list[float] = []  # steady-state gathers (max over ranks), no group formation
        self._stop = threading.Event()
        self._sup = threading.Thread(target=self._supervise, args=(supervise_interval_s,), daemon=True,
                                     name="vep-supervisor")
        self._sup.start()
        log.info("isolated hub up: devices=%s pids=%s", self.devices, [c.pid for c in self._children])

    # ------------------------------------------------------------------ supervision
    def _child(self, i: int) -> _Child:
        return self._children[i]

    def _supervise(self, interval: float) -> None:
        while not self._stop.wait(interval):
            for i in range(len(self._children)):
                if self._stop.is_set() or self._children[i].alive():
                    continue
                code = self._children[i].proc.returncode
                log.error("worker process for device %s (pid %d) exited with %s: restarting",
                          self.devices[i], self._children[i].pid, code)
                try:
                    self._restart(i)
                except Exception as e:  # noqa: BLE001 — try again at the next interval
                    log.error("restart of device %s failed: %s", self.devices[i], e)

    def _restart(self, i: int) -> None:
        dead = self._children[i]
        dead.close_pipes()  # the dead child's pipes and shared-memory mappings
        remove_segments(dead.pid)  # and the segments it could not unlink itself
        _remove_bus_segments(dead.pid)
        self._group_ok = False  # the survivors' group lost a rank: re-form before the next gather
        child = _Child(self.devices[i], self._cfg_json, owner=i, first_start=False, plan_devices=self.devices)
        try:
            with self._lock:
                mine = [n for n, h in self.cameras.items() if h.worker_index == i]
                for n in mine:  # re-add before the fresh child takes calls (until then: restarting)
                    spec = self._specs[n]
                    res = child.call("start_camera", *spec["args"])
                    self.cameras[n].cam = res["cam"]
                    if self._proxy.get(n):
                        child.call("set_proxy", n, True)
                self._children[i] = child
                self.child_restarts[i] += 1
        except BaseException:
            # a half-initialised child must not survive (the next supervision round starts
            # another one): it holds a GPU context and some of the cameras
            child.close(timeout_s=5.0)
            raise
        log.info("device %s: fresh worker process pid %d, %d cameras re-added", self.devices[i], child.pid, len(mine))

    # ------------------------------------------------------------------ lifecycle (Hub API)
    def _loads(self) -> list[int]:
        loads = [0] * len(self._children)
        for h in self.cameras.values():
            loads[h.worker_index] += 1
        return loads

    def archive_dir(self) -> str:
        if not self.cfg.buffer.on_disk:
            return ""
        return self.cfg.buffer.on_disk_folder or os.path.join(self.cfg.data_dir, "archive")

    def start_camera(self, name: str, rtsp: str, rtmp: str = "", disk_path: Optional[str] = None,
                     timeout_ms: int = 5000, reconnect_delay_ms: int = 1000) -> CameraHandle:
        with self._lock:
            if name in self.cameras:
                raise CameraExists(f"camera {name!r} already running")
            wi = place_camera(name, self._loads(), self.cfg.gpu.placement)
            args = (name, rtsp, rtmp or "", self.archive_dir() if disk_path is None else disk_path, timeout_ms,
                    reconnect_delay_ms)
            res = self._children[wi].call("start_camera", *args)
            h = CameraHandle(name, wi, res["cam"], rtsp, rtmp)
            self.cameras[name] = h
            self._specs[name] = {"args": args}
            return h

    def stop_camera(self, name: str) -> None:
        with self._lock:
            h = self.cameras.pop(name, None)
            self._specs.pop(name, None)
            self._proxy.pop(name, None)
        if h is None:
            raise CameraNotFound(name)
        try:
            self._children[h.worker_index].call("stop_camera", name)
        except WorkerRestarting:
            pass  # the fresh child will not re-add it

    def has(self, name: str) -> bool:
        return name in self.cameras

    def handle(self, name: str) -> CameraHandle:
        h = self.cameras.get(name)
        if h is None:
            raise CameraNotFound(name)
        return h

    def _call(self, name: str, method: str, *args, **kwargs):
        h = self.handle(name)
        return self._children[h.worker_index].call(method, name, *args, **kwargs)

    # ------------------------------------------------------------------ rank group / consumer batch
    def _on_all(self, method: str, per_child_args: list, **kwargs) -> list:
        """Collective ``method`` on every child concurrently (all ranks must enter at once), each
        on the child's collective connection."""
        futs = [self._pool.submit(self._children[i].call_group, method, *per_child_args[i], **kwargs)
                for i in range(len(self._children))]
        out, err = [], None
        for f in futs:
            try:
                out.append(f.result(timeout=self.group_timeout_s + 30))
            except Exception as e:  # noqa: BLE001 — first error wins, after every rank returned
                out.append(None)
                err = err or e
        if err is not None:
            raise err
        return out

    def form_group(self) -> int:
        """(Re-)form the children's process group with a fresh rendezvous. Returns its epoch."""
        with self._group_lock:
            if not all(c.alive() for c in self._children):
                raise WorkerRestarting("a worker process is restarting")
            # survivors of a failed collective may still be blocked in it: abort their
            # communicators (over the control pool) so the collective connections come free
            for c in self._children:
                if c.group_pending():
                    try:
                        c.call("group_abort")
                    except Exception as e:  # noqa: BLE001
                        log.warning("group abort on device %s failed: %s", c.device, e)
            deadline = time.time() + self.group_timeout_s
            while any(c.group_pending() for c in self._children):
                if time.time() > deadline:
                    raise RuntimeError("a worker's collective did not return after the abort")
                time.sleep(0.05)
            self._group_epoch += 1
            port = _free_port()
            world = len(self._children)
            # RCCL needs one rank per GPU: with several worker processes per GPU (or CPU
            # workers) the group runs on gloo
            gpus = [d for d in self.devices if d >= 0]
            backend = "nccl" if gpus and len(set(gpus)) == len(self.devices) else "gloo"
            try:
                self._on_all("group_form", [(self._group_epoch, port, r, world, self.group_timeout_s, backend)
                                            for r in range(world)])
            except Exception:
                self._group_ok = False
                raise
            self._group_ok = True
            return self._group_epoch

    def consumer_batch(self, device=None, names=None, copy: bool = True, to_host: bool = True):
        """Node-wide letterboxed batch of the newest frame of every running camera (or of
        ``names``, in that order): ``(tensor [N, S, S, 3] uint8 (or NV12 rows), names)``.

        One all-gather across the worker processes (RCCL over xGMI between GPUs) assembles it on
        every rank's GPU — where ``gpu.consumer_hook`` consumers receive it — and the rank of
        ``device`` (default: the first) DMAs it into shared memory, returned here as a CPU tensor
        (``copy=False``: a view of the segment, valid until the next call; this process never
        touches a GPU). Rows of cameras that have not published a frame yet are zero.
        ``to_host=False``: gather on the ranks only (their consumer hooks get the batch), return
        (None, names)."""
        if int(self.cfg.gpu.letterbox_size) <= 0:
            raise RuntimeError("consumer batch disabled (gpu.letterbox_size is 0)")
        with self._lock:
            order = list(names) if names is not None else sorted(self.cameras)
            hs = [self.handle(n) for n in order]
        per = [[] for _ in range(len(self._children))]
        pos = []
        for h in hs:
            pos.append((h.worker_index, len(per[h.worker_index])))
            per[h.worker_index].append(h.name)
        k = max(1, max(len(p) for p in per))
        perm = [r * k + j for r, j in pos]
        dst = (0 if device is None else self.devices.index(device)) if to_host else -1
        with self._gather_lock:  # one collective at a time, in the same order on every rank
            return self._gather(per, k, order, perm, dst, copy)

    def _gather(self, per, k, order, perm, dst, copy):
        import numpy as np
        import torch

        world = len(self._children)
        if not self._group_ok:
            self.form_group()
        epoch = self._group_epoch

        def read(res, shm):
            if "segment" not in res:
                return res
            buf = shm.buffer(res["segment"], res["nbytes"])
            arr = np.frombuffer(buf, dtype=np.uint8)
            t = torch.from_numpy(arr.copy() if copy else arr)
            res["tensor"] = t.view(*res["shape"])
            return res

        futs = []
        for r in range(world):
            kw = dict(to_host=(r == dst))
            futs.append(self._pool.submit(self._children[r].call_group, "consumer_gather", epoch, per[r], k, order,
                                          perm, read=read if r == dst else None, **kw))
        results, err = [], None
        for f in futs:
            try:
                results.append(f.result(timeout=self.group_timeout_s + 30))
            except Exception as e:  # noqa: BLE001
                results.append(None)
                err = err or e
        if err is not None:
            self._group_ok = False  # a failed collective may have left the group unusable
            raise err
        bad = results[0].get("rank_errors") or []
        if bad:  # every rank joined, but some sent zero rows: not a whole batch
            raise RuntimeError(f"consumer gather: ranks {bad} failed locally: "
                               f"{[results[r].get('error') for r in bad if results[r]]}")
        self.gather_ms.append(max(r["gather_ms"] for r in results))
        if len(self.gather_ms) > 4096:
            del self.gather_ms[:2048]
        return (results[dst]["tensor"] if dst >= 0 else None), order

    def shutdown(self) -> None:
        self._stop.set()
        self._sup.join(timeout=5)
        for name in list(self.cameras):
            try:
                self.stop_camera(name)
            except (CameraNotFound, WorkerRestarting):
                pass
        for c in self._children:
            c.close()
        self._pool.shutdown(wait=False)

    # ------------------------------------------------------------------ state / control / frames
    def host_plane(self) -> list[dict]:
        """Each worker process's host domain (Hub.host_plane of every child)."""
        out = []
        for i in range(len(self._children)):
            try:
                out += self._child(i).call("host_plane")
            except Exception:  # noqa: BLE001 — a restarting child
                out.append({"device": self.devices[i], "index": i, "restarting": True})
        return out

    def state(self, name: str) -> dict:
        h = self.handle(name)
        child = self._children[h.worker_index]
        try:
            st = self._call(name, "state")
        except WorkerRestarting as e:
            st = {"status": "restarting", "running": False, "restarting": True, "error": str(e),
                  "health": "starting"}
        st["device"] = self.devices[h.worker_index]
        st["worker_pid"] = child.pid
        st["worker_restarts"] = self.child_restarts[h.worker_index]
        return st

    def logs(self, name: str, last: int = 100) -> tuple[str, str]:
        try:
            return tuple(self._call(name, "logs", last))
        except WorkerRestarting as e:
            return "", str(e)

    def touch(self, name: str, keyframe_only: Optional[bool] = None) -> None:
        self.handle(name)
        if not self.bus.touch(name, -1 if keyframe_only is None else int(bool(keyframe_only))):
            raise WorkerRestarting(f"camera {name!r}: its worker process is restarting")

    def set_proxy(self, name: str, on: bool) -> None:
        self._proxy[name] = bool(on)
        self._call(name, "set_proxy", bool(on))

    def proxy(self, name: str) -> bool:
        return bool(self._call(name, "proxy"))

    def latest_frame_bytes(self, name: str, after: int = 0, wait_ms: int = 0):
        """(seq, serialized VideoFrame, meta) or None, from the frame bus: the child's pump DMAs
        the frame into shared memory, copied out here once (the bytes grpcio sends)."""
        self.handle(name)
        r = self.bus.frame(name, after, wait_ms, -1, -1, False)  # (a read: hub.touch marks demand)
        if r is None:
            return None
        info = self.bus.info(name) or {}
        return r[0], r[1], {"seq": r[0], "shm_pinned": bool(info.get("pinned"))}

    def latest_frame(self, name: str, after: int = 0):
        return self._call(name, "latest_frame", after)

    def wait_decoded(self, name: str, n: int = 1, timeout_s: float = 10.0) -> bool:
        return bool(self._call(name, "wait_decoded", n, timeout_s))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _count_gpus() -> list[int]:
    try:
        import torch

        return list(range(torch.cuda.device_count()))  # (does not initialise the GPU here)
    except Exception:  # noqa: BLE001
        return []
