"""Hub: the node-level data-plane owner (one native Worker per local GPU, camera placement,
ingest sessions, archiver, latest-frame access).

Reference parity: replaces the per-camera Docker container + Redis pair
(services/rtsp_process_manager.go:50-150 starts a container per camera; python/ workers publish
frames to Redis). Here every camera is a native IngestSession thread feeding a Camera on the GPU
Worker chosen by the placement policy (camera data parallelism inside one process; across
processes/nodes see ``video_edge_ai_proxy_amd.parallel``).
"""
from __future__ import annotations

import hashlib
import logging
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Optional

from .._native import gpu_count, native
from ..config import Config
from ..utils import now_ms

log = logging.getLogger("vep.hub")

_CHW = {"none": 0, "fp16": 1, "bf16": 2, "fp32": 3}


def new_bus_tag() -> str:
    """A frame-bus tag unique to one hub instance on this node (pid + random suffix)."""
    import secrets

    return f"n{os.getpid()}{secrets.token_hex(3)}"


class CameraNotFound(KeyError):
    pass


class CameraExists(ValueError):
    pass


@dataclass
class CameraHandle:
    name: str
    worker_index: int
    cam: int
    rtsp: str
    rtmp: str = ""
    session: Optional[object] = None
    created_ms: int = field(default_factory=now_ms)


def place_camera(name: str, loads: list[int], policy: str = "least_loaded") -> int:
    """Camera -> worker index. ``hash`` is stable across restarts; ``least_loaded`` balances."""
    if not loads:
        raise RuntimeError("no workers")
    if policy == "hash":
        h = int(hashlib.md5(name.encode()).hexdigest(), 16)
        return h % len(loads)
    return min(range(len(loads)), key=lambda i: (loads[i], i))


class Hub:
    def __init__(self, cfg: Config, devices: Optional[list[int]] = None, bus_owner: int = 0,
                 host_domains: Optional[list[dict]] = None):
        self.cfg = cfg
        if devices is None:
            devices = list(cfg.gpu.devices) if cfg.gpu.devices else list(range(gpu_count()))
        if not devices:
            devices = [-1]  # CPU backend (no GPU visible)
        self.devices = devices
        g = cfg.gpu
        # per-GPU host data plane (hostplan.h): each worker's ingest sockets, parse strands and
        # GPU feeder threads run on its own CPU set (the GPU's NUMA-local CPUs, split among the
        # workers sharing them), sized from the process's CPU budget / workers
        if host_domains is None:
            host_domains = native.plan_host_domains(list(devices), [str(c) for c in (g.host_cpus or [])])
        self.host_domains = host_domains
        self.workers = []
        for d, dom in zip(devices, host_domains):
            w = native.Worker(device=d, letterbox_size=int(g.letterbox_size),
                              chw_dtype=_CHW.get(g.letterbox_dtype, 0), mean=list(g.mean),
                              std=list(g.std), max_cameras=int(g.max_cameras_per_gpu),
                              letterbox_format=1 if g.letterbox_format == "nv12" else 0,
                              decoder=str(getattr(g, "decoder", "native")), host_domain=dom)
            w.start()
            self.workers.append(w)
        # Consumer batch: with letterbox_size > 0 every worker letterboxes each frame it publishes
        # into row <camera slot> of a torch-owned tensor on its own GPU; consumer_batch() assembles
        # the node-wide batch from them.
        self.consumer: list = []
        if int(g.letterbox_size) > 0:
            import torch

            S = int(g.letterbox_size)
            shape = (S * S * 3 // 2,) if g.letterbox_format == "nv12" else (S, S, 3)
            for w, d in zip(self.workers, devices):
                dev = torch.device("cuda", d) if d >= 0 else torch.device("cpu")
                t = torch.zeros((int(g.max_cameras_per_gpu), *shape), dtype=torch.uint8, device=dev)
                w.set_consumer_buffers(t.data_ptr(), 0, int(g.max_cameras_per_gpu))
                self.consumer.append(t)
        self._snaps: list = [None] * len(self.consumer)
        self._cons_lock = threading.Lock()  # one consumer batch at a time (shared snapshot tensors)
        # Frame bus (cfg.bus_tag set: serving processes read frames from shared memory): one owner
        # per worker, index bus_owner + k; the pump DMAs a camera's newest frame on demand.
        self.bus = []
        if cfg.bus_tag:
            for k, w in enumerate(self.workers):
                o = native.BusOwner(cfg.bus_tag, bus_owner + k, int(g.max_cameras_per_gpu))
                o.attach(w)
                self.bus.append(o)
        self.archiver = native.Archiver()
        self.cameras: dict[str, CameraHandle] = {}
        self._lock = threading.RLock()
        log.info("hub up: devices=%s", devices)

    # ------------------------------------------------------------------ lifecycle
    def _loads(self) -> list[int]:
        loads = [0] * len(self.workers)
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
            w = self.workers[wi]
            cam = w.add_camera(name, self.cfg.ring_slots)
            w.set_idle_cutoff_ms(cam, int(self.cfg.gpu.idle_cutoff_ms))
            h = CameraHandle(name, wi, cam, rtsp, rtmp)
            disk = self.archive_dir() if disk_path is None else disk_path
            h.session = native.IngestSession(w, cam, name, rtsp, rtmp or "", disk or "",
                                             self.archiver, timeout_ms, reconnect_delay_ms, 30000)
            h.session.start()
            self.cameras[name] = h
            if self.bus:
                self.bus[wi].add(cam, name)
            log.info("camera %s -> worker %d (device %s) slot %d", name, wi, self.devices[wi], cam)
            return h

    def stop_camera(self, name: str) -> None:
        with self._lock:
            h = self.cameras.pop(name, None)
        if h is None:
            raise CameraNotFound(name)
        if self.bus:
            self.bus[h.worker_index].remove(h.cam)
        h.session.stop()
        self.workers[h.worker_index].remove_camera(h.cam)

    def has(self, name: str) -> bool:
        return name in self.cameras

    def handle(self, name: str) -> CameraHandle:
        h = self.cameras.get(name)
        if h is None:
            raise CameraNotFound(name)
        return h

    def worker_of(self, name: str):
        h = self.handle(name)
        return self.workers[h.worker_index], h.cam

    def consumer_batch(self, device=None, names: Optional[list[str]] = None):
        """Node-wide letterboxed batch of the newest frame of every running camera (or of
        ``names``, in that order): ``(tensor [N, S, S, 3] uint8 (or NV12 rows), names)`` on
        ``device`` (default: the first worker's device). Each GPU's rows are gathered from its own
        consumer tensor and the per-GPU slices are concatenated on the destination with peer
        copies over xGMI (one process, many GPUs; the multi-process form is
        ``parallel.ConsumerBatch``, one RCCL all-gather). Rows of cameras that have not published
        a frame yet are zero."""
        from ..parallel import gather_to_device

        if not self.consumer:
            raise RuntimeError("consumer batch disabled (gpu.letterbox_size is 0)")
        with self._lock:
            order = list(names) if names is not None else sorted(self.cameras)
            hs = [self.handle(n) for n in order]
        if device is None:
            device = self.consumer[0].device
        with self._cons_lock:
            return self._consumer_batch(hs, order, device, gather_to_device)

    def _consumer_batch(self, hs, order, device, gather_to_device):
        import torch

        parts, where = [], []
        for wi, t in enumerate(self.consumer):
            mine = [(k, h.cam) for k, h in enumerate(hs) if h.worker_index == wi]
            if not mine:
                continue
            # a consistent snapshot of the rows in use (the lanes keep letterboxing into the
            # live rows; reading them directly could catch a row mid-rewrite), on the current
            # stream: the row selection below is ordered after it without a host wait
            snap = self.snapshot(wi, max(c for _, c in mine) + 1)
            idx = torch.tensor([c for _, c in mine], dtype=torch.long, device=t.device)
            parts.append(snap.index_select(0, idx))
            where += [k for k, _ in mine]
        if not parts:
            return torch.zeros((0, *self.consumer[0].shape[1:]), dtype=torch.uint8, device=device), []
        cat = gather_to_device(parts, torch.device(device))
        inv = torch.empty(len(where), dtype=torch.long)
        inv[torch.tensor(where, dtype=torch.long)] = torch.arange(len(where))
        return cat.index_select(0, inv.to(cat.device)), order

    def snapshot(self, wi: int, rows: int):
        """Consistent copy of worker wi's consumer rows [0, rows) (Worker.snapshot_consumer) into
        a per-worker snapshot tensor, enqueued on the device's current stream."""
        import torch

        t = self.consumer[wi]
        if self._snaps[wi] is None:
            self._snaps[wi] = torch.empty_like(t)
        snap = self._snaps[wi]
        stream = torch.cuda.current_stream(t.device).cuda_stream if t.is_cuda else 0
        n = snap[:rows].numel()
        self.workers[wi].snapshot_consumer(snap.data_ptr(), n, rows, stream)
        return snap[:rows]

    def shutdown(self) -> None:
        for name in list(self.cameras):
            try:
                self.stop_camera(name)
            except CameraNotFound:
                pass
        for o in self.bus:
            o.stop()
        self.bus = []  # (unlinks the segments now, not at garbage collection)
        for w in self.workers:
            w.stop()
        self.archiver.flush()

    # ------------------------------------------------------------------ state
    def host_plane(self) -> list[dict]:
        """Each worker's host domain: device, NUMA node, CPU list, parse / io threads planned and
        the parse strands its live ingest services run (0 until its first camera)."""
        out = []
        loads = self._loads()
        for i, w in enumerate(self.workers):
            d = dict(w.host_domain)
            d.pop("cpus", None)  # (cpulist says it compactly)
            d["ingest_parse_threads"] = w.ingest_parse_threads
            d["cameras"] = loads[i]
            d["pid"] = os.getpid()
            out.append(d)
        return out

    def state(self, name: str) -> dict:
        h = self.handle(name)
        w = self.workers[h.worker_index]
        st = h.session.state()
        st.update(w.stats(h.cam))
        st["device"] = self.devices[h.worker_index]
        return st

    def logs(self, name: str, last: int = 100) -> tuple[str, str]:
        w, cam = self.worker_of(name)
        return w.logs(cam, False, last), w.logs(cam, True, last)

    # ------------------------------------------------------------------ control
    def touch(self, name: str, keyframe_only: Optional[bool] = None) -> None:
        """A client asked for a frame: refresh last_query (and keyframe-only mode)."""
        w, cam = self.worker_of(name)
        if keyframe_only is not None:
            w.set_keyframe_only(cam, bool(keyframe_only))
        w.set_last_query(cam, now_ms())

    def set_proxy(self, name: str, on: bool) -> None:
        w, cam = self.worker_of(name)
        w.set_proxy(cam, bool(on))
        w.set_last_query(cam, now_ms())

    def proxy(self, name: str) -> bool:
        w, cam = self.worker_of(name)
        return bool(w.proxy(cam))

    # ------------------------------------------------------------------ frames
    def latest_frame_bytes(self, name: str, after: int = 0, wait_ms: int = 0):
        """(seq, serialized VideoFrame, meta) of the newest frame with seq > after, or None."""
        w, cam = self.worker_of(name)
        pub = w.published(cam)
        if pub < after:
            # the caller's cursor belongs to an older ring of this camera (a restarted worker
            # process or a resolution change starts a new ring at 0): start over
            after = 0
        if wait_ms > 0 and pub <= after:
            w.wait_frame(cam, after, wait_ms)
        return w.video_frame(cam, after, name)

    def latest_frame(self, name: str, after: int = 0):
        w, cam = self.worker_of(name)
        return w.read_latest(cam, after)

    def wait_decoded(self, name: str, n: int = 1, timeout_s: float = 10.0) -> bool:
        w, cam = self.worker_of(name)
        deadline = time.time() + timeout_s
        while time.time() < deadline:
            if w.published(cam) >= n:
                return True
            w.wait_frame(cam, w.published(cam), 50)
        return False
