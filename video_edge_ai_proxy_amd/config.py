"""Hub configuration: the reference's ``/data/chrysalis/conf.yaml`` schema plus a ``gpu:`` section.

Reference parity: server/globals/config.go:23-64 (struct + yaml keys) and the built-in defaults
of server/main.go:51-78 used when no conf.yaml exists. Differences:

* both ``buffer.in_memory`` (parsed by the reference code) and ``buffer.n_memory`` (documented
  in its README) are accepted;
* the REST port stays forced to 8080 unless ``--port`` is given on the CLI (main.go:82);
* ``redis`` is accepted and ignored (frames/control live in HBM / native atomics);
* new ``gpu`` section: devices, ring slots, letterbox consumer batch, placement policy.
"""
from __future__ import annotations

import dataclasses
import os
import re
from dataclasses import dataclass, field
from pathlib import Path

import yaml

DEFAULT_DATA_DIR = "/data/chrysalis"


@dataclass
class RedisConfig:  # accepted for compatibility; unused
    connection: str = "redis:6379"
    database: int = 0
    password: str = ""


@dataclass
class AnnotationConfig:
    endpoint: str = "https://event.chryscloud.com/api/v1/annotate"
    unacked_limit: int = 1000
    poll_duration_ms: int = 300
    max_batch_size: int = 299


@dataclass
class ApiConfig:
    endpoint: str = "https://api.chryscloud.com"


@dataclass
class BufferConfig:
    in_memory: int = 1
    on_disk: bool = False
    on_disk_clean_older_than: str = "30s"
    on_disk_folder: str = ""
    on_disk_schedule: str = "@every 5m"


@dataclass
class GpuConfig:
    devices: list = field(default_factory=list)  # [] = every visible GPU; [-1] = CPU backend
    placement: str = "least_loaded"              # least_loaded | hash
    max_cameras_per_gpu: int = 256
    ring_slots: int = 0                          # 0 = max(2, buffer.in_memory)
    letterbox_size: int = 0                      # >0: maintain a batched consumer tensor
    letterbox_dtype: str = "none"                # none | fp16 | bf16 | fp32
    letterbox_format: str = "bgr"                # bgr (HWC u8) | nv12 (gather-friendly)
    mean: list = field(default_factory=lambda: [0.0, 0.0, 0.0])
    std: list = field(default_factory=lambda: [1.0, 1.0, 1.0])
    idle_cutoff_ms: int = 10000                  # rtsp_to_rtmp.py:144-145
    isolation: str = "thread"                    # thread (one process) | process (a supervised
                                                 # worker process per GPU, engine/isolated.py)
    decoder: str = "native"                      # native (CPU parse + gfx950 reconstruction) |
                                                 # vcn (rocDecode on the video core) | auto
    workers_per_gpu: int = 1                     # process isolation: worker processes per GPU, each
                                                 # owning a camera group (a crash costs 1/k of the
                                                 # GPU's cameras)
    consumer_rate_hz: float = 0.0                # >0: gather the node's consumer batch this often
                                                 # and hand it to consumer_hook (engine/consumer.py)
    host_cpus: list = field(default_factory=list)  # per-worker CPU lists ("0-15", ...) overriding the
                                                 # GPU-local (NUMA) split of the host data plane;
                                                 # [] = detect (hostplan.h); env VEP_HOST_CPUS
                                                 # "0-15;16-31;..." also sets it
    consumer_hook: str = ""                      # process isolation: "module:function" each
                                                 # worker process calls with every gathered
                                                 # node batch (fn(batch, names, rank), on its GPU)


@dataclass
class ServingConfig:
    """Frame serving. ``frontends`` > 0 runs that many serving processes, all bound to
    ``grpc_port`` with SO_REUSEPORT (the kernel spreads client connections over them); they read
    frames from the node's frame bus (shared memory, csrc/vep/bus.h) and forward the other RPCs to
    the main process. -1 = one per GPU; 0 = serve from the main process; -2 (default) = auto: one
    per GPU when the node has more than one GPU; on one GPU, two when the CPU budget has 8 CPUs
    beyond the GPU's 16-CPU decode share (server/app.py auto_frontends), else the main process.

    ``native`` (default): VideoLatestImage is answered by the native HTTP/2 gRPC endpoint
    (csrc/vep/rpcsrv.h: C++, no interpreter lock, straight from the frame bus); the other methods
    go to the grpcio server, which then listens on an internal loopback port. ``native: false``
    serves every method with grpcio (round 4's path)."""
    frontends: int = -2
    threads: int = 256          # handler threads per serving process (each request waits <= 3 x 1 s)
    bus: bool = False           # main-process serving also reads the frame bus (shared DMA per frame)
    native: bool = True
    io_threads: int = 2         # native endpoint: epoll threads per serving process


@dataclass
class Config:
    version: str = "0.1.0"
    title: str = "vep MI355X video edge hub"
    description: str = ""
    mode: str = "release"
    port: int = 8080
    grpc_port: int = 50001
    data_dir: str = DEFAULT_DATA_DIR
    redis: RedisConfig = field(default_factory=RedisConfig)
    annotation: AnnotationConfig = field(default_factory=AnnotationConfig)
    api: ApiConfig = field(default_factory=ApiConfig)
    buffer: BufferConfig = field(default_factory=BufferConfig)
    gpu: GpuConfig = field(default_factory=GpuConfig)
    serving: ServingConfig = field(default_factory=ServingConfig)
    # frame-bus tag of this hub instance (set at start-up when the bus is in use; not a YAML key)
    bus_tag: str = ""

    @property
    def ring_slots(self) -> int:
        return self.gpu.ring_slots or max(2, int(self.buffer.in_memory))


def _merge(dc, data: dict):
    if not isinstance(data, dict):
        return dc
    fields = {f.name: f for f in dataclasses.fields(dc)}
    for k, v in data.items():
        if k == "n_memory" and isinstance(dc, BufferConfig):
            k = "in_memory"
        if k not in fields:
            continue
        cur = getattr(dc, k)
        if dataclasses.is_dataclass(cur):
            _merge(cur, v or {})
        elif k == "grpc_port" and isinstance(v, str):
            setattr(dc, k, int(v.rsplit(":", 1)[-1]) if v else cur)
        else:
            setattr(dc, k, type(cur)(v) if cur is not None and v is not None and not isinstance(cur, list) else v)
    return dc


def load_config(path: str | os.PathLike | None = None, data_dir: str | None = None) -> Config:
    """Load ``<data_dir>/conf.yaml`` (or ``path``); missing file -> reference defaults."""
    cfg = Config()
    if data_dir:
        cfg.data_dir = str(data_dir)
    p = Path(path) if path else Path(cfg.data_dir) / "conf.yaml"
    if p.exists():
        with open(p) as f:
            data = yaml.safe_load(f) or {}
        _merge(cfg, data)
        if data_dir:
            cfg.data_dir = str(data_dir)
    if os.environ.get("VEP_HOST_CPUS"):
        cfg.gpu.host_cpus = [s.strip() for s in os.environ["VEP_HOST_CPUS"].split(";")]
    return cfg


_DUR = re.compile(r"(\d+(?:\.\d+)?)(ns|us|µs|ms|s|m|h)")
_UNIT = {"ns": 1e-9, "us": 1e-6, "µs": 1e-6, "ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}


def parse_duration(s: str) -> float:
    """Go ``time.ParseDuration`` subset -> seconds (e.g. "30s", "5m", "1h30m", "250ms")."""
    s = s.strip()
    if not s:
        raise ValueError("empty duration")
    neg = s.startswith("-")
    s = s.lstrip("+-")
    pos, total = 0, 0.0
    for m in _DUR.finditer(s):
        if m.start() != pos:
            raise ValueError(f"invalid duration {s!r}")
        total += float(m.group(1)) * _UNIT[m.group(2)]
        pos = m.end()
    if pos != len(s):
        raise ValueError(f"invalid duration {s!r}")
    return -total if neg else total
