"""Hub daemon bootstrap (``vep serve``).

Reference parity: server/main.go:44-164 — load conf.yaml or defaults, open the registry store,
build services, start cron jobs, REST on :8080 and gRPC on :50001, graceful shutdown on SIGINT.
Differences: no Redis (frames/control in native memory), stored cameras are re-spawned at boot.
"""
from __future__ import annotations

import logging
import os
import signal
import threading
from dataclasses import dataclass
from typing import Optional

from ..config import Config, load_config
from ..engine.hub import Hub, new_bus_tag
from ..services.annotation import AnnotationConsumer, AnnotationQueue
from ..services.cron import start_cron_jobs
from ..services.edge import EdgeService
from ..services.process_manager import ProcessManager
from ..services.settings import SettingsManager
from ..services.storage import Storage
from ..utils import host_cpu_budget
from .grpc_server import BusFrames, ImageService, serve
from .metrics import Metrics
from .rest import create_app

log = logging.getLogger("vep.app")


@dataclass
class HubApp:
    cfg: Config
    storage: Storage
    hub: Hub
    pm: ProcessManager
    settings: SettingsManager
    edge: EdgeService
    queue: AnnotationQueue
    consumer: AnnotationConsumer
    image: ImageService
    grpc_server: object
    rest_server: Optional[object]
    rest_thread: Optional[threading.Thread]
    cron: list
    metrics: Metrics
    frontends: Optional[object] = None  # server.frontend.FrontendPool (serving.frontends > 0)
    public_grpc_port: int = 0
    native_server: Optional[object] = None  # native.RpcServer (serving.native, main-process serving)
    consumer_loop: Optional[object] = None  # engine.consumer.ConsumerLoop (gpu.consumer_rate_hz > 0)

    @property
    def grpc_port(self) -> int:
        return self.public_grpc_port or self.grpc_server.bound_port

    @property
    def rest_port(self) -> int:
        return self._rest_port

    def stop(self):
        log.info("shutting down")
        if self.frontends is not None:
            self.frontends.close()
        if self.native_server is not None:
            self.native_server.stop()
        try:
            self.grpc_server.stop(grace=2).wait(5)
        except Exception:
            pass
        if self.rest_server is not None:
            self.rest_server.should_exit = True
            if self.rest_thread:
                self.rest_thread.join(timeout=5)
        for j in self.cron:
            j.stop()
        if self.consumer_loop is not None:
            self.consumer_loop.stop()
        self.queue.stop()
        self.hub.shutdown()
        self.storage.close()


# One GPU saturates its host parse on ~16 CPUs (the headline's host domain); CPUs beyond that
# are spare, and 8 of them pay for two serving processes (their writev / TCP work then runs off the
# decoding process's CPUs; docs/ROUND6.md).
SERVING_SPARE_CPUS = 8
DECODE_CPUS_PER_GPU = 16


def auto_frontends(ngpu: int, budget: int) -> int:
    """serving.frontends -2: one serving process per GPU on a multi-GPU node; on one GPU, two when
    the CPU budget leaves SERVING_SPARE_CPUS beyond the GPU's decode share, else none (the main
    process serves)."""
    if ngpu > 1:
        return ngpu
    return 2 if budget - DECODE_CPUS_PER_GPU >= SERVING_SPARE_CPUS else 0


def build_app(cfg: Config, host: str = "0.0.0.0", rest_port: Optional[int] = None,
              grpc_port: Optional[int] = None, devices=None, start_rest: bool = True,
              restore: bool = True) -> HubApp:
    os.makedirs(cfg.data_dir, exist_ok=True)
    gport = cfg.grpc_port if grpc_port is None else grpc_port
    # Serving processes (serving.frontends): started first — this process may initialise a GPU
    # below, and a process holding a GPU context must not start programs. They read frames from
    # the frame bus, so every decoding process publishes one (cfg.bus_tag); the isolated hub's
    # workers always do (the main process then serves from the bus too, without calling them).
    nfront = int(cfg.serving.frontends)
    ngpu = len(devices if devices is not None else (cfg.gpu.devices or _gpu_count()))
    if nfront == -2:  # auto: serving processes on multi-GPU nodes, and on one GPU with CPUs to spare
        nfront = auto_frontends(ngpu, host_cpu_budget())
    elif nfront < 0:
        nfront = max(1, ngpu)
    # main-process serving through the native endpoint: it reads the frame bus
    native_main = nfront == 0 and bool(cfg.serving.native)
    use_bus = nfront > 0 or cfg.gpu.isolation == "process" or cfg.serving.bus or native_main
    if use_bus and not cfg.bus_tag:
        cfg.bus_tag = new_bus_tag()
    frontends, control = None, None
    if nfront > 0:
        from .frontend import FrontendPool

        if not gport:
            gport = _free_port(host)
        control = f"127.0.0.1:{_free_port('127.0.0.1')}"
        frontends = FrontendPool(nfront, cfg.bus_tag, f"{host}:{gport}", control, int(cfg.serving.threads),
                                 stats_path=os.path.join(cfg.data_dir, f"serving-{cfg.bus_tag}"),
                                 native=bool(cfg.serving.native), io_threads=int(cfg.serving.io_threads))
    elif native_main:
        control = f"127.0.0.1:{_free_port('127.0.0.1')}"  # grpcio: the non-frame methods
    storage = Storage(os.path.join(cfg.data_dir, "registry.db"))
    if cfg.gpu.isolation == "process":
        from ..engine.isolated import ProcessHub

        hub = ProcessHub(cfg, devices)
    else:
        hub = Hub(cfg, devices)
    pm = ProcessManager(storage, hub)
    settings = SettingsManager(storage)
    edge = EdgeService()
    queue = AnnotationQueue(os.path.join(cfg.data_dir, "annotations.db"))
    consumer = AnnotationConsumer(settings, edge, cfg.annotation.endpoint)
    queue.start_consuming(consumer, cfg.annotation.unacked_limit, cfg.annotation.poll_duration_ms,
                          cfg.annotation.max_batch_size)
    image = ImageService(pm, settings, edge, queue, cfg.api.endpoint, bus=BusFrames(cfg.bus_tag) if use_bus else None)
    # with serving processes / the native endpoint this server is their control port (non-frame
    # RPCs); else public
    gsrv = serve(image, control if control is not None else f"{host}:{gport}", workers=int(cfg.serving.threads))
    native_server = None
    if native_main:
        from .._native import native as _n
        from .frontend import NativeForwarder

        fwd = NativeForwarder(control)
        native_server = _n.RpcServer(host if host else "0.0.0.0", int(gport or 0), cfg.bus_tag,
                                     io_threads=int(cfg.serving.io_threads), wait_threads=int(cfg.serving.threads),
                                     handler=fwd, reuseport=False)  # (holds fwd: the control channel)
    cron = start_cron_jobs(cfg)
    metrics = Metrics(hub, image, frontends)
    rest_server = rest_thread = None
    rport = cfg.port if rest_port is None else rest_port
    if start_rest:
        import socket

        import uvicorn

        app = create_app(pm, settings, metrics)
        sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        sock.bind((host, rport))
        rport = sock.getsockname()[1]
        ucfg = uvicorn.Config(app, log_level="warning", lifespan="off")
        rest_server = uvicorn.Server(ucfg)
        rest_thread = threading.Thread(target=rest_server.run, kwargs={"sockets": [sock]},
                                       daemon=True, name="vep-rest")
        rest_thread.start()
    public = gport if frontends is not None else (native_server.port if native_server is not None else 0)
    happ = HubApp(cfg, storage, hub, pm, settings, edge, queue, consumer, image, gsrv,
                  rest_server, rest_thread, cron, metrics, frontends, public, native_server)
    metrics.native = native_server
    happ._rest_port = rport  # type: ignore[attr-defined]
    if float(cfg.gpu.consumer_rate_hz) > 0 and int(cfg.gpu.letterbox_size) > 0:
        from ..engine.consumer import ConsumerLoop

        happ.consumer_loop = ConsumerLoop(hub, float(cfg.gpu.consumer_rate_hz), cfg.gpu.consumer_hook).start()
        metrics.consumer = happ.consumer_loop
    if restore:
        restored = pm.restore()
        if restored:
            log.info("restored %d cameras from the registry", len(restored))
    log.info("vep ready: REST :%s gRPC :%s devices=%s serving processes=%d native=%s", rport, happ.grpc_port,
             hub.devices, nfront, bool(cfg.serving.native))
    return happ


def _free_port(host: str) -> int:
    import socket

    with socket.socket() as s:
        s.bind((host if host not in ("", "0.0.0.0") else "127.0.0.1", 0))
        return s.getsockname()[1]


def _gpu_count() -> list:
    try:
        import torch

        return list(range(torch.cuda.device_count()))  # (does not initialise the GPU)
    except Exception:  # noqa: BLE001
        return []


def run_forever(cfg: Config, **kw) -> None:
    app = build_app(cfg, **kw)
    done = threading.Event()

    def on_sig(*_):
        done.set()

    signal.signal(signal.SIGINT, on_sig)
    signal.signal(signal.SIGTERM, on_sig)
    done.wait()
    app.stop()
