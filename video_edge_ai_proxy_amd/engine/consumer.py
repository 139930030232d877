"""Steady-state consumer of the node's letterboxed batch (``gpu.consumer_rate_hz``).

The north star of the MI355X design (BASELINE.json): annotation / inference consumers take the
newest frame of every camera of the node as one batched tensor, assembled on the GPUs. In the
reference the consumer side is the annotation batch consumer fed by a Redis queue
(server/batch/annotation_consumer.go:54-121); here frames never leave HBM for it.

``ConsumerLoop`` drives ``hub.consumer_batch()`` at a fixed rate:
  * in-process hub (one process, many GPUs): each GPU's rows are snapshot (Worker.snapshot_consumer)
    and concatenated on the first GPU; ``gpu.consumer_hook`` is called here with the batch;
  * isolated hub (worker processes): one RCCL all-gather across the worker processes per call;
    every rank hands the node batch to ``gpu.consumer_hook`` on its own GPU (engine/child.py), and
    nothing is copied to this process (``to_host=False``).
The per-call gather time is recorded (steady state: group formation is not part of it) and
exposed through ``stats()`` / ``/metrics``.
"""
from __future__ import annotations

import importlib
import logging
import statistics
import threading
import time
from typing import Callable, Optional

log = logging.getLogger("vep.consumer")


def load_hook(spec: str) -> Optional[Callable]:
    if not spec:
        return None
    mod, _, fn = spec.partition(":")
    return getattr(importlib.import_module(mod), fn)


class ConsumerLoop:
    def __init__(self, hub, rate_hz: float, hook: str = ""):
        self.hub = hub
        self.period = 1.0 / float(rate_hz)
        self.isolated = hasattr(hub, "form_group")
        # the isolated hub's ranks call the hook themselves (cfg.gpu.consumer_hook reaches them)
        self.hook = None if self.isolated else load_hook(hook)
        self.gathers = 0
        self.errors = 0
        self.last_error = ""
        self.ms: list[float] = []
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._run, daemon=True, name="vep-consumer")

    def start(self) -> "ConsumerLoop":
        self._th.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        self._th.join(timeout=30)

    def step(self) -> None:
        if not self.hub.cameras:
            return
        t0 = time.perf_counter()
        if self.isolated:
            self.hub.consumer_batch(to_host=False)
            ms = self.hub.gather_ms[-1] if self.hub.gather_ms else (time.perf_counter() - t0) * 1e3
        else:
            import torch

            batch, names = self.hub.consumer_batch()
            if batch.is_cuda:
                torch.cuda.current_stream(batch.device).synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            if self.hook is not None:
                self.hook(batch, names, 0)
        self.gathers += 1
        self.ms.append(ms)
        if len(self.ms) > 4096:
            del self.ms[:2048]

    def _run(self) -> None:
        nxt = time.perf_counter()
        while not self._stop.is_set():
            try:
                self.step()
            except Exception as e:  # noqa: BLE001 — a restarting worker: try again next period
                self.errors += 1
                self.last_error = f"{type(e).__name__}: {e}"
                if self.errors <= 3 or self.errors % 100 == 0:
                    log.warning("consumer batch failed (%d so far): %s", self.errors, self.last_error)
            nxt += self.period
            delay = nxt - time.perf_counter()
            if delay < 0:
                nxt = time.perf_counter()  # running behind: no burst to catch up
            self._stop.wait(max(0.0, delay))

    def stats(self) -> dict:
        ms = sorted(self.ms[-1024:])
        return {"gathers": self.gathers, "errors": self.errors, "last_error": self.last_error,
                "rate_hz": round(1.0 / self.period, 3),
                "gather_ms_p50": round(statistics.median(ms), 3) if ms else None,
                "gather_ms_p99": round(ms[max(0, int(len(ms) * 0.99) - 1)], 3) if ms else None,
                "gather_ms_mean": round(statistics.fmean(ms), 3) if ms else None}
