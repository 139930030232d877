"""Camera data parallelism across GPUs and processes.

* :func:`shard_cameras` — deterministic camera -> rank/GPU placement (rendezvous hashing: adding
  a camera or a GPU moves only the cameras that must move).
* :func:`init_distributed` — one process per GPU, ``torch.distributed`` over RCCL ("nccl") on
  ROCm, gloo on CPU hosts; rendezvous on 127.0.0.1 by default.
* :class:`ConsumerBatch` — the batched, letterboxed frame tensor every worker maintains for
  annotation / inference consumers; ``gather()`` assembles the node-wide batch either with one
  RCCL all-gather over xGMI (multi-process) or with peer copies (single process, many GPUs).

The reference scaled by running one Docker container per camera on one host with no GPU and no
collective communication at all (0 NCCL/MPI/Gloo call sites); camera-level data
parallelism is the only parallelism that applies (no model is trained, there is no tensor /
sequence dimension to split — a GOP must be decoded serially).
"""
from __future__ import annotations

import hashlib
import os
from typing import Iterable, Optional

import torch
import torch.distributed as dist


def shard_cameras(names: Iterable[str], world: int, capacity: Optional[int] = None) -> dict[str, int]:
    """Rendezvous (highest-random-weight) hashing with an optional per-rank capacity.

    Deterministic across processes and restarts; with ``capacity`` the overflow spills to the
    next-best rank so load stays within ``capacity`` cameras per rank."""
    names = list(names)
    if world <= 0:
        raise ValueError("world must be positive")
    if capacity is not None and capacity * world < len(names):
        raise ValueError(f"{len(names)} cameras exceed {world} x {capacity} capacity")
    load = [0] * world
    out: dict[str, int] = {}
    for n in sorted(names):
        scores = sorted(range(world), key=lambda r: hashlib.sha1(f"{n}|{r}".encode()).digest(),
                        reverse=True)
        for r in scores:
            if capacity is None or load[r] < capacity:
                out[n] = r
                load[r] += 1
                break
    return out


def balanced_shard(n_cameras: int, world: int) -> list[range]:
    """Contiguous equal split used by the benchmark (weak scaling: fixed cameras per rank)."""
    per, rem = divmod(n_cameras, world)
    out, start = [], 0
    for r in range(world):
        k = per + (1 if r < rem else 0)
        out.append(range(start, start + k))
        start += k
    return out


def init_distributed(backend: Optional[str] = None) -> tuple[int, int, int]:
    """Initialise torch.distributed from the torchrun environment. Returns (rank, world, local)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    return rank, world, local


class ConsumerBatch:
    """``[cams, S, S, 3]`` uint8 letterboxed batch (or NV12 rows) gathered across ranks with one
    RCCL all-gather.

    The native Worker letterboxes every frame it publishes into its *live* rows (``self.live``)
    on its lane streams, whenever that camera's batch runs. A gather therefore never reads the
    live rows directly — a lane's next letterbox kernel could rewrite a row while the collective
    reads it (a row half one frame, half the next). ``gather()`` first takes a snapshot
    (``Worker.snapshot_consumer``: a device copy enqueued on the current stream after every
    letterbox write already enqueued, and before any later one — the lanes wait on its event, the
    host never does) into one of two snapshot buffers, then all-gathers that. The next gather uses
    the other buffer after making the stream wait for the collective that last read it, so a
    gather in flight is never overwritten.

    Gathering the uint8 HWC tensor (1.2 MB per 640x640 camera; NV12 0.6 MB) instead of the
    normalised fp16/bf16 CHW tensor halves the xGMI bytes; consumers normalise after the gather."""

    def __init__(self, worker, cams: int, size: int, device: torch.device, world: int = 1,
                 fmt: str = "bgr"):
        self.worker = worker
        self.cams, self.size, self.world, self.fmt = cams, size, world, fmt
        self.device = device
        shape = (size * size * 3 // 2,) if fmt == "nv12" else (size, size, 3)
        self.live = torch.zeros((cams, *shape), dtype=torch.uint8, device=device)
        worker.set_consumer_buffers(self.live.data_ptr(), 0, cams)
        self.bufs = [torch.zeros((cams, *shape), dtype=torch.uint8, device=device) for _ in range(2)]
        # a process group of any size (a 1-rank RCCL group included) gathers through the
        # collective; without one the local batch is the node batch
        self.collective = world > 1 or (dist.is_available() and dist.is_initialized())
        self.out = [torch.zeros((world * cams, *shape), dtype=torch.uint8, device=device)
                    for _ in range(2)] if self.collective else None
        self.handles = [None, None]
        self.tick = 0

    def prepare(self) -> torch.Tensor:
        """The live rows the worker letterboxes into (kept for callers of the round-2 API; the
        rows are written in place, nothing to switch)."""
        return self.live

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream if self.live.is_cuda else 0

    def gather(self, async_op: bool = True):
        """Snapshot the live rows and all-gather them. Returns (tensor, work)."""
        b = self.tick & 1
        h = self.handles[b]
        if h is not None:  # the collective that last read snapshot b (a stream wait on RCCL)
            h.wait()
            self.handles[b] = None
        snap = self.bufs[b]
        self.worker.snapshot_consumer(snap.data_ptr(), snap.numel(), self.cams, self._stream())
        self.tick += 1
        if not self.collective:
            return snap, None
        w = dist.all_gather_into_tensor(self.out[b], snap, async_op=async_op)
        self.handles[b] = w if async_op else None
        return self.out[b], w

    def drain(self):
        for k in range(2):
            if self.handles[k] is not None:
                self.handles[k].wait()
                self.handles[k] = None


def gather_to_device(batches: list[torch.Tensor], device: torch.device) -> torch.Tensor:
    """Single-process multi-GPU: concatenate per-GPU consumer batches on one device with peer
    copies over xGMI (non_blocking copies on the destination's current stream)."""
    total = sum(b.shape[0] for b in batches)
    out = torch.empty((total, *batches[0].shape[1:]), dtype=batches[0].dtype, device=device)
    off = 0
    for b in batches:
        out[off:off + b.shape[0]].copy_(b, non_blocking=True)
        off += b.shape[0]
    return out
