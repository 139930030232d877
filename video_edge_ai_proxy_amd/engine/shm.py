"""Shared-memory frame transport between the isolated hub's worker processes and the front-end.

A worker process (engine/child.py) owns one :class:`ShmSlot` per front-end connection: the
serialized ``VideoFrame`` of a ``VideoLatestImage`` request (or a gathered consumer batch) is
written straight into it — on a GPU the slot is page-locked (``Worker.register_host``), so the
frame leaves HBM by one DMA into memory the front-end maps — and only ``(name, length)`` travels
over the control connection. The front-end (:class:`ShmReader`) copies the bytes out once (into
the ``bytes`` object grpcio sends) before it hands the connection back, so a slot is never
rewritten while it is being read: one connection, one request in flight, one slot.

Replaces the pickled-socket transport (a 6.2 MB frame was pickled, written to a socket, read and
unpickled: four copies and the parent's GIL held through two of them). The reference moved frames
through Redis (python/read_image.py:121 publishes, server/grpcapi/grpc_api.go:191-197 reads).
"""
from __future__ import annotations

import ctypes
import mmap
import os
import secrets
import tempfile

SHM_DIR = "/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir()
_PAGE = mmap.PAGESIZE


def _path(name: str) -> str:
    return os.path.join(SHM_DIR, name)


def segment_prefix(pid: int) -> str:
    return f"vep-{pid}-"


def remove_segments(pid: int) -> int:
    """Unlink the segments a (dead) worker process left behind. Returns how many."""
    pre, n = segment_prefix(pid), 0
    try:
        names = os.listdir(SHM_DIR)
    except OSError:
        return 0
    for f in names:
        if f.startswith(pre):
            try:
                os.unlink(_path(f))
                n += 1
            except OSError:
                pass
    return n


class ShmSlot:
    """Writer side: a growable shared-memory segment at a stable address until it grows."""

    def __init__(self, worker=None):
        self.worker = worker  # native Worker that page-locks the segment (None: CPU / plain)
        self.name = ""
        self.cap = 0
        self.addr = 0
        self.pinned = False
        self._mm = None
        self._anchor = None

    def ensure(self, n: int) -> None:
        if n <= self.cap:
            return
        self.close()
        size = max(_PAGE, (int(n * 1.125) + _PAGE - 1) // _PAGE * _PAGE)
        name = segment_prefix(os.getpid()) + secrets.token_hex(6)
        fd = os.open(_path(name), os.O_RDWR | os.O_CREAT | os.O_EXCL, 0o600)
        try:
            os.ftruncate(fd, size)
            mm = mmap.mmap(fd, size, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        finally:
            os.close(fd)
        self._mm, self.name, self.cap = mm, name, size
        self._anchor = ctypes.c_char.from_buffer(mm)
        self.addr = ctypes.addressof(self._anchor)
        self.pinned = bool(self.worker is not None and self.worker.register_host(self.addr, size))

    def view(self, n: int) -> memoryview:
        return memoryview(self._mm)[:n]

    def close(self) -> None:
        if self._mm is None:
            return
        if self.pinned:
            self.worker.unregister_host(self.addr)
        self._anchor = None
        self._mm.close()
        try:
            os.unlink(_path(self.name))
        except OSError:
            pass
        self._mm, self.name, self.cap, self.addr, self.pinned = None, "", 0, 0, False


class ShmReader:
    """Reader side of one connection: maps the worker's current segment for that connection."""

    def __init__(self):
        self.name = ""
        self._mm = None

    def _map(self, name: str) -> None:
        if name == self.name:
            return
        self.close()
        fd = os.open(_path(name), os.O_RDONLY)
        try:
            size = os.fstat(fd).st_size
            self._mm = mmap.mmap(fd, size, mmap.MAP_SHARED, mmap.PROT_READ)
        finally:
            os.close(fd)
        self.name = name

    def read(self, name: str, length: int) -> bytes:
        """One copy of the first ``length`` bytes of the segment (into a fresh bytes object)."""
        self._map(name)
        return self._mm[:length]

    def buffer(self, name: str, length: int) -> memoryview:
        self._map(name)
        return memoryview(self._mm)[:length]

    def close(self) -> None:
        if self._mm is not None:
            try:
                self._mm.close()
            except BufferError:  # a caller still holds a view: the mapping goes with it
                pass
        self._mm, self.name = None, ""
