"""Camera process manager: registry records + native ingest sessions.

Reference parity: server/services/rtsp_process_manager.go —
  * ``Start`` (:50-150): requires name and rtsp_endpoint; starts the camera's worker (a Docker
    container there, a native IngestSession on a GPU Worker here); with an RTMP endpoint sets
    ``last_query`` + ``proxy_rtmp`` and ``rtmp_stream_status.streaming``; persists the record under
    ``/rtspprocess/<name>``.
  * ``Stop`` (:153-188): stops the session and deletes the record.
  * ``Info`` (:283-335): stored record + live ContainerState + last 100 log lines (base64).
  * ``List`` (:236-280): Info for every record; self-heals records whose session vanished.
  * ``ListStream`` (:191-233): like List, skipping missing sessions, honouring cancellation.
  * ``UpdateProcessInfo`` (:338-356).
New: :meth:`restore` re-spawns every stored camera at boot (the reference relied on Docker's
``restart: always`` for that — SURVEY.md §5 checkpoint/resume row).
"""
from __future__ import annotations

import hashlib
import json
import logging
import re
import threading
from typing import Callable, Optional

from ..engine.hub import CameraExists, CameraNotFound, Hub
from ..models import (DEFAULT_IMAGE_TAG, PREFIX_RTSP_PROCESS, ContainerState, DockerLogs,
                      RTMPStreamStatus, StreamProcess)
from ..utils import now_ms
from .storage import KeyNotFound, Storage

log = logging.getLogger("vep.process")

_NAME = re.compile(r"^[A-Za-z0-9_.\-]+$")


class ProcessError(RuntimeError):
    pass


class ProcessNotFound(ProcessError):
    pass


class ProcessNotFoundDatastore(ProcessError):
    pass


class ProcessManager:
    def __init__(self, storage: Storage, hub: Hub):
        self.storage = storage
        self.hub = hub
        self._lock = threading.RLock()

    # ------------------------------------------------------------------ helpers
    def _get_record(self, name: str) -> StreamProcess:
        try:
            return StreamProcess.from_json(json.loads(self.storage.get(PREFIX_RTSP_PROCESS, name)))
        except KeyNotFound:
            raise ProcessNotFoundDatastore(f"process {name!r} not found in datastore")

    def _put(self, sp: StreamProcess) -> None:
        rec = sp.to_json()
        rec.pop("logs", None)  # logs are volatile (ring in native memory)
        self.storage.put(PREFIX_RTSP_PROCESS, sp.name, json.dumps(rec).encode())

    def _records(self) -> list[StreamProcess]:
        out = []
        for v in self.storage.list(PREFIX_RTSP_PROCESS).values():
            try:
                out.append(StreamProcess.from_json(json.loads(v)))
            except (ValueError, TypeError) as e:
                log.error("corrupt process record skipped: %s", e)
        return out

    # ------------------------------------------------------------------ API
    def start(self, sp: StreamProcess) -> StreamProcess:
        if not sp.rtsp_endpoint:
            raise ProcessError("rtsp endpoint required")
        if not sp.name:
            # the reference computes md5(rtsp) but never uses it (Appendix A.12): we use it
            sp.name = hashlib.md5(sp.rtsp_endpoint.encode()).hexdigest()
        if not _NAME.match(sp.name):
            raise ProcessError(f"invalid process name {sp.name!r}")
        with self._lock:
            if self.hub.has(sp.name):
                raise ProcessError(f"process {sp.name!r} already exists")
            sp.image_tag = sp.image_tag or DEFAULT_IMAGE_TAG
            try:
                h = self.hub.start_camera(sp.name, sp.rtsp_endpoint, sp.rtmp_endpoint or "")
            except (CameraExists, RuntimeError, ValueError) as e:
                raise ProcessError(str(e))
            if sp.rtmp_endpoint:
                self.hub.set_proxy(sp.name, True)
                if sp.rtmp_stream_status is None:
                    sp.rtmp_stream_status = RTMPStreamStatus()
                sp.rtmp_stream_status.streaming = True
            sp.container_id = f"vep-{self.hub.devices[h.worker_index]}-{h.cam}-{sp.name}"
            sp.status = "running"
            sp.created = sp.created or now_ms()
            sp.modified = now_ms()
            st = self.hub.state(sp.name)
            sp.state = ContainerState.from_session(st)
            self._put(sp)
            return sp

    def stop(self, name: str) -> None:
        with self._lock:
            try:
                self.hub.stop_camera(name)
            except CameraNotFound:
                # a stored record without a live session can still be removed
                try:
                    self._get_record(name)
                except ProcessNotFoundDatastore:
                    raise ProcessNotFound(f"process {name!r} not found")
            self.storage.delete(PREFIX_RTSP_PROCESS, name)

    def info(self, name: str, persist: bool = True) -> StreamProcess:
        if not self.hub.has(name):
            raise ProcessNotFound(f"process {name!r} not found")
        sp = self._get_record(name)
        st = self.hub.state(name)
        h = self.hub.handle(name)
        sp.container_id = sp.container_id or f"vep-{self.hub.devices[h.worker_index]}-{h.cam}-{name}"
        sp.state = ContainerState.from_session(st)
        sp.status = sp.state.Status
        out, err = self.hub.logs(name, 100)
        sp.logs = DockerLogs.from_text(out, err)
        sp.modified = now_ms()
        if persist:
            self._put(sp)
        return sp

    def list(self) -> list[StreamProcess]:
        procs, gone = [], []
        for rec in self._records():
            try:
                procs.append(self.info(rec.name))
            except ProcessNotFound:
                gone.append(rec.name)
        for n in gone:  # self-heal (rtsp_process_manager.go:253-278)
            self.storage.delete(PREFIX_RTSP_PROCESS, n)
        return procs

    def list_stream(self, found: Callable[[StreamProcess], None],
                    cancelled: Optional[Callable[[], bool]] = None) -> None:
        for rec in self._records():
            if cancelled and cancelled():
                return
            try:
                found(self.info(rec.name))
            except ProcessNotFound:
                continue

    def update_process_info(self, sp: StreamProcess) -> StreamProcess:
        sp.modified = now_ms()
        self._put(sp)
        return sp

    def restore(self) -> list[str]:
        """Re-spawn a session for every stored record (boot-time resume)."""
        started = []
        for rec in self._records():
            if self.hub.has(rec.name):
                continue
            try:
                self.hub.start_camera(rec.name, rec.rtsp_endpoint, rec.rtmp_endpoint or "")
                if rec.rtmp_stream_status and rec.rtmp_stream_status.streaming and rec.rtmp_endpoint:
                    self.hub.set_proxy(rec.name, True)
                started.append(rec.name)
            except Exception as e:  # keep booting; the record stays for a later retry
                log.error("failed to restore camera %s: %s", rec.name, e)
        return started
