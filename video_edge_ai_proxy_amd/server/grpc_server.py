"""gRPC ``chrys.cloud.videostreaming.v1beta1.Image`` service.

Reference parity (server/grpcapi/):
  * ``VideoLatestImage`` (grpc_api.go:133-235): 15 s deadline per stream; per request: store
    keyframe-only mode + ``last_query`` (wakes the lazy decoder), then return the newest frame
    after the caller's cursor, waiting up to 3 x 1 s (XREAD BLOCK 1 s, 3 attempts) and sending an
    empty ``VideoFrame`` if none arrives. The cursor is kept per (client connection, device) —
    the reference kept one handler-wide cursor per device shared by every client (Appendix A.9).
  * ``ListStreams`` (:100-131), ``Annotate`` (grpc_annotation_api.go), ``Proxy``
    (grpc_proxy_api.go), ``Storage`` (grpc_storage_api.go) with the same validation/status codes.
Frames are served zero-copy from the camera's HBM ring: the native layer D2H-copies the slot into
one pre-encoded protobuf buffer; the response serializer is the identity. With a frame bus
(``bus=BusFrames(tag)``: serving processes, isolated workers) the frame comes from the node's
shared-memory bus instead (csrc/vep/bus.h): the owner's pump DMAs it once for every reader.
"""
from __future__ import annotations

import logging
import threading
import time
from collections import OrderedDict
from concurrent import futures
from typing import Optional

import grpc

from ..engine.hub import CameraNotFound
from ..engine.isolated import WorkerRestarting
from ..models import RTMPStreamStatus
from ..proto import SERVICE, pb
from ..services.edge import Forbidden
from ..services.process_manager import ProcessError, ProcessManager
from ..utils import now_ms, parse_rtmp_key

log = logging.getLogger("vep.grpc")

MAX_MSG = 256 * 1024 * 1024  # 4K BGR24 frames are 24.9 MB; grpcio's default is 4 MiB
# Multi-MB frame messages: let the peer send 16 MB HTTP/2 frames, read the socket in large
# chunks and keep a deep flow-control lookahead (measured: the Python client's receive CPU per
# 1080p frame drops from ~14 ms to ~9 ms on loopback).
FRAME_CHANNEL_OPTS = [("grpc.max_receive_message_length", MAX_MSG), ("grpc.max_send_message_length", MAX_MSG),
                      ("grpc.http2.max_frame_size", 16777215), ("grpc.http2.lookahead_bytes", 64 << 20),
                      ("grpc.experimental.tcp_read_chunk_size", 4 << 20),
                      ("grpc.experimental.tcp_min_read_chunk_size", 256 << 10),
                      ("grpc.experimental.tcp_max_read_chunk_size", 8 << 20)]
STREAM_DEADLINE_S = 15.0
WAIT_ATTEMPTS, WAIT_BLOCK_MS = 3, 1000
MAX_CURSORS = 65536  # (client, camera) cursors kept, least recently used evicted first
_EMPTY = b""  # serialized empty VideoFrame


class BusFrames:
    """Frames from the node's frame bus (any camera of any owner process, no GPU context here).
    The newest frame's bytes are kept per camera, so the clients of one camera in this process
    share one copy out of shared memory as well as the owner's one DMA."""

    def __init__(self, tag: str):
        from .._native import native

        self.reader = native.BusReader(tag)
        self._last: dict[str, tuple[int, bytes]] = {}

    def has(self, dev: str) -> bool:
        return self.reader.has(dev)

    def frame(self, dev: str, after: int, wait_ms: int, key_frame_only: bool):
        """(seq, serialized VideoFrame) of the newest frame with seq > after, or None."""
        held = self._last.get(dev)
        r = self.reader.frame(dev, after, wait_ms, 1 if key_frame_only else 0, held[0] if held else -1)
        if r is None:
            return None
        seq, data = r
        if data is None:  # the frame this process already copied out
            return held
        self._last[dev] = (seq, data)
        return seq, data


class ImageService:
    def __init__(self, process_manager: Optional[ProcessManager], settings_manager=None, edge_service=None,
                 annotation_queue=None, api_endpoint: str = "", bus: Optional[BusFrames] = None):
        self.pm = process_manager
        self.hub = process_manager.hub if process_manager is not None else None
        self.bus = bus
        self.settings = settings_manager
        self.edge = edge_service
        self.queue = annotation_queue
        self.api_endpoint = api_endpoint
        # per (client peer, camera) sequence of the last frame sent; least recently used entries
        # are evicted one at a time past MAX_CURSORS (no wholesale reset of every client)
        self._cursors: "OrderedDict[tuple[str, str], int]" = OrderedDict()
        self._cur_lock = threading.Lock()
        self._edge_key: Optional[str] = None
        self.frames_served = 0
        self.latencies_ms: list[float] = []

    # ------------------------------------------------------------------ frames
    def _cursor(self, peer: str, dev: str) -> int:
        with self._cur_lock:
            return self._cursors.get((peer, dev), 0)

    def _set_cursor(self, peer: str, dev: str, seq: int) -> None:
        with self._cur_lock:
            key = (peer, dev)
            self._cursors[key] = seq
            self._cursors.move_to_end(key)
            while len(self._cursors) > MAX_CURSORS:
                self._cursors.popitem(last=False)

    def _served(self, peer: str, dev: str, seq: int, t0: float) -> None:
        self._set_cursor(peer, dev, seq)
        self.frames_served += 1
        self.latencies_ms.append((time.perf_counter() - t0) * 1e3)
        if len(self.latencies_ms) > 10000:
            del self.latencies_ms[:5000]

    def _bus_frame(self, dev: str, key_frame_only: bool, peer: str, t0: float) -> bytes:
        after = self._cursor(peer, dev)
        for _ in range(WAIT_ATTEMPTS):
            r = self.bus.frame(dev, after, WAIT_BLOCK_MS, key_frame_only)  # (marks the demand too)
            if r is not None:
                self._served(peer, dev, r[0], t0)
                return r[1]
            if not self.bus.has(dev):
                break  # unknown camera, or its owner is restarting: an empty frame
            time.sleep(0.016)
        return _EMPTY

    def frame_for(self, dev: str, key_frame_only: bool, peer: str = "") -> bytes:
        t0 = time.perf_counter()
        if self.bus is not None:
            return self._bus_frame(dev, key_frame_only, peer, t0)
        if not self.hub.has(dev):
            return _EMPTY
        try:
            self.hub.touch(dev, key_frame_only)
            after = self._cursor(peer, dev)
            for _ in range(WAIT_ATTEMPTS):
                r = self.hub.latest_frame_bytes(dev, after, WAIT_BLOCK_MS)
                if r is not None:
                    seq, data, _meta = r
                    self._served(peer, dev, seq, t0)
                    return data
                time.sleep(0.016)
        except (CameraNotFound, WorkerRestarting):
            pass  # removed meanwhile / its worker process is being restarted: an empty frame
        return _EMPTY

    def VideoLatestImage(self, request_iterator, context):
        deadline = time.time() + STREAM_DEADLINE_S
        peer = context.peer() or ""
        for req in request_iterator:
            if time.time() > deadline:
                context.abort(grpc.StatusCode.DEADLINE_EXCEEDED, "stream deadline exceeded")
            if not context.is_active():
                return
            yield self.frame_for(req.device_id, req.key_frame_only, peer)

    # ------------------------------------------------------------------ listing
    def ListStreams(self, request, context):
        out = []

        def found(sp):
            st = sp.state
            m = pb.ListStream(name=sp.name, status=sp.status or "", dead=st.Dead, error=st.Error,
                              exit_code=st.ExitCode, oomkilled=st.OOMKilled, paused=st.Paused,
                              pid=st.Pid, restarting=st.Restarting, running=st.Running)
            if st.Health is not None:
                m.failing_streak = st.Health.FailingStreak
                m.health_status = st.Health.Status
            out.append(m)

        self.pm.list_stream(found, lambda: not context.is_active())
        yield from out

    # ------------------------------------------------------------------ annotate
    def Annotate(self, req, context):
        if self._edge_key is None:
            try:
                s = self.settings.get()
            except Exception:
                context.abort(grpc.StatusCode.INVALID_ARGUMENT, "failed to read settings")
            if not s.edge_key:
                context.abort(grpc.StatusCode.INVALID_ARGUMENT,
                              "Can't find edge key in settings. required to use annotations.")
            self._edge_key = s.edge_key
        if not req.device_name or not req.type or req.start_timestamp < 0:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, "device_name and type (event type) required")
        week = 7 * 24 * 3600 * 1000
        now = now_ms()
        if req.start_timestamp < now - week or req.start_timestamp > now + week:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT,
                          "start_timestamp must not be older than 7 days and not more than 7 days in the future")
        if self.queue is None or not self.queue.publish(req.SerializeToString()):
            context.abort(grpc.StatusCode.INTERNAL, "failed to publish to msg queue")
        return pb.AnnotateResponse(device_name=req.device_name, start_timestamp=req.start_timestamp,
                                   type=req.type)

    # ------------------------------------------------------------------ proxy / storage
    def Proxy(self, req, context):
        dev = req.device_id
        if not dev:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, "device id required")
        try:
            info = self.pm.info(dev)
        except ProcessError as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        if not info.rtmp_endpoint and req.passthrough:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT,
                          f"device {dev} doesn't have an associated RTMP stream")
        self.hub.set_proxy(dev, req.passthrough)
        if info.rtmp_stream_status is None:
            info.rtmp_stream_status = RTMPStreamStatus()
        info.rtmp_stream_status.streaming = req.passthrough
        self.pm.update_process_info(info)
        return pb.ProxyResponse(device_id=dev, passthrough=info.rtmp_stream_status.streaming)

    def Storage(self, req, context):
        dev = req.device_id
        if not dev:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, "device id required")
        try:
            info = self.pm.info(dev)
        except ProcessError as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        if not info.rtmp_endpoint:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"device {dev} doesn't have an associated RTMP stream")
        try:
            key = parse_rtmp_key(info.rtmp_endpoint)
            if not self.api_endpoint:
                raise RuntimeError("missing cloud API endpoint in settings")
            ek, es = self.settings.current_edge_key_and_secret()
            self.edge.call_api_with_body("PUT", f"{self.api_endpoint}/api/v1/edge/storage/{key}",
                                         {"enable": bool(req.start)}, ek, es)
        except Forbidden:
            context.abort(grpc.StatusCode.PERMISSION_DENIED, "permission denied")
        except Exception as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT,
                          f"cannot enable or disable storage on cloud: {e}")
        if info.rtmp_stream_status is None:
            info.rtmp_stream_status = RTMPStreamStatus()
        info.rtmp_stream_status.storing = req.start
        self.pm.update_process_info(info)
        return pb.StorageResponse(device_id=dev, start=req.start)


def _identity(b: bytes) -> bytes:
    return b


def make_handler(svc: ImageService) -> grpc.GenericRpcHandler:
    handlers = {
        "VideoLatestImage": grpc.stream_stream_rpc_method_handler(
            svc.VideoLatestImage, request_deserializer=pb.VideoFrameRequest.FromString,
            response_serializer=_identity),
        "ListStreams": grpc.unary_stream_rpc_method_handler(
            svc.ListStreams, request_deserializer=pb.ListStreamRequest.FromString,
            response_serializer=pb.ListStream.SerializeToString),
        "Annotate": grpc.unary_unary_rpc_method_handler(
            svc.Annotate, request_deserializer=pb.AnnotateRequest.FromString,
            response_serializer=pb.AnnotateResponse.SerializeToString),
        "Proxy": grpc.unary_unary_rpc_method_handler(
            svc.Proxy, request_deserializer=pb.ProxyRequest.FromString,
            response_serializer=pb.ProxyResponse.SerializeToString),
        "Storage": grpc.unary_unary_rpc_method_handler(
            svc.Storage, request_deserializer=pb.StorageRequest.FromString,
            response_serializer=pb.StorageResponse.SerializeToString),
    }
    return grpc.method_handlers_generic_handler(SERVICE.full_name, handlers)


def serve(svc: ImageService, address: str = "0.0.0.0:50001", workers: int = 64,
          reuseport: bool = False, handler: Optional[grpc.GenericRpcHandler] = None,
          tune_malloc: bool = False) -> grpc.Server:
    """Start the Image service on ``address``. ``workers`` handler threads (a VideoLatestImage
    request holds one for up to 3 x 1 s of waiting). ``tune_malloc`` keeps frame-sized buffers in
    the heap (native.tune_malloc_for_frames): worth it in a process that does nothing but serve
    frames (the serving processes); off by default since it changes glibc's policy process-wide."""
    if tune_malloc:
        from .._native import native

        native.tune_malloc_for_frames(64)
    opts = FRAME_CHANNEL_OPTS + [("grpc.so_reuseport", 1 if reuseport else 0)]
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=workers), options=opts,
                         maximum_concurrent_rpcs=None)
    server.add_generic_rpc_handlers((handler or make_handler(svc),))
    port = server.add_insecure_port(address)
    if port == 0:
        raise RuntimeError(f"cannot bind gRPC server to {address}")
    server.start()
    server.bound_port = port  # type: ignore[attr-defined]
    return server


class ImageClient:
    """Client stub (the reference used protoc-generated ``ImageStub``)."""

    def __init__(self, target: str, own_connection: bool = False):
        # own_connection: not grpc-core's process-wide subchannel pool (channels to one target
        # share a TCP connection by default; the server keeps its cursors per connection)
        opts = FRAME_CHANNEL_OPTS + ([("grpc.use_local_subchannel_pool", 1)] if own_connection else [])
        self.channel = grpc.insecure_channel(target, options=opts)
        p = SERVICE.path
        self.VideoLatestImage = self.channel.stream_stream(
            p("VideoLatestImage"), request_serializer=pb.VideoFrameRequest.SerializeToString,
            response_deserializer=pb.VideoFrame.FromString)
        self.ListStreams = self.channel.unary_stream(
            p("ListStreams"), request_serializer=pb.ListStreamRequest.SerializeToString,
            response_deserializer=pb.ListStream.FromString)
        self.Annotate = self.channel.unary_unary(
            p("Annotate"), request_serializer=pb.AnnotateRequest.SerializeToString,
            response_deserializer=pb.AnnotateResponse.FromString)
        self.Proxy = self.channel.unary_unary(
            p("Proxy"), request_serializer=pb.ProxyRequest.SerializeToString,
            response_deserializer=pb.ProxyResponse.FromString)
        self.Storage = self.channel.unary_unary(
            p("Storage"), request_serializer=pb.StorageRequest.SerializeToString,
            response_deserializer=pb.StorageResponse.FromString)

    def latest_frame(self, device_id: str, key_frame_only: bool = False, timeout: float = 20.0):
        it = self.VideoLatestImage(iter([pb.VideoFrameRequest(device_id=device_id,
                                                              key_frame_only=key_frame_only)]),
                                   timeout=timeout)
        for vf in it:
            return vf
        return None

    def close(self):
        self.channel.close()
