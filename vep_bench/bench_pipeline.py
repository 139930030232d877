"""BASELINE config 5 side loads for bench.py (``--rtmp --annotate``): RTMP pass-through of every
camera to a loopback RTMP server, and asynchronous annotation upload through the production
path — gRPC ``Annotate`` -> durable queue -> batch consumer -> signed HTTP POST — to a loopback
HTTP endpoint standing in for the cloud API.

Reference parity:
  * pass-through: python/rtsp_to_rtmp.py:127-182 (the proxy flag's rising edge flushes the GOP,
    then every packet is muxed to FLV / RTMP);
  * annotation: server/grpcapi/grpc_annotation_api.go:15-57 (validation, publish to
    ``annotationqueue``), server/batch/annotation_consumer.go:54-121 (batches of <= 299 every
    300 ms, JSON ``{"data": [...]}`` POSTed through the signed EdgeService).
"""
from __future__ import annotations

import json
import os
import tempfile
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer


class _CloudSink:
    """Loopback stand-in for the cloud annotation endpoint: counts signed POSTs."""

    def __init__(self):
        sink = self
        self.posts = 0
        self.annotations = 0
        self.unsigned = 0
        self.lock = threading.Lock()

        class H(BaseHTTPRequestHandler):
            def do_POST(self):  # noqa: N802
                n = int(self.headers.get("Content-Length", "0"))
                body = self.rfile.read(n)
                signed = bool(self.headers.get("X-ChrysEdge-Auth")) and bool(self.headers.get("Content-MD5"))
                try:
                    k = len(json.loads(body).get("data", []))
                except ValueError:
                    k = 0
                with sink.lock:
                    sink.posts += 1
                    sink.annotations += k
                    sink.unsigned += 0 if signed else 1
                self.send_response(200)
                self.send_header("Content-Length", "2")
                self.end_headers()
                self.wfile.write(b"{}")

            def log_message(self, *a):  # quiet
                pass

        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.httpd.server_address[1]}/api/v1/annotations"
        self.th = threading.Thread(target=self.httpd.serve_forever, daemon=True)
        self.th.start()

    def close(self):
        self.httpd.shutdown()
        self.httpd.server_close()


class AnnotationLoad:
    """Annotate RPCs at ``rate`` per camera per second while running; the production consumer
    uploads the queued annotations in batches to the loopback cloud sink."""

    def __init__(self, cameras: list[str], rate: float = 5.0):
        from video_edge_ai_proxy_amd.models import Settings
        from video_edge_ai_proxy_amd.services.annotation import AnnotationConsumer, AnnotationQueue
        from video_edge_ai_proxy_amd.services.edge import EdgeService
        from video_edge_ai_proxy_amd.services.settings import SettingsManager
        from video_edge_ai_proxy_amd.services.storage import Storage
        from video_edge_ai_proxy_amd.server.grpc_server import ImageClient, ImageService, serve

        self.tmp = tempfile.TemporaryDirectory(prefix="vep-annot-")
        storage = Storage(os.path.join(self.tmp.name, "kv.sqlite"))
        self.settings = SettingsManager(storage)
        self.settings.overwrite(Settings(edge_key="bench-edge-key", edge_secret="bench-edge-secret"))
        self.cloud = _CloudSink()
        self.queue = AnnotationQueue(os.path.join(self.tmp.name, "queue.sqlite"))
        self.consumer = AnnotationConsumer(self.settings, EdgeService(timeout_s=5.0), self.cloud.url)
        self.queue.start_consuming(self.consumer, unacked_limit=1000, poll_ms=300, max_batch=299)

        class _PM:  # Annotate needs no process manager / hub
            hub = None

        self.svc = ImageService(_PM(), self.settings, None, self.queue)
        self.server = serve(self.svc, "127.0.0.1:0", workers=8)
        self.client = ImageClient(f"127.0.0.1:{self.server.bound_port}")
        self.cameras = list(cameras)
        self.rate = rate
        self.sent = 0
        self.rpc_errors = 0
        self.error = ""
        self._stop = threading.Event()
        self._th = None

    def start(self):
        from video_edge_ai_proxy_amd.proto import pb

        def run():
            try:
                loop()
            except Exception as e:  # noqa: BLE001 — surfaces in the stats, never silently
                self.error = f"{type(e).__name__}: {e}"

        def loop():
            period = 1.0 / max(1e-3, self.rate * len(self.cameras))
            nxt = time.perf_counter()
            k = 0
            while not self._stop.is_set():
                cam = self.cameras[k % len(self.cameras)]
                req = pb.AnnotateRequest(device_name=cam, type="object_detected", start_timestamp=int(time.time() * 1000),
                                         object_type="person", confidence=0.9, width=640, height=640,
                                         ml_model="bench", object_tracking_id=str(k))
                try:
                    self.client.Annotate(req, timeout=5)
                    self.sent += 1
                except Exception:  # noqa: BLE001 — counted
                    self.rpc_errors += 1
                k += 1
                nxt += period
                time.sleep(max(0.0, nxt - time.perf_counter()))

        self._th = threading.Thread(target=run, daemon=True, name="bench-annotate")
        self._th.start()

    def stop(self, drain_s: float = 3.0) -> dict:
        self._stop.set()
        if self._th is not None:
            self._th.join(timeout=10)
        deadline = time.time() + drain_s  # let the consumer upload what is queued
        while time.time() < deadline and self.consumer.sent < self.sent:
            time.sleep(0.05)
        counts = self.queue.counts()
        out = {"annotate_rpcs": self.sent, "annotate_rpc_errors": self.rpc_errors,
               "annotations_uploaded": self.consumer.sent, "upload_posts": self.cloud.posts,
               "upload_failed_batches": self.consumer.failed_batches, "unsigned_posts": self.cloud.unsigned,
               "queue_left": counts, "error": self.error}
        return out

    def close(self):
        self.queue.close()
        self.client.close()
        self.server.stop(0)
        self.cloud.close()
        self.tmp.cleanup()
