"""Durable annotation queue + batched uploader.

Reference parity:
  * queue: rmq over Redis lists, queue ``annotationqueue``; ``PublishBytes``; batch consumer
    with unacked limit 1000, poll 300 ms, batch <= 299 (grpc_api.go:69-75, main.go:59-64);
  * consumer: proto -> JSON ``{"data": [annotation...]}`` POSTed to ``annotation.endpoint``
    through the signed EdgeService; error -> Reject; a 5 s ticker re-queues rejected messages
    (batch/annotation_consumer.go:22-175).
Fixes: rejected batches are *not* also acked; missing credentials
reject the batch (the reference returned leaving them unacked forever); unacked messages from a
crashed run are returned to ``ready`` at startup.

Storage is SQLite WAL (states: ready / unacked / rejected), so queued annotations survive a
restart like Redis lists with persistence would.
"""
from __future__ import annotations

import logging
import sqlite3
import threading
import time
from pathlib import Path
from typing import Callable

log = logging.getLogger("vep.annotation")

READY, UNACKED, REJECTED = "ready", "unacked", "rejected"


class Batch(list):
    """A consumed batch of (id, payload); ack() or reject() exactly once."""

    def __init__(self, queue: "AnnotationQueue", rows):
        super().__init__(rows)
        self._q = queue
        self.settled = False

    def payloads(self) -> list[bytes]:
        return [p for _, p in self]

    def ack(self) -> None:
        if not self.settled:
            self._q._settle([i for i, _ in self], None)
            self.settled = True

    def reject(self) -> None:
        if not self.settled:
            self._q._settle([i for i, _ in self], REJECTED)
            self.settled = True


class AnnotationQueue:
    def __init__(self, path: str, name: str = "annotationqueue"):
        Path(path).parent.mkdir(parents=True, exist_ok=True)
        self.name = name
        self._lock = threading.RLock()
        self._db = sqlite3.connect(path, check_same_thread=False, isolation_level=None)
        self._db.execute("PRAGMA journal_mode=WAL")
        self._db.execute(
            "CREATE TABLE IF NOT EXISTS q (id INTEGER PRIMARY KEY AUTOINCREMENT, queue TEXT, "
            "payload BLOB, state TEXT, ts INTEGER)")
        self._db.execute("CREATE INDEX IF NOT EXISTS q_state ON q(queue, state, id)")
        with self._lock:  # recover deliveries of a crashed consumer
            self._db.execute("UPDATE q SET state=? WHERE queue=? AND state=?", (READY, name, UNACKED))
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []

    # ---- producer ----
    def publish(self, payload: bytes) -> bool:
        try:
            with self._lock:
                self._db.execute("INSERT INTO q (queue, payload, state, ts) VALUES (?,?,?,?)",
                                 (self.name, bytes(payload), READY, int(time.time() * 1000)))
            return True
        except sqlite3.Error as e:
            log.error("publish failed: %s", e)
            return False

    # ---- consumer side ----
    def counts(self) -> dict[str, int]:
        with self._lock:
            rows = self._db.execute("SELECT state, COUNT(*) FROM q WHERE queue=? GROUP BY state",
                                    (self.name,)).fetchall()
        c = {READY: 0, UNACKED: 0, REJECTED: 0}
        c.update(dict(rows))
        return c

    def take(self, n: int) -> Batch:
        with self._lock:
            rows = self._db.execute(
                "SELECT id, payload FROM q WHERE queue=? AND state=? ORDER BY id LIMIT ?",
                (self.name, READY, n)).fetchall()
            if rows:
                self._db.executemany("UPDATE q SET state=? WHERE id=?", [(UNACKED, r[0]) for r in rows])
        return Batch(self, [(r[0], bytes(r[1])) for r in rows])

    def _settle(self, ids, state):
        with self._lock:
            if state is None:
                self._db.executemany("DELETE FROM q WHERE id=?", [(i,) for i in ids])
            else:
                self._db.executemany("UPDATE q SET state=? WHERE id=?", [(state, i) for i in ids])

    def return_all_rejected(self) -> int:
        with self._lock:
            cur = self._db.execute("UPDATE q SET state=? WHERE queue=? AND state=?",
                                   (READY, self.name, REJECTED))
            return cur.rowcount

    def start_consuming(self, consumer: Callable[[Batch], None], unacked_limit: int = 1000,
                        poll_ms: int = 300, max_batch: int = 299, requeue_every_s: float = 5.0):
        def poll_loop():
            while not self._stop.wait(poll_ms / 1000.0):
                self.poll_once(consumer, unacked_limit, max_batch)

        def requeue_loop():
            while not self._stop.wait(requeue_every_s):
                n = self.return_all_rejected()
                if n:
                    log.info("re-queued %d previously rejected annotations", n)

        for fn in (poll_loop, requeue_loop):
            t = threading.Thread(target=fn, daemon=True, name=f"annotation-{fn.__name__}")
            t.start()
            self._threads.append(t)

    def poll_once(self, consumer, unacked_limit=1000, max_batch=299) -> int:
        room = unacked_limit - self.counts()[UNACKED]
        n = min(max_batch, room)
        if n <= 0:
            return 0
        b = self.take(n)
        if not b:
            return 0
        try:
            consumer(b)
        except Exception as e:  # never lose a batch to a consumer bug
            log.error("annotation consumer failed: %s", e)
            b.reject()
        if not b.settled:
            b.reject()
        return len(b)

    def stop(self):
        self._stop.set()
        for t in self._threads:
            t.join(timeout=2)
        self._threads.clear()

    def close(self):
        self.stop()
        with self._lock:
            self._db.close()


def request_to_annotation(req) -> dict:
    """AnnotateRequest -> cloud JSON (annotation_consumer.go:124-175; ObjectCoordinate unmapped
    in the reference — mapped here as ``object_coordinate``). Key names: parity-unpinned (the
    ``ai`` Go package is not vendored in the reference)."""
    a = {
        "device_name": req.device_name,
        "remote_stream_id": req.remote_stream_id,
        "event_type": req.type,
        "start_timestamp": req.start_timestamp,
        "end_timestamp": req.end_timestamp,
        "object_type": req.object_type,
        "object_id": req.object_id,
        "object_tracking_id": req.object_tracking_id,
        "confidence": req.confidence,
        "object_signature": list(req.object_signature),
        "ml_model": req.ml_model,
        "ml_model_version": req.ml_model_version,
        "width": req.width,
        "height": req.height,
        "is_keyframe": req.is_keyframe,
        "video_type": req.video_type,
        "offset_timestamp": req.offset_timestamp,
        "offset_duration": req.offset_duration,
        "offset_frame_id": req.offset_frame_id,
        "offset_packet_id": req.offset_packet_id,
        "custom_meta_1": req.custom_meta_1,
        "custom_meta_2": req.custom_meta_2,
        "custom_meta_3": req.custom_meta_3,
        "custom_meta_4": req.custom_meta_4,
        "custom_meta_5": req.custom_meta_5,
    }
    if req.HasField("location"):
        a["location"] = {"lat": req.location.lat, "lon": req.location.lon}
    if req.HasField("object_bouding_box"):
        b = req.object_bouding_box
        a["object_bounding_box"] = {"top": b.top, "left": b.left, "width": b.width, "height": b.height}
    if req.HasField("object_coordinate"):
        c = req.object_coordinate
        a["object_coordinate"] = {"x": c.x, "y": c.y, "z": c.z}
    if len(req.mask):
        a["object_mask"] = [{"x": m.x, "y": m.y, "z": m.z} for m in req.mask]
    return a


class AnnotationConsumer:
    """Batch consumer: decode -> JSON -> signed POST; reject on any failure."""

    def __init__(self, settings_manager, edge_service, endpoint: str):
        self.settings = settings_manager
        self.edge = edge_service
        self.endpoint = endpoint
        self.sent = 0
        self.failed_batches = 0

    def __call__(self, batch: Batch) -> None:
        from ..proto import pb

        if not self.endpoint:
            log.error("annotation endpoint is not configured (annotation.endpoint in conf.yaml)")
            batch.reject()
            return
        try:
            key, secret = self.settings.current_edge_key_and_secret()
        except LookupError as e:
            log.error("%s", e)
            batch.reject()
            return
        data = []
        for payload in batch.payloads():
            try:
                req = pb.AnnotateRequest.FromString(payload)
            except Exception as e:  # undecodable: drop (reference drops too)
                log.error("failed to unmarshal annotation: %s", e)
                continue
            data.append(request_to_annotation(req))
        try:
            self.edge.call_api_with_body("POST", self.endpoint, {"data": data}, key, secret)
        except Exception as e:
            log.error("error calling annotation API: %s", e)
            self.failed_batches += 1
            batch.reject()
            return
        self.sent += len(data)
        batch.ack()
