"""Signed HTTP calls to the cloud API (annotation upload, storage on/off).

Reference parity: server/services/edge_service.go:31-64:
  * body = JSON(payload); ``Content-MD5`` = hex(md5(body))
  * ``X-Chrys-Date`` = unix time in ms (seconds * 1000, as the reference computes it)
  * ``X-ChrysEdge-Auth`` = ``<edge_key>:<HMAC-SHA256(date + md5, edge_secret)>``
  * 2xx -> body; 401/403 -> :class:`Forbidden`; anything else -> :class:`EdgeApiError`.
The HMAC digest is base64-encoded (go-microkit ``ComputeHmac``; its source is not vendored in the
reference, so this encoding is parity-unpinned and covered by a known-vector test of our own).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import json
import time
from typing import Any

import requests


class EdgeApiError(RuntimeError):
    pass


class Forbidden(EdgeApiError):
    pass


def sign(payload: bytes, edge_key: str, edge_secret: str, ts_ms: int | None = None) -> dict[str, str]:
    content_md5 = hashlib.md5(payload).hexdigest()
    ts = str(int(time.time()) * 1000 if ts_ms is None else ts_ms)
    mac = hmac.new(edge_secret.encode(), (ts + content_md5).encode(), hashlib.sha256).digest()
    return {
        "X-ChrysEdge-Auth": f"{edge_key}:{base64.b64encode(mac).decode()}",
        "X-Chrys-Date": ts,
        "Content-MD5": content_md5,
        "Content-Type": "application/json",
    }


class EdgeService:
    def __init__(self, timeout_s: float = 10.0, retries: int = 3):
        self.timeout_s = timeout_s
        self.retries = retries  # resty SetRetryCount(3) in annotation_consumer.go:23
        self.session = requests.Session()

    def call_api_with_body(self, method: str, url: str, body: Any, edge_key: str,
                           edge_secret: str) -> bytes:
        payload = json.dumps(body, separators=(",", ":")).encode()
        last: Exception | None = None
        for attempt in range(self.retries + 1):
            headers = sign(payload, edge_key, edge_secret)
            try:
                r = self.session.request(method, url, data=payload, headers=headers,
                                         timeout=self.timeout_s)
            except requests.RequestException as e:  # network error: retry
                last = e
                time.sleep(min(0.1 * 2 ** attempt, 1.0))
                continue
            if 200 <= r.status_code <= 300:
                return r.content
            if r.status_code in (401, 403):
                raise Forbidden(f"invalid response code from cloud API: {r.status_code}")
            last = EdgeApiError(f"invalid response code from cloud API: {r.status_code}, {r.text[:200]}")
            if r.status_code < 500:
                break
        raise last if isinstance(last, EdgeApiError) else EdgeApiError(str(last))
