"""Small helpers: time, RTMP key parsing, structured logging."""
from __future__ import annotations

import json
import logging
import sys
import time
from urllib.parse import urlparse


def now_ms() -> int:
    return int(time.time() * 1000)


def parse_rtmp_key(url: str) -> str:
    """Stream key = last path segment of an rtmp:// URL (server/utils/parser_utils.go:10-25).

    Unlike the reference (which returns "" with no error for non-rtmp schemes, Appendix A.14)
    a non-rtmp URL raises ValueError."""
    u = urlparse(url)
    if u.scheme != "rtmp":
        raise ValueError(f"not an rtmp URL: {url!r}")
    parts = [p for p in u.path.split("/") if p]
    if not parts:
        raise ValueError(f"rtmp URL has no stream key: {url!r}")
    return parts[-1]


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        d = {"ts": round(record.created, 3), "level": record.levelname.lower(),
             "logger": record.name, "msg": record.getMessage()}
        if record.exc_info:
            d["exc"] = self.formatException(record.exc_info)
        return json.dumps(d)


def setup_logging(level: str = "info", json_logs: bool = True) -> logging.Logger:
    root = logging.getLogger("vep")
    if not root.handlers:
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(JsonFormatter() if json_logs else logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
        root.addHandler(h)
    root.setLevel(getattr(logging, level.upper(), logging.INFO))
    return root


log = logging.getLogger("vep")
