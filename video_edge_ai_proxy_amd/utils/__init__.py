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


def host_cpu_budget() -> int:
    """CPUs this process may actually run on: the smaller of its affinity mask and the cgroup
    CPU quota (cgroup v2 ``cpu.max`` or v1 ``cfs_quota_us``). ``os.cpu_count()`` reports the
    whole machine, which on a shared GPU node is many times the share a rank gets."""
    import os

    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(p)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                p = int(f.read())
            if q > 0 and p > 0:
                quota = q / p
        except (OSError, ValueError):
            pass
    if quota is not None:
        n = min(n, max(1, int(quota)))
    return max(1, n)


def parse_threads_per_rank(local_world: int, reserve: int = 1) -> int:
    """Host parse threads for one rank: the node's CPU budget split over the ranks that share
    it, minus ``reserve`` for the rank's launcher / lane / gRPC threads, with no constant cap
    (15 on a 16-CPU single-GPU share, the measured optimum: profiles/r2/sweep_threads_s2.txt).
    The GPU ranks' own plan is the native ``plan_host_domains`` (hostplan.h: the same split,
    pinned to each GPU's NUMA-local CPUs); this is the fallback without the extension."""
    share = host_cpu_budget() // max(1, local_world)
    return max(2, share - reserve)
