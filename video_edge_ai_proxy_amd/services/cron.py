"""On-disk MP4 buffer cleanup on a cron schedule.

Reference parity: server/cron_jobs.go:27-83 — when ``buffer.on_disk`` is set, a UTC cron job on
``buffer.on_disk_schedule`` walks ``buffer.on_disk_folder`` and deletes ``*.mp4`` files whose
mtime + ``on_disk_clean_older_than`` is in the past. Schedules: robfig/cron syntax subset —
``@every <go-duration>``, ``@hourly``/``@daily``/``@midnight``/``@weekly``/``@monthly``/``@yearly``
and 5-field ``min hour dom month dow`` expressions with ``*``, lists, ranges and ``/step``.
"""
from __future__ import annotations

import datetime as dt
import logging
import os
import threading
import time

from ..config import parse_duration

log = logging.getLogger("vep.cron")

_MACROS = {"@yearly": "0 0 1 1 *", "@annually": "0 0 1 1 *", "@monthly": "0 0 1 * *",
           "@weekly": "0 0 * * 0", "@daily": "0 0 * * *", "@midnight": "0 0 * * *",
           "@hourly": "0 * * * *"}


def _field(spec: str, lo: int, hi: int) -> set[int]:
    out: set[int] = set()
    for part in spec.split(","):
        step = 1
        if "/" in part:
            part, s = part.split("/", 1)
            step = int(s)
        if part in ("*", "?"):
            a, b = lo, hi
        elif "-" in part:
            a, b = map(int, part.split("-", 1))
        else:
            a = b = int(part)
            if step != 1:
                b = hi
        if a < lo or b > hi or a > b:
            raise ValueError(f"cron field {spec!r} out of range [{lo},{hi}]")
        out.update(range(a, b + 1, step))
    return out


class Schedule:
    def __init__(self, spec: str):
        spec = spec.strip()
        self.every: float | None = None
        if spec.startswith("@every"):
            self.every = parse_duration(spec.split(None, 1)[1])
            if self.every <= 0:
                raise ValueError("@every needs a positive duration")
            return
        spec = _MACROS.get(spec, spec)
        parts = spec.split()
        if len(parts) != 5:
            raise ValueError(f"unsupported cron spec {spec!r}")
        self.minute = _field(parts[0], 0, 59)
        self.hour = _field(parts[1], 0, 23)
        self.dom = _field(parts[2], 1, 31)
        self.month = _field(parts[3], 1, 12)
        self.dow = {d % 7 for d in _field(parts[4], 0, 7)}
        self._dom_star = parts[2] in ("*", "?")
        self._dow_star = parts[4] in ("*", "?")

    def next_after(self, t: float) -> float:
        if self.every is not None:
            return t + self.every
        cur = dt.datetime.fromtimestamp(t, tz=dt.timezone.utc).replace(second=0, microsecond=0)
        cur += dt.timedelta(minutes=1)
        for _ in range(366 * 24 * 60):
            dom_ok = cur.day in self.dom
            dow_ok = (cur.isoweekday() % 7) in self.dow
            day_ok = (dom_ok and dow_ok) if (self._dom_star or self._dow_star) else (dom_ok or dow_ok)
            if cur.month in self.month and day_ok and cur.hour in self.hour and cur.minute in self.minute:
                return cur.timestamp()
            cur += dt.timedelta(minutes=1)
        raise ValueError("cron spec never fires")


def cleanup_mp4(folder: str, older_than_s: float, now: float | None = None) -> list[str]:
    """Delete *.mp4 under folder with mtime + older_than < now. Returns deleted paths."""
    now = time.time() if now is None else now
    removed = []
    if not folder or not os.path.isdir(folder):
        return removed
    for root, _dirs, files in os.walk(folder):
        for f in files:
            if not f.endswith(".mp4"):
                continue
            p = os.path.join(root, f)
            try:
                if os.path.getmtime(p) + older_than_s < now:
                    os.remove(p)
                    removed.append(p)
            except OSError as e:
                log.error("failed to remove %s: %s", p, e)
    return removed


class CleanupJob:
    def __init__(self, folder: str, schedule: str, older_than: str):
        self.folder = folder
        self.schedule = Schedule(schedule)
        self.older_than_s = parse_duration(older_than)
        self._stop = threading.Event()
        self._th: threading.Thread | None = None
        self.runs = 0
        self.removed = 0

    def start(self):
        def loop():
            nxt = self.schedule.next_after(time.time())
            while not self._stop.wait(max(0.0, min(1.0, nxt - time.time()))):
                if time.time() >= nxt:
                    self.removed += len(cleanup_mp4(self.folder, self.older_than_s))
                    self.runs += 1
                    nxt = self.schedule.next_after(time.time())

        self._th = threading.Thread(target=loop, daemon=True, name="vep-cron-cleanup")
        self._th.start()
        log.info("started buffer on_disk_cleanup folder=%s", self.folder)
        return self

    def stop(self):
        self._stop.set()
        if self._th:
            self._th.join(timeout=2)


def start_cron_jobs(cfg) -> list[CleanupJob]:
    jobs = []
    if cfg.buffer.on_disk:
        folder = cfg.buffer.on_disk_folder or os.path.join(cfg.data_dir, "archive")
        jobs.append(CleanupJob(folder, cfg.buffer.on_disk_schedule,
                               cfg.buffer.on_disk_clean_older_than).start())
    return jobs
