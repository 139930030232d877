"""Embedded key-value registry (process + settings records) on SQLite (WAL).

Reference parity: server/services/storage.go (Badger v2 at /data/chrysalis): ``Put/Get/Del``
by (prefix, key) and ``List(prefix)`` returning every value under a prefix (storage.go:37-90).
Keys are stored as ``prefix + key`` exactly like the reference, so ``/rtspprocess/<name>`` and
``/settings/default`` keep their meaning.
"""
from __future__ import annotations

import os
import sqlite3
import threading
from pathlib import Path


class KeyNotFound(KeyError):
    pass


class Storage:
    def __init__(self, path: str | os.PathLike):
        p = Path(path)
        if p.suffix != ".db":
            p.mkdir(parents=True, exist_ok=True)
            p = p / "vep.db"
        else:
            p.parent.mkdir(parents=True, exist_ok=True)
        self.path = str(p)
        self._lock = threading.RLock()
        self._db = sqlite3.connect(self.path, check_same_thread=False, isolation_level=None)
        self._db.execute("PRAGMA journal_mode=WAL")
        self._db.execute("PRAGMA synchronous=NORMAL")
        self._db.execute("CREATE TABLE IF NOT EXISTS kv (k TEXT PRIMARY KEY, v BLOB NOT NULL)")

    def put(self, prefix: str, key: str, value: bytes) -> None:
        with self._lock:
            self._db.execute("INSERT OR REPLACE INTO kv (k, v) VALUES (?, ?)", (prefix + key, bytes(value)))

    def get(self, prefix: str, key: str) -> bytes:
        with self._lock:
            row = self._db.execute("SELECT v FROM kv WHERE k = ?", (prefix + key,)).fetchone()
        if row is None:
            raise KeyNotFound(prefix + key)
        return bytes(row[0])

    def delete(self, prefix: str, key: str) -> None:
        with self._lock:
            self._db.execute("DELETE FROM kv WHERE k = ?", (prefix + key,))

    def list(self, prefix: str) -> dict[str, bytes]:
        """All values whose key starts with prefix (key -> value, copied out)."""
        hi = prefix[:-1] + chr(ord(prefix[-1]) + 1) if prefix else "\U0010ffff"
        with self._lock:
            rows = self._db.execute("SELECT k, v FROM kv WHERE k >= ? AND k < ? ORDER BY k",
                                    (prefix, hi)).fetchall()
        return {k: bytes(v) for k, v in rows}

    def close(self) -> None:
        with self._lock:
            self._db.close()
