"""Edge key/secret settings record.

Reference parity: server/services/settings_manager.go:28-122 — one record ``/settings/default``;
``Get`` returns a default-named empty record when none is stored; ``Overwrite`` replaces key and
secret and stamps created/modified (ms). The cached key/secret are read under the lock here (the
reference read them unlocked, SURVEY.md §5 race-detection row).
"""
from __future__ import annotations

import json
import threading

from ..models import PREFIX_SETTINGS, SETTINGS_DEFAULT_KEY, Settings
from ..utils import now_ms
from .storage import KeyNotFound, Storage


class MissingEdgeCredentials(LookupError):
    pass


class SettingsManager:
    def __init__(self, storage: Storage):
        self.storage = storage
        self._lock = threading.RLock()
        self._key = ""
        self._secret = ""

    def _default(self) -> Settings:
        try:
            s = Settings.from_json(json.loads(self.storage.get(PREFIX_SETTINGS, SETTINGS_DEFAULT_KEY)))
        except KeyNotFound:
            s = Settings(name=SETTINGS_DEFAULT_KEY)
        with self._lock:
            if s.edge_key:
                self._key = s.edge_key
            if s.edge_secret:
                self._secret = s.edge_secret
        return s

    def get(self) -> Settings:
        return self._default()

    def overwrite(self, new: Settings) -> Settings:
        s = self._default()
        s.name = s.name or SETTINGS_DEFAULT_KEY
        s.edge_key = new.edge_key
        s.edge_secret = new.edge_secret
        now = now_ms()
        if s.created <= 0:
            s.created = now
        s.modified = now
        with self._lock:
            self._key, self._secret = s.edge_key, s.edge_secret
            self.storage.put(PREFIX_SETTINGS, s.name, json.dumps(s.to_json()).encode())
        return s

    def current_edge_key_and_secret(self) -> tuple[str, str]:
        with self._lock:
            if self._key and self._secret:
                return self._key, self._secret
        self._default()
        with self._lock:
            if not (self._key and self._secret):
                raise MissingEdgeCredentials(
                    "edge key and secret are not configured (POST /api/v1/settings)")
            return self._key, self._secret
