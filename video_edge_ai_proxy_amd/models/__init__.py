"""Data models of the control plane (JSON shapes identical to the reference REST API).

Reference parity: server/models/StreamProcess.go:22-43, Settings.go:17-29,
web/src/app/models/StreamProcess.ts:15-27 (Docker ContainerState fields consumed by the portal).
"""
from __future__ import annotations

import base64
import dataclasses
import datetime as _dt
from dataclasses import dataclass, field
from typing import Any, Optional

PREFIX_RTSP_PROCESS = "/rtspprocess/"
PREFIX_SETTINGS = "/settings/"
SETTINGS_DEFAULT_KEY = "default"
DEFAULT_IMAGE_TAG = "vep/native-session:0.1"  # reference: chryscloud/chrysedgeproxy:0.0.2


def iso_ms(ms: int) -> str:
    """Docker-style RFC3339Nano timestamp ("0001-01-01T00:00:00Z" for never)."""
    if not ms:
        return "0001-01-01T00:00:00Z"
    t = _dt.datetime.fromtimestamp(ms / 1000.0, tz=_dt.timezone.utc)
    return t.strftime("%Y-%m-%dT%H:%M:%S.") + f"{t.microsecond:06d}000Z"


@dataclass
class Health:
    Status: str = "starting"
    FailingStreak: int = 0
    Log: list = field(default_factory=list)


@dataclass
class ContainerState:
    """Same field names as docker/api/types.ContainerState (the portal reads them verbatim)."""
    Status: str = "created"
    Running: bool = False
    Paused: bool = False
    Restarting: bool = False
    OOMKilled: bool = False
    Dead: bool = False
    Pid: int = 0
    ExitCode: int = 0
    Error: str = ""
    StartedAt: str = "0001-01-01T00:00:00Z"
    FinishedAt: str = "0001-01-01T00:00:00Z"
    Health: Optional[Health] = None

    @classmethod
    def from_session(cls, s: dict) -> "ContainerState":
        return cls(
            Status=s.get("status", "created"),
            Running=bool(s.get("running")),
            Paused=bool(s.get("paused")),
            Restarting=bool(s.get("restarting")),
            OOMKilled=bool(s.get("oomkilled")),
            Dead=bool(s.get("dead")),
            Pid=int(s.get("pid", 0)),
            ExitCode=int(s.get("exit_code", 0)),
            Error=s.get("error", ""),
            StartedAt=iso_ms(s.get("started_at_ms", 0)),
            FinishedAt=iso_ms(s.get("finished_at_ms", 0)),
            Health=Health(Status=s.get("health", "starting"),
                          FailingStreak=int(s.get("failing_streak", 0))),
        )


@dataclass
class DockerLogs:
    stdout: str = ""  # base64 (the portal atob()s it: process-details.component.ts:58-68)
    stderr: str = ""

    @classmethod
    def from_text(cls, out: str, err: str) -> "DockerLogs":
        return cls(base64.b64encode(out.encode()).decode(), base64.b64encode(err.encode()).decode())


@dataclass
class RTMPStreamStatus:
    streaming: bool = False
    storing: bool = False


@dataclass
class StreamProcess:
    name: str = ""
    image_tag: str = ""
    rtsp_endpoint: str = ""
    rtmp_endpoint: str = ""
    container_id: str = ""
    status: str = ""
    state: Optional[ContainerState] = None
    logs: Optional[DockerLogs] = None
    created: int = 0
    modified: int = 0
    rtmp_stream_status: Optional[RTMPStreamStatus] = None

    def to_json(self) -> dict[str, Any]:
        """omitempty semantics of the Go struct tags (rtsp_endpoint is always present)."""
        d: dict[str, Any] = {}
        for f in dataclasses.fields(self):
            v = getattr(self, f.name)
            if f.name != "rtsp_endpoint" and (v is None or v == "" or v == 0):
                continue
            d[f.name] = dataclasses.asdict(v) if dataclasses.is_dataclass(v) else v
        return d

    @classmethod
    def from_json(cls, d: dict) -> "StreamProcess":
        sp = cls()
        for k in ("name", "image_tag", "rtsp_endpoint", "rtmp_endpoint", "container_id", "status"):
            v = d.get(k)
            if v is not None:
                if not isinstance(v, str):
                    raise ValueError(f"{k} must be a string")
                setattr(sp, k, v)
        for k in ("created", "modified"):
            if d.get(k) is not None:
                setattr(sp, k, int(d[k]))
        if isinstance(d.get("state"), dict):
            st = dict(d["state"])
            h = st.pop("Health", None)
            known = {f.name for f in dataclasses.fields(ContainerState)}
            sp.state = ContainerState(**{k: v for k, v in st.items() if k in known})
            if isinstance(h, dict):
                sp.state.Health = Health(**{k: v for k, v in h.items() if k in ("Status", "FailingStreak", "Log")})
        if isinstance(d.get("logs"), dict):
            sp.logs = DockerLogs(d["logs"].get("stdout", ""), d["logs"].get("stderr", ""))
        if isinstance(d.get("rtmp_stream_status"), dict):
            r = d["rtmp_stream_status"]
            sp.rtmp_stream_status = RTMPStreamStatus(bool(r.get("streaming")), bool(r.get("storing")))
        return sp


@dataclass
class Settings:
    name: str = ""
    edge_key: str = ""
    edge_secret: str = ""
    created: int = 0
    modified: int = 0

    def to_json(self) -> dict[str, Any]:
        d = {"name": self.name}
        for k in ("edge_key", "edge_secret", "created", "modified"):
            v = getattr(self, k)
            if v:
                d[k] = v
        return d

    @classmethod
    def from_json(cls, d: dict) -> "Settings":
        return cls(name=str(d.get("name", "")), edge_key=str(d.get("edge_key", "") or ""),
                   edge_secret=str(d.get("edge_secret", "") or ""),
                   created=int(d.get("created", 0) or 0), modified=int(d.get("modified", 0) or 0))
