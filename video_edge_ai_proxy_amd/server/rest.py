"""REST API (``/api/v1``), static portal and Prometheus metrics.

Reference parity: server/router/config_routes.go:25-50 (CORS ``*`` + six routes),
server/api/rtsp_process.go:39-106, api/settings.go:38-62, api/error.go:20-31:

  POST   /api/v1/process          400 bad JSON / missing rtsp_endpoint, 409 start failure, 200
  DELETE /api/v1/process/{name}   400 / 409 / 200
  GET    /api/v1/process/{name}   400 / 200 + StreamProcess JSON
  GET    /api/v1/processlist      500 / 200 + [StreamProcess]
  GET    /api/v1/settings         500 / 200 + Settings
  POST   /api/v1/settings         400 / 500 / 202
Errors are ``{"code": int, "message": str}``. New: ``/metrics`` (Prometheus), ``/healthz``,
``GET /api/v1/process/{name}/frame`` (latest frame as PPM, for the portal preview), and the
portal itself at ``/`` (replaces the Angular build, which needs a node toolchain).
"""
from __future__ import annotations

import json
import logging
from pathlib import Path

from fastapi import FastAPI, Request
from fastapi.middleware.cors import CORSMiddleware
from fastapi.responses import HTMLResponse, JSONResponse, Response

from ..models import Settings, StreamProcess
from ..services.process_manager import ProcessError, ProcessManager
from ..services.settings import SettingsManager

log = logging.getLogger("vep.rest")
PORTAL = Path(__file__).with_name("portal.html")


def err(code: int, message: str) -> JSONResponse:
    return JSONResponse(status_code=code, content={"code": code, "message": message})


def create_app(pm: ProcessManager, sm: SettingsManager, metrics=None) -> FastAPI:
    app = FastAPI(title="vep", docs_url=None, redoc_url=None, openapi_url=None)
    app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_methods=["*"], allow_headers=["*"],
                       allow_credentials=False)

    async def body_json(request: Request):
        raw = await request.body()
        try:
            data = json.loads(raw or b"null")
        except ValueError as e:
            raise ValueError(f"invalid JSON: {e}")
        if not isinstance(data, dict):
            raise ValueError("JSON object expected")
        return data

    @app.post("/api/v1/process")
    async def start_process(request: Request):
        try:
            sp = StreamProcess.from_json(await body_json(request))
        except ValueError as e:
            return err(400, str(e))
        if not sp.rtsp_endpoint:
            return err(400, "RTSP endpoint required")
        from ..models import RTMPStreamStatus

        sp.rtmp_stream_status = RTMPStreamStatus(streaming=True, storing=False)
        try:
            pm.start(sp)
        except ProcessError as e:
            return err(409, str(e))
        return Response(status_code=200)

    @app.delete("/api/v1/process/{name}")
    def stop_process(name: str):
        if not name:
            return err(400, "required device_id")
        try:
            pm.stop(name)
        except ProcessError as e:
            return err(409, str(e))
        return Response(status_code=200)

    @app.get("/api/v1/process/{name}")
    def info(name: str):
        try:
            return pm.info(name).to_json()
        except ProcessError as e:
            return err(400, str(e))

    @app.get("/api/v1/process/{name}/frame")
    def frame(name: str):
        try:
            pm.hub.touch(name)
            r = pm.hub.latest_frame(name, 0)
        except KeyError:
            return err(404, f"process {name!r} not found")
        if r is None:
            return err(404, "no frame decoded yet")
        meta, img = r
        h, w = img.shape[:2]
        ppm = f"P6 {w} {h} 255\n".encode() + img[:, :, ::-1].tobytes()  # BGR -> RGB
        return Response(content=ppm, media_type="image/x-portable-pixmap")

    @app.get("/api/v1/processlist")
    def plist():
        try:
            return [p.to_json() for p in pm.list()]
        except Exception as e:
            return err(500, str(e))

    @app.get("/api/v1/settings")
    def get_settings():
        try:
            return sm.get().to_json()
        except Exception as e:
            return err(500, str(e))

    @app.post("/api/v1/settings")
    async def put_settings(request: Request):
        try:
            s = Settings.from_json(await body_json(request))
        except (ValueError, TypeError) as e:
            return err(400, str(e))
        try:
            sm.overwrite(s)
        except Exception as e:
            return err(500, str(e))
        return Response(status_code=202)

    @app.get("/healthz")
    def healthz():
        from .._native import native

        out = {"ok": True, "cameras": len(pm.hub.cameras), "devices": pm.hub.devices,
               "decoder_backends": [w.decoder for w in pm.hub.workers],
               "vcn_available": bool(native.rocdecode_available()),
               "direct_host_reads": [bool(w.direct_reads) for w in pm.hub.workers],
               # per-GPU host data plane: each worker's CPU list, NUMA node and parse threads
               "host_plane": pm.hub.host_plane() if hasattr(pm.hub, "host_plane") else []}
        if metrics is not None and metrics.consumer is not None:
            out["consumer"] = metrics.consumer.stats()
        return out

    @app.get("/metrics")
    def prom():
        if metrics is None:
            return Response(status_code=404)
        body, ctype = metrics.render()
        return Response(content=body, media_type=ctype)

    @app.get("/", response_class=HTMLResponse)
    def portal():
        return PORTAL.read_text()

    return app
