"""gpu.consumer_rate_hz: the daemon's steady-state consumer of the node batch (engine/consumer.py).

In-process hub: snapshots of every GPU's consumer rows, the hook called with the node batch.
Isolated hub: one collective gather per call across the worker processes; the hook runs on every
rank (with the whole node batch), nothing is copied back to the parent; the steady-state gather
time (group formation excluded) is recorded."""
import os
import sys
import time

from test_isolated_hub import _isolated_cfg, _settle, farm

HOOK = """import os
def hook(batch, names, rank):
    with open(os.path.join(os.environ["VEP_TEST_HOOK_DIR"], f"rank{rank}"), "a") as f:
        f.write(f"{tuple(batch.shape)} {','.join(names)}\\n")
"""


def _hook_module(tmp_path, monkeypatch):
    (tmp_path / "vep_test_hook.py").write_text(HOOK)
    monkeypatch.setenv("PYTHONPATH", str(tmp_path) + os.pathsep + os.environ.get("PYTHONPATH", ""))
    monkeypatch.setenv("VEP_TEST_HOOK_DIR", str(tmp_path))
    monkeypatch.syspath_prepend(str(tmp_path))


def _lines(tmp_path, rank):
    p = tmp_path / f"rank{rank}"
    return p.read_text().splitlines() if p.exists() else []


def test_consumer_loop_in_process_hub(native, tmp_path, monkeypatch):
    from video_edge_ai_proxy_amd.engine.consumer import ConsumerLoop
    from video_edge_ai_proxy_amd.engine.hub import Hub

    _hook_module(tmp_path, monkeypatch)
    srv = farm(native, 2)
    cfg = _isolated_cfg(tmp_path, 16)
    cfg.gpu.isolation = "thread"
    hub = Hub(cfg, devices=[-1])
    try:
        for i in range(2):
            hub.start_camera(f"c{i}", f"rtsp://127.0.0.1:{srv.port}/c{i}")
        _settle(hub, ["c0", "c1"])
        loop = ConsumerLoop(hub, 20.0, "vep_test_hook:hook").start()
        time.sleep(1.5)
        loop.stop()
        st = loop.stats()
        assert st["gathers"] >= 10 and st["errors"] == 0 and st["gather_ms_p50"] is not None, st
        lines = _lines(tmp_path, 0)
        assert len(lines) == st["gathers"] and lines[-1] == "(2, 16, 16, 3) c0,c1"
    finally:
        hub.shutdown()
        srv.stop()


def test_consumer_loop_isolated_hub_every_rank(native, tmp_path, monkeypatch):
    from video_edge_ai_proxy_amd.engine.consumer import ConsumerLoop
    from video_edge_ai_proxy_amd.engine.isolated import ProcessHub

    _hook_module(tmp_path, monkeypatch)
    srv = farm(native, 3)
    cfg = _isolated_cfg(tmp_path, 16)
    cfg.gpu.consumer_hook = "vep_test_hook:hook"
    hub = ProcessHub(cfg, devices=[-1, -1], supervise_interval_s=0.2)
    try:
        names = [f"c{i}" for i in range(3)]
        for n in names:
            hub.start_camera(n, f"rtsp://127.0.0.1:{srv.port}/{n}")
        _settle(hub, names)
        loop = ConsumerLoop(hub, 10.0).start()
        time.sleep(2.0)
        loop.stop()
        st = loop.stats()
        assert st["gathers"] >= 8 and st["errors"] == 0, st
        assert st["gather_ms_p50"] is not None and st["gather_ms_p50"] < 1000
        for rank in (0, 1):  # the hook ran on every rank with the whole node batch
            lines = _lines(tmp_path, rank)
            assert len(lines) >= st["gathers"] - 1 and lines[-1] == "(3, 16, 16, 3) c0,c1,c2", lines[-3:]
        assert len(hub.gather_ms) == st["gathers"]  # steady state only: no group formation in it
    finally:
        hub.shutdown()
        srv.stop()
