"""Per-GPU host data plane (csrc/vep/hostplan.h): each GPU worker's ingest sockets, parse strands,
fan-out pool and GPU feeder threads run on its own CPU set, sized from the process's CPU budget
split over the workers (no constant cap), so decode capacity grows with the GPUs of a node.
Replaces the reference's one-container-per-camera CPU shares
(/root/reference/server/services/rtsp_process_manager.go:70-81)."""
import os
import time

import pytest

from conftest import synth


def test_cpulist_roundtrip(native):
    assert native.parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert native.format_cpulist([0, 1, 2, 3, 8, 10, 11]) == "0-3,8,10-11"
    assert native.parse_cpulist(" 5 , 2-3") == [2, 3, 5]
    with pytest.raises(Exception):
        native.parse_cpulist("3-1")


def test_plan_splits_the_budget_without_a_cap(native):
    aff = native.affinity_cpus()
    budget = native.cpu_budget()
    one = native.plan_host_domains([-1])
    assert one[0]["cpus"] == aff and one[0]["cpu_share"] == min(budget, len(aff))
    share = one[0]["cpu_share"]
    assert one[0]["parse_threads"] == max(1, share - (1 if 4 <= share < 16 else 0))
    if len(aff) >= 2:
        two = native.plan_host_domains([-1, -1])
        assert not set(two[0]["cpus"]) & set(two[1]["cpus"])  # disjoint halves
        assert sorted(two[0]["cpus"] + two[1]["cpus"]) == aff
        assert all(d["source"] == "split" for d in two)
    # explicit lists (gpu.host_cpus) win, intersected with the mask
    ex = native.plan_host_domains([-1, -1], [str(aff[0]), native.format_cpulist(aff)])
    assert ex[0]["cpus"] == [aff[0]] and ex[0]["parse_threads"] == 1 and ex[0]["source"] == "explicit"
    assert ex[1]["cpus"] == aff
    # more workers than CPUs: they share
    many = native.plan_host_domains([-1] * (len(aff) + 1))
    assert all(d["cpus"] for d in many) and all(d["parse_threads"] >= 1 for d in many)


def _threads_by_name():
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/comm") as f:
                name = f.read().strip()
            with open(f"/proc/self/task/{tid}/status") as f:
                allowed = [l.split(":", 1)[1].strip() for l in f if l.startswith("Cpus_allowed_list")][0]
        except OSError:
            continue
        out.setdefault(name, []).append(allowed)
    return out


@pytest.mark.skipif(len(os.sched_getaffinity(0)) < 2, reason="needs 2 CPUs")
def test_hub_workers_get_their_own_pinned_ingest_pools(native, tmp_path):
    """Two workers (GPUs): each camera's parse runs on its worker's own strand pool, pinned to the
    worker's CPUs; /healthz's host_plane reports the lists and the live pools."""
    from video_edge_ai_proxy_amd.config import Config
    from video_edge_ai_proxy_amd.engine.hub import Hub

    srv = native.RtspServer("127.0.0.1", 0)
    for i in range(2):
        c = native.SynthConfig()
        c.width, c.height, c.gop, c.fps, c.seed = 160, 96, 10, 30, 3 + i
        srv.add_stream(f"/c{i}", c, realtime=True, cached_frames=10)
    srv.start()
    aff = sorted(os.sched_getaffinity(0))
    cfg = Config()
    cfg.data_dir = str(tmp_path)
    cfg.gpu.host_cpus = [str(aff[0]), str(aff[1])]
    hub = Hub(cfg, devices=[-1, -1])
    try:
        hp = hub.host_plane()
        assert [d["cpulist"] for d in hp] == [str(aff[0]), str(aff[1])]
        assert all(d["ingest_parse_threads"] == 0 for d in hp)  # no camera yet: no pool
        for i in range(2):
            hub.start_camera(f"c{i}", f"rtsp://127.0.0.1:{srv.port}/c{i}")
        assert {h.worker_index for h in hub.cameras.values()} == {0, 1}
        deadline = time.time() + 20
        while time.time() < deadline and not all(hub.wait_decoded(f"c{i}", 1, 0.2) for i in range(2)):
            for i in range(2):
                hub.touch(f"c{i}")
        assert all(hub.wait_decoded(f"c{i}", 1, 5) for i in range(2))
        hp = hub.host_plane()
        assert all(d["ingest_parse_threads"] == 1 for d in hp)
        threads = _threads_by_name()
        # one parse strand per worker, each pinned to that worker's CPU; the feeder threads too
        assert sorted(threads["vep-parse"]) == sorted([str(aff[0]), str(aff[1])])
        assert sorted(threads["vep-worker"]) == sorted([str(aff[0]), str(aff[1])])
    finally:
        hub.shutdown()
        srv.stop()


def test_process_isolated_children_split_the_plan(native, tmp_path):
    """gpu.isolation: process — every worker process takes its own entry of the node's plan and
    pins itself to it (the children agree without talking: the plan is deterministic)."""
    from video_edge_ai_proxy_amd.config import Config
    from video_edge_ai_proxy_amd.engine.isolated import ProcessHub

    aff = sorted(os.sched_getaffinity(0))
    if len(aff) < 2:
        pytest.skip("needs 2 CPUs")
    cfg = Config()
    cfg.data_dir = str(tmp_path)
    cfg.gpu.isolation = "process"
    hub = ProcessHub(cfg, devices=[-1, -1])
    try:
        hp = hub.host_plane()
        assert len(hp) == 2 and hp[0]["pid"] != hp[1]["pid"]
        got = [native.parse_cpulist(d["cpulist"]) for d in hp]
        assert not set(got[0]) & set(got[1]) and sorted(got[0] + got[1]) == aff
        for d in hp:  # the whole child process is pinned to its domain
            with open(f"/proc/{d['pid']}/status") as f:
                allowed = [l.split(":", 1)[1].strip() for l in f if l.startswith("Cpus_allowed_list")][0]
            assert native.parse_cpulist(allowed) == native.parse_cpulist(d["cpulist"])
    finally:
        hub.shutdown()
