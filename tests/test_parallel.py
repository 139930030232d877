"""Camera data parallelism: sharding, gloo multi-process all-gather, 2-rank bench (CPU)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_deterministic_and_balanced():
    from video_edge_ai_proxy_amd.parallel import balanced_shard, shard_cameras

    names = [f"cam{i}" for i in range(256)]
    a = shard_cameras(names, 8, capacity=32)
    b = shard_cameras(list(reversed(names)), 8, capacity=32)
    assert a == b
    loads = [list(a.values()).count(r) for r in range(8)]
    assert loads == [32] * 8
    # adding one GPU moves only cameras to the new rank (no capacity limit)
    u = shard_cameras(names, 8)
    v = shard_cameras(names, 9)
    moved = [n for n in names if u[n] != v[n]]
    assert all(v[n] == 8 for n in moved)
    assert [len(r) for r in balanced_shard(10, 4)] == [3, 3, 2, 2]
    with pytest.raises(ValueError):
        shard_cameras(names, 2, capacity=10)


def _gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from video_edge_ai_proxy_amd import native
    from video_edge_ai_proxy_amd.parallel import ConsumerBatch, init_distributed

    init_distributed("gloo")
    w = native.Worker(device=-1, letterbox_size=32, max_cameras=2)
    cb = ConsumerBatch(w, 2, 32, torch.device("cpu"), world)
    cfg = native.SynthConfig()
    cfg.width, cfg.height, cfg.gop, cfg.seed = 64, 48, 4, 100 + rank
    rb = native.ReplayBench(w, 2, cfg, cached_frames=4, threads=1, prefix=f"r{rank}")
    for _ in range(3):
        cb.prepare()
        rb.step()
        out, work = cb.gather(async_op=False)
    cb.drain()
    # each rank's slice of the gathered batch equals what that rank produced
    local = cb.bufs[(cb.tick - 1) & 1]
    ok = torch.equal(out[rank * 2:(rank + 1) * 2], local) and out.shape == (world * 2, 32, 32, 3)
    sums = out.view(world, -1).float().sum(1).tolist()
    q.put((rank, ok, sums))
    dist.destroy_process_group()


def test_consumer_batch_allgather_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res)
    sums = {r: s for r, _, s in res}
    assert sums[0] == sums[1]  # both ranks hold the identical node-wide batch
    assert sums[0][0] != sums[0][1]  # different cameras per rank (different seeds)


def test_bench_two_ranks_gloo():
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--cpu", "--width", "96", "--height", "64",
           "--cams-per-gpu", "2", "--letterbox", "32", "--latency-samples", "3", "--threads", "1",
           "--frames-per-step", "2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_ranks"] == 2 and d["n_gpus"] == 0 and d["config"]["global_batch"] == 4 and d["config"]["all_gather"]
    assert d["value"] > 0 and d["config"]["parallelism"] == "camera-dp2"
    assert d["gather_verified"] is True and d["frames_per_step"] == 2


def test_parse_threads_split_cpu_budget(monkeypatch):
    from video_edge_ai_proxy_amd import utils

    monkeypatch.setattr(utils, "host_cpu_budget", lambda: 16)
    assert utils.parse_threads_per_rank(1) == 15      # single-GPU share: the measured optimum
    monkeypatch.setattr(utils, "host_cpu_budget", lambda: 128)
    assert utils.parse_threads_per_rank(8) == 15      # 16 CPUs per rank
    monkeypatch.setattr(utils, "host_cpu_budget", lambda: 256)
    assert utils.parse_threads_per_rank(8) == 31      # no constant cap: 32 CPUs per rank
    monkeypatch.setattr(utils, "host_cpu_budget", lambda: 64)
    assert utils.parse_threads_per_rank(8) == 7       # 8 per rank, 1 left for launch/lanes
    monkeypatch.setattr(utils, "host_cpu_budget", lambda: 4)
    assert utils.parse_threads_per_rank(8) == 2       # floor
    assert utils.host_cpu_budget.__call__() >= 1


def test_hub_consumer_batch_cpu(native, tmp_path):
    """`vep serve`'s consumer API: every worker letterboxes each published frame into its
    torch-owned consumer tensor; Hub.consumer_batch() returns the node-wide batch in the
    requested camera order (rows compared with the fp32 letterbox reference of the camera's
    latest frame, within rounding)."""
    import time

    import torch

    from video_edge_ai_proxy_amd.config import Config
    from video_edge_ai_proxy_amd.engine.hub import Hub
    from video_edge_ai_proxy_amd.ops import letterbox_reference

    srv = native.RtspServer("127.0.0.1", 0)
    for i, (w, h) in enumerate([(320, 240), (256, 144)]):
        c = native.SynthConfig()
        c.width, c.height, c.gop, c.fps, c.seed = w, h, 10, 30, 3 + i
        srv.add_stream(f"/c{i}", c, realtime=True, cached_frames=20)
    srv.start()
    cfg = Config()
    cfg.data_dir = str(tmp_path)
    cfg.gpu.devices = [-1, -1]  # two CPU-backend workers: the multi-worker assembly path
    cfg.gpu.letterbox_size = 64
    cfg.gpu.max_cameras_per_gpu = 4
    hub = Hub(cfg)
    try:
        for i in range(2):
            hub.start_camera(f"c{i}", f"rtsp://127.0.0.1:{srv.port}/c{i}", disk_path="")
        assert {hub.handle("c0").worker_index, hub.handle("c1").worker_index} == {0, 1}
        deadline = time.time() + 10
        while time.time() < deadline:
            for n in ("c0", "c1"):
                w, cam = hub.worker_of(n)
                w.set_last_query(cam, int(time.time() * 1000))
            if all(hub.worker_of(n)[0].published(hub.worker_of(n)[1]) >= 3 for n in ("c0", "c1")):
                break
            time.sleep(0.05)
        # freeze decoding (no more queries) so the rows and the latest frames stay put
        for n in ("c0", "c1"):
            w, cam = hub.worker_of(n)
            w.set_idle_cutoff_ms(cam, 1)
        time.sleep(0.3)
        batch, names = hub.consumer_batch(names=["c1", "c0"])
        assert names == ["c1", "c0"] and tuple(batch.shape) == (2, 64, 64, 3)
        for row, n in zip(batch, names):
            w, cam = hub.worker_of(n)
            meta, img = w.read_latest(cam, 0)
            ref, _ = letterbox_reference(torch.from_numpy(img), 64)
            assert (row.int() - ref.int()).abs().max().item() <= 1, n
    finally:
        hub.shutdown()
        srv.stop()


def test_bench_keyframe_only_rtsp_cpu():
    """BASELINE config 3 shape: every access unit crosses the live ingest, only IDR pictures are
    decoded (keyframe-only cameras); the JSON reports both rates."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--source", "rtsp", "--keyframe-only",
           "--steps", "2", "--warmup", "1", "--width", "96", "--height", "64", "--cams-per-gpu", "2",
           "--gop", "6", "--letterbox", "32", "--latency-samples", "0", "--threads", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["keyframe_only"] and d["source"] == "rtsp" and d["frames_dropped"] == 0
    # only keyframes decode: about one picture per GOP of ingested access units
    assert 0 < d["frames_decoded"] < d["access_units_ingested"]


@pytest.mark.parametrize("fmt", [["--bit-depth", "10"], ["--chroma-format", "2"]], ids=["high10", "422"])
def test_bench_high_formats_rtsp_cpu(fmt):
    """The headline bench with H.264 High 10 / High 4:2:2 streams (CPU backend): every picture
    decodes and publishes, the JSON names the profile and reports the launch statistics."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--source", "rtsp", "--steps", "1",
           "--warmup", "1", "--width", "96", "--height", "64", "--cams-per-gpu", "2", "--gop", "6",
           "--letterbox", "32", "--latency-samples", "0", "--threads", "1"] + fmt
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["frames_dropped"] == 0 and d["frames_decoded"] >= 12
    assert ("High 10" if fmt[0] == "--bit-depth" else "High 4:2:2") in d["data"]
    assert d["rank0_pictures_per_launch"] > 0


def test_hostprof_samples_native_threads(native, tmp_path):
    """The extension's SIGPROF sampler records where host CPU time goes (parse hot spots)."""
    import time

    out = tmp_path / "prof.txt"
    cfg = native.SynthConfig()
    cfg.width, cfg.height, cfg.compressed = 320, 240, True
    enc = native.SynthH264(cfg)
    aus = [enc.next() for _ in range(10)]
    native.hostprof_start(200)
    t0 = time.time()
    while time.time() - t0 < 1.0:
        dec = native.CpuDecoder()
        for au in aus:
            dec.decode(au)
    n = native.hostprof_stop(str(out))
    rows = [l.split(maxsplit=3) for l in out.read_text().splitlines()]
    assert n > 0 and sum(int(r[0]) for r in rows) == min(n, 1 << 21)
    assert any("_vep" in r[1] for r in rows)  # samples inside the extension, with offsets


def test_bench_config5_rtmp_annotation_cpu():
    """BASELINE config 5 shape on the CPU backend: H.265 cameras through the live ingest with RTMP
    pass-through to a loopback RTMP server and Annotate RPCs uploaded by the production queue +
    batch consumer to a loopback cloud endpoint; the JSON reports all three. (40 steps: the RTMP
    counts cover the timed region only, and a few steps of these tiny pictures can be decoded
    before the pass-through senders' first message lands.)"""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--codec", "h265", "--rtmp", "--annotate",
           "--annotate-rate", "20", "--steps", "40", "--warmup", "2", "--width", "128", "--height", "96",
           "--cams-per-gpu", "2", "--gop", "8", "--letterbox", "32", "--clients", "2", "--client-procs", "1",
           "--latency-seconds", "1", "--latency-samples", "5", "--threads", "2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["source"] == "rtsp" and d["frames_dropped"] == 0 and d["decode_errors"] == 0
    assert d["access_units_skipped"] == 0
    # (the timed region of these tiny pictures can end before a loaded host's pass-through
    # senders deliver their first message: count from the start of the run)
    assert d["rtmp_passthrough"]["video_messages_since_start"] > 0
    ann = d["annotation"]
    assert ann["annotate_rpcs"] > 0 and ann["annotate_rpc_errors"] == 0 and not ann["error"]
    assert ann["annotations_uploaded"] == ann["annotate_rpcs"] and ann["unsigned_posts"] == 0
    assert d["p50_latency_ms"] is not None and d["serve_p50_latency_ms"] is not None


def test_bench_eight_ranks_gloo():
    """World = 8 rehearsal of the camera-DP bench (gloo, CPU backend): rank spawn, barriers, the
    all-gather of the consumer batch every step, the MAX / SUM reductions and rank 0's JSON."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "8", "--steps", "3", "--warmup", "1", "--cpu", "--width", "64", "--height", "48",
           "--cams-per-gpu", "1", "--letterbox", "16", "--latency-samples", "2", "--clients", "1",
           "--client-procs", "1", "--latency-seconds", "1", "--threads", "1", "--gop", "6"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_ranks"] == 8 and d["config"]["global_batch"] == 8 and d["config"]["all_gather"]
    assert d["config"]["parallelism"] == "camera-dp8" and d["frames_dropped"] == 0 and d["value"] > 0
    # every rank checked the rows it received against their owners' checksums
    assert d["gather_verified"] is True and d["gather_check"]["mismatching_rows"] == 0
    assert d["gather_check"]["checked_gathers"] >= 8 and d["collective_backend"] == "gloo"
    assert d["frames_per_step"] == 6 and d["rccl_world"] == 0
