#!/usr/bin/env python3
"""Headline benchmark: decoded FPS (whole node) + p50 VideoLatestImage latency, 256x1080p RTSP.

One rank per GPU (torch.distributed over RCCL when WORLD_SIZE > 1). Each rank owns
``--cams-per-gpu`` synthetic 1080p30 H.264 cameras (camera data parallelism, weak scaling).

Default ``--source rtsp`` (the stated metric): every rank serves its cameras from an in-process
loopback RTSP camera farm (RTP over TCP-interleaved, FU-A), and the production ingest — RtspClient
+ RTP depacketizer on the epoll loops, the lazy decoder's CABAC/CAVLC host parse on the parse
strands, the GPU worker's batched gfx950 reconstruction + NV12->BGR24 into each camera's HBM ring
+ letterbox into the consumer batch — decodes them. One *step* is ``cams-per-gpu`` decoded
pictures; the farm is unthrottled during the timed region, so ``value`` is the node's decode
capacity (decoded pictures / s summed over ranks, time = max over ranks). With N > 1 the
letterboxed consumer batch is all-gathered over RCCL once per frame interval, overlapped with
decode, and every rank checks what it received: per-row checksums of each rank's snapshot are
all-gathered next to the rows and compared with the checksums of the gathered rows
(``gather_verified``).

One *step* is ``--frames-per-step`` frame intervals of every camera (default: one GOP, 30 frames):
``cams-per-gpu x frames-per-step`` decoded pictures per rank, so ``--steps 20`` times ~3 s of
decoding at the headline rate and every step covers whole GOPs (IDR, P and B pictures in the
stream's own proportions) rather than a transient.

Latency (headline ``p50_latency_ms`` / ``p99_latency_ms``): after the timed loop the farm switches
to real time (``--fps``), and ``--clients`` concurrent gRPC clients running in separate processes
(started before this process touches the GPU) each issue back-to-back VideoLatestImage requests
for their own live camera through the production gRPC server: request sent -> the camera's next
BGR24 VideoFrame received and parsed. ``serve_p50_latency_ms`` is one request on a fresh
connected channel (the newest frame already in the ring).

``--source replay`` is the decode-only capacity (pre-encoded AUs fed straight to the parse pool,
no network stack), labelled as such in the JSON.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# The worker's serving stream + 3 decode lanes + their 3 copy streams (and, multi-rank, torch's
# and RCCL's streams): give the process 8 hardware queues (HIP's default is 4) so no decode lane
# or all-gather shares a queue with another. Must be set before HIP initialises.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "decoded FPS (whole node) + p50 VideoLatestImage latency, 256×1080p RTSP"
CODEC = {"h264": "H.264", "h265": "H.265"}
ENTROPY = {"h264": "CAVLC macroblock-layer", "h265": "CABAC coding-tree"}


def parse_args():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    # a step is --frames-per-step frame intervals of every camera (~155 ms at the headline rate)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--frames-per-step", type=int, default=0,
                    help="frame intervals of every camera per step (0 = one GOP, --gop; keyframe-only: 1)")
    ap.add_argument("--cams-per-gpu", type=int, default=32)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--fps", type=int, default=30)
    ap.add_argument("--gop", type=int, default=30)
    ap.add_argument("--motion", type=float, default=0.05)
    ap.add_argument("--codec", choices=["h264", "h265"], default="h264",
                    help="h265 = BASELINE config 5 codec (e.g. --width 3840 --height 2160)")
    ap.add_argument("--content", choices=["avc", "pcm"], default="avc",
                    help="avc = compressed CAVLC streams (general decoder); pcm = I_PCM/P_Skip fast path")
    ap.add_argument("--profile", choices=["baseline", "main", "high"], default="high",
                    help="H.264 profile of the compressed streams: baseline = CAVLC I/P; main = CABAC "
                         "I/P/B; high = main + 8x8 transform / Intra_8x8 (what IP cameras send)")
    ap.add_argument("--bframes", type=int, default=2, help="main/high: B pictures per mini-GOP (pyramid)")
    ap.add_argument("--cavlc", action="store_true", help="main/high: CAVLC instead of CABAC")
    ap.add_argument("--qp", type=int, default=None,
                    help="encoder QP of the compressed streams (default: 25 main/high, 27 baseline)")
    ap.add_argument("--noise", type=float, default=8.0, help="static scene texture amplitude")
    ap.add_argument("--temporal-noise", type=float, default=None,
                    help="per-frame sensor noise (default: 1.5 main/high -> ~3.9 Mbit/s at 1080p30, "
                         "1.0 baseline -> ~4.5 Mbit/s)")
    ap.add_argument("--refs", type=int, default=1, help="max_num_ref_frames of the compressed streams")
    ap.add_argument("--slices", type=int, default=0,
                    help="slices per picture of the synthetic streams (0: 8 for 4K H.265 — config 5 — else 1); "
                         "the independent slices of an H.265 picture are parsed in parallel")
    ap.add_argument("--interlaced", type=int, choices=[0, 1, 2], default=0,
                    help="h264 main/high: 1 = interlaced SPS coding frame pictures, 2 = every frame a field "
                         "pair (PAFF: CAVLC I/P fields, 4x4 transforms, no B pictures); fps counts frames")
    ap.add_argument("--bit-depth", type=int, choices=[8, 10], default=8,
                    help="10: H.265 Main10 / H.264 High 10 (main / high profiles, progressive) streams (u16 "
                         "surfaces on the GPU, narrowed to 8 bits for BGR24)")
    ap.add_argument("--chroma-format", type=int, choices=[1, 2], default=1,
                    help="h264 main/high, progressive: 2 = High 4:2:2 streams (NV16 surfaces, 4:2:0 display "
                         "conversion for BGR24)")
    ap.add_argument("--threads", type=int, default=0,
                    help="host parse threads per rank (0 = the rank's host domain: its part of the CPU "
                         "budget - 1, pinned to its GPU's NUMA-local CPUs)")
    ap.add_argument("--parse-window", type=int, default=8,
                    help="ticks a camera's parse may run ahead of the tick being launched")
    ap.add_argument("--pack-threads", type=int, default=4, help="host index/staging threads per rank")
    ap.add_argument("--cache-gops", type=int, default=1,
                    help="distinct pre-encoded GOPs replayed per camera (working-set size)")
    ap.add_argument("--lanes", type=int, default=0,
                    help="independent GPU pipelines per worker (0 = runtime default)")
    ap.add_argument("--stages", type=int, default=0,
                    help="ticks in flight per GPU lane (0 = runtime default)")
    ap.add_argument("--lane-queue", type=int, default=0,
                    help="batches queued per GPU lane launcher thread (0 = runtime default)")
    ap.add_argument("--letterbox", type=int, default=640)
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--consumer-format", choices=["nv12", "bgr"], default="nv12",
                    help="letterboxed consumer batch layout gathered over xGMI (nv12 = 1.5 B/px)")
    ap.add_argument("--ring-slots", type=int, default=2)
    ap.add_argument("--latency-samples", type=int, default=100)
    ap.add_argument("--cpu", action="store_true", help="CPU backend (plumbing check, no GPU)")
    ap.add_argument("--ref-equivalent", action="store_true",
                    help="with --cpu: the reference-equivalent CPU path (CPU parse + CPU reconstruction + CPU "
                         "BGR24, the tobytes + SerializeToString copy chain per frame; read_image.py:87-121)")
    ap.add_argument("--ref-cpu", choices=["on", "off"], default="on",
                    help="GPU runs: after the measurement, rank 0 runs the same cameras / steps / clients "
                         "through the reference-equivalent CPU path on its host domain's CPUs and reports "
                         "reference_equivalent_cpu_fps and vs_baseline = value / (that x ranks)")
    ap.add_argument("--source", choices=["replay", "rtsp", "records"], default="rtsp",
                    help="replay = pre-encoded AUs fed to the decode pipeline (decode-only); rtsp = an "
                         "in-process loopback RTSP camera farm, unthrottled, with the production "
                         "ingest (RtspClient + RTP depacketizer + lazy decoder) inside the timed loop; "
                         "records = the GPU-side ceiling: every camera's GOPs parsed once up front and the "
                         "reconstruction jobs (records) replayed into the GPU lanes, no host parse in the loop")
    ap.add_argument("--rtmp", action="store_true",
                    help="BASELINE config 5: every camera's RTMP pass-through on, to a loopback RTMP server "
                         "(rtsp source)")
    ap.add_argument("--annotate", action="store_true",
                    help="BASELINE config 5: Annotate RPCs during the timed region, uploaded by the production "
                         "queue + batch consumer to a loopback cloud endpoint (rtsp source)")
    ap.add_argument("--annotate-rate", type=float, default=5.0, help="annotations per camera per second")
    ap.add_argument("--keyframe-only", action="store_true",
                    help="BASELINE config 3 (selective I-frame decode): every camera in keyframe-only "
                         "mode (the reference's read_image.py --keyframe_only); needs --source rtsp so "
                         "every access unit still crosses ingest and only IDR pictures are decoded")
    ap.add_argument("--clients", type=int, default=32,
                    help="concurrent gRPC clients for the latency run (one camera each)")
    ap.add_argument("--client-procs", type=int, default=0,
                    help="processes the latency clients run in (0 = half the rank's CPU budget)")
    ap.add_argument("--serving", choices=["native", "grpcio"], default="native",
                    help="latency run's gRPC endpoint: the native HTTP/2 server on the worker's frame bus "
                         "(vep serve's default) or the grpcio ImageService")
    ap.add_argument("--latency-seconds", type=float, default=4.0,
                    help="duration of the concurrent-client latency run")
    a = ap.parse_args()
    if a.keyframe_only and a.source != "rtsp":
        ap.error("--keyframe-only needs --source rtsp (the ingest filters the access units)")
    if (a.rtmp or a.annotate) and a.source != "rtsp":
        ap.error("--rtmp / --annotate need --source rtsp")
    if a.qp is None:
        a.qp = 27 if a.profile == "baseline" else 25
    if a.slices <= 0:
        a.slices = 8 if a.codec == "h265" and a.width * a.height >= 3840 * 2160 else 1
    if a.temporal_noise is None:
        a.temporal_noise = 1.0 if a.profile == "baseline" else 1.5
    if a.frames_per_step <= 0:  # (keyframe-only cameras decode one picture per GOP: a step is a GOP)
        a.frames_per_step = 1 if a.keyframe_only else a.gop
    return a


class GatherCheck:
    """Correctness of the consumer-batch all-gather: every checked gather also all-gathers the
    per-row checksums of each rank's snapshot (computed on the stream that took the snapshot), and
    once the rows have arrived each rank compares the checksums of the rows it received with the
    ones their owners sent. Mismatches are counted on the device (no host sync in the loop)."""

    def __init__(self, torch, dist, world, cams, row, dev, nbuf, every=4):
        self.torch, self.dist, self.every = torch, dist, every
        words = row // 4 if row % 4 == 0 else row
        self.view = torch.int32 if row % 4 == 0 else torch.uint8
        self.w = torch.arange(words, dtype=torch.int64, device=dev) % 65521 + 1
        self.local = [torch.empty(cams, dtype=torch.int64, device=dev) for _ in range(nbuf)]
        self.remote = [torch.empty(world * cams, dtype=torch.int64, device=dev) for _ in range(nbuf)]
        self.handles = [None] * nbuf
        self.bad = torch.zeros((), dtype=torch.int64, device=dev)
        self.checks = self.rows = 0
        self.n = 0

    def sums(self, rows):
        return (rows.view(self.view).to(self.torch.int64) * self.w).sum(dim=1)

    def issue(self, b, snap):
        """After the snapshot of buffer b was enqueued: its checksums, gathered (every `every`-th)."""
        self.n += 1
        if (self.n - 1) % self.every:
            self.handles[b] = None
            return
        self.local[b].copy_(self.sums(snap))
        self.handles[b] = self.dist.all_gather_into_tensor(self.remote[b], self.local[b], async_op=True)

    def verify(self, b, gathered):
        """After the rows' gather of buffer b was waited on."""
        h, self.handles[b] = self.handles[b], None
        if h is None:
            return
        h.wait()
        self.bad += (self.sums(gathered) != self.remote[b]).sum()
        self.checks += 1
        self.rows += gathered.shape[0]

    def result(self, dev):
        """(verified, checks, rows checked, mismatching rows), summed over ranks."""
        t = self.torch.tensor([int(self.bad.item()), self.checks, self.rows], dtype=self.torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        bad, checks, rows = (int(v) for v in t.tolist())
        return checks > 0 and bad == 0, checks, rows, bad


def start_client_pool(a):
    """Latency clients in fresh processes, started before this process touches the GPU."""
    from vep_bench.latency_clients import ClientPool
    from video_edge_ai_proxy_amd.utils import host_cpu_budget

    if a.clients <= 0 and a.latency_samples <= 0:
        return None
    n = max(1, a.clients)
    procs = a.client_procs or max(1, min(n, host_cpu_budget() // 2))
    return ClientPool(procs, (n + procs - 1) // procs)


def latency_fields(a, lat, live_fps=None):
    """The JSON latency block of bench_latency.measure() results."""
    from vep_bench.bench_latency import summarize

    def r3(x):
        return round(x, 3) if x is not None else None

    nx, sv, srv = summarize(lat["next"]), summarize(lat["serve"]), summarize(lat["server_ms"])
    out = {
        "p50_latency_ms": r3(nx[0]),
        "p99_latency_ms": r3(nx[1]),
        "latency_definition": (f"{a.clients} concurrent gRPC clients in separate processes (one connected "
                               "channel and one live camera each), back-to-back VideoLatestImage requests "
                               f"while every camera streams at {a.fps} fps: request sent -> the camera's next "
                               f"{a.width}x{a.height} BGR24 VideoFrame received and parsed (includes waiting for "
                               f"it, up to one frame interval); {len(lat['next'])} samples over "
                               f"{a.latency_seconds:g} s"),
        "latency_frames_served_per_s": round(lat["frames_served"] / a.latency_seconds, 1),
        "serving_endpoint": ("native HTTP/2 gRPC endpoint (csrc/vep/rpcsrv.h) on the worker's frame bus"
                             if a.serving == "native" else "grpcio ImageService"),
        "server_p50_ms": r3(srv[0]),
        "server_p99_ms": r3(srv[1]),
        "server_latency_definition": "server side: request received -> serialized frame queued for the "
                                     "connection (includes waiting for the next frame)",
        "serve_p50_latency_ms": r3(sv[0]),
        "serve_p99_latency_ms": r3(sv[1]),
        "serve_latency_definition": "one request per fresh connected channel, no concurrent clients: the "
                                    f"newest frame already in the HBM ring; {len(lat['serve'])} samples",
    }
    if live_fps is not None:
        out["latency_live_fps_per_camera"] = round(live_fps, 2)
    return out


def n_gpus_scope(res):
    """The headline names a whole node (8 GPUs, 256 cameras); a run on fewer GPUs is that share."""
    n = res.get("n_gpus") or 0
    if 0 < n < 8:
        cams = res["config"]["cams_per_gpu"] * n
        return f"per-GPU share: {n} of the node's 8 GPUs ({cams} of 256 cameras); not a whole-node number"
    return None


def spawn_ranks(n: int) -> int:
    """`--gpus N` without a torch.distributed environment: run N fresh rank processes (one per
    GPU) through torch.distributed.run and return their exit code. Called before this process
    touches the GPU, so the parent never holds a device context while its children run."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__),
           *sys.argv[1:]]
    return subprocess.call(cmd)


def describe_streams(a, compressed):
    if compressed and a.codec == "h265":
        return (f"HEVC {'Main10' if a.bit_depth == 10 else 'Main'} CABAC I/P/B, {a.bframes} B per mini-GOP, CTB 32, merge/AMVP/TMVP, "
                f"deblocking, {a.slices} slice{'s' if a.slices > 1 else ''} per picture")
    if compressed and a.profile == "baseline":
        return "Baseline CAVLC I/P"
    if compressed and a.interlaced == 2:
        return (f"{a.profile.capitalize()} profile interlaced, every frame a field pair (PAFF), CAVLC "
                f"I/P{'/B' if a.bframes else ''} fields{f', {a.bframes} B pairs per mini-GOP' if a.bframes else ''}")
    if compressed:
        hp = ("High 4:2:2" if a.chroma_format == 2 else "High 10" if a.bit_depth == 10 else a.profile.capitalize()) \
            if a.profile != "baseline" else a.profile.capitalize()
        return (f"{hp} profile{' 10-bit' if a.chroma_format == 2 and a.bit_depth == 10 else ''} "
                f"{'CAVLC' if a.cavlc else 'CABAC'} I/P/B, "
                f"{a.bframes} B per mini-GOP{' (pyramid)' if a.bframes >= 2 else ''}"
                f"{', 8x8 transform + Intra_8x8' if a.profile == 'high' else ''}")
    return "I_PCM/P_Skip fast path"


def make_cfg(vep, a, rank, compressed):
    cfg = vep.SynthConfig()
    cfg.width, cfg.height, cfg.fps, cfg.gop, cfg.motion = a.width, a.height, a.fps, a.gop, a.motion
    cfg.codec = a.codec
    cfg.seed = 1 + rank * 100003
    cfg.slices = a.slices
    cfg.bit_depth = a.bit_depth if (a.codec == "h265" or (a.profile != "baseline" and a.interlaced == 0)) else 8
    cfg.chroma_format = a.chroma_format if (a.codec == "h264" and a.profile != "baseline" and a.interlaced == 0) else 1
    if compressed:
        cfg.compressed = True
        cfg.qp, cfg.noise, cfg.temporal_noise, cfg.refs = a.qp, a.noise, a.temporal_noise, a.refs
        cfg.profile, cfg.bframes, cfg.cabac = a.profile, a.bframes, not a.cavlc
        if a.codec == "h264" and a.profile != "baseline":
            cfg.interlaced = a.interlaced
    return cfg


class RtspFarm:
    """`--source rtsp`: a loopback RTSP camera farm (one served stream per camera, pre-encoded
    GOPs looped, unthrottled) and one production IngestSession per camera (RTSP client + RTP
    depacketizer + Camera::on_access_unit lazy decoder -> Worker batches). Every picture of the
    timed region crossed the network stack, the depacketizer and the host parse inside it."""

    def __init__(self, vep, worker, a, rank, compressed):
        import threading

        self.worker = worker
        self.srv = vep.RtspServer("127.0.0.1", 0)
        self.cams = a.cams_per_gpu
        self.stream_bytes = 0

        def add(i):  # (the farm pre-encodes each camera's GOPs: in parallel, GIL released)
            c = make_cfg(vep, a, rank, compressed)
            c.seed = c.seed + i * 7919
            c.idr_phase = (i * a.gop) // self.cams  # unsynchronised cameras
            self.srv.add_stream(f"/cam{i}", c, realtime=False, cached_frames=a.gop * a.cache_gops)

        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(max(1, min(self.cams, (os.cpu_count() or 4), 16))) as ex:
            list(ex.map(add, range(self.cams)))
        self.srv.start()
        # BASELINE config 5: RTMP pass-through of every camera to a loopback RTMP server
        self.sink = None
        if a.rtmp:
            self.sink = vep.RtmpSink("127.0.0.1", 0)
            self.sink.set_keep_bodies(False)
            self.sink.start()
        worker.start()
        self.idx = [worker.add_camera(f"r{rank}rtsp{i}", a.ring_slots) for i in range(self.cams)]
        for cam in self.idx:
            worker.set_keyframe_only(cam, a.keyframe_only)
            if self.sink is not None:
                worker.set_proxy(cam, True)
        self._touch()
        self.sessions = []
        for i, cam in enumerate(self.idx):
            # lossless: while a camera's parse backlog is deep its socket is paused (TCP
            # back-pressure on the unthrottled farm) instead of dropping AUs to the next keyframe
            rtmp = f"rtmp://127.0.0.1:{self.sink.port}/live/r{rank}cam{i}" if self.sink is not None else ""
            sess = vep.IngestSession(worker, cam, f"r{rank}rtsp{i}", f"rtsp://127.0.0.1:{self.srv.port}/cam{i}",
                                     rtmp_url=rtmp, lossless=True)
            sess.start()
            self.sessions.append(sess)
        self.stop_evt = threading.Event()
        self.toucher = threading.Thread(target=self._touch_loop, daemon=True)
        self.toucher.start()

    def _touch(self):  # a client is watching every camera (the lazy decoder's last_query)
        now = int(time.time() * 1000)
        for cam in self.idx:
            self.worker.set_last_query(cam, now)

    def _touch_loop(self):
        while not self.stop_evt.wait(0.5):
            self._touch()

    def wait_pictures(self, target, timeout_s=120.0):
        deadline = time.perf_counter() + timeout_s
        while self.worker.pictures < target:
            if time.perf_counter() > deadline:
                raise RuntimeError(f"rtsp farm stalled at {self.worker.pictures}/{target} pictures")
            time.sleep(0.0002)

    def settle(self, min_s=1.0, max_s=6.0, window_s=0.25):
        """Before the warmup steps: let the unthrottled pipeline reach its steady state (the
        sockets' start-up backlog drained: nearly every decoded picture is published again rather
        than collapsed into a catch-up batch), so a short timed window measures the steady rate.
        Returns the seconds it took."""
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < max_s:
            p0, f0 = self.worker.pictures, self.worker.frames
            time.sleep(window_s)
            dp, df = self.worker.pictures - p0, self.worker.frames - f0
            if time.perf_counter() - t0 >= min_s and dp > 0 and df >= 0.9 * dp:
                break
        return round(time.perf_counter() - t0, 2)

    def stats(self):
        st = [self.worker.stats(c) for c in self.idx]
        out = {"packets": sum(x["packets"] for x in st), "bytes_in": sum(x["bytes_in"] for x in st),
               "errors": sum(x["errors"] for x in st), "decoded": sum(x["decoded"] for x in st),
               "skipped": sum(x["skipped"] for x in st)}
        if self.sink is not None:
            out["rtmp_messages"] = self.sink.video_messages
            out["rtmp_bytes"] = self.sink.video_bytes
            out["rtmp_keyframes"] = self.sink.keyframes
        return out

    def go_live(self, fps, timeout_s=20.0):
        """Switch the farm to real time and wait until the ingest backlog of the unthrottled run has
        drained (the decode rate has fallen to the cameras' frame rate)."""
        self.srv.set_pacing(1)
        for sess in self.sessions:  # live cameras: the production (lossy) ingest
            sess.set_lossless(False)
        deadline = time.perf_counter() + timeout_s
        target = self.cams * fps * 1.25
        while time.perf_counter() < deadline:
            p0 = self.worker.pictures
            time.sleep(0.5)
            if (self.worker.pictures - p0) / 0.5 <= target:
                return True
        return False

    def close(self):
        self.stop_evt.set()
        for sess in self.sessions:
            sess.stop()
        self.srv.stop()
        if self.sink is not None:
            self.sink.stop()
        self.worker.stop()


def thread_cpu() -> dict:
    """CPU seconds of this process's threads by name (/proc/self/task/*/comm; the native threads
    name themselves by role: vep-parse, vep-io, vep-worker, vep-farm, ...)."""
    tick = os.sysconf("SC_CLK_TCK")
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/comm") as f:
                name = f.read().strip()
            with open(f"/proc/self/task/{tid}/stat") as f:
                st = f.read().rsplit(")", 1)[1].split()
        except OSError:  # (a thread that ended meanwhile)
            continue
        name = name if name.startswith("vep-") else "other (python / grpc / hip)"
        out[name] = out.get(name, 0.0) + (int(st[11]) + int(st[12])) / tick  # utime + stime
    return out


def cpu_cores_by_thread(c0: dict, c1: dict, elapsed: float) -> dict:
    d = {k: round((c1.get(k, 0.0) - c0.get(k, 0.0)) / elapsed, 2) for k in set(c0) | set(c1)}
    d = {k: v for k, v in sorted(d.items(), key=lambda kv: -kv[1]) if v > 0}
    d["total"] = round(sum(d.values()), 2)
    return d


def avc_cycles_per_mb(worker) -> dict:
    """VEP_AVC_PROF=1: the H.264 wavefront kernels' per-phase clocks, per macroblock."""
    pr = worker.avc_profile()
    out = {}
    for ph in ("intra", "dbk"):
        n = max(1, pr[f"{ph}_mbs"])
        out[f"{ph}_cycles_per_mb"] = {k[len(ph) + 1:]: round(v / n, 1) for k, v in pr.items()
                                      if k.startswith(ph) and not k.endswith("mbs")}
        out[f"{ph}_mbs"] = pr[f"{ph}_mbs"]
    return out


def run_rtsp(a, vep, torch, dist, worker, world, rank, use_gpu, dev, row, compressed, pool):
    """`--source rtsp`: the timed loop waits for the live pipeline (loopback RTSP farm ->
    IngestSession -> lazy decoder -> Worker batches) to decode `cams` more pictures per step."""
    from vep_bench.bench_latency import measure

    cams = a.cams_per_gpu
    # the worker letterboxes every published frame into the live rows; each step's all-gather
    # reads a consistent snapshot of them (Worker.snapshot_consumer: ordered after the letterbox
    # writes already enqueued, before any later one), double-buffered so the next snapshot never
    # overwrites rows a gather in flight still reads
    live = torch.zeros((cams, row), dtype=torch.uint8, device=dev)
    gather = world > 1 and not a.no_gather
    snaps = [torch.empty((cams, row), dtype=torch.uint8, device=dev) for _ in range(2)] if gather else None
    gathered = [torch.empty((world * cams, row), dtype=torch.uint8, device=dev) for _ in range(2)] if gather else None
    check = GatherCheck(torch, dist, world, cams, row, dev, 2) if gather else None
    F = a.frames_per_step
    worker.set_consumer_buffers(live.data_ptr(), 0, cams)

    def sync():
        if use_gpu:
            torch.cuda.synchronize()

    farm = RtspFarm(vep, worker, a, rank, compressed)
    lat = None
    live_fps = None
    annot = None
    side = {}
    try:
        if a.annotate:  # (runs from the warmup on: the counts cover warmup + timed region)
            from vep_bench.bench_pipeline import AnnotationLoad

            annot = AnnotationLoad([f"r{rank}rtsp{i}" for i in range(cams)], rate=a.annotate_rate)
            annot.start()
        settle_s = farm.settle()
        farm.wait_pictures(farm.worker.pictures + cams * max(1, a.warmup * a.frames_per_step), timeout_s=300.0)
        if world > 1:
            dist.barrier()
        sync()
        p0, f0, d0, s0 = worker.pictures, worker.frames, worker.dropped, farm.stats()
        sh0 = worker.shed
        rg0 = worker.records_gathered
        g0 = worker.gpu_ms_total
        bt0, mg0 = worker.batches, worker.merged
        hostprof = os.environ.get("VEP_HOSTPROF")  # path: SIGPROF samples of every thread, timed region
        if hostprof:
            vep.hostprof_start(1000)
        handles = [None, None]
        cpu0 = thread_cpu()
        t0 = time.perf_counter()
        for i in range(a.steps * F):  # (a step: F frame intervals of every camera)
            farm.wait_pictures(p0 + cams * (i + 1))
            if gather:  # RCCL all-gather of the letterboxed consumer batch, overlapped with decode
                b = i & 1
                if handles[b] is not None:  # (a stream wait: the gather that last read snapshot b)
                    handles[b].wait()
                    check.verify(b, gathered[b])
                stream = torch.cuda.current_stream().cuda_stream if use_gpu else 0
                worker.snapshot_consumer(snaps[b].data_ptr(), snaps[b].numel(), cams, stream)
                handles[b] = dist.all_gather_into_tensor(gathered[b], snaps[b], async_op=True)
                check.issue(b, snaps[b])
        for b, h in enumerate(handles):
            if h is not None:
                h.wait()
                check.verify(b, gathered[b])
        sync()
        t1 = time.perf_counter()
        # every counter is sampled at the end of this rank's timed region, before the barrier: the
        # unthrottled farm keeps feeding (and the worker decoding) while a rank waits for the others
        rg1 = worker.records_gathered
        pictures, frames, dropped = worker.pictures - p0, worker.frames - f0, worker.dropped - d0
        shed = worker.shed - sh0
        batches, merged = worker.batches - bt0, worker.merged - mg0
        s1 = farm.stats()
        cpu1 = thread_cpu()
        if world > 1:
            dist.barrier()
        elapsed = t1 - t0
        if hostprof:
            vep.hostprof_stop(hostprof)
        gpu_ms = worker.gpu_ms_total - g0
        # where the host's CPU went in the timed region (the in-process farm included): cores busy
        # per thread role, this rank's process
        side["rank0_host_cpu_cores_by_thread"] = cpu_cores_by_thread(cpu0, cpu1, t1 - t0)
        wire_bytes = s1["bytes_in"] - s0["bytes_in"]
        errors = s1["errors"] - s0["errors"]
        aus = s1["packets"] - s0["packets"]  # access units through Camera::on_access_unit
        skipped = s1["skipped"] - s0["skipped"]  # AUs the ingest dropped (parse backlog full)
        if farm.sink is not None:
            side["rtmp_passthrough"] = {
                "video_messages": s1["rtmp_messages"] - s0["rtmp_messages"],
                "video_bytes": s1["rtmp_bytes"] - s0["rtmp_bytes"],
                "keyframes": s1["rtmp_keyframes"] - s0["rtmp_keyframes"],
                "messages_per_s": round((s1["rtmp_messages"] - s0["rtmp_messages"]) / elapsed, 1),
                "video_messages_since_start": s1["rtmp_messages"],
                "definition": "FLV video messages the loopback RTMP server received from the cameras' pass-through "
                              "senders during the timed region (packet copy, no transcode)"}
        if annot is not None:
            side["annotation"] = annot.stop()
            side["annotation"]["rate_per_camera_per_s"] = a.annotate_rate
            annot.close()
            annot = None
        if gather:
            verified, checks, rows_checked, bad_rows = check.result(dev)
            side["gather_check"] = {"gather_verified": verified, "checked_gathers": checks, "rows_checked": rows_checked,
                                    "mismatching_rows": bad_rows,
                                    "definition": "every 4th all-gather of the consumer batch also all-gathers each rank's "
                                                  "per-row checksums (int32 words x position weights); every rank compares "
                                                  "them with the checksums of the rows it received (summed over ranks)"}
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            fr = torch.tensor([pictures, frames, dropped, errors, wire_bytes, aus, skipped, shed], dtype=torch.float64,
                              device=dev)
            dist.all_reduce(fr, op=dist.ReduceOp.SUM)
            pictures, frames, dropped, errors, wire_bytes, aus, skipped, shed = (int(v) for v in fr.tolist())
        # latency: every rank's cameras go live (real-time farm) with the production ingest
        # (lossy: a camera that outruns the decoder skips to its next keyframe), rank 0 measures
        if pool is not None or world > 1:
            settled = farm.go_live(a.fps)
            ls0 = farm.stats()["skipped"]
            if world > 1:
                dist.barrier()
            if pool is not None:
                lp0, lt0 = worker.pictures, time.perf_counter()
                lat = measure(pool, worker, farm.idx, duration_s=a.latency_seconds,
                              serve_samples=a.latency_samples, native=a.serving == "native")
                live_fps = (worker.pictures - lp0) / (time.perf_counter() - lt0) / cams
                lat["settled"] = settled
                lat["live_skipped"] = farm.stats()["skipped"] - ls0
            if world > 1:
                dist.barrier()
    finally:
        if annot is not None:
            annot.close()
        farm.close()
        if pool is not None:
            pool.close()
    backend = dist.get_backend() if world > 1 else None
    if world > 1:  # (every collective is done; rank 0's reference-equivalent run needs none)
        dist.destroy_process_group()
    if rank == 0:
        fps = pictures / elapsed
        res = {
            "metric": METRIC,
            "value": round(fps, 2),
            "unit": "frames/s",
            "n_gpus": world if use_gpu else 0,
            "n_ranks": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "frames_per_step": a.frames_per_step,
            "step_definition": f"{a.frames_per_step} frame intervals of every camera: {cams} x {a.frames_per_step} "
                               "decoded pictures per rank",
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "rccl_world": world if (use_gpu and world > 1) else 0,
            "collective_backend": backend,
            "gather_verified": side.get("gather_check", {}).get("gather_verified") if world > 1 else None,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "uint8 (BGR24 frames; bf16-capable consumer path)",
            "data": (f"synthetic {CODEC[a.codec]} camera streams ({describe_streams(a, compressed)}, QP {a.qp}, "
                     f"GOP {a.gop}) served by an in-process loopback RTSP farm (RTP/TCP interleaved, "
                     f"FU-A), unthrottled in the timed region; {wire_bytes * 8 / max(1, aus) * a.fps / 1e6:.1f} "
                     f"Mbit/s per camera at {a.fps} fps"),
            "source": "rtsp",
            "keyframe_only": a.keyframe_only,
            "config": {
                "model": f"{cams * max(world, 1)}x{a.width}x{a.height}p{a.fps} {CODEC[a.codec]} cameras",
                "global_batch": cams * max(world, 1),
                "seq_len": a.gop,
                "parallelism": f"camera-dp{max(world, 1)}",
                "cams_per_gpu": cams,
                "letterbox": a.letterbox,
                "consumer_format": a.consumer_format,
                "all_gather": gather,
                "gathered_bytes_per_rank_per_step": cams * row if gather else 0,
            },
            "frame_count_definition": "pictures the live pipeline decoded (RTSP receive -> RTP "
                                      "depacketize -> host parse -> GPU reconstruct) during the timed "
                                      "region; the newest of each camera's batch is converted to BGR24 "
                                      "and committed to its HBM ring (frames_published); older ones of "
                                      "a catch-up batch are superseded before any client could read them",
            "frames_decoded": pictures,
            "frames_published": frames,
            "access_units_ingested": aus,
            "access_units_per_s": round(aus / elapsed, 1),
            "access_units_skipped": skipped,
            "settle_s": settle_s,
            "ingest_mode": {"timed_region": "lossless: a camera's socket is paused while its parse backlog is deep "
                                            "(TCP back-pressure on the unthrottled farm), so no access unit is "
                                            "skipped by construction",
                            "latency_phase": "lossy (the production default): a camera that outruns its parse "
                                             "drops to its next keyframe; live_phase_access_units_skipped counts them"},
            "frames_dropped": dropped,
            "frames_shed": shed,
            "frames_shed_definition": "outputs not published because the worker shed their reconstruction: a camera "
                                      "whose queued job reached a keyframe restarted from it (GOP catch-up collapse "
                                      "under load); frames_decoded counts only reconstructed pictures",
            "decode_errors": errors,
            "concurrent_clients": a.clients,
            "rank0_gpu_kernel_ms_per_step": round(gpu_ms / a.steps, 4),
            "rank0_pictures_per_launch": round(pictures / max(1, batches), 3),
            "rank0_launches_merged": merged,
            "rank0_record_bytes_gathered_per_step": (rg1 - rg0) // max(1, a.steps),
            "keyframe_coalesce_window_us": worker.kf_window_us if a.keyframe_only else None,
            "parse_threads_per_rank": a.threads,
            "rank0_host_domain": a.host_domain,
            "rocdecode_available": bool(vep.rocdecode_available()),
            "decoder_backend": decoder_backend(a, compressed),
            "per_gpu_fps": round(fps / max(world, 1), 2),
        }
        if os.environ.get("VEP_AVC_PROF") == "1":
            res.update(avc_cycles_per_mb(worker))
        if lat is not None:
            res.update(latency_fields(a, lat, live_fps))
            res["latency_farm_settled"] = lat["settled"]
            res["live_phase_access_units_skipped"] = lat["live_skipped"]
        res.update(side)  # (rank 0's side loads)
        if n_gpus_scope(res):
            res["scope"] = n_gpus_scope(res)
        if use_gpu and not a.cpu and a.ref_cpu == "on":
            res.update(reference_fields(a, res, world))
        elif a.cpu and a.ref_equivalent:
            res["source_definition"] = REF_CPU_DEFINITION
            res["ref_copy_bytes"] = worker.ref_copy_bytes
        print(json.dumps(res), flush=True)
    if dropped or errors:
        print(f"bench: {dropped} frames dropped, {errors} decode errors in the timed region", file=sys.stderr,
              flush=True)
        sys.exit(3)


def payload_path(a, compressed, worker, ip0, sg0, rg0=0, end=None):
    """What reaches the GPU per picture, from the worker's own byte counters (`end`: the
    (in-place, staged, gathered) counters sampled when the timed region ended)."""
    ip1, sg1, rg1 = end or (worker.bytes_inplace, worker.bytes_staged, worker.records_gathered)
    inplace = (ip1 - ip0) // max(1, a.steps)
    staged = (sg1 - sg0) // max(1, a.steps)
    if compressed:
        gathered = (rg1 - rg0) // max(1, a.steps)
        how = ("the H.264 records sit in pinned pool memory and a gather kernel pulls them over PCIe "
               "(no host copy); the H.265 records are copied into the pinned staging buffer and sent H2D"
               if gathered else "copied into the pinned staging buffer by the host and sent H2D per batch")
        return {"gpu_input": "per-macroblock reconstruction records (modes, motion vectors, dequantised "
                             "coefficients) built by the host parse; " + how + "; slice bytes never reach the GPU",
                "record_bytes_gathered_per_step": gathered,
                "slice_bytes_read_in_place_per_step": inplace, "slice_bytes_staged_per_step": staged}
    return {"gpu_input": "I_PCM slice bytes: the decode kernel reads them from pinned host memory over PCIe"
                         if worker.direct_reads else "I_PCM slice bytes gathered into HBM, decode reads HBM",
            "slice_bytes_read_in_place_per_step": inplace, "slice_bytes_staged_per_step": staged}


REF_CPU_DEFINITION = (
    "reference-equivalent CPU path (SURVEY.md §6 / BASELINE.md: FFmpeg, Redis and the Go server cannot run "
    "here): the same cameras, streams, RTSP farm, steps and latency clients, decoded by this repo's CPU backend "
    "on rank 0's host-domain CPUs (its CPU share) - CPU CABAC parse, CPU reconstruction (the portable scalar "
    "bit-exact reference, no SIMD: libavcodec's SIMD decoder is faster, so vs_baseline is an upper bound), CPU "
    "NV12->BGR24 and the read_image.py:97/:119 tobytes + SerializeToString copy chain per published frame; "
    "whole-node value = per-share rate x ranks (each GPU has its own CPU share)")


def reference_equivalent(a):
    """Rank 0, after the GPU measurement: the same command on the CPU backend in a fresh process
    (bench.py --cpu --ref-equivalent) on this rank's host-domain CPUs; its JSON line."""
    import subprocess

    args = [a for a in sys.argv[1:]]
    drop = {"--gpus", "--ref-cpu", "--warmup"}
    out, skip = [], False
    for x in args:
        if skip:
            skip = False
            continue
        key = x.split("=")[0]
        if key in drop:
            skip = "=" not in x
            continue
        out.append(x)
    cmd = [sys.executable, os.path.abspath(__file__), *out, "--cpu", "--ref-equivalent", "--ref-cpu", "off",
           "--warmup", "1"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT") and not k.startswith("TORCHELASTIC")}
    env["VEP_HOST_CPUS"] = a.host_domain["cpulist"]
    t0 = time.perf_counter()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=420)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if not lines:
        return {"error": f"reference-equivalent run failed (rc {r.returncode}): {r.stderr[-400:]}"}
    d = json.loads(lines[-1])
    d["wall_s"] = round(time.perf_counter() - t0, 1)
    return d


def reference_fields(a, res, world):
    """reference_equivalent_cpu_fps and vs_baseline for the GPU run's JSON (rank 0)."""
    ref = reference_equivalent(a)
    if "value" not in ref:
        return {"reference_equivalent": ref}
    per_share = ref["value"]
    node = per_share * max(1, world)
    keep = ("value", "frames_decoded", "frames_published", "decode_errors", "access_units_ingested", "ms_per_step",
            "p50_latency_ms", "p99_latency_ms", "latency_frames_served_per_s", "rank0_host_cpu_cores_by_thread",
            "rank0_host_domain", "steps", "warmup", "wall_s")
    return {
        "reference_equivalent_cpu_fps": round(node, 2),
        "reference_equivalent_cpu_fps_per_share": per_share,
        "reference_equivalent_p50_latency_ms": ref.get("p50_latency_ms"),
        "reference_equivalent_definition": REF_CPU_DEFINITION,
        "reference_equivalent_run": {k: ref.get(k) for k in keep},
        "vs_baseline": round(res["value"] / node, 3) if node > 0 else None,
        "vs_baseline_definition": "value / reference_equivalent_cpu_fps (BASELINE.json publishes no number; "
                                  "this ratio is against the labelled reference-equivalent CPU path above)",
    }


def decoder_backend(a, compressed):
    if compressed and a.codec == "h265":
        return ("native H.265 Main decoder: CPU CABAC coding-tree parse + merge/AMVP into reconstruction "
                "records; gfx950 HIP motion compensation, level-scheduled intra + residual transform blocks, "
                "deblocking, SAO, NV12->BGR24 (rocDecode absent in image)")
    if compressed:
        return ("native H.264 decoder: CPU " + ("CAVLC" if a.profile == "baseline" or a.cavlc else "CABAC") +
                " macroblock-layer parse + dequant; gfx950 HIP motion compensation, intra + deblocking "
                "wavefronts, NV12->BGR24 (rocDecode absent in image)")
    return ("native subset decoder: CPU " + ENTROPY[a.codec] + " parse + gfx950 HIP PCM reconstruct/"
            "NV12->BGR24 (rocDecode absent in image)")


def main():
    a = parse_args()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ and not a.cpu:
        sys.exit(spawn_ranks(a.gpus))
    # rank 0's latency clients: fresh processes, started before this process touches the GPU
    pool = start_client_pool(a) if int(os.environ.get("RANK", "0")) == 0 else None
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = (not a.cpu) and torch.cuda.is_available()
    if world > 1:
        if use_gpu:
            torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl" if use_gpu else "gloo")
    dev = torch.device("cuda", local) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(local)

    from video_edge_ai_proxy_amd import native as vep

    # this rank's host domain (hostplan.h): the node's ranks split the CPUs, each rank's share
    # pinned to its GPU's NUMA-local CPUs and sized from the CPU budget (no constant cap)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    plan_devs = list(range(local_world)) if use_gpu else [-1] * local_world
    # VEP_HOST_CPUS "a-b;c-d;..." (one CPU list per local rank) overrides the NUMA-local plan
    explicit = [x.strip() for x in os.environ["VEP_HOST_CPUS"].split(";")] if os.environ.get("VEP_HOST_CPUS") else []
    dom = vep.plan_host_domains(plan_devs, explicit)[local]
    if a.threads > 0:
        dom["parse_threads"] = a.threads
    a.threads = dom["parse_threads"]
    a.host_domain = {k: dom[k] for k in ("cpulist", "numa_node", "pci_bus_id", "cpu_share", "parse_threads",
                                         "io_threads", "source")}
    cams = a.cams_per_gpu
    S = a.letterbox
    worker = vep.Worker(device=local if use_gpu else -1, letterbox_size=S, chw_dtype=0,
                        max_cameras=cams, pack_threads=a.pack_threads,
                        letterbox_format=1 if a.consumer_format == "nv12" else 0, lanes=a.lanes,
                        stages=a.stages, queue=a.lane_queue, host_domain=dom,
                        ref_copies=bool(a.cpu and a.ref_equivalent), backpressure=bool(a.cpu and a.ref_equivalent))
    row = S * S * 3 // 2 if a.consumer_format == "nv12" else S * S * 3
    compressed = a.content == "avc"  # (h265: general HEVC Main streams, CPU reconstruction)
    cfg = make_cfg(vep, a, rank, compressed)
    stream_desc = describe_streams(a, compressed)
    if a.source == "rtsp":
        return run_rtsp(a, vep, torch, dist, worker, world, rank, use_gpu, dev, row, compressed, pool)
    rb = vep.ReplayBench(worker, cams, cfg, cached_frames=a.gop * a.cache_gops, threads=a.threads,
                         ring_slots=a.ring_slots, prefix=f"r{rank}cam", window=a.parse_window,
                         records=a.source == "records")

    # The native worker keeps up to `worker.inflight` ticks per lane launched but unpublished,
    # and one all-gather may still be reading an older tick: inflight + 2 consumer buffers.
    LAG = worker.inflight if use_gpu else 0
    NB = LAG + 2
    bufs = [torch.empty((cams, row), dtype=torch.uint8, device=dev) for _ in range(NB)]
    gather = world > 1 and not a.no_gather
    gathered = [torch.empty((world * cams, row), dtype=torch.uint8, device=dev)
                for _ in range(NB)] if gather else None
    handles = [None] * NB
    check = GatherCheck(torch, dist, world, cams, row, dev, NB) if gather else None
    side = {}
    F = a.frames_per_step
    pending = []  # ticks launched whose consumer batch has not been handed to the gather yet
    seq_of = {}   # tick -> the worker's launch sequence (lane threads publish asynchronously)

    def sync():
        if use_gpu:
            torch.cuda.synchronize()

    def issue_gather(t):
        k = t % NB
        seq = seq_of.pop(t)
        if gather:
            worker.wait_published(seq)  # every lane has written tick t's letterbox rows
            handles[k] = dist.all_gather_into_tensor(gathered[k], bufs[k], async_op=True)
            check.issue(k, bufs[k])

    def step(i):
        b = i % NB
        if handles[b] is not None:  # buffer b may still feed the all-gather of tick i - NB
            handles[b].wait()
            handles[b] = None
            check.verify(b, gathered[b])
            sync()
        worker.set_consumer_buffers(bufs[b].data_ptr(), 0, cams)
        rb.step()  # enqueues tick i
        seq_of[i] = worker.launch_seq if use_gpu else 0
        pending.append(i)
        while pending and pending[0] <= i - LAG:
            issue_gather(pending.pop(0))

    def drain():
        rb.drain()  # publishes every launched tick
        while pending:
            issue_gather(pending.pop(0))
        for k in range(NB):
            if handles[k] is not None:
                handles[k].wait()
                handles[k] = None
                check.verify(k, gathered[k])
        sync()

    for i in range(a.warmup * F):
        step(i)
    # the parse pipeline runs ahead of the launched tick: launch what it has already parsed and
    # stop it, so every tick of the timed region is parsed inside the timed region
    rb.quiesce()
    drain()
    if world > 1:
        dist.barrier()
    sync()
    f0, p0, b0, g0 = worker.frames, rb.parse_ms, rb.batch_ms, worker.gpu_ms_total
    d0, pf0, l0 = worker.dropped, rb.parse_failures, rb.frames
    pw0 = rb.parse_wait_ms
    ip0, sg0, rg0 = worker.bytes_inplace, worker.bytes_staged, worker.records_gathered
    tm0 = worker.timings()
    t0 = time.perf_counter()
    for i in range(a.steps * F):  # (a step: F ticks, one frame interval of every camera each)
        step(a.warmup * F + i)
    drain()
    t1 = time.perf_counter()
    end_bytes = (worker.bytes_inplace, worker.bytes_staged, worker.records_gathered)
    # frames committed to the camera rings (readable by clients), not jobs launched; sampled at the
    # end of this rank's timed region, before the barrier
    frames = worker.frames - f0
    launched = rb.frames - l0
    dropped = (worker.dropped - d0) + (rb.parse_failures - pf0)
    parse_ms, batch_ms, gpu_ms = rb.parse_ms - p0, rb.batch_ms - b0, worker.gpu_ms_total - g0
    parse_wait_ms = rb.parse_wait_ms - pw0
    tm1 = worker.timings()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    if gather:
        verified, checks, rows_checked, bad_rows = check.result(dev)
        side["gather_check"] = {"gather_verified": verified, "checked_gathers": checks, "rows_checked": rows_checked,
                                "mismatching_rows": bad_rows}
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        fr = torch.tensor([frames, dropped, launched], dtype=torch.float64, device=dev)
        dist.all_reduce(fr, op=dist.ReduceOp.SUM)
        frames, dropped, launched = (int(v) for v in fr.tolist())

    lat = None
    if pool is not None:
        from vep_bench.bench_latency import measure, ticking

        # cameras decode at their frame rate meanwhile; the single-process tick must not touch
        # the collective: decode-only ticks here
        worker.set_consumer_buffers(bufs[0].data_ptr(), 0, cams)
        with ticking(lambda: (rb.step(), rb.drain()), float(a.fps)):
            time.sleep(0.5)
            lat = measure(pool, worker, list(rb.cameras), duration_s=a.latency_seconds,
                          serve_samples=a.latency_samples, native=a.serving == "native")
        pool.close()
    if world > 1:
        dist.barrier()

    bitrate_mbps = rb.stream_bytes * 8 / max(1, rb.stream_frames) * a.fps / 1e6
    if rank == 0:
        fps = frames / elapsed
        res = {
            "metric": METRIC,
            "value": round(fps, 2),
            "unit": "frames/s",
            "n_gpus": world if use_gpu else 0,
            "n_ranks": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "frames_per_step": a.frames_per_step,
            "step_definition": f"{a.frames_per_step} frame intervals of every camera: {cams} x {a.frames_per_step} "
                               "decoded pictures per rank",
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "rccl_world": world if (use_gpu and world > 1) else 0,
            "collective_backend": (dist.get_backend() if world > 1 else None),
            "gather_verified": side.get("gather_check", {}).get("gather_verified") if world > 1 else None,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "uint8 (BGR24 frames; bf16-capable consumer path)",
            "data": (f"synthetic compressed {CODEC[a.codec]} camera streams ({stream_desc}, QP {a.qp}, GOP "
                     f"{a.gop}, {bitrate_mbps:.1f} Mbit/s per camera: textured scene, moving objects, "
                     "sensor noise), pre-encoded per camera and replayed" if compressed else
                     f"synthetic {CODEC[a.codec]} I_PCM/P_Skip fast-path streams (random-noise "
                     f"background + moving object, GOP {a.gop}, {a.motion:.0%} motion), pre-encoded "
                     "per camera and replayed"),
            "config": {
                "model": f"{cams * max(world, 1)}x{a.width}x{a.height}p{a.fps} {CODEC[a.codec]} cameras",
                "global_batch": cams * max(world, 1),
                "seq_len": a.gop,
                "parallelism": f"camera-dp{max(world, 1)}",
                "cams_per_gpu": cams,
                "letterbox": S,
                "consumer_format": a.consumer_format,
                "gathered_bytes_per_rank_per_step": cams * row if gather else 0,
                "all_gather": gather,
            },
            "rocdecode_available": bool(vep.rocdecode_available()),
            "decoder_backend": decoder_backend(a, compressed),
            "source": ("records (GPU-side ceiling: each camera's looped GOPs parsed once before the timed "
                       "region; the timed loop replays the parsed reconstruction jobs - records gathered over "
                       "PCIe, GPU reconstruction, BGR24, ring publish, letterbox - with no host parse)"
                       if a.source == "records" else
                       "replay (decode-only: pre-encoded access units fed to the parse pool; no RTSP "
                       "receive / depacketization in the timed region)"),
            "per_gpu_fps": round(fps / max(world, 1), 2),
            "frames_published": frames,
            "frames_launched": launched,
            "frames_dropped": dropped,
            "frame_count_definition": "frames committed to camera HBM rings during the timed "
                                      "region (parse -> GPU reconstruct -> BGR24 -> ring publish); "
                                      "dropped = parse failures + frames the worker did not publish",
            "rank0_host_parse_ms_per_step": round(parse_ms / a.steps, 4),
            "rank0_parse_wait_ms_per_step": round(parse_wait_ms / a.steps, 4),
            "rank0_batch_ms_per_step": round(batch_ms / a.steps, 4),
            "rank0_gpu_kernel_ms_per_step": round(gpu_ms / a.steps, 4),
            "gpu_lanes": worker.lanes,
            "parse_threads_per_rank": a.threads,
            "rank0_host_domain": a.host_domain,
            "gpu_stages": worker.stages,
            "gpu_inflight_per_lane": worker.inflight,
            "payload_path": payload_path(a, compressed, worker, ip0, sg0, rg0, end_bytes),
            "rank0_launch_breakdown_ms_per_step": {
                k: round((v - tm0[k]) / a.steps, 4) for k, v in tm1.items()},
        }
        if os.environ.get("VEP_AVC_PROF") == "1":
            res.update(avc_cycles_per_mb(worker))
        if lat is not None:
            res.update(latency_fields(a, lat))
        res.update(side)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if dropped:
        print(f"bench: {dropped} frames dropped in the timed region", file=sys.stderr, flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
