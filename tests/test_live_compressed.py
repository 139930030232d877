"""Live compressed streams end to end (CPU backend; the GPU twin is in test_gpu_integration.py):
loopback RTSP farm (RTP over TCP, FU-A fragmentation) -> native IngestSession -> the lazy
decoder (fast path first, switching to the general H.264 decoder on first contact) -> the
camera's frame ring. Every published frame is compared, pixel for pixel, with the CPU reference
decoder's output for the same access unit — Baseline CAVLC and High-profile CABAC IBBP, GOP
catch-up after a late first query, keyframe-only mode, the idle cutoff and 1080p IDRs that
arrive as dozens of FU-A fragments.

Reference behaviour: python/read_image.py:57-128 (decode on demand, keyframe-only, idle stop),
python/rtsp_to_rtmp.py:61-92 (RTSP ingest)."""
import threading
import time

import numpy as np
import pytest

FPS = 60  # realtime pacing of the farm (fast, but each AU still crosses the socket in order)


def stream_cfg(native, profile, w=320, h=240, gop=10, seed=21):
    c = native.SynthConfig()
    c.width, c.height, c.gop, c.fps, c.seed = w, h, gop, FPS, seed
    c.compressed = True
    c.profile = profile
    c.bframes = 2
    c.objects = 3
    c.temporal_noise = 1.0
    return c


def reference(native, cfg, n_cached, loops=2):
    """Newest output frame (BGR) after each AU of the looped cache, keyed by coding index k
    (the farm stamps RTP time k * 90000 / fps on the k-th AU it sends)."""
    enc = native.SynthH264(cfg)
    aus = [enc.next() for _ in range(n_cached)]
    dec = native.CpuDecoder()
    ref = {}
    step = 90000 // cfg.fps
    for k in range(n_cached * loops):
        a = aus[k % n_cached]
        au = native.AccessUnit.from_nals(a.nals(), pts=k * step, dts=k * step, keyframe=a.keyframe)
        img = dec.decode(au)
        if img is not None:
            ref[dec.last_pts // step] = img
    return ref, aus


def ref_index(k, n_cached):
    # the stream is a loop of n_cached AUs starting at an IDR: from the second pass on every
    # pass decodes exactly like the second one
    return k if k < 2 * n_cached else n_cached + (k - n_cached) % n_cached


class Live:
    def __init__(self, native, cfg, n_cached, touch=True, keyframe_only=False, device=-1):
        self.srv = native.RtspServer("127.0.0.1", 0)
        self.srv.add_stream("/cam", cfg, realtime=True, cached_frames=n_cached)
        self.srv.start()
        self.w = native.Worker(device=device)
        self.w.start()
        self.cam = self.w.add_camera("live", 4)
        self.w.set_keyframe_only(self.cam, keyframe_only)
        self.touching = touch
        self.stop_evt = threading.Event()
        if touch:
            self.w.set_last_query(self.cam, int(time.time() * 1000))
        self.toucher = threading.Thread(target=self._touch_loop, daemon=True)
        self.toucher.start()
        self.sess = native.IngestSession(self.w, self.cam, "live", f"rtsp://127.0.0.1:{self.srv.port}/cam")
        self.sess.start()

    def _touch_loop(self):
        while not self.stop_evt.wait(0.05):
            if self.touching:
                self.w.set_last_query(self.cam, int(time.time() * 1000))

    def frames(self, seconds, max_frames=1000):
        """(pts, BGR, meta) of every frame newer than the previous read, until `max_frames` were
        read or `seconds` passed (a deadline for a frame count, so a loaded host only slows the
        test down)."""
        out, seq = [], 0
        end = time.time() + seconds
        while time.time() < end and len(out) < max_frames:
            r = self.w.read_latest(self.cam, seq)
            if r is None:
                time.sleep(0.002)
                continue
            meta, img = r
            seq = meta["seq"]
            out.append((meta["pts"], img.copy(), meta))
        return out

    def close(self):
        self.stop_evt.set()
        self.sess.stop()
        self.srv.stop()
        self.w.stop()


def check_frames(got, ref, n_cached, step):
    assert got, "no frame published"
    for pts, img, meta in got:
        k = pts // step
        want = ref.get(ref_index(k, n_cached))
        assert want is not None, f"AU {k}: the reference decoder outputs no frame there"
        assert np.array_equal(img, want), f"AU {k} ({meta['frame_type']}) differs in {int((img != want).sum())} samples"


@pytest.mark.parametrize("profile", ["baseline", "high"])
def test_live_compressed_stream_bit_exact(native, profile):
    """Compressed CAVLC (Baseline) and CABAC IBBP (High) cameras through the whole live path:
    the camera starts on the fast path, switches to the general decoder on first contact, and
    every frame it publishes equals the reference decoder's."""
    n = 20
    cfg = stream_cfg(native, profile)
    ref, _ = reference(native, cfg, n, loops=4)
    live = Live(native, cfg, n)
    try:
        got = live.frames(60, max_frames=15)
        st = live.w.stats(live.cam)
    finally:
        live.close()
    assert st["errors"] == 0 and st["skipped"] == 0, (st, live.w.logs(live.cam, True, 20))
    check_frames(got, ref, n, 90000 // FPS)
    assert len(got) >= 15 and st["decoder"] == "general" and st["errors"] == 0
    if profile == "high":
        assert {m["frame_type"] for _, _, m in got} >= {"B", "P"}


@pytest.mark.parametrize("device", [-1, pytest.param(0, marks=pytest.mark.gpu)])
@pytest.mark.parametrize("chunk", [2, 3, 4, 5, 6, 7, 9, 11])
def test_backlog_across_idr_publishes_the_output_picture(native, chunk, device):
    """A worker that falls behind merges a camera's queued jobs into one (GOP catch-up collapse);
    a backlog that reaches an IDR restarts from it (the queued pictures are dropped). The IDR
    bumps the previous GOP's pictures out of the reorder buffer: a frame whose reconstruction was
    dropped must not be published (it would be a stale surface). Deterministic twin of a live-farm
    flake ("AU 27 (P) differs") that showed up only on a loaded host."""
    n = 20
    cfg = stream_cfg(native, "high")
    ref, aus = reference(native, cfg, n, loops=2)
    step = 90000 // cfg.fps
    wk = native.Worker(device=device)
    cam = wk.add_camera("backlog", 4)
    seq, checked = 0, 0
    for k0 in range(0, 2 * n, chunk):
        batch = []
        for k in range(k0, min(k0 + chunk, 2 * n)):
            a = aus[k % n]
            batch.append(native.AccessUnit.from_nals(a.nals(), pts=k * step, dts=k * step, keyframe=a.keyframe))
        wk.decode_many([(cam, batch)])  # one merged job per chunk
        r = wk.read_latest(cam, seq)
        if r is None:
            continue
        meta, img = r
        seq = meta["seq"]
        k = meta["pts"] // step
        assert np.array_equal(img, ref[k]), f"chunk ending at AU {k0 + chunk - 1}: AU {k} ({meta['frame_type']}) stale"
        checked += 1
    assert checked >= 2 * n // chunk - 5  # (a chunk that crosses an IDR may publish nothing)


def test_live_gop_catch_up_after_late_query(native):
    """No client for the first half second (nothing decoded), then a query mid-GOP: the lazy
    decoder catches up from the GOP's keyframe and the first frame it publishes is already the
    correct current picture (its references were reconstructed in the same batch)."""
    n = 30
    cfg = stream_cfg(native, "high", gop=30)
    ref, _ = reference(native, cfg, n, loops=3)
    live = Live(native, cfg, n, touch=False)
    try:
        # wait (by AU count, not wall clock) until the camera is 14..24 AUs into a GOP (B pictures:
        # output trails coding order by a few pictures)
        deadline = time.time() + 60
        while time.time() < deadline and not 14 <= live.w.stats(live.cam)["packets"] % n <= 24:
            time.sleep(0.005)
        assert live.w.stats(live.cam)["decoded"] == 0  # no last_query yet: nothing decoded
        p0 = live.w.stats(live.cam)["packets"]
        live.touching = True
        live.w.set_last_query(live.cam, int(time.time() * 1000))
        got = live.frames(60, max_frames=3)
    finally:
        live.close()
    check_frames(got, ref, n, 90000 // FPS)
    first_k = got[0][0] // (90000 // FPS)
    # the first published frame is the current picture (output trails coding order by <= 2 B
    # pictures), not the GOP's keyframe or an early picture of it. Relative to the AU count at the
    # query, so a loaded host that lets the stream cross into the next GOP meanwhile still passes.
    assert first_k >= p0 - 4, f"first published frame {first_k} trails the stream ({p0} AUs at the query)"
    if first_k // n == p0 // n:
        assert first_k % n > 5, "the first published frame should be well inside the GOP (catch-up)"


def test_live_keyframe_only(native):
    """keyframe_only (VideoLatestImage key_frame_only): only IDR pictures are reconstructed and
    published, each equal to the reference decoder's IDR picture."""
    n = 20
    cfg = stream_cfg(native, "high")
    ref, aus = reference(native, cfg, n, loops=4)
    live = Live(native, cfg, n, keyframe_only=True)
    try:
        got = live.frames(1.2)
    finally:
        live.close()
    step = 90000 // FPS
    assert got
    for pts, img, meta in got:
        k = pts // step
        assert aus[k % n].keyframe and meta["frame_type"] == "I", f"AU {k} is not a keyframe"
    # an IDR picture is output with its own AU only once the reorder buffer lets it out: compare
    # against the reference picture decoded from that IDR alone
    for pts, img, meta in got:
        k = pts // step
        dec = native.CpuDecoder()
        a = aus[k % n]
        out = dec.decode(native.AccessUnit.from_nals(a.nals(), pts=pts, keyframe=True))
        if out is None:
            out = dec.flush()[-1]
        assert np.array_equal(img, out)


def test_live_idle_cutoff_stops_decoding(native):
    """The camera stops decoding once no client has asked for idle_cutoff_ms (10 s in the
    reference, read_image.py:77-78; shortened here) and resumes on the next query."""
    n = 20
    cfg = stream_cfg(native, "baseline")
    live = Live(native, cfg, n)
    try:
        live.w.set_idle_cutoff_ms(live.cam, 300)
        live.frames(0.4)
        live.touching = False
        time.sleep(0.6)  # past the cutoff
        d0 = live.w.stats(live.cam)["decoded"]
        time.sleep(0.5)
        d1 = live.w.stats(live.cam)["decoded"]
        assert d1 == d0, "decoding continued after the idle cutoff"
        live.touching = True
        live.w.set_last_query(live.cam, int(time.time() * 1000))
        time.sleep(0.5)
        assert live.w.stats(live.cam)["decoded"] > d1
    finally:
        live.close()


def test_live_1080p_fu_a_idr(native):
    """1080p compressed IDRs (~100+ kB) arrive as dozens of FU-A fragments; the reassembled
    pictures decode bit-exact."""
    n = 8
    c = native.SynthConfig()
    c.width, c.height, c.gop, c.fps, c.seed = 1920, 1080, 4, 10, 5
    c.compressed = True
    c.temporal_noise = 2.0
    c.qp = 24
    enc = native.SynthH264(c)
    aus = [enc.next() for _ in range(n)]
    assert max(a.size for a in aus if a.keyframe) > 60000
    dec = native.CpuDecoder()
    ref = {}
    for k in range(2 * n):
        a = aus[k % n]
        ref[k] = dec.decode(native.AccessUnit.from_nals(a.nals(), pts=k * 9000, keyframe=a.keyframe))
    srv = native.RtspServer("127.0.0.1", 0)
    srv.add_stream("/hd", c, realtime=True, cached_frames=n)
    srv.start()
    w = native.Worker(device=-1)
    w.start()
    cam = w.add_camera("hd", 2)
    w.set_last_query(cam, int(time.time() * 1000) + 60000)
    sess = native.IngestSession(w, cam, "hd", f"rtsp://127.0.0.1:{srv.port}/hd")
    sess.start()
    got, seq = [], 0
    try:
        end = time.time() + 12.0  # (CPU decode of 1080p: slow when the suite runs in parallel)
        while time.time() < end and len(got) < 6:
            r = w.read_latest(cam, seq)
            if r is None:
                time.sleep(0.005)
                continue
            meta, img = r
            seq = meta["seq"]
            got.append((meta["pts"] // 9000, img.copy()))
    finally:
        sess.stop()
        srv.stop()
        w.stop()
    assert len(got) >= 3
    for k, img in got:
        want = ref[k if k < 2 * n else n + (k - n) % n]
        assert np.array_equal(img, want), f"AU {k} differs"


def test_rtmp_passthrough_never_stalls_ingest(native):
    """RTMP pass-through runs on its own sender thread with a bounded queue: a server that
    accepts the TCP connection and then never answers the handshake (the worst case: every send
    blocks until the timeout) does not slow the camera's ingest or decoding."""
    import socket

    hang = socket.socket()
    hang.bind(("127.0.0.1", 0))
    hang.listen(4)
    port = hang.getsockname()[1]
    accepted = []
    threading.Thread(target=lambda: accepted.append(hang.accept()), daemon=True).start()
    n = 20
    cfg = stream_cfg(native, "baseline")
    srv = native.RtspServer("127.0.0.1", 0)
    srv.add_stream("/cam", cfg, realtime=True, cached_frames=n)
    srv.start()
    w = native.Worker(device=-1)
    w.start()
    cam = w.add_camera("px", 2)
    w.set_last_query(cam, int(time.time() * 1000) + 60000)
    w.set_proxy(cam, True)
    # a long socket timeout: were the camera's decode behind the blocked handshake, it would make
    # no progress for 30 s, far beyond the catch-up deadline below
    sess = native.IngestSession(w, cam, "px", f"rtsp://127.0.0.1:{srv.port}/cam",
                                rtmp_url=f"rtmp://127.0.0.1:{port}/live/px", timeout_ms=30000)
    sess.start()
    try:
        deadline = time.time() + 60
        while time.time() < deadline and sess.state()["aus"] < 20:
            time.sleep(0.01)
        d0, a0 = w.stats(cam)["decoded"], sess.state()["aus"]
        # the RTMP handshake hangs all this time: 60 more AUs must arrive AND be decoded
        while time.time() < deadline and sess.state()["aus"] - a0 < 60:
            time.sleep(0.01)
        a1 = sess.state()["aus"]
        # the decode of those AUs (deadline-bounded: a loaded host only slows it down)
        catch_up = time.time() + 10
        while time.time() < catch_up and w.stats(cam)["decoded"] - d0 < 0.8 * (a1 - a0):
            time.sleep(0.01)
        d1 = w.stats(cam)["decoded"]
        diag = (w.stats(cam), w.logs(cam, True, 20), w.logs(cam, False, 20), native.ingest_pool_stats()
                if hasattr(native, "ingest_pool_stats") else None)
    finally:
        sess.stop()
        srv.stop()
        w.stop()
        hang.close()
    assert accepted, "the pass-through never tried to connect"
    assert a1 - a0 >= 60, f"ingest stalled behind RTMP: {a1 - a0} AUs"
    assert d1 - d0 >= 0.8 * (a1 - a0), f"decoding stalled behind RTMP: {d1 - d0} frames for {a1 - a0} AUs: {diag}"


def hevc_reference(native, cfg, n_cached, loops=4):
    """H.265 twin of reference(): newest output frame (BGR) per coding index of the looped cache."""
    enc = native.SynthH264(cfg)
    aus = [enc.next() for _ in range(n_cached)]
    dec = native.HevcDecoder()
    ref = {}
    step = 90000 // cfg.fps
    for k in range(n_cached * loops):
        a = aus[k % n_cached]
        au = native.AccessUnit.from_nals(a.nals(), pts=k * step, dts=k * step, keyframe=a.keyframe, codec=1)
        for pts, poc, t, (y, uv) in dec.decode(au):
            ref[pts // step] = native.nv12_to_bgr_cpu(y, uv, 0, 0, cfg.width, cfg.height)
    return ref


def test_live_hevc_stream_bit_exact(native):
    """A compressed H.265 Main camera (CABAC I/P/B) through the live path: RTSP (RFC 7798 FU
    fragmentation) -> fast-path attempt -> general HEVC decoder in records mode -> worker (CPU
    mirror here, gfx950 kernels in the GPU twin) -> ring; every published frame equals the
    reference decoder's."""
    n = 20
    cfg = stream_cfg(native, "main", w=320, h=240)
    cfg.codec = "h265"
    ref = hevc_reference(native, cfg, n)
    live = Live(native, cfg, n)
    try:
        got = live.frames(60, max_frames=15)
        st = live.w.stats(live.cam)
    finally:
        live.close()
    assert st["errors"] == 0 and st["skipped"] == 0, (st, live.w.logs(live.cam, True, 20))
    check_frames(got, ref, n, 90000 // FPS)
    assert len(got) >= 15 and st["decoder"] == "general" and st["errors"] == 0
