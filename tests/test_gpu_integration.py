"""Live path on the GPU: RTSP farm -> native ingest -> gfx950 decode -> gRPC frames."""
import time

import numpy as np
import pytest

from conftest import synth

pytestmark = pytest.mark.gpu


def test_live_rtsp_to_grpc_on_gpu(native, tmp_path):
    from video_edge_ai_proxy_amd.config import Config
    from video_edge_ai_proxy_amd.models import StreamProcess
    from video_edge_ai_proxy_amd.server.app import build_app
    from video_edge_ai_proxy_amd.server.grpc_server import ImageClient

    srv = native.RtspServer("127.0.0.1", 0)
    cfg = native.SynthConfig()
    cfg.width, cfg.height, cfg.gop, cfg.seed = 1920, 1080, 15, 21
    srv.add_stream("/hd", cfg, realtime=True, cached_frames=30)
    srv.start()
    c = Config()
    c.data_dir = str(tmp_path)
    c.gpu.devices = [0]
    c.gpu.letterbox_size = 640
    app = build_app(c, host="127.0.0.1", rest_port=0, grpc_port=0, start_rest=False)
    try:
        app.pm.start(StreamProcess(name="hd", rtsp_endpoint=f"rtsp://127.0.0.1:{srv.port}/hd"))
        cli = ImageClient(f"127.0.0.1:{app.grpc_port}")
        vf = None
        t0 = time.time()
        while time.time() - t0 < 20:
            vf = cli.latest_frame("hd")
            if vf.width:
                break
            time.sleep(0.1)
        assert vf.width == 1920 and vf.height == 1080
        img = np.frombuffer(vf.data, np.uint8).reshape(1080, 1920, 3)
        ref = synth(native, 1920, 1080, gop=15, seed=21)
        dec = native.CpuDecoder()
        pics = [dec.decode(ref.next()) for _ in range(30)]
        assert any(np.array_equal(img, p) for p in pics)
        frames = [cli.latest_frame("hd") for _ in range(10)]
        assert all(f.width == 1920 for f in frames)
        st = app.hub.state("hd")
        assert st["decoded"] >= 10 and st["errors"] == 0 and st["device"] == 0
        cli.close()
    finally:
        app.stop()
        srv.stop()


@pytest.mark.parametrize("profile", ["baseline", "high"])
def test_live_compressed_rtsp_on_gpu(native, profile):
    """Compressed live cameras (CAVLC Baseline, CABAC IBBP High) through RTSP ingest on the
    gfx950 path: every published frame equals the CPU reference decoder's (test_live_compressed
    is the CPU-backend twin)."""
    from test_live_compressed import FPS, Live, check_frames, reference, stream_cfg

    n = 20
    cfg = stream_cfg(native, profile, w=640, h=360)
    ref, _ = reference(native, cfg, n, loops=4)
    live = Live(native, cfg, n, device=0)
    try:
        got = live.frames(1.5)
        st = live.w.stats(live.cam)
    finally:
        live.close()
    check_frames(got, ref, n, 90000 // FPS)
    assert len(got) >= 15 and st["decoder"] == "general" and st["errors"] == 0


def test_live_hevc_rtsp_on_gpu(native):
    """A compressed H.265 Main camera through RTSP ingest on the gfx950 HEVC kernels: every
    published frame equals the CPU reference decoder's."""
    from test_live_compressed import FPS, Live, check_frames, hevc_reference, stream_cfg

    n = 20
    cfg = stream_cfg(native, "main", w=640, h=360)
    cfg.codec = "h265"
    ref = hevc_reference(native, cfg, n)
    live = Live(native, cfg, n, device=0)
    try:
        got = live.frames(1.5)
        st = live.w.stats(live.cam)
    finally:
        live.close()
    check_frames(got, ref, n, 90000 // FPS)
    assert len(got) >= 15 and st["decoder"] == "general" and st["errors"] == 0

