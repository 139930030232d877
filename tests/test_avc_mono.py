"""4:0:0 (monochrome) H.264, High profile: no chroma syntax in the macroblock layer (no
intra_chroma_pred_mode, the luma-only coded_block_pattern mapping of Table 9-4, 256-byte I_PCM),
CropUnit 1. The decoder keeps the chroma planes at 128 (grey): intra DC without neighbours, motion
compensation from grey references, default weights and deblocking all leave 128 unchanged, so the
GPU kernels need no 4:0:0 variant. Closed loop against the High encoder's `mono` mode (CAVLC and
CABAC, B pictures, coverage mode), then the camera runtime on the CPU backend and on
gfx950. Parity note: the 4:0:0 coded_block_pattern tables are transcribed from the standard's
Table 9-4 from memory; no third-party decoder in the image pins them."""
import numpy as np
import pytest


def mono_cfg(native, cabac, **kw):
    c = native.SynthConfig()
    c.width, c.height, c.gop, c.fps, c.seed = 176, 144, 8, 30, 5
    c.compressed = True
    c.profile = "high"
    c.cabac = cabac
    c.mono = True
    c.bframes = kw.pop("bframes", 2)
    for k, v in kw.items():
        setattr(c, k, v)
    return c


CASES = [dict(cabac=True), dict(cabac=False), dict(cabac=True, coverage=True), dict(cabac=False, coverage=True),
         dict(cabac=True, bframes=0)]
IDS = ["cabac", "cavlc", "cabac-coverage", "cavlc-coverage", "cabac-p"]


@pytest.mark.parametrize("kw", CASES, ids=IDS)
def test_mono_closed_loop(native, kw):
    kw = dict(kw)
    cabac = kw.pop("cabac")
    enc = native.SynthH264(mono_cfg(native, cabac, **kw))
    dec = native.CpuDecoder()
    for i in range(16):
        au = enc.next()
        dec.decode(au)
        y, uv = enc.picture()
        gy, guv = dec.surface()
        if dec.last_pts != enc.last_pts:
            continue  # (B reordering: compare when the decoder's newest output is this picture)
        assert np.array_equal(y, gy), f"AU {i}: luma"
        assert (guv == 128).all(), f"AU {i}: chroma not grey"
    assert dec.general


def _run_worker(native, device, kw):
    kw = dict(kw)
    cabac = kw.pop("cabac")
    cfg = mono_cfg(native, cabac, **kw)
    enc = native.SynthH264(cfg)
    ref = native.CpuDecoder()
    aus, want = [], {}
    for _ in range(16):
        au = enc.next()
        aus.append(au)
        img = ref.decode(au)
        if img is not None:
            want[ref.last_pts] = img
    wk = native.Worker(device=device)
    cam = wk.add_camera("mono", 4)
    seq, checked = 0, 0
    for au in aus:
        wk.decode_now(cam, au)
        r = wk.read_latest(cam, seq)
        if r is None:
            continue
        meta, got = r
        seq = meta["seq"]
        assert np.array_equal(got, want[meta["pts"]]), f"pts {meta['pts']}"
        b, g, rr = (got[..., k].astype(int) for k in range(3))
        assert (np.abs(b - g) <= 1).all() and (np.abs(g - rr) <= 1).all(), "a grey picture is not grey"
        checked += 1
    assert checked >= 12 and wk.stats(cam)["decoder"] == "general"


@pytest.mark.parametrize("kw", CASES[:3], ids=IDS[:3])
def test_mono_camera_cpu_backend(native, kw):
    _run_worker(native, -1, kw)


@pytest.mark.gpu
@pytest.mark.parametrize("kw", CASES, ids=IDS)
def test_mono_camera_gpu_bit_exact(native, kw):
    _run_worker(native, 0, kw)
