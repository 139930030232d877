import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu_count():
    try:
        from video_edge_ai_proxy_amd import native

        return native.device_count()
    except Exception:
        return 0


def pytest_collection_modifyitems(config, items):
    if _gpu_count() > 0:
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def native():
    from video_edge_ai_proxy_amd import native as n

    return n


def synth(native, w=640, h=480, gop=10, motion=0.05, seed=1, slices=1, zero=False, fps=30,
          codec="h264", merge_cands=1, compressed=False, coverage=False, refs=1, qp=28,
          deblock_idc=0, objects=3):
    c = native.SynthConfig()
    c.width, c.height, c.gop, c.motion, c.seed, c.slices, c.fps = w, h, gop, motion, seed, slices, fps
    c.zero_samples = zero
    c.codec = codec
    c.merge_cands = merge_cands
    c.compressed, c.coverage, c.refs, c.qp = compressed, coverage, refs, qp
    c.deblock_idc, c.objects = deblock_idc, objects
    return native.SynthH264(c)


def check_surface(wk, cam, pts, full, w, h, cf=1):
    """The DPB surface behind camera `cam`'s newest published frame (Worker.read_surface: full
    sample depth, before the 8-bit narrowing for BGR24) equals the encoder's reconstruction of that
    picture, `full[pts]` = (y, uv) coded planes (uint16 above 8 bits; 4:2:2 chroma has h rows).
    Returns the luma plane read back."""
    import numpy as np

    r = wk.read_surface(cam)
    assert r is not None, "no surface for the published frame"
    spts, (y, uv) = r
    assert spts == pts, (spts, pts)
    wy, wuv = full[pts]
    assert y.dtype == wy.dtype, (y.dtype, wy.dtype)
    ch = h if cf == 2 else h // 2
    dy = y[:h, :w] != wy[:h, :w]
    assert not dy.any(), f"pts {pts}: {int(dy.sum())} luma samples differ at full depth"
    duv = uv[:ch, :w] != wuv[:ch, :w]
    assert not duv.any(), f"pts {pts}: {int(duv.sum())} chroma samples differ at full depth"
    return y[:h, :w]


def high_encoder(native, w=176, h=144, **kw):
    """Main / High-profile synthetic encoder (avc::AvcHighEncoder); kw = AvcHighConfig fields."""
    c = native.AvcHighConfig()
    c.width, c.height = w, h
    for k, v in kw.items():
        if not hasattr(c, k):
            raise AttributeError(k)
        setattr(c, k, v)
    return native.AvcHighEncoder(c)


def roundtrip(native, enc, n):
    """Encode n pictures and decode them on the CPU: ({pts: encoder NV12}, {pts: decoder NV12},
    decoder, access units). Decoder frames are collected from every reorder-buffer output."""
    dec = native.CpuDecoder()
    rec, got, aus = {}, {}, []
    for _ in range(n):
        au = enc.next()
        aus.append(au)
        y, uv = enc.picture()
        rec[enc.last_pts] = (y.copy(), uv.copy())
        dec.decode(au)
        for pts, planes in dec.frames():
            got[pts] = planes
    for pts, planes in dec.flush_frames():
        got[pts] = planes
    return rec, got, dec, aus
