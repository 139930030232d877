"""VCN decoder backend (csrc/vep/vcn.cpp): cameras decoded through the rocDecode API.

The image ships no librocdecode and the video core cannot be reached from it, so VCN itself is
unmeasured here. These tests load `tests/native/libvep_rocdec_stub.so` (csrc/tests/rocdec_stub.cpp,
built by csrc/build.py), a test double of librocdecode compiled against the same ROCm API
header: its parser decodes with the framework's CPU decoders and drives the real callback
protocol (sequence -> decode_picture -> display_picture, pts echoed), and its decoder hands out
pitched NV12 surfaces from a bounded pool that is only refilled when the application marks
surfaces for reuse. What is checked is the backend's side of the contract: decoder creation
from the sequence callback, surface mapping (pitch, display crop), the worker's surface copy +
conversion, pts/metadata mapping through reordering, keyframe-only draining, and that every
surface goes back to the parser (a leak exhausts the pool within a GOP).

Reference parity: the reference decodes with libavcodec per camera (python/read_image.py:87);
SURVEY.md N2(a) names the rocDecode backend.
"""
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
STUB = ROOT / "tests" / "native" / "libvep_rocdec_stub.so"


@pytest.fixture(scope="module")
def vcn(native):
    if not STUB.exists():
        pytest.fail(f"{STUB} missing: run `python csrc/build.py`")
    os.environ["VEP_ROCDEC_STUB_HOST"] = "1"  # CPU backend: surfaces in host memory
    assert native.vcn_load(str(STUB)), native.vcn_load_error()
    assert native.rocdecode_available()
    assert native.vcn_library() == str(STUB)
    yield native


def synth(native, codec, w, h, bframes, gop=8, profile="high"):
    c = native.SynthConfig()
    c.width, c.height, c.gop, c.codec, c.compressed = w, h, gop, codec, True
    c.bframes = bframes
    if codec == "h264":
        c.profile = profile
    return native.SynthH264(c)


def reference_frames(native, codec, aus):
    """pts -> BGR of every picture the framework's own CPU decoder outputs."""
    want = {}
    if codec == "h264":
        dec = native.CpuDecoder()
        for au in aus:
            img = dec.decode(au)
            if img is not None:
                want[dec.last_pts] = img
    else:
        dec = native.HevcDecoder()
        for au in aus:
            for pts, _poc, _t, (y, uv) in dec.decode(au):
                h, w = y.shape
                want[pts] = native.nv12_to_bgr_cpu(y, uv, 0, 0, w, h)
    return want


def run_vcn_camera(native, device, codec, w, h, n, bframes, gop=8):
    s = synth(native, codec, w, h, bframes, gop)
    aus = [s.next() for _ in range(n)]
    want = reference_frames(native, codec, aus)
    wk = native.Worker(device=device, decoder="vcn")
    assert wk.decoder == "vcn"
    cam = wk.add_camera("vcn_cam", 4)
    seq, published = 0, 0
    for au in aus:
        wk.decode_now(cam, au)
        r = wk.read_latest(cam, seq)
        if r is None:
            continue  # reordering: nothing reached display order yet
        meta, got = r
        seq = meta["seq"]
        ref = want[meta["pts"]]
        assert got.shape == ref.shape == (h, w, 3)
        assert np.array_equal(got, ref), f"pts {meta['pts']}: {int((got != ref).sum())} samples differ"
        published += 1
    st = wk.stats(cam)
    assert st["backend"] == "vcn" and st["errors"] == 0, (st, wk.logs(cam, True))
    wk.stop()
    return published


def test_vcn_absent_is_reported_and_enforced(native):
    """Without librocdecode: the probe says so with a reason, decoder='vcn' refuses to start,
    'auto' falls back to the native decoder (fresh process: the loader state is per process)."""
    code = (
        "import os; os.environ.pop('VEP_ROCDECODE_LIB', None)\n"
        "from video_edge_ai_proxy_amd import native\n"
        "assert not native.rocdecode_available()\n"
        "assert native.vcn_load_error()\n"
        "assert native.Worker(device=-1, decoder='auto').decoder == 'native'\n"
        "try:\n"
        "    native.Worker(device=-1, decoder='vcn')\n"
        "    raise SystemExit('vcn worker started without rocDecode')\n"
        "except Exception as e:\n"
        "    assert 'rocDecode' in str(e), e\n"
        "try:\n"
        "    native.Worker(device=-1, decoder='bogus')\n"
        "    raise SystemExit('bad decoder accepted')\n"
        "except Exception:\n"
        "    pass\n"
        "print('ok')\n"
    )
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("codec,w,h,bframes", [
    ("h264", 320, 180, 2),   # High CABAC IBBP, coded 320x192 cropped to 180 rows
    ("h264", 176, 144, 0),
    ("h265", 200, 120, 2),
    ("h265", 160, 96, 0),
], ids=["h264-high-ibbp-crop", "h264-ipp", "h265-ibbp", "h265-ipp"])
def test_vcn_camera_cpu_backend(vcn, codec, w, h, bframes):
    # 40 pictures over 5 GOPs: far more than the decoder's surface pool, so an unreleased
    # surface would fail the run
    n = 40
    published = run_vcn_camera(vcn, -1, codec, w, h, n, bframes)
    assert published >= n - 3


def test_vcn_keyframe_only_drains_reorder_queue(vcn):
    """keyframe_only: the IDR is published at once even with B pictures pending (the session
    flushes the parser; the next keyframe re-sends the parameter sets)."""
    import time

    s = synth(vcn, "h264", 176, 144, 2, gop=4)
    aus = [s.next() for _ in range(8)]
    dec = vcn.CpuDecoder()  # the IDR alone, flushed out of the reorder buffer
    dec.decode(aus[0])
    frames = dec.flush_frames()
    assert frames, "CPU decoder has no output for the IDR"
    pts, (y, uv) = frames[-1]
    wk = vcn.Worker(device=-1, decoder="vcn")
    wk.start()
    cam = wk.add_camera("k", 4)
    wk.set_keyframe_only(cam, True)
    wk.set_last_query(cam, int(time.time() * 1000))
    assert wk.submit_au(cam, aus[0])
    wk.flush()
    meta, got = wk.read_latest(cam, 0)
    assert meta["is_keyframe"] and meta["pts"] == pts
    assert np.array_equal(got, vcn.nv12_to_bgr_cpu(y, uv, 0, 0, 176, 144))
    # the rest of the GOP is not decoded; the next keyframe is
    for au in aus[1:4]:
        assert not wk.submit_au(cam, au)
    assert wk.submit_au(cam, aus[4])
    wk.flush()
    meta2, _ = wk.read_latest(cam, meta["seq"])
    assert meta2["is_keyframe"] and meta2["pts"] == aus[4].pts
    assert wk.stats(cam)["errors"] == 0, wk.logs(cam, True)
    wk.stop()


@pytest.mark.gpu
@pytest.mark.parametrize("codec,w,h,bframes", [("h264", 320, 180, 2), ("h265", 200, 120, 2)],
                         ids=["h264-high-ibbp", "h265-ibbp"])
def test_vcn_camera_gpu(native, codec, w, h, bframes):
    """gfx950: surfaces in HBM (hipMalloc by the stub decoder), copied into the camera surface on
    the lane stream and converted by the decode_convert kernel."""
    assert native.device_count() > 0
    os.environ.pop("VEP_ROCDEC_STUB_HOST", None)
    assert native.vcn_load(str(STUB)), native.vcn_load_error()
    n = 24
    assert run_vcn_camera(native, 0, codec, w, h, n, bframes) >= n - 3
