"""General H.265 streams through the camera runtime: a stream beyond the PCM / skip subset
switches the camera to the general HEVC decoder (hevc_dec.h); each published picture reaches
the surface as an update of the changed 16x16 blocks and goes through the shared apply /
convert kernels. Every published frame must equal the encoder's reconstruction of that picture
(converted by the CPU reference of the colour conversion), bit-exact: on the CPU backend here
and on gfx950 in the GPU variant."""
import numpy as np
import pytest

from conftest import check_surface


def synth_hevc(native, w, h, **kw):
    c = native.SynthConfig()
    c.width, c.height, c.gop, c.codec, c.compressed = w, h, 8, "h265", True
    c.bframes = 0
    for k, v in kw.items():
        setattr(c, k, v)
    return native.SynthH264(c)


def run_camera(native, device, w, h, n, **kw):
    s = synth_hevc(native, w, h, **kw)
    wk = native.Worker(device=device)
    cam = wk.add_camera("hevc", 4)
    want, full = {}, {}
    published = 0
    seq = 0
    low_bits = False
    for _ in range(n):
        au = s.next()
        y, uv = s.picture()
        full[s.last_pts] = (y.copy(), uv.copy())
        if y.dtype == np.uint16:  # Main10: the worker publishes the surface rounded to 8 bits
            y, uv = (np.minimum((p.astype(np.int32) + 2) >> 2, 255).astype(np.uint8) for p in (y, uv))
        want[s.last_pts] = native.nv12_to_bgr_cpu(y, uv, 0, 0, w, h)
        wk.decode_now(cam, au)
        r = wk.read_latest(cam, seq)
        if r is None:
            continue  # reordering: the picture was reconstructed, nothing left the DPB
        meta, got = r
        seq = meta["seq"]
        assert got.shape == (h, w, 3)
        ref = want[meta["pts"]]
        assert np.array_equal(got, ref), f"pts {meta['pts']}: {int((got != ref).sum())} samples differ"
        # the reconstruction itself at full depth (Main10: before the 8-bit narrowing)
        ys = check_surface(wk, cam, meta["pts"], full, w, h)
        low_bits |= ys.dtype == np.uint16 and bool((ys & 3).any())
        published += 1
    st = wk.stats(cam)
    assert st["decoder"] == "general"
    assert kw.get("bit_depth", 8) == 8 or published == 0 or low_bits, "no sample below the 8-bit grid"
    return published


@pytest.mark.parametrize("kw", [dict(), dict(bframes=2), dict(coverage=True, bframes=1, slices=2)],
                         ids=["ippp", "ibbp", "coverage"])
def test_hevc_camera_cpu_backend(native, kw):
    n = 14
    published = run_camera(native, -1, 200, 120, n, **kw)
    assert published >= n - 3


@pytest.mark.parametrize("kw", [dict(bit_depth=10), dict(bit_depth=10, coverage=True, bframes=2, slices=2)],
                         ids=["main10", "main10-coverage"])
def test_hevc_camera_main10_cpu_backend(native, kw):
    """Main10 cameras: 16-bit surfaces, narrowed to 8 bits for the BGR24 ring."""
    n = 12
    assert run_camera(native, -1, 200, 120, n, **kw) >= n - 4


def test_hevc_camera_keyframe_only(native):
    """keyframe_only: the IDR is published at once even with reordering (B pictures)."""
    s = synth_hevc(native, 160, 96, bframes=2)
    wk = native.Worker(device=-1)
    cam = wk.add_camera("k", 4)
    wk.set_keyframe_only(cam, True)
    au = s.next()
    y, uv = s.picture()
    assert wk.decode_now(cam, au)
    meta, got = wk.read_latest(cam, 0)
    assert np.array_equal(got, native.nv12_to_bgr_cpu(y, uv, 0, 0, 160, 96))


@pytest.mark.parametrize("device", [-1, pytest.param(0, marks=pytest.mark.gpu)])
@pytest.mark.parametrize("chunk", [3, 5])
def test_hevc_backlog_across_irap(native, chunk, device):
    """The H.265 twin of test_live_compressed.py::test_backlog_across_idr_publishes_the_output_picture:
    backlogs merged into one job per chunk (a chunk that reaches an IRAP restarts from it) publish
    only frames whose reconstruction they hold, each equal to the encoder's picture."""
    w, h = 200, 120
    s = synth_hevc(native, w, h, bframes=2)
    aus, want = [], {}
    for _ in range(24):
        aus.append(s.next())
        y, uv = s.picture()
        want[s.last_pts] = native.nv12_to_bgr_cpu(y, uv, 0, 0, w, h)
    wk = native.Worker(device=device)
    cam = wk.add_camera("hevc-backlog", 4)
    seq, checked = 0, 0
    for k0 in range(0, len(aus), chunk):
        wk.decode_many([(cam, aus[k0:k0 + chunk])])
        r = wk.read_latest(cam, seq)
        if r is None:
            continue
        meta, got = r
        seq = meta["seq"]
        ref = want[meta["pts"]]
        assert np.array_equal(got, ref), f"chunk at AU {k0}: pts {meta['pts']} stale ({int((got != ref).sum())} samples)"
        checked += 1
    assert checked >= len(aus) // chunk - 4


def test_hevc_open_gop_closed_loop(native):
    """Open GOPs (every IRAP after the first a CRA, coded before the RASL B pictures that precede
    it in display order): the camera decodes every picture bit-exactly, RASL ones included."""
    w, h = 160, 96
    s = synth_hevc(native, w, h, bframes=2, open_gop=True)
    wk = native.Worker(device=-1)
    cam = wk.add_camera("open-gop", 4)
    want, seq, types, published = {}, 0, set(), 0
    for _ in range(30):
        au = s.next()
        y, uv = s.picture()
        want[s.last_pts] = native.nv12_to_bgr_cpu(y, uv, 0, 0, w, h)
        types |= {(bytes(n)[0] >> 1) & 0x3F for n in au.nals()}
        wk.decode_now(cam, au)
        r = wk.read_latest(cam, seq)
        if r is None:
            continue
        meta, got = r
        seq = meta["seq"]
        assert np.array_equal(got, want[meta["pts"]]), f"pts {meta['pts']}"
        published += 1
    assert {19, 21, 8} <= types  # IDR, CRA, RASL_N
    assert published >= 26 and wk.stats(cam)["errors"] == 0


@pytest.mark.parametrize("device", [-1, pytest.param(0, marks=pytest.mark.gpu)])
@pytest.mark.parametrize("chunk", [2, 3, 4, 5, 6, 7, 9, 11])
def test_hevc_backlog_across_cra(native, chunk, device):
    """Open-GOP twin of test_hevc_backlog_across_irap: a merged backlog that restarts from a CRA
    drops the previous GOP's pictures, which the CRA's RASL pictures predict from. Neither those
    dropped pictures (bumped out by later jobs) nor the RASL pictures may be published; every
    published frame equals the encoder's picture."""
    w, h = 160, 96
    s = synth_hevc(native, w, h, bframes=2, open_gop=True)
    aus, want = [], {}
    for _ in range(40):
        aus.append(s.next())
        y, uv = s.picture()
        want[s.last_pts] = native.nv12_to_bgr_cpu(y, uv, 0, 0, w, h)
    wk = native.Worker(device=device)
    cam = wk.add_camera("hevc-cra-backlog", 4)
    seq, checked = 0, 0
    for k0 in range(0, len(aus), chunk):
        wk.decode_many([(cam, aus[k0:k0 + chunk])])
        r = wk.read_latest(cam, seq)
        if r is None:
            continue
        meta, got = r
        seq = meta["seq"]
        ref = want[meta["pts"]]
        assert np.array_equal(got, ref), f"chunk at AU {k0}: pts {meta['pts']} stale ({int((got != ref).sum())} samples)"
        checked += 1
    assert checked >= len(aus) // chunk - 6


def test_repeated_pts_across_a_merge_is_published(native):
    """A dropped picture's (slot, pts) entry is erased once matched and expires: a source whose
    pts restart (looped file, reconnect) still publishes the later pictures that reuse them."""
    w, h = 160, 96
    s = synth_hevc(native, w, h, bframes=2)
    aus = [s.next() for _ in range(16)]
    wk = native.Worker(device=-1)
    cam = wk.add_camera("pts-repeat", 4)
    wk.decode_many([(cam, aus[0:5])])
    wk.decode_many([(cam, aus[5:10])])   # reaches the IDR at AU 8: drops a backlog
    for k in range(10, 16):
        wk.decode_now(cam, aus[k])
    base = wk.stats(cam)["decoded"]
    # the same stream again from its IDR (pts repeat): every output picture is published
    s2 = synth_hevc(native, w, h, bframes=2)
    for _ in range(24):
        wk.decode_now(cam, s2.next())
    assert wk.stats(cam)["decoded"] - base >= 20
