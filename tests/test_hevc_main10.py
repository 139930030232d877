"""HEVC Main10: 10-bit 4:2:0 streams (SPS bit_depth 10, general_profile_idc 2). The synthetic
encoder codes a 10-bit source (the 8-bit scene << 2 plus a dither in the low bits) through the
shared CTU layer; the decoder keeps the samples in 16-bit surfaces. Checked here:

* the reference CPU decoder reproduces the encoder's reconstruction bit for bit on every syntax
  path (coverage streams: QP below 0 via QpBdOffset, 10-bit SAO offsets up to 31, PCM below the
  sample bit depth, weighted prediction with scaled offsets, scaling lists, tiles / WPP, ...);
* the records path's CPU mirror (hevc_kern.h math, which the gfx950 kernels run) equals the
  reference decoder (tests/test_gpu_hevc_main10.py runs the kernels themselves);
* the reconstruction tracks the 10-bit source (PSNR at 10-bit peak), i.e. the bit-depth
  scaling of MC, transforms, dequantisation and loop filters is consistent, not only
  self-consistent;
* (the primitives against the spec formulas at bit depth 10: tests/test_spec_oracle_hevc10.py);
* the worker publishes Main10 cameras as BGR24 (the 10-bit surface narrowed to 8 bits, then
  the BT.601 conversion).

Parity with libavcodec (read_image.py:87) is unpinned: no third-party 10-bit stream exists in
this image.
"""
import numpy as np
import pytest

from test_hevc_general import encoder

from video_edge_ai_proxy_amd import _vep as v

CONFIGS = [
    dict(),
    dict(bframes=2),
    dict(coverage=True, seed=21),
    dict(coverage=True, bframes=2, seed=23),
    dict(coverage=True, qp=4, seed=25),  # SliceQpY near 0; CU QPs below 0 (QpBdOffsetY = 12)
    dict(coverage=True, qp=45, bframes=1, slices=3, seed=27),
    dict(coverage=True, weighted=True, bframes=2, seed=29),
    dict(coverage=True, scaling_lists=True, lossless=True, seed=31),
    dict(coverage=True, tile_cols=2, tile_rows=2, seed=33, width=256, height=128),
    dict(coverage=True, wpp=True, segments=2, seed=35, width=256, height=128),
    dict(coverage=True, long_term=True, bframes=1, seed=37),
]


def roundtrip(n=10, **kw):
    e, d = encoder(bit_depth=10, **kw), v.HevcDecoder()
    recon, outs = {}, []
    for _ in range(n):
        au = e.next()
        y, uv = e.picture()
        recon[e.last_pts] = (y.copy(), uv.copy(), e.last_type)
        outs += d.decode(au)
    outs += d.flush()
    return recon, outs


@pytest.mark.parametrize("kw", CONFIGS, ids=[str(i) for i in range(len(CONFIGS))])
def test_main10_roundtrip_bit_exact(kw):
    recon, outs = roundtrip(**kw)
    assert len(outs) == len(recon) > 0
    for pts, poc, t, (y, uv) in outs:
        ry, ruv, rt = recon[pts]
        assert y.dtype == np.uint16 and uv.dtype == np.uint16
        assert t == rt
        assert np.array_equal(y, ry), f"luma mismatch at pts {pts} ({t})"
        assert np.array_equal(uv, ruv), f"chroma mismatch at pts {pts} ({t})"


@pytest.mark.parametrize("kw", CONFIGS, ids=[str(i) for i in range(len(CONFIGS))])
def test_main10_records_mirror_matches_reference(kw):
    e = encoder(bit_depth=10, **kw)
    ref, rec = v.HevcDecoder(), v.HevcRecordsDecoder()
    a, b = [], []
    for _ in range(10):
        au = e.next()
        a += ref.decode(au)
        b += rec.decode(au)
    a += ref.flush()
    b += rec.flush()
    assert len(a) == len(b) > 0
    for (pa, qa, ta, (ya, uva)), (pb, qb, tb, (yb, uvb), _) in zip(a, b):
        assert (pa, qa, ta) == (pb, qb, tb)
        assert yb.dtype == np.uint16
        assert np.array_equal(ya, yb), f"luma differs at poc {qa} ({ta}): {int((ya != yb).sum())} samples"
        assert np.array_equal(uva, uvb), f"chroma differs at poc {qa} ({ta}): {int((uva != uvb).sum())} samples"


def psnr10(a, b):
    m = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return 99.0 if m == 0 else 10 * np.log10(1023.0 ** 2 / m)


@pytest.mark.parametrize("kw,floor", [(dict(qp=22), 36.0), (dict(qp=32, bframes=2), 30.0)])
def test_main10_quality_tracks_the_10bit_source(kw, floor):
    e = encoder(bit_depth=10, width=192, height=128, gop=16, **kw)
    sizes = []
    for _ in range(8):
        au = e.next()
        sizes.append(au.size)
        y, uv = e.picture()
        sy, suv = e.source()
        assert sy.dtype == np.uint16 and int(sy.max()) > 255  # a real 10-bit source
        assert psnr10(y, sy) > floor
        assert psnr10(uv, suv) > floor
    assert sizes[0] > 2 * max(sizes[1:])


def test_main10_parameter_sets_and_profile():
    e = encoder(bit_depth=10)
    e.next()
    sps = e.sps_nal
    # general_profile_idc (5 bits after profile_space / tier) in the first PTL byte of the SPS
    # (NAL header 2 bytes, then sps_video_parameter_set_id / max_sub_layers / temporal_id_nesting)
    assert (sps[3] & 0x1F) == 2
    # a fresh decoder given the IDR decodes 10-bit planes (values above the 8-bit range)
    e2 = encoder(bit_depth=10)
    d2 = v.HevcDecoder()
    outs = d2.decode(e2.next()) + d2.flush()
    assert outs and outs[0][3][0].dtype == np.uint16 and int(outs[0][3][0].max()) > 255


def test_8bit_streams_keep_8bit_planes():
    e, d = encoder(), v.HevcDecoder()
    outs = d.decode(e.next()) + d.flush()
    assert outs[0][3][0].dtype == np.uint8


def test_main10_camera_publishes_bgr():
    """A Main10 camera on the CPU backend: records -> mirror -> 16-bit surfaces -> narrowed
    8-bit NV12 -> BGR24 ring frames; the frame equals the conversion of the decoder's picture
    rounded to 8 bits."""
    from video_edge_ai_proxy_amd import native

    e = encoder(bit_depth=10, width=128, height=96, bframes=0)
    w = native.Worker(device=-1, max_cameras=1)
    w.start()
    try:
        cam = w.add_camera("m10", 3)
        ref = v.HevcDecoder()
        last = None
        for _ in range(4):
            au = e.next()
            w.decode_now(cam, au)
            outs = ref.decode(au)
            if outs:
                last = outs[-1]
        w.flush()
        assert w.published(cam) >= 3
        _, img = w.read_latest(cam, 0)
        y, uv = last[3]
        y8 = np.minimum((y.astype(np.int32) + 2) >> 2, 255).astype(np.uint8)
        uv8 = np.minimum((uv.astype(np.int32) + 2) >> 2, 255).astype(np.uint8)
        want = v.nv12_to_bgr_cpu(y8, uv8, 0, 0, 128, 96)
        assert img.shape == (96, 128, 3)
        assert np.array_equal(img, want)
    finally:
        w.stop()
