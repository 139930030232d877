"""General H.265 Main decoder (csrc/vep/hevc_dec.cpp, hevc_ctu.cpp, hevc_recon.cpp) against the
closed-loop synthetic encoder (hevc_enc.cpp).

The encoder drives the same CTU layer in write mode and keeps its reconstruction, so every
decoded picture must equal the encoder's reconstruction bit for bit; `coverage` streams
randomise every syntax decision (CU / TU trees, AMP, 35 intra modes, PCM, merge / AMVP, bi-
prediction, transform skip, sign hiding, QP deltas, SAO, per-slice deblocking). The PSNR checks
against the source pin the transform / scan / dequantisation conventions (the encoder's
forward transform is an independent floating-point DCT/DST). Parity with a third-party HEVC
decoder is unpinned: no HEVC bitstream from another encoder exists in this image.
Reference behaviour: libavcodec's hevc decoder behind PyAV (python/read_image.py:87).
"""
import numpy as np
import pytest

from video_edge_ai_proxy_amd import _vep as v


def encoder(**kw):
    c = v.HevcEncConfig()
    c.width, c.height, c.gop, c.qp = 128, 96, 8, 30
    for k, x in kw.items():
        setattr(c, k, x)
    return v.HevcEncoder(c)


def roundtrip(n=12, **kw):
    e, d = encoder(**kw), v.HevcDecoder()
    recon, outs, stats = {}, [], {}
    for _ in range(n):
        au = e.next()
        y, uv = e.picture()
        recon[e.last_pts] = (y.copy(), uv.copy(), e.last_type)
        outs += d.decode(au)
        for k, x in d.stats.items():
            stats[k] = stats.get(k, 0) + x
    outs += d.flush()
    return recon, outs, stats


CONFIGS = [
    dict(),
    dict(bframes=2),
    dict(coverage=True),
    dict(coverage=True, bframes=2, seed=3),
    dict(coverage=True, bframes=3, slices=3, log2_ctb=4, seed=5),
    dict(coverage=True, bframes=1, log2_ctb=6, width=200, height=136, seed=7),
    dict(coverage=True, amp=False, sao=False, tskip=False, sign_hiding=False, cu_qp_delta=False, seed=11),
    dict(coverage=True, deblock=False, pcm=False, tmvp=False, bframes=2, seed=13),
    dict(coverage=True, qp=12, seed=17),   # large levels: escape codes, Rice parameter growth
    dict(coverage=True, qp=45, bframes=1, slices=2, seed=19),
]


@pytest.mark.parametrize("kw", CONFIGS, ids=[str(i) for i in range(len(CONFIGS))])
def test_hevc_roundtrip_bit_exact(kw):
    recon, outs, _ = roundtrip(**kw)
    assert len(outs) == len(recon)
    pocs = [o[0] for o in outs]
    assert pocs == sorted(pocs), "output must be in display order"
    for pts, poc, t, (y, uv) in outs:
        ry, ruv, rt = recon[pts]
        assert t == rt
        assert np.array_equal(y, ry), f"luma mismatch at pts {pts} ({t})"
        assert np.array_equal(uv, ruv), f"chroma mismatch at pts {pts} ({t})"


def test_hevc_coverage_exercises_every_cu_kind():
    total = {}
    for seed in (1, 2, 3):
        _, _, st = roundtrip(n=10, coverage=True, bframes=2, seed=seed, log2_ctb=4)
        for k, x in st.items():
            total[k] = total.get(k, 0) + x
    for k in ("intra", "inter", "skip", "pcm", "merge", "bi", "tskip", "amp"):
        assert total[k] > 0, (k, total)


def psnr(a, b):
    m = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return 99.0 if m == 0 else 10 * np.log10(255.0 ** 2 / m)


@pytest.mark.parametrize("kw,floor", [(dict(qp=22), 36.0), (dict(qp=32, bframes=2), 30.0)])
def test_hevc_camera_quality(kw, floor):
    e = encoder(width=192, height=128, gop=16, **kw)
    sizes = []
    for _ in range(10):
        au = e.next()
        sizes.append(au.size)
        y, uv = e.picture()
        sy, suv = e.source()
        assert psnr(y, sy) > floor
        assert psnr(uv, suv) > floor
    assert sizes[0] > 2 * max(sizes[1:]), "inter pictures must be much smaller than the IDR"


def test_hevc_corrupt_slice_raises_and_recovers():
    e, d = encoder(bframes=0), v.HevcDecoder()
    aus = [e.next() for _ in range(12)]
    for au in aus[:3]:
        d.decode(au)
    nals = aus[3].nals()
    bad = v.AccessUnit.from_nals([n[: len(n) // 3] for n in nals], pts=aus[3].pts, codec=1)
    with pytest.raises(Exception):
        d.decode(bad)
    # a following P picture may reference the lost one; the next IDR (gop 8) restarts cleanly
    for au in aus[4:8]:
        try:
            d.decode(au)
        except Exception:
            pass
    out = d.decode(aus[8])
    out += d.flush()
    assert out and out[-1][2] == "I"


def test_hevc_stream_starting_mid_gop_is_rejected_until_idr():
    e, d = encoder(), v.HevcDecoder()
    aus = [e.next() for _ in range(10)]
    with pytest.raises(Exception):
        d.decode(aus[2])  # no parameter sets yet
    out = []
    for au in aus[8:]:
        out += d.decode(au)
    out += d.flush()
    assert len(out) == 2


def test_hevc_mid_gop_size_change_is_rejected():
    """A repeated SPS with another picture size before a P picture (corrupt / spliced stream)
    must not make the P picture predict from surfaces of the old size."""
    a = encoder(width=128, height=96)
    b = encoder(width=160, height=96)
    aus = [a.next() for _ in range(3)]
    d = v.HevcDecoder()
    for au in aus[:2]:
        d.decode(au)
    bad = v.AccessUnit.from_nals([b.sps_nal] + aus[2].nals(), pts=aus[2].pts, codec=1)
    with pytest.raises(Exception, match="size"):
        d.decode(bad)
