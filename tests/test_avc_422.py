"""H.264 4:2:2 (High 4:2:2 profile, profile_idc 122; 8 to 10 bits, progressive, CABAC and CAVLC).

4:2:2 changes the chroma of every macroblock to 8x16 per component: a 2x4 chroma DC (its own scan,
transform and QP'C + 3 scaling), CAVLC coeff_token / total_zeros tables for nC = -2, CABAC chroma
DC contexts Min(i / 2, 2), eight 4x4 AC blocks per component with their neighbour geometry, 8x16
intra chroma prediction (plane with yCF = 4), full-height chroma motion compensation (vertical
quarter-sample positions scaled to eighths) and chroma deblocking of every horizontal 4x4 edge.
The surfaces are NV16; the published BGR24 goes through a 4:2:0 display conversion (chroma rows
averaged in pairs: codec.h narrow_surface, the GPU narrow kernel).

The synthetic High encoder (AvcHighConfig.chroma_format = 2) codes through the decoder's own
macroblock layer and reconstruction, so the closed loop pins that both directions agree; the
4:2:2-specific arithmetic is checked against the independent spec oracle
(tests/test_spec_oracle_avc422.py). Parity with a third-party 4:2:2 stream / decoder is unpinned
(none in the image)."""
import numpy as np
import pytest

from conftest import check_surface, high_encoder, roundtrip

CONFIGS = {
    "cabac-ibbp": dict(bframes=2),
    "cavlc-ibp": dict(bframes=1, cabac=False),
    "cabac-cov": dict(bframes=2, coverage=True),
    "cavlc-cov": dict(bframes=2, coverage=True, cabac=False, direct_spatial=False),
    "cov-wp-scaling-slices": dict(bframes=3, coverage=True, scaling=True, slices=3, weighted_b=1, weighted_p=True,
                                  chroma_qp_offset=-3, second_chroma_qp_offset=4),
    "cov-dbk2-t4x4": dict(bframes=2, coverage=True, t8x8=False, slices=2, deblock_idc=2),
    "10bit-cov": dict(bframes=2, coverage=True, bit_depth=10),
    "10bit-cavlc-negqp": dict(bframes=1, cabac=False, bit_depth=10, qp=-6),
}


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_422_roundtrip_bit_exact(native, name):
    kw = dict(CONFIGS[name])
    enc = high_encoder(native, 176, 144, gop=12, seed=9, chroma_format=2, **kw)
    rec, got, dec, _ = roundtrip(native, enc, 20)
    assert len(rec) == 20 and set(got) == set(rec)
    for pts in sorted(rec):
        (ey, euv), (gy, guv) = rec[pts], got[pts]
        assert euv.shape == (144, 176) and guv.shape == (144, 176)  # NV16: full-height chroma
        assert np.array_equal(ey, gy) and np.array_equal(euv, guv), f"{name}: pts {pts} differs"
    st = dec.mb_stats
    if kw.get("coverage"):
        assert st["pcm"] > 0 and st["i4x4"] > 0 and st["i16x16"] > 0 and st["skip"] > 0


def test_422_parameter_sets(native):
    enc = high_encoder(native, 176, 144, chroma_format=2)
    sps = native.parse_sps(enc.sps_nal)
    assert sps["profile_idc"] == 122 and sps["chroma_format_idc"] == 2
    with pytest.raises(native.NativeError):
        high_encoder(native, 176, 144, chroma_format=2, interlaced=True, fields=True, cabac=False)


@pytest.mark.parametrize("bd", [8, 10])
def test_422_quality_tracks_the_source(native, bd):
    """The chroma is coded at full vertical resolution: the reconstruction's chroma is close to the
    4:2:2 source's, like its luma (PSNR at the depth's peak)."""
    enc = high_encoder(native, 320, 240, bframes=2, gop=12, seed=3, qp=24 - 6 * (bd - 8), bit_depth=bd,
                       chroma_format=2)
    peak = (1 << bd) - 1

    def psnr(a, b):
        e = a.astype(float) - b.astype(float)
        return 10 * np.log10(peak ** 2 / max(1e-9, (e ** 2).mean()))

    for _ in range(10):
        enc.next()
        (sy, suv), (ry, ruv) = enc.source(), enc.picture()
        assert suv.shape[0] == sy.shape[0]
        assert psnr(ry[:240, :320], sy[:240, :320]) > 38
        assert psnr(ruv[:240, :320], suv[:240, :320]) > 40


def test_422_display_conversion(native):
    """decode() returns BGR24 through the 4:2:0 display conversion: chroma rows averaged in pairs
    before the BT.601 conversion (the GPU narrow kernel does the same)."""
    enc = high_encoder(native, 176, 144, gop=6, seed=2, bframes=0, chroma_format=2)
    dec = native.CpuDecoder()
    au = enc.next()
    y, uv = enc.picture()
    bgr = dec.decode(au)
    uv420 = ((uv[0::2].astype(np.int32) + uv[1::2] + 1) >> 1).astype(np.uint8)
    assert np.array_equal(bgr, native.nv12_to_bgr_cpu(y, uv420, 0, 0, 176, 144))


def synth_422(native, w, h, **kw):
    c = native.SynthConfig()
    c.width, c.height, c.gop, c.codec, c.compressed, c.profile = w, h, 8, "h264", True, "high"
    c.bframes = 0
    c.chroma_format = 2
    for k, v in kw.items():
        setattr(c, k, v)
    return native.SynthH264(c)


def run_camera(native, device, w, h, n, **kw):
    bd = kw.get("bit_depth", 8)
    s = synth_422(native, w, h, **kw)
    wk = native.Worker(device=device)
    cam = wk.add_camera("c422", 4)
    want, full, published, seq, low_bits = {}, {}, 0, 0, False
    for _ in range(n):
        au = s.next()
        y, uv = s.picture()
        full[s.last_pts] = (y.copy(), uv.copy())
        uv = (uv[0::2].astype(np.int32) + uv[1::2] + 1) >> 1  # 4:2:0 display conversion
        y = y.astype(np.int32)
        if bd > 8:
            sh = bd - 8
            y, uv = (np.minimum((p + (1 << (sh - 1))) >> sh, 255) for p in (y, uv))
        want[s.last_pts] = native.nv12_to_bgr_cpu(y.astype(np.uint8), uv.astype(np.uint8), 0, 0, w, h)
        wk.decode_now(cam, au)
        r = wk.read_latest(cam, seq)
        if r is None:
            continue
        meta, got = r
        seq = meta["seq"]
        ref = want[meta["pts"]]
        assert np.array_equal(got, ref), f"pts {meta['pts']}: {int((got != ref).sum())} samples differ"
        # the NV16 reconstruction itself at full depth (before the 4:2:0 display conversion and
        # the 8-bit narrowing)
        ys = check_surface(wk, cam, meta["pts"], full, w, h, cf=2)
        low_bits |= bd > 8 and bool(((ys & ((1 << (bd - 8)) - 1)) != 0).any())
        published += 1
    assert wk.stats(cam)["decoder"] == "general"
    assert bd == 8 or published == 0 or low_bits, "no sample below the 8-bit grid: the check would be vacuous"
    return published


@pytest.mark.parametrize("kw", [dict(), dict(coverage=True, bframes=2, slices=2), dict(bit_depth=10, coverage=True)],
                         ids=["422", "422-coverage", "422-10bit"])
def test_422_camera_cpu_backend(native, kw):
    assert run_camera(native, -1, 176, 144, 12, **kw) >= 8


def test_422_cropping_cpu_backend(native):
    """A height that is not a multiple of 16: 4:2:2's CropUnitY is 1 (SubHeightC), not 4:2:0's 2,
    so 1088 -> 1080 is frame_crop_bottom_offset 8 (writer and parser, §7.4.2.1.1)."""
    assert run_camera(native, -1, 176, 136, 8, bframes=1) >= 4


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,n,kw", [
    (176, 144, 14, dict(coverage=True, bframes=2, slices=2)),
    (176, 144, 12, dict(coverage=True, bframes=1, cabac=False, weighted_p=True, weighted_b=1)),
    (176, 144, 12, dict(coverage=True, bframes=2, bit_depth=10, deblock_idc=2, slices=3)),
    (1920, 1080, 6, dict(bframes=2, qp=24, temporal_noise=2.0)),
], ids=["cov-cabac", "cov-cavlc-wp", "cov-10bit-dbk2", "1080p-ibbp"])
def test_422_gpu_bit_exact(native, w, h, n, kw):
    """gfx950: NV16 surfaces, avc_inter_kernel<P, 2> + avc_hbd_kernel<P, 2>, narrow + convert."""
    assert run_camera(native, 0, w, h, n, **kw) >= n // 2


@pytest.mark.parametrize("kw", [dict(chroma_format=2), dict(chroma_format=2, bit_depth=10, cabac=False),
                                dict(bit_depth=10)], ids=["422", "422-10bit-cavlc", "high10"])
def test_422_and_high10_corruption_never_crashes(native, kw):
    """Bit flips in 4:2:2 / High 10 slices: the decoder raises or decodes (never crashes, never
    writes outside its pools: every record is validated), and recovers at the next IDR."""
    import random

    rnd = random.Random(11)
    enc = high_encoder(native, 176, 144, bframes=2, gop=8, seed=4, coverage=True, **kw)
    aus = [enc.next() for _ in range(24)]
    clean = native.CpuDecoder()
    want = {}
    for a in aus:
        clean.decode(a)
        for pts, (y, uv) in clean.frames():
            want[pts] = (y, uv)
    for trial in range(10):
        dec = native.CpuDecoder()
        bad = rnd.randrange(1, 14)
        for i, a in enumerate(aus):
            if i == bad:
                nals = [bytearray(n) for n in a.nals()]
                sl = [k for k, x in enumerate(nals) if (x[0] & 0x1F) in (1, 5)][0]
                for _ in range(rnd.randint(1, 5)):
                    pos = rnd.randrange(3, len(nals[sl]))
                    nals[sl][pos] ^= 1 << rnd.randrange(8)
                a = native.AccessUnit.from_nals([bytes(x) for x in nals], pts=a.pts, dts=a.dts, keyframe=a.keyframe)
            try:
                dec.decode(a)
            except (native.NativeError, native.UnsupportedStream):
                continue
            if i >= 16:
                for pts, (y, uv) in dec.frames():
                    if pts < 18 * 3000:
                        continue
                    assert np.array_equal(y, want[pts][0]) and np.array_equal(uv, want[pts][1]), f"trial {trial}"
