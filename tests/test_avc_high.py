"""Main / High profile H.264 on the CPU reference decoder.

* A real third-party High-profile clip: imageio's `realshort.mp4` (320x240, CABAC, 8x8
  transform + Intra_8x8, Intra_4x4, P pictures, two IDRs), present in this image under
  /opt/conda. Nothing in the image can decode it for a pixel reference (no FFmpeg / PyAV /
  OpenCV), so parity is *unpinned*: the test checks that every access unit decodes through the
  CABAC engine without a desync (any CABAC table or binarization error desynchronises the
  arithmetic decoder within a few macroblocks and ends in a range / overrun error or a wrong
  end_of_slice position), that the syntax it exercises is what the clip is known to contain,
  and that the pictures are temporally coherent (a desync or a wrong predictor produces
  garbage that breaks frame-to-frame similarity).
* Closed-loop High-profile streams from the synthetic encoder (CABAC / CAVLC, B pyramids,
  8x8, weighted prediction) where the encoder's reconstruction is the reference.
"""
import os

import numpy as np
import pytest

CLIP = "/opt/conda/lib/python3.9/site-packages/imageio/resources/images/realshort.mp4"


def clip_aus(native):
    from video_edge_ai_proxy_amd.utils import mp4

    buf = open(CLIP, "rb").read()
    tr = mp4.parse(buf)
    out = []
    for i, (nals, key, dts, pts) in enumerate(mp4.samples(buf, tr)):
        au = native.AccessUnit.from_nals((tr.param_sets if i == 0 else []) + nals, keyframe=key,
                                         pts=pts, dts=dts)
        out.append(au)
    return tr, out


def psnr(a, b):
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return 99.0 if mse == 0 else 10 * np.log10(255.0 ** 2 / mse)


@pytest.mark.skipif(not os.path.exists(CLIP), reason="imageio sample clip not in this image")
def test_third_party_high_profile_cabac_clip(native):
    tr, aus = clip_aus(native)
    assert tr.codec == "avc1" and (tr.width, tr.height) == (320, 240) and len(aus) == 36
    dec = native.CpuDecoder()
    frames = [dec.decode(au) for au in aus]
    assert all(f is not None and f.shape == (240, 320, 3) for f in frames)
    st = dec.mb_stats
    # CABAC High profile syntax the clip is known to use
    assert st["types"] == "I" + "P" * 29 + "I" + "P" * 5
    assert st["i8x8"] > 0 and st["i4x4"] > 0 and st["t8x8"] > 1000 and st["skip"] > 0 and st["inter"] > 1000
    # natural content, temporally coherent (a CABAC desync or drift destroys both)
    for f in frames:
        assert f.std() > 20
    sims = [psnr(frames[i], frames[i + 1]) for i in range(len(frames) - 1)]
    assert min(sims) > 14 and np.median(sims) > 20, sims
    # the clip's two GOPs show the same scene (the IDR at 30 re-anchors it)
    assert psnr(frames[29], frames[30]) > 15


@pytest.mark.skipif(not os.path.exists(CLIP), reason="imageio sample clip not in this image")
def test_third_party_clip_corruption_never_crashes(native):
    """Bit flips in the CABAC slice data of the real clip: every access unit either decodes or
    raises; the stream recovers at its next IDR."""
    import random

    _, aus = clip_aus(native)
    clean = native.CpuDecoder()
    want = [clean.decode(a) for a in aus]
    rnd = random.Random(11)
    for trial in range(6):
        dec = native.CpuDecoder()
        bad_at = rnd.randrange(1, 29)
        broken = False
        for i, au in enumerate(aus):
            if i == bad_at:
                nals = [bytearray(n) for n in au.nals()]
                k = [j for j, x in enumerate(nals) if (x[0] & 0x1F) in (1, 5)][0]
                for _ in range(rnd.randint(1, 4)):
                    pos = rnd.randrange(4, len(nals[k]))
                    nals[k][pos] ^= 1 << rnd.randrange(8)
                au = native.AccessUnit.from_nals([bytes(x) for x in nals], keyframe=au.keyframe)
            try:
                got = dec.decode(au)
            except (native.NativeError, native.UnsupportedStream):
                broken = True
                continue
            if i >= 30:
                assert got is not None and np.array_equal(got, want[i]), f"trial {trial}: frame {i}"
        assert isinstance(broken, bool)
