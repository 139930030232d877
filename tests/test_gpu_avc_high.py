"""Main / High-profile H.264 on gfx950: CABAC and CAVLC streams with B pictures (pyramids,
spatial / temporal direct), 8x8 transform + Intra_8x8, explicit / implicit weighted
prediction, scaling matrices and multiple slices from the closed-loop High encoder. Every frame
the GPU worker publishes equals the CPU reference decoder's output and the encoder's own
reconstruction of that picture, bit-exact, at 176x144 (coverage streams: every MB / sub-MB
type) and 1080p (realistic IBBP); interlaced streams of frame pictures and of field pairs."""
import numpy as np
import pytest

from conftest import high_encoder

pytestmark = pytest.mark.gpu

PAFF = dict(interlaced=True, fields=True, cabac=False, t8x8=False, bframes=0)

GPU_CONFIGS = {
    "cov-cabac-spatial": (176, 144, 16, dict(bframes=2, coverage=True)),
    "cov-cavlc-temporal-implicit": (176, 144, 16, dict(bframes=3, coverage=True, cabac=False,
                                                       direct_spatial=False, weighted_b=2)),
    "cov-scaling-slices-explicit": (352, 288, 12, dict(bframes=2, coverage=True, scaling=True, slices=3,
                                                       weighted_p=True, weighted_b=1, deblock_idc=2,
                                                       chroma_qp_offset=-2, second_chroma_qp_offset=3)),
    "high-1080p-ibbp": (1920, 1080, 8, dict(bframes=2, qp=26, temporal_noise=2.0)),
    # interlaced SPS coding frame pictures (1080i-style: 1088 coded rows in map units of 2 MB rows)
    "interlaced-frames-cov": (176, 144, 12, dict(bframes=2, coverage=True, interlaced=True)),
    "interlaced-1080-ibbp": (1920, 1080, 6, dict(bframes=2, qp=26, interlaced=True)),
    # long-term references, MMCO 1-4 / 6 and list modifications (marking coverage)
    "marking-cov-ibbp": (176, 144, 30, dict(bframes=2, refs=3, coverage=True, marking=True)),
    "marking-1080-p": (1920, 1080, 12, dict(bframes=0, refs=4, qp=26, marking=True)),
    # field pairs (PAFF): half-height field pictures in field slots, the published frame woven
    "paff-cov": (176, 144, 24, dict(coverage=True, **PAFF)),
    "paff-1080-refs2": (1920, 1080, 12, dict(qp=26, refs=2, temporal_noise=2.0, **PAFF)),
    "paff-b-cov-temporal": (176, 144, 36, dict(PAFF, bframes=2, coverage=True, direct_spatial=False, weighted_b=2)),
    "paff-b-1080-ibbp": (1920, 1080, 18, dict(PAFF, bframes=2, qp=26, temporal_noise=2.0)),
    "paff-marking-cov": (176, 144, 40, dict(PAFF, bframes=2, refs=3, coverage=True, marking=True)),
    "paff-high-8x8-cov": (176, 144, 36, dict(PAFF, bframes=2, t8x8=True, coverage=True)),
}


@pytest.mark.parametrize("name", sorted(GPU_CONFIGS))
def test_high_profile_gpu_bit_exact(native, name):
    w, h, n, kw = GPU_CONFIGS[name]
    enc = high_encoder(native, w, h, gop=12, seed=11, **kw)
    ref = native.CpuDecoder()
    wk = native.Worker(device=0)
    cam = wk.add_camera("hi", 4)
    rec = {}
    published = 0
    for i in range(n):
        au = enc.next()
        y, uv = enc.picture()
        rec[enc.last_pts] = y.copy()
        want = ref.decode(au)
        ok = wk.decode_now(cam, au)
        if want is None:
            continue  # B reordering: nothing leaves the reorder buffer with this picture
        assert ok
        meta, got = wk.read_latest(cam, 0)
        assert got.shape == (h, w, 3)
        assert meta["pts"] == ref.last_pts
        assert np.array_equal(got, want), f"{name}: AU {i} differs in {int((got != want).sum())} samples"
        gy, _ = ref.surface()
        assert np.array_equal(gy, rec[ref.last_pts]), f"{name}: AU {i}: decoder != encoder reconstruction"
        published += 1
    # (reorder depth 2: several pictures leave together at an IDR; field pairs: 2 AUs per frame)
    assert published >= (n // 4 if kw.get("fields") else n // 2)
    assert wk.stats(cam)["decoder"] == "general"
