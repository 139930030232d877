"""H.265 coding tools on gfx950 through the camera runtime (records -> hevc_mc / hevc_tu /
deblock / SAO kernels -> NV12->BGR24): tiles, WPP, dependent slice segments, scaling lists,
explicit weighted prediction, long-term references and transquant-bypass CUs. Every published
frame must equal the closed-loop encoder's reconstruction, bit-exact, at CIF (coverage streams:
every syntax path randomised) and at 1080p (camera-style streams with the tool on). The CPU-
backend variant of the same paths runs in the CPU suite (test_hevc_tools.py, and
test_hevc_tools_camera_cpu below)."""
import pytest

from test_hevc_camera import run_camera

CIF_TOOLS = {
    "tiles": dict(tile_cols=3, tile_rows=2, coverage=True, bframes=1),
    "wpp": dict(wpp=True, coverage=True, bframes=1, slices=2),
    "dependent": dict(segments=3, coverage=True, slices=2),
    "tiles_wpp_dep": dict(tile_cols=2, tile_rows=2, wpp=True, segments=2, coverage=True),
    "scaling": dict(scaling_lists=True, coverage=True, bframes=1),
    "weighted": dict(weighted_p=True, coverage=True, bframes=2),
    "long_term": dict(long_term=True, coverage=True, bframes=1),
    "lossless": dict(lossless=True, coverage=True),
}

HD_TOOLS = {
    "1080p-tiles-wpp": dict(tile_cols=4, tile_rows=2, wpp=True, bframes=2, qp=30, temporal_noise=2.0),
    "1080p-scaling-weighted-lt": dict(scaling_lists=True, weighted_p=True, long_term=True, bframes=2, qp=30,
                                      temporal_noise=2.0),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CIF_TOOLS))
def test_hevc_tools_gpu_cif(native, name):
    n = 10
    published = run_camera(native, 0, 352, 288, n, **CIF_TOOLS[name])
    assert published >= n // 2


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(HD_TOOLS))
def test_hevc_tools_gpu_1080p(native, name):
    n = 8
    published = run_camera(native, 0, 1920, 1080, n, **HD_TOOLS[name])
    assert published >= n // 2


@pytest.mark.parametrize("name", ["tiles_wpp_dep", "weighted", "lossless", "long_term"])
def test_hevc_tools_camera_cpu(native, name):
    n = 8
    published = run_camera(native, -1, 176, 144, n, **CIF_TOOLS[name])
    assert published >= n // 2
