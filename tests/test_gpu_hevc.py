"""General H.265 Main streams on gfx950: every frame the GPU worker publishes equals the closed-
loop encoder's reconstruction (CPU HEVC decoder -> changed-block update -> GPU apply / convert),
bit-exact, for coverage streams (every CU / PU / TU syntax path) and a realistic 1080p IBBP
camera."""
import pytest

from test_hevc_camera import run_camera

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("w,h,n,kw", [
    (200, 120, 14, dict(coverage=True, bframes=1, slices=2)),
    (352, 288, 12, dict(coverage=True, bframes=2)),
    (1920, 1080, 8, dict(bframes=2, qp=30, temporal_noise=2.0)),
], ids=["cov-200x120", "cov-cif", "1080p-ibbp"])
def test_hevc_gpu_bit_exact(native, w, h, n, kw):
    published = run_camera(native, 0, w, h, n, **kw)
    assert published >= n // 2


@pytest.mark.parametrize("queue", ["1", "0"], ids=["tu-queue", "tu-levels"])
def test_hevc_gpu_intra_tu_scheduling(native, monkeypatch, queue):
    """Both schedules of the intra transform blocks are bit-exact: one queue launch per round
    (edge-word exchange between blocks) and one launch per dependency level."""
    monkeypatch.setenv("VEP_HEVC_TU_QUEUE", queue)
    published = run_camera(native, 0, 200, 120, 14, coverage=True, bframes=1, slices=2)
    assert published >= 7
