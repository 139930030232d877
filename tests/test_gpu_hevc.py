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


@pytest.mark.parametrize("env", [{"VEP_HEVC_TU_QUEUE": "1"}, {"VEP_HEVC_TU_QUEUE": "0"},
                                 {"VEP_HEVC_TU_WINDOW": "3"}, {"VEP_HEVC_TU_WINDOW": "8"},
                                 {"VEP_HEVC_TU_WINDOW": "-1"}],
                         ids=["tu-queue", "tu-levels", "tu-window3", "tu-window8", "tu-picture"])
def test_hevc_gpu_intra_tu_scheduling(native, monkeypatch, env):
    """Every schedule of the intra transform blocks is bit-exact: one queue launch per round
    (edge-word exchange between blocks), one launch per dependency level, and one queue launch
    per window of k levels (the exchange also spans windows), and one workgroup per picture
    (every dependency wait inside the workgroup)."""
    monkeypatch.delenv("VEP_HEVC_TU_QUEUE", raising=False)
    monkeypatch.delenv("VEP_HEVC_TU_WINDOW", raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    published = run_camera(native, 0, 200, 120, 14, coverage=True, bframes=1, slices=2)
    assert published >= 7
