"""HEVC Main10 on gfx950: the reconstruction kernels on u16 DPB surfaces (HevcDesc kHevcWide,
bit depth 10), the launch_narrow step to 8-bit NV12 and the BT.601 conversion. Every published
frame must equal the closed-loop encoder's 10-bit reconstruction rounded to 8 bits and
converted by the CPU reference, bit-exact, for coverage streams (every CU / PU / TU syntax
path incl. PCM below the bit depth, 10-bit SAO offsets, negative QPs) and under every intra
TU schedule."""
import pytest

from test_hevc_camera import run_camera

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("w,h,n,kw", [
    (200, 120, 14, dict(coverage=True, bframes=1, slices=2, bit_depth=10)),
    (352, 288, 12, dict(coverage=True, bframes=2, bit_depth=10, qp=8)),
    (1920, 1080, 6, dict(bframes=2, qp=30, temporal_noise=2.0, bit_depth=10)),
], ids=["cov-200x120", "cov-cif-lowqp", "1080p-ibbp"])
def test_hevc_main10_gpu_bit_exact(native, w, h, n, kw):
    published = run_camera(native, 0, w, h, n, **kw)
    assert published >= n // 2


@pytest.mark.parametrize("env", [{"VEP_HEVC_TU_WINDOW": "0"}, {"VEP_HEVC_TU_WINDOW": "-1"}],
                         ids=["tu-levels", "tu-picture"])
def test_hevc_main10_gpu_tu_schedules(native, monkeypatch, env):
    monkeypatch.delenv("VEP_HEVC_TU_WINDOW", raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    assert run_camera(native, 0, 200, 120, 12, coverage=True, bframes=1, bit_depth=10) >= 6
