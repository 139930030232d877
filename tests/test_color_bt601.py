"""Colour conversion against an independent float BT.601 limited-range formula (±1 LSB), not the
fixed-point oracle that shares the kernel's constants (ops.nv12_to_bgr_reference). swscale's
default matrix is what the reference's read_image.py:94 ``frame.to_ndarray('bgr24')`` applies."""
import numpy as np
import pytest
import torch

from video_edge_ai_proxy_amd import ops


def _planes(H, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    y = torch.randint(0, 256, (H, W), dtype=torch.uint8, generator=g)
    uv = torch.randint(0, 256, (H // 2, W), dtype=torch.uint8, generator=g)
    # every (Y, U, V) corner and the limited-range edges appear too
    vals = torch.tensor([0, 1, 15, 16, 17, 127, 128, 129, 234, 235, 236, 239, 240, 241, 254, 255], dtype=torch.uint8)
    n = len(vals)
    y[:n, :n] = vals.view(-1, 1).expand(n, n)
    uv[: n // 2, : 2 * n : 2] = vals.view(1, -1).expand(n // 2, n)
    uv[: n // 2, 1 : 2 * n : 2] = vals.view(-1, 1)[: n // 2].expand(n // 2, n)
    return y, uv


def test_float_formula_sanity():
    y = torch.tensor([[16, 235], [16, 235]], dtype=torch.uint8)
    uv = torch.tensor([[128, 128, 128, 128]], dtype=torch.uint8)
    out = ops.nv12_to_bgr_bt601_float(y, uv)
    assert out[0, 0].tolist() == [0, 0, 0] and out[0, 1].tolist() == [255, 255, 255]
    # 100% red (BT.601 limited: Y 81, Cb 90, Cr 240) -> about (0, 0, 255) BGR
    red = ops.nv12_to_bgr_bt601_float(torch.tensor([[81, 81], [81, 81]], dtype=torch.uint8),
                                      torch.tensor([[90, 240, 90, 240]], dtype=torch.uint8))
    b, g, r = red[0, 0].tolist()
    assert b <= 2 and g <= 2 and r >= 253


def test_cpu_conversion_within_one_lsb_of_float_bt601(native):
    H, W = 96, 160
    y, uv = _planes(H, W)
    got = torch.from_numpy(np.ascontiguousarray(native.nv12_to_bgr_cpu(y.numpy(), uv.numpy(), 0, 0, W, H)))
    want = ops.nv12_to_bgr_bt601_float(y, uv)
    d = (got.to(torch.int16) - want.to(torch.int16)).abs()
    assert int(d.max()) <= 1, f"max |diff| {int(d.max())}"
    # and the fixed-point oracle agrees with the CPU path exactly
    assert torch.equal(got, ops.nv12_to_bgr_reference(y, uv))


@pytest.mark.gpu
def test_gpu_conversion_within_one_lsb_of_float_bt601():
    H, W = 1088, 1920
    y, uv = _planes(H, W, seed=3)
    got = ops.nv12_to_bgr(y.cuda(), uv.cuda(), 1920, 1080).cpu()
    want = ops.nv12_to_bgr_bt601_float(y, uv, 1920, 1080)
    d = (got.to(torch.int16) - want.to(torch.int16)).abs()
    assert int(d.max()) <= 1, f"max |diff| {int(d.max())}"
    assert float((d > 0).float().mean()) < 0.05  # (rounding differences only)
