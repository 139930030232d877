"""Tensor-level ops backed by the gfx950 HIP kernels (and their plain-PyTorch references).

* :func:`nv12_to_bgr` — BT.601 limited-range NV12 -> packed BGR24 (the kernel behind
  ``VideoFrame.data``; reference: python/read_image.py:94 ``to_ndarray(format='bgr24')``).
* :func:`pcm_decode_bgr` — fused I_PCM macroblock reconstruction + conversion.
* :func:`letterbox` — NV12 -> letterboxed model input (HWC uint8 and/or normalised CHW).

The ``*_reference`` functions are the fp32 PyTorch oracles the GPU tests compare against.
Calling a GPU op on a host with no HIP device raises (no silent CPU fallback).
"""
from __future__ import annotations

import torch

from .._native import native, require_gpu

_CHW_DTYPES = {None: 0, torch.float16: 1, torch.bfloat16: 2, torch.float32: 3}


def _stream_ptr(t: torch.Tensor) -> int:
    return int(torch.cuda.current_stream(t.device).cuda_stream)


def _check_nv12(y: torch.Tensor, uv: torch.Tensor):
    if not (y.is_cuda and uv.is_cuda):
        raise ValueError("nv12 planes must be device tensors")
    if y.dtype != torch.uint8 or uv.dtype != torch.uint8:
        raise TypeError("nv12 planes must be uint8")
    if not (y.is_contiguous() and uv.is_contiguous()):
        raise ValueError("nv12 planes must be contiguous")
    H, W = y.shape
    if W % 16 or H % 16:
        raise ValueError("coded NV12 size must be macroblock aligned (multiple of 16)")
    if tuple(uv.shape) != (H // 2, W):
        raise ValueError(f"uv plane must be {(H // 2, W)}, got {tuple(uv.shape)}")
    return H, W


def nv12_to_bgr(y: torch.Tensor, uv: torch.Tensor, width: int | None = None,
                height: int | None = None, crop_left: int = 0, crop_top: int = 0,
                out: torch.Tensor | None = None) -> torch.Tensor:
    """Convert a macroblock-aligned NV12 surface to a ``[height, width, 3]`` BGR24 tensor."""
    require_gpu()
    H, W = _check_nv12(y, uv)
    width = W - crop_left if width is None else width
    height = H - crop_top if height is None else height
    if out is None:
        out = torch.empty((height, width, 3), dtype=torch.uint8, device=y.device)
    assert out.is_contiguous() and tuple(out.shape) == (height, width, 3)
    native.nv12_to_bgr(y.data_ptr(), uv.data_ptr(), 0, 0, 0, 0, W // 16, H // 16, width,
                       height, crop_left, crop_top, out.data_ptr(), _stream_ptr(y))
    return out


def mb_mask_prefix(mb_slot: torch.Tensor):
    """Dense per-MB slot map -> (coded-MB bitmask words, exclusive per-word popcount prefix,
    raster-order permutation of the payload slots) — the compact form the kernel consumes."""
    s = mb_slot.detach().to("cpu", torch.int64)
    n = s.numel()
    words = (n + 31) // 32
    coded = torch.zeros(words * 32, dtype=torch.int64)
    coded[:n] = (s >= 0).to(torch.int64)
    bits = coded.view(words, 32) << torch.arange(32, dtype=torch.int64)
    mask = bits.sum(1)
    counts = coded.view(words, 32).sum(1)
    prefix = torch.cumsum(counts, 0) - counts
    order = s[s >= 0]
    to_i32 = lambda t: torch.where(t >= 2**31, t - 2**32, t).to(torch.int32)
    return to_i32(mask), prefix.to(torch.int32), order


def pcm_decode_bgr(y: torch.Tensor, uv: torch.Tensor, mb_slot: torch.Tensor,
                   payload: torch.Tensor, width: int | None = None,
                   height: int | None = None) -> torch.Tensor:
    """Apply I_PCM macroblocks (``mb_slot[mb]`` -> 384-byte slot in ``payload``, -1 = keep) to
    the NV12 surface in place and return the converted BGR24 picture."""
    require_gpu()
    H, W = _check_nv12(y, uv)
    if mb_slot.dtype != torch.int32 or mb_slot.numel() != (H // 16) * (W // 16):
        raise ValueError("mb_slot must be int32 with one entry per macroblock")
    if payload.dtype != torch.uint8 or payload.numel() % 384:
        raise ValueError("payload must be uint8 with 384-byte slots")
    nslots = payload.numel() // 384
    if nslots and int(mb_slot.max().item()) >= nslots:
        raise ValueError("mb_slot references a payload slot out of range")
    width = W if width is None else width
    height = H if height is None else height
    mask, prefix, order = mb_mask_prefix(mb_slot)
    offsets = (order * 384).to(torch.int32).to(y.device)  # samples read in place from payload
    mask, prefix = mask.to(y.device), prefix.to(y.device)
    payload = payload.to(y.device).contiguous()
    out = torch.empty((height, width, 3), dtype=torch.uint8, device=y.device)
    native.nv12_to_bgr(y.data_ptr(), uv.data_ptr(), mask.data_ptr(), prefix.data_ptr(),
                       offsets.data_ptr(), payload.data_ptr(), W // 16, H // 16, width, height,
                       0, 0, out.data_ptr(), _stream_ptr(y))
    torch.cuda.current_stream(y.device).synchronize()  # host-built index tensors go out of scope
    return out


def letterbox_geometry(src_w: int, src_h: int, size: int, even: bool = False):
    """(new_w, new_h, pad_x, pad_y) of the centred aspect-preserving fit (even: NV12-aligned)."""
    return tuple(native.letterbox_geometry(src_w, src_h, size, even))


def letterbox_nv12(y: torch.Tensor, uv: torch.Tensor, size: int = 640, width: int | None = None,
                   height: int | None = None, crop_left: int = 0, crop_top: int = 0,
                   pad_value: int = 114) -> torch.Tensor:
    """NV12 -> letterboxed NV12 ``[S*S*3/2]`` uint8 (Y and UV planes resized independently):
    the compact consumer format that crosses xGMI in the all-gather."""
    require_gpu()
    H, W = _check_nv12(y, uv)
    width = W - crop_left if width is None else width
    height = H - crop_top if height is None else height
    if size % 8:
        raise ValueError("size must be a multiple of 8")
    out = torch.empty((size * size * 3 // 2,), dtype=torch.uint8, device=y.device)
    native.letterbox(y.data_ptr(), uv.data_ptr(), W, width, height, crop_left, crop_top, size,
                     out.data_ptr(), 0, 0, [0.0] * 3, [1.0] * 3, int(pad_value), _stream_ptr(y), 1)
    return out


def nv12_to_chw(batch: torch.Tensor, size: int, dtype: torch.dtype = torch.bfloat16,
                mean=(0.0, 0.0, 0.0), std=(1.0, 1.0, 1.0)) -> torch.Tensor:
    """Consumer-side: ``[N, S*S*3/2]`` NV12 batch -> ``[N, 3, S, S]`` normalised RGB (BT.601)."""
    require_gpu()
    if batch.dtype != torch.uint8 or not batch.is_contiguous():
        raise ValueError("batch must be contiguous uint8")
    n = batch.numel() // (size * size * 3 // 2)
    if n * size * size * 3 // 2 != batch.numel():
        raise ValueError("batch size is not a whole number of S x S NV12 pictures")
    out = torch.empty((n, 3, size, size), dtype=dtype, device=batch.device)
    native.nv12_to_chw(batch.data_ptr(), out.data_ptr(), n, size, _CHW_DTYPES[dtype],
                       list(map(float, mean)), list(map(float, std)), _stream_ptr(batch))
    return out


def letterbox_nv12_reference(y: torch.Tensor, uv: torch.Tensor, size: int, width: int,
                             height: int, pad_value: int = 114) -> torch.Tensor:
    """fp32 torch reference of :func:`letterbox_nv12` (per-plane bilinear, align_corners=False)."""
    import torch.nn.functional as F

    nw, nh, px, py = letterbox_geometry(width, height, size, even=True)
    ypad = round(16 + pad_value * 219 / 255)
    Y = y[:height, :width].float()[None, None]
    yo = torch.full((size, size), float(ypad), device=y.device)
    yo[py:py + nh, px:px + nw] = F.interpolate(Y, size=(nh, nw), mode="bilinear",
                                               align_corners=False)[0, 0]
    cw, chh = (width + 1) // 2, (height + 1) // 2
    C = uv[:chh, :cw * 2].float().view(chh, cw, 2).permute(2, 0, 1)[None]
    co = torch.full((2, size // 2, size // 2), 128.0, device=y.device)
    co[:, py // 2:py // 2 + nh // 2, px // 2:px // 2 + nw // 2] = F.interpolate(
        C, size=(nh // 2, nw // 2), mode="bilinear", align_corners=False)[0]
    out_y = (yo + 0.5).clamp(0, 255).floor().to(torch.uint8).flatten()
    out_c = (co + 0.5).clamp(0, 255).floor().to(torch.uint8).permute(1, 2, 0).flatten()
    return torch.cat([out_y, out_c])


def letterbox(y: torch.Tensor, uv: torch.Tensor, size: int = 640, width: int | None = None,
              height: int | None = None, crop_left: int = 0, crop_top: int = 0,
              chw_dtype: torch.dtype | None = None, mean=(0.0, 0.0, 0.0), std=(1.0, 1.0, 1.0),
              pad_value: int = 114, hwc: bool = True):
    """NV12 -> (hwc uint8 [S,S,3] BGR or None, chw [3,S,S] RGB normalised or None)."""
    require_gpu()
    H, W = _check_nv12(y, uv)
    width = W - crop_left if width is None else width
    height = H - crop_top if height is None else height
    if size % 4:
        raise ValueError("size must be a multiple of 4")
    out_hwc = torch.empty((size, size, 3), dtype=torch.uint8, device=y.device) if hwc else None
    out_chw = (torch.empty((3, size, size), dtype=chw_dtype, device=y.device)
               if chw_dtype is not None else None)
    native.letterbox(y.data_ptr(), uv.data_ptr(), W, width, height, crop_left, crop_top, size,
                     out_hwc.data_ptr() if out_hwc is not None else 0,
                     out_chw.data_ptr() if out_chw is not None else 0,
                     _CHW_DTYPES[chw_dtype], list(map(float, mean)), list(map(float, std)),
                     int(pad_value), _stream_ptr(y))
    return out_hwc, out_chw


# ----------------------------------------------------------------------------- references

def nv12_to_bgr_reference(y: torch.Tensor, uv: torch.Tensor, width=None, height=None,
                          crop_left=0, crop_top=0) -> torch.Tensor:
    """Bit-exact oracle of the conversion kernel's integer arithmetic (BT.601 limited range,
    nearest chroma): each channel = floor((c + k*d + 2^15) / 2^16) with the kernel's 16.16
    coefficients. It shares the kernel's constants, so it pins the implementation, not the colour
    science: ``nv12_to_bgr_bt601_float`` is the independent check (±1 LSB)."""
    H, W = y.shape
    width = W - crop_left if width is None else width
    height = H - crop_top if height is None else height
    Y = y[crop_top:crop_top + height, crop_left:crop_left + width].to(torch.int64)
    xs = torch.arange(crop_left, crop_left + width, device=y.device) // 2 * 2
    ys = torch.arange(crop_top, crop_top + height, device=y.device) // 2
    U = uv[ys][:, xs].to(torch.int64)
    V = uv[ys][:, xs + 1].to(torch.int64)
    c = (Y - 16) * 76309 + 32768
    d, e = U - 128, V - 128
    r = torch.div(c + 104597 * e, 65536, rounding_mode="floor")
    g = torch.div(c - 25675 * d - 53279 * e, 65536, rounding_mode="floor")
    b = torch.div(c + 132201 * d, 65536, rounding_mode="floor")
    return torch.stack([b, g, r], dim=-1).clamp(0, 255).to(torch.uint8)


def nv12_to_bgr_bt601_float(y: torch.Tensor, uv: torch.Tensor, width=None, height=None,
                            crop_left=0, crop_top=0) -> torch.Tensor:
    """Independent float64 BT.601 limited-range YCbCr -> BGR (what swscale's default converts,
    read_image.py:94 ``to_ndarray('bgr24')``), derived from the standard's definitions rather than
    from any fixed-point constants: Kr = 0.299, Kb = 0.114, luma scaled by 255/219 from
    [16, 235], chroma by 255/224 around 128; round to nearest, clip to [0, 255]. Nearest chroma
    sample (4:2:0, the sample at or left of / above the luma position)."""
    H, W = y.shape
    width = W - crop_left if width is None else width
    height = H - crop_top if height is None else height
    kr, kb = 0.299, 0.114
    kg = 1.0 - kr - kb
    Y = (y[crop_top:crop_top + height, crop_left:crop_left + width].to(torch.float64) - 16.0) * (255.0 / 219.0)
    xs = torch.arange(crop_left, crop_left + width, device=y.device) // 2 * 2
    ys = torch.arange(crop_top, crop_top + height, device=y.device) // 2
    pb = (uv[ys][:, xs].to(torch.float64) - 128.0) * (255.0 / 224.0)
    pr = (uv[ys][:, xs + 1].to(torch.float64) - 128.0) * (255.0 / 224.0)
    r = Y + 2.0 * (1.0 - kr) * pr
    b = Y + 2.0 * (1.0 - kb) * pb
    g = Y - (2.0 * (1.0 - kb) * kb / kg) * pb - (2.0 * (1.0 - kr) * kr / kg) * pr
    bgr = torch.stack([b, g, r], dim=-1)
    return torch.floor(bgr + 0.5).clamp(0, 255).to(torch.uint8)


def letterbox_reference(bgr: torch.Tensor, size: int = 640, pad_value: int = 114,
                        chw_dtype=None, mean=(0.0, 0.0, 0.0), std=(1.0, 1.0, 1.0)):
    """fp32 torch reference: bilinear (align_corners=False) resize + centred pad."""
    import torch.nn.functional as F

    h, w = bgr.shape[:2]
    nw, nh, px, py = letterbox_geometry(w, h, size)
    x = bgr.permute(2, 0, 1)[None].float()
    r = F.interpolate(x, size=(nh, nw), mode="bilinear", align_corners=False, antialias=False)[0]
    canvas = torch.full((3, size, size), float(pad_value), device=bgr.device)
    canvas[:, py:py + nh, px:px + nw] = r
    hwc = (canvas + 0.5).clamp(0, 255).floor().to(torch.uint8).permute(1, 2, 0).contiguous()
    chw = None
    if chw_dtype is not None:
        rgb = canvas.flip(0) / 255.0
        m = torch.tensor(mean, device=bgr.device).view(3, 1, 1)
        s = torch.tensor(std, device=bgr.device).view(3, 1, 1)
        chw = ((rgb - m) / s).to(chw_dtype)
    return hwc, chw
