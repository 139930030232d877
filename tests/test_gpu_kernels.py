"""gfx950 kernel numerics vs plain-PyTorch / CPU references (run on an MI355X)."""
import numpy as np
import pytest
import torch

from conftest import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("w,h,slices", [(640, 480, 1), (1920, 1080, 4), (352, 288, 2)])
def test_decode_convert_bit_exact_vs_cpu_decoder(native, w, h, slices):
    enc = synth(native, w, h, gop=6, motion=0.1, slices=slices)
    ref = native.CpuDecoder()
    wk = native.Worker(device=0)
    cam = wk.add_camera("c", 2)
    for i in range(13):  # crosses two IDR boundaries
        au = enc.next()
        want = ref.decode(au)
        assert wk.decode_now(cam, au)
        meta, got = wk.read_latest(cam, 0)
        assert got.shape == (h, w, 3)
        assert np.array_equal(got, want), f"frame {i} mismatch"
        assert meta["frame_type"] == ("I" if i % 6 == 0 else "P")


def test_decode_with_emulation_prevention_bytes(native):
    enc = synth(native, 320, 240, gop=4, zero=True)
    ref = native.CpuDecoder()
    wk = native.Worker(device=0)
    cam = wk.add_camera("epb", 1)
    saw_epb = False
    for _ in range(6):
        au = enc.next()
        saw_epb |= any(native.find_epb(n) for n in au.nals())
        want = ref.decode(au)
        wk.decode_now(cam, au)
        _, got = wk.read_latest(cam, 0)
        assert np.array_equal(got, want)
    assert saw_epb


def test_nv12_to_bgr_op_vs_torch_reference():
    from video_edge_ai_proxy_amd import ops

    g = torch.Generator().manual_seed(0)
    H, W = 1088, 1920
    y = torch.randint(0, 256, (H, W), dtype=torch.uint8, generator=g).cuda()
    uv = torch.randint(0, 256, (H // 2, W), dtype=torch.uint8, generator=g).cuda()
    got = ops.nv12_to_bgr(y, uv, 1920, 1080)
    want = ops.nv12_to_bgr_reference(y, uv, 1920, 1080)
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    # ragged crop (width not a multiple of 16) goes through the scalar edge path
    got2 = ops.nv12_to_bgr(y, uv, 1900, 1070, crop_left=0, crop_top=2)
    want2 = ops.nv12_to_bgr_reference(y, uv, 1900, 1070, crop_left=0, crop_top=2)
    assert torch.equal(got2, want2)


def test_pcm_decode_op_scatter():
    from video_edge_ai_proxy_amd import ops

    H, W = 64, 96
    y = torch.full((H, W), 16, dtype=torch.uint8, device="cuda")
    uv = torch.full((H // 2, W), 128, dtype=torch.uint8, device="cuda")
    mbs = (H // 16) * (W // 16)
    slot = torch.full((mbs,), -1, dtype=torch.int32)
    slot[5] = 0
    slot[17] = 1
    payload = torch.randint(16, 236, (2 * 384,), dtype=torch.uint8)
    out = ops.pcm_decode_bgr(y, uv, slot.cuda(), payload.cuda())
    torch.cuda.synchronize()
    # host oracle of the surface
    yh = torch.full((H, W), 16, dtype=torch.uint8)
    uvh = torch.full((H // 2, W), 128, dtype=torch.uint8)
    for mb, s in ((5, 0), (17, 1)):
        p = payload[s * 384:(s + 1) * 384]
        mx, my = mb % (W // 16), mb // (W // 16)
        yh[my * 16:my * 16 + 16, mx * 16:mx * 16 + 16] = p[:256].view(16, 16)
        uvh[my * 8:my * 8 + 8, mx * 16:mx * 16 + 16:2] = p[256:320].view(8, 8)
        uvh[my * 8:my * 8 + 8, mx * 16 + 1:mx * 16 + 16:2] = p[320:384].view(8, 8)
    assert torch.equal(y.cpu(), yh) and torch.equal(uv.cpu(), uvh)
    assert torch.equal(out.cpu(), ops.nv12_to_bgr_reference(yh, uvh))


@pytest.mark.parametrize("src", [(1920, 1080), (640, 480), (352, 288)])
def test_letterbox_vs_torch_reference(src):
    from video_edge_ai_proxy_amd import ops

    w, h = src
    H, W = (h + 15) // 16 * 16, (w + 15) // 16 * 16
    g = torch.Generator().manual_seed(1)
    y = torch.randint(16, 236, (H, W), dtype=torch.uint8, generator=g).cuda()
    uv = torch.randint(16, 241, (H // 2, W), dtype=torch.uint8, generator=g).cuda()
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    hwc, chw = ops.letterbox(y, uv, 640, w, h, chw_dtype=torch.float32, mean=mean, std=std)
    bgr = ops.nv12_to_bgr_reference(y, uv, w, h)
    rh, rc = ops.letterbox_reference(bgr, 640, chw_dtype=torch.float32, mean=mean, std=std)
    torch.cuda.synchronize()
    diff = (hwc.int() - rh.int()).abs()
    assert diff.max().item() <= 1
    assert (diff > 0).float().mean().item() < 0.01
    assert torch.allclose(chw, rc, atol=2.0 / 255 / 0.224)
    _, c16 = ops.letterbox(y, uv, 640, w, h, chw_dtype=torch.bfloat16, mean=mean, std=std, hwc=False)
    assert torch.allclose(c16.float(), rc, atol=0.05)


def test_worker_consumer_batch_matches_op(native):
    from video_edge_ai_proxy_amd import ops

    wk = native.Worker(device=0, letterbox_size=320, max_cameras=4)
    buf = torch.zeros((4, 320, 320, 3), dtype=torch.uint8, device="cuda")
    wk.set_consumer_buffers(buf.data_ptr(), 0, 4)
    ref = native.CpuDecoder()
    enc = synth(native, 640, 480, gop=5)
    cams = [wk.add_camera(f"c{i}", 2) for i in range(2)]
    au = enc.next()
    want = ref.decode(au)
    for c in cams:
        wk.decode_now(c, au)
    want_t = torch.from_numpy(want).cuda()
    rh, _ = ops.letterbox_reference(want_t, 320)
    for c in cams:
        d = (buf[c].int() - rh.int()).abs()
        assert d.max().item() <= 1


def test_replay_bench_runs(native):
    wk = native.Worker(device=0, letterbox_size=640, max_cameras=8)
    cfg = native.SynthConfig()
    cfg.width, cfg.height, cfg.gop = 1920, 1080, 10
    rb = native.ReplayBench(wk, 8, cfg, cached_frames=10, threads=4)
    for _ in range(12):
        rb.step()
    rb.drain()  # two ticks stay in flight until drained
    assert rb.frames == 96
    for c in rb.cameras:
        st = wk.stats(c)
        assert st["decoded"] == 12 and st["errors"] == 0


@pytest.mark.parametrize("src", [(1920, 1080), (640, 480), (352, 288)])
def test_letterbox_nv12_vs_reference(src):
    from video_edge_ai_proxy_amd import ops

    w, h = src
    H, W = (h + 15) // 16 * 16, (w + 15) // 16 * 16
    g = torch.Generator().manual_seed(2)
    y = torch.randint(16, 236, (H, W), dtype=torch.uint8, generator=g).cuda()
    uv = torch.randint(16, 241, (H // 2, W), dtype=torch.uint8, generator=g).cuda()
    got = ops.letterbox_nv12(y, uv, 640, w, h)
    want = ops.letterbox_nv12_reference(y, uv, 640, w, h)
    torch.cuda.synchronize()
    d = (got.int() - want.int()).abs()
    assert d.max().item() <= 1 and (d > 0).float().mean().item() < 0.01


def test_nv12_to_chw_vs_reference():
    from video_edge_ai_proxy_amd import ops

    S, n = 64, 3
    g = torch.Generator().manual_seed(3)
    batch = torch.randint(0, 256, (n, S * S * 3 // 2), dtype=torch.uint8, generator=g)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    got = ops.nv12_to_chw(batch.cuda(), S, torch.float32, mean, std)
    got16 = ops.nv12_to_chw(batch.cuda(), S, torch.bfloat16, mean, std)
    torch.cuda.synchronize()
    for i in range(n):
        yp = batch[i, :S * S].view(S, S)
        uvp = batch[i, S * S:].view(S // 2, S)
        bgr = ops.nv12_to_bgr_reference(yp, uvp).float() / 255.0
        rgb = bgr.flip(-1).permute(2, 0, 1)
        ref = (rgb - torch.tensor(mean).view(3, 1, 1)) / torch.tensor(std).view(3, 1, 1)
        assert torch.allclose(got[i].cpu(), ref, atol=1e-5)
        assert torch.allclose(got16[i].float().cpu(), ref, atol=0.03)


def test_worker_nv12_consumer_batch(native):
    from video_edge_ai_proxy_amd import ops

    S = 320
    wk = native.Worker(device=0, letterbox_size=S, max_cameras=2, letterbox_format=1)
    buf = torch.zeros((2, S * S * 3 // 2), dtype=torch.uint8, device="cuda")
    wk.set_consumer_buffers(buf.data_ptr(), 0, 2)
    enc = synth(native, 640, 480, gop=5)
    ref = native.CpuDecoder()
    cam = wk.add_camera("c", 3)
    for _ in range(3):
        au = enc.next()
        ref.decode(au)
        wk.decode_now(cam, au)
    yh, uvh = ref.surface()
    want = ops.letterbox_nv12_reference(torch.from_numpy(yh), torch.from_numpy(uvh), S, 640, 480)
    d = (buf[cam].cpu().int() - want.int()).abs()
    assert d.max().item() <= 1


@pytest.mark.parametrize("w,h,slices", [(3840, 2160, 1), (1920, 1080, 3)])
def test_hevc_decode_on_gpu_bit_exact_vs_cpu(native, w, h, slices):
    """The H.265 subset shares the MB-update format, so the same gfx950 kernel reconstructs it."""
    enc = synth(native, w, h, gop=4, motion=0.1, slices=slices, codec="h265", merge_cands=2)
    ref = native.CpuDecoder()
    wk = native.Worker(device=0)
    cam = wk.add_camera("hevc", 3)
    for i in range(6):
        au = enc.next()
        want = ref.decode(au)
        assert wk.decode_now(cam, au)
        meta, got = wk.read_latest(cam, 0)
        assert got.shape == (h, w, 3)
        assert np.array_equal(got, want), f"frame {i} mismatch"
        assert meta["frame_type"] == ("I" if i % 4 == 0 else "P")


def test_pinned_aus_are_read_in_place(native):
    """AUs finalised into the pinned ingest pool are gathered by the GPU without a host copy."""
    wk = native.Worker(device=0)
    assert native.pinned_pool_stats()["enabled"]
    cam = wk.add_camera("pin", 3)
    enc = synth(native, 640, 480, gop=4, motion=0.2)
    ref = native.CpuDecoder()
    for i in range(6):
        au = enc.next()
        want = ref.decode(au)
        if i % 2 == 0:
            assert au.pin() and au.pinned
        wk.decode_now(cam, au)
        _, got = wk.read_latest(cam, 0)
        assert np.array_equal(got, want), i
    assert wk.bytes_inplace > 0 and wk.bytes_staged > 0


def test_speculative_keyframe_walk_is_verified_gpu(native):
    from test_runtime_semantics import run_speculation_check

    run_speculation_check(native, 0)
