"""General H.264 path on gfx950: the inter / intra-wavefront / deblocking-wavefront kernels
(gpu_avc.hip) against the CPU reference decoder (avc.cpp), bit-exact, on real compressed
synthetic streams (CAVLC intra 4x4/16x16, P partitions down to 4x4, multi-reference, slices,
deblocking on/off/slice-edge)."""
import numpy as np
import pytest

from conftest import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize(
    "w,h,refs,slices,dbk",
    [(176, 144, 3, 2, 0), (320, 240, 1, 1, 1), (352, 288, 2, 3, 2), (1280, 720, 1, 1, 0)],
)
def test_general_decode_bit_exact_vs_cpu(native, w, h, refs, slices, dbk):
    enc = synth(native, w, h, gop=8, seed=3, slices=slices, compressed=True, coverage=True,
                refs=refs, deblock_idc=dbk)
    ref = native.CpuDecoder()
    wk = native.Worker(device=0)
    cam = wk.add_camera("avc", 3)
    for i in range(18):  # crosses two IDRs
        au = enc.next()
        want = ref.decode(au)
        assert wk.decode_now(cam, au)
        meta, got = wk.read_latest(cam, 0)
        assert got.shape == (h, w, 3)
        assert np.array_equal(got, want), f"frame {i} differs in {int((got != want).sum())} samples"
    assert ref.general and wk.stats(cam)["decoder"] == "general"


def test_general_decode_batched_cameras_and_catch_up(native):
    """Several cameras in one launch (round-batched inter / wavefront kernels) and a GOP
    catch-up job (several pictures of one camera reconstructed in sequence in one batch)."""
    encs = [synth(native, 640, 360, gop=10, seed=10 + k, compressed=True, coverage=k % 2 == 1,
                  refs=1 + k % 3) for k in range(4)]
    refs = [native.CpuDecoder() for _ in encs]
    wk = native.Worker(device=0)
    cams = [wk.add_camera(f"c{k}", 3) for k in range(4)]
    backlog = [[] for _ in encs]
    for step in range(14):
        for k, (e, r) in enumerate(zip(encs, refs)):
            au = e.next()
            want = r.decode(au)
            backlog[k].append((au, want))
        if step % 3 != 2:
            continue  # let AUs pile up: the next submit carries several pictures per camera
        wk.decode_many([(cams[k], [a for a, _ in backlog[k]]) for k in range(4)])
        for k in range(4):
            _, got = wk.read_latest(cams[k], 0)
            assert np.array_equal(got, backlog[k][-1][1]), f"camera {k} step {step}"
            backlog[k].clear()


def test_general_decode_1080p_psnr(native):
    """A realistic (non-coverage) 1080p stream: GPU output equals the CPU reference and the
    encoder's closed loop, and is close to the source scene."""
    enc = synth(native, 1920, 1080, gop=30, seed=5, compressed=True, qp=26)
    ref = native.CpuDecoder()
    wk = native.Worker(device=0)
    cam = wk.add_camera("hd", 3)
    for i in range(6):
        au = enc.next()
        want = ref.decode(au)
        assert wk.decode_now(cam, au)
        _, got = wk.read_latest(cam, 0)
        assert np.array_equal(got, want), f"frame {i}"
        y, _ = enc.picture()
        gy, _ = ref.surface()
        assert np.array_equal(y, gy)


@pytest.mark.parametrize("lane_threads", [False, True])
def test_lanes_pipeline_bit_exact(native, lane_threads):
    """Cameras spread over 3 GPU lanes (independent streams + staging), batches kept in flight
    across launches (launch_async without a sync per tick), optionally with one launcher thread
    per lane: every published frame equals the CPU decoder's, and wait_published() covers
    exactly the launched sequence."""
    ncam = 5
    encs = [synth(native, 320, 240, gop=6, seed=40 + k, compressed=True, coverage=k % 2 == 0)
            for k in range(ncam)]
    refs = [native.CpuDecoder() for _ in encs]
    wk = native.Worker(device=0, lanes=3, stages=2, queue=2, lane_threads=lane_threads)
    assert wk.lanes == 3
    cams = [wk.add_camera(f"l{k}", 2) for k in range(ncam)]
    want = [[] for _ in range(ncam)]
    for step in range(9):
        batch = []
        for k in range(ncam):
            au = encs[k].next()
            want[k].append(refs[k].decode(au))
            batch.append((cams[k], [au]))
        wk.decode_many(batch, sync=False)
        seq = wk.launch_seq
        if step >= 2:
            wk.wait_published(seq - 2)
    wk.complete_all()
    for k in range(ncam):
        _, got = wk.read_latest(cams[k], 0)
        assert np.array_equal(got, want[k][-1]), f"camera {k}"


def test_lane_merge_bit_exact(native):
    """Lane launcher threads merge the batches queued behind their in-flight ones into one launch
    (Worker::merge_queued): many one-camera batches submitted without waiting queue up and merge,
    a merge never holds two jobs of one camera, and every frame stays bit-exact (a merge that put
    dependent pictures in one round would corrupt every later picture of that camera)."""
    ncam = 6
    encs = [synth(native, 320, 240, gop=8, seed=70 + k, compressed=True, coverage=k % 2 == 1)
            for k in range(ncam)]
    refs = [native.CpuDecoder() for _ in encs]
    wk = native.Worker(device=0, lanes=2, stages=2, queue=16, lane_threads=True)
    cams = [wk.add_camera(f"m{k}", 2) for k in range(ncam)]
    want = [None] * ncam
    for rnd in range(4):
        wk.hold_lanes(True)  # the launchers leave the batches queued: 12 per lane (queue 16)
        for step in range(4):
            for k in range(ncam):  # one batch per camera: consecutive batches repeat every camera
                au = encs[k].next()
                want[k] = refs[k].decode(au)
                wk.decode_many([(cams[k], [au])], sync=False)
        wk.hold_lanes(False)
        wk.complete_all()
    assert wk.merged > 0
    assert wk.frames == 16 * ncam
    for k in range(ncam):
        _, got = wk.read_latest(cams[k], 0)
        assert np.array_equal(got, want[k]), f"camera {k}"


def test_corrupt_slices_on_gpu_recover_at_idr(native):
    """Bit errors in slice data through the GPU worker: a rejected picture is dropped (the
    camera waits for the next keyframe); whatever the kernels are given has passed
    avc::validate; from the next IDR on the output equals the clean stream's, bit-exact."""
    import random

    rnd = random.Random(3)
    gop = 6
    clean = synth(native, 176, 144, gop=gop, seed=12, compressed=True, coverage=True, refs=2)
    aus = [clean.next() for _ in range(3 * gop)]
    ref = native.CpuDecoder()
    want = [ref.decode(a) for a in aus]
    for trial in range(8):
        wk = native.Worker(device=0)
        cam = wk.add_camera(f"fz{trial}", 3)
        bad_at = rnd.randrange(1, 2 * gop)
        for i, au in enumerate(aus):
            if i == bad_at:
                nals = [bytearray(n) for n in au.nals()]
                n = nals[[k for k, x in enumerate(nals) if (x[0] & 0x1F) in (1, 5)][0]]
                for _ in range(rnd.randint(1, 6)):
                    pos = rnd.randrange(2, len(n))
                    n[pos] ^= 1 << rnd.randrange(8)
                au = native.AccessUnit.from_nals([bytes(x) for x in nals], keyframe=au.keyframe)
            ok = wk.decode_now(cam, au)
            if i >= (bad_at // gop + 1) * gop:
                assert ok, f"trial {trial}: frame {i} after the IDR was dropped"
                _, got = wk.read_latest(cam, 0)
                assert np.array_equal(got, want[i]), f"trial {trial}: frame {i} differs"


CLIP = "/opt/conda/lib/python3.9/site-packages/imageio/resources/images/realshort.mp4"


@pytest.mark.skipif(not __import__("os").path.exists(CLIP), reason="imageio sample clip not in this image")
def test_third_party_high_profile_clip_bit_exact_vs_cpu(native):
    """A real High-profile CABAC clip (8x8 transform, Intra_8x8 / 4x4, P pictures): every frame
    the GPU worker publishes equals the CPU reference decoder's, bit-exact."""
    from video_edge_ai_proxy_amd.utils import mp4

    buf = open(CLIP, "rb").read()
    tr = mp4.parse(buf)
    ref = native.CpuDecoder()
    wk = native.Worker(device=0)
    cam = wk.add_camera("clip", 3)
    for i, (nals, key, dts, pts) in enumerate(mp4.samples(buf, tr)):
        au = native.AccessUnit.from_nals((tr.param_sets if i == 0 else []) + nals, keyframe=key, pts=pts, dts=dts)
        want = ref.decode(au)
        assert wk.decode_now(cam, au)
        _, got = wk.read_latest(cam, 0)
        assert np.array_equal(got, want), f"frame {i} differs in {int((got != want).sum())} samples"
    st = ref.mb_stats
    assert st["i8x8"] > 0 and st["t8x8"] > 0
    assert wk.stats(cam)["decoder"] == "general"
