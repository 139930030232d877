"""Interlaced H.264 field pictures (PAFF: every frame coded as a top and a bottom field picture).

A field picture is decoded as a half-height picture into a field slot (frame slot s = field slots
2s and 2s + 1, top field rows then bottom field rows); the frame leaves the reorder buffer once
its second field is decoded and the output weaves the two fields. What differs from a frame
picture, all exercised here by the closed-loop encoder (`AvcHighConfig.fields`):

* the field scan of 4x4 levels (Table 8-13), POC per field (top 2k, bottom 2k + 1);
* P-field reference lists: frames by FrameNumWrap, split into fields alternating parity starting
  with the current one (§8.2.4.2.5), the first field of the current frame included;
* chroma vectors into the opposite-parity field offset by a quarter sample (Table 8-10);
* deblocking: horizontal intra MB edges get bS 3, vertical vector threshold 2 (§8.7.2.1);
* sliding-window marking on frames (a field pair is one frame of the DPB);
* B fields: lists by POC around the current field's (a frame's POC the lowest of its reference
  fields'), alternated by parity (§8.2.4.2.4 / §8.2.4.2.5); spatial and temporal direct from the
  colocated field (RefPicList1[0], its own motion table), implicit weights from field POCs.

Coverage is CAVLC I / P / B fields, 4x4 and 8x8 transforms (the 8x8 field scan is written from
the standard's table, which no source here holds to check against: the closed loop pins only the
encoder / decoder agreement, parity unpinned). CABAC field pictures need the field-coded context
tables (ctxIdx 277..398 / 436..459), which no source in this image holds (parity unpinned), and
are reported as UnsupportedStream (the VCN backend's job), as are streams mixing frame and field
pictures between IDRs. The encoder and decoder share the macroblock layer, so the
closed loop pins their agreement; the field-specific rules above are each written from the spec
tables (field scan, chroma offset, bS), and PSNR to the source checks the fields are the source's
rows."""
import numpy as np
import pytest

from conftest import high_encoder, roundtrip

PAFF = dict(interlaced=True, fields=True, cabac=False, t8x8=False, bframes=0)
PAFF_B = dict(PAFF, bframes=2)


def paff_encoder(native, w=176, h=144, **kw):
    cfg = dict(PAFF)
    cfg.update(kw)
    return high_encoder(native, w, h, **cfg)


@pytest.mark.parametrize("kw", [dict(), dict(refs=3, gop=8), dict(coverage=True), dict(slices=2, weighted_p=True),
                                dict(deblock_idc=2, qp=20, temporal_noise=2.0)],
                         ids=["ip", "refs3", "coverage", "slices-wp", "dbk2-noise"])
def test_paff_closed_loop_bit_exact(native, kw):
    kw.setdefault("gop", 6)
    enc = paff_encoder(native, seed=3, **kw)
    rec, got, dec, aus = roundtrip(native, enc, 24)  # 24 field pictures = 12 frames
    assert len(rec) == 12 and set(got) == set(rec)
    for pts in rec:
        assert np.array_equal(rec[pts][0], got[pts][0]) and np.array_equal(rec[pts][1], got[pts][1]), pts
    assert dec.pictures_decoded == 24  # one decoded picture per field
    assert dec.info["coded_height"] == 160 and dec.info["height"] == 144


@pytest.mark.parametrize("kw", [dict(bframes=1), dict(bframes=2, weighted_b=2), dict(bframes=2, direct_spatial=False),
                                dict(bframes=3, coverage=True), dict(bframes=2, weighted_b=1, refs=2, coverage=True),
                                dict(bframes=2, slices=2, direct_spatial=False, coverage=True),
                                dict(bframes=2, t8x8=True), dict(bframes=2, t8x8=True, coverage=True, scaling=True)],
                         ids=["ibp", "ibbp-implicit", "ibbp-temporal", "cov-b3", "cov-explicit-refs2",
                              "cov-temporal-slices", "high-8x8", "high-8x8-cov-scaling"])
def test_paff_b_fields_closed_loop(native, kw):
    """Non-reference B field pairs between I / P anchor pairs: the decoder's B-field lists, direct
    modes and implicit weights against the encoder's (every MB / sub-MB type in coverage mode)."""
    cfg = dict(PAFF)
    cfg.update(kw)
    enc = high_encoder(native, 176, 144, gop=9, seed=3, **cfg)
    rec, got, dec, aus = roundtrip(native, enc, 36)
    assert len(rec) == 18 and set(got) == set(rec)
    for pts in rec:
        assert np.array_equal(rec[pts][0], got[pts][0]) and np.array_equal(rec[pts][1], got[pts][1]), pts
    st = dec.mb_stats
    assert "B" in st["types"] and st["bipred"] > 0 and st["list1_only"] > 0
    if kw.get("t8x8"):  # 8x8 transform with the 8x8 field scan, Intra_8x8
        assert st["t8x8"] > 0 and st["i8x8"] > 0


def test_paff_output_per_pair_and_quality(native):
    """The top field's access unit outputs nothing; the bottom field's outputs the woven frame,
    which is close to the source frame (the fields are the source's alternate rows)."""
    enc = paff_encoder(native, 176, 144, gop=8, seed=5, qp=22)
    dec = native.CpuDecoder()
    outs = 0
    for i in range(16):
        au = enc.next()
        img = dec.decode(au)
        if i % 2 == 0:
            assert img is None, f"field {i}: a top field completes no frame"
            continue
        outs += 1
        y, _ = enc.picture()
        sy, _ = enc.source()
        mse = np.mean((y[:144].astype(np.float64) - sy[:144].astype(np.float64)) ** 2)
        psnr = 10 * np.log10(255.0 ** 2 / max(mse, 1e-9))
        assert psnr > 33, f"frame {i // 2}: PSNR {psnr:.1f} dB"
    assert outs == 8


def test_paff_pair_in_one_access_unit(native):
    """Both fields of a frame in one access unit (one RTP timestamp for the pair): the decoder
    takes the pictures apart and outputs the same frames."""
    enc = paff_encoder(native, seed=7, gop=6)
    aus = [enc.next() for _ in range(16)]
    ref = native.CpuDecoder()
    want = []
    for au in aus:
        img = ref.decode(au)
        if img is not None:
            want.append(img)
    dec = native.CpuDecoder()
    got = []
    for k in range(0, 16, 2):
        top, bot = aus[k], aus[k + 1]
        pair = native.AccessUnit.from_nals(list(top.nals()) + list(bot.nals()), top.pts, top.dts, top.keyframe)
        img = dec.decode(pair)
        assert img is not None
        got.append(img)
    assert len(got) == len(want) == 8
    for a, b in zip(got, want):
        assert np.array_equal(a, b)


def test_paff_worker_cpu_backend(native):
    """The camera runtime (CPU backend): field pictures into half-height field surfaces, the
    published frame woven from its pair, equal to the reference decoder's."""
    enc = paff_encoder(native, 176, 144, gop=6, seed=9, refs=2)
    ref = native.CpuDecoder()
    wk = native.Worker(device=-1)
    cam = wk.add_camera("paff", 4)
    published = 0
    for i in range(20):
        au = enc.next()
        want = ref.decode(au)
        ok = wk.decode_now(cam, au)
        if want is None:
            continue
        assert ok
        meta, got = wk.read_latest(cam, 0)
        assert meta["pts"] == ref.last_pts
        assert np.array_equal(got, want), f"AU {i} differs in {int((got != want).sum())} samples"
        published += 1
    assert published == 10


def _bits(b):
    return "".join(f"{x:08b}" for x in b)


def _unescape(nal):
    out, zeros = bytearray(), 0
    for x in nal:
        if zeros >= 2 and x == 3:
            zeros = 0
            continue
        out.append(x)
        zeros = zeros + 1 if x == 0 else 0
    return bytes(out)


def _escape(rbsp):
    out, zeros = bytearray(), 0
    for x in rbsp:
        if zeros >= 2 and x <= 3:
            out.append(3)
            zeros = 0
        out.append(x)
        zeros = zeros + 1 if x == 0 else 0
    return bytes(out)


def _ue_end(bits, pos):
    z = 0
    while bits[pos + z] == "0":
        z += 1
    return pos + 2 * z + 1


def _frame_idr_to_top_field(nal):
    """An interlaced frame IDR slice of the High encoder (log2_max_frame_num 16, POC lsb 16,
    delta_pic_order_cnt_bottom se(1)) rewritten as a top field IDR slice header: field_pic_flag 1,
    bottom_field_flag 0, no delta_pic_order_cnt_bottom (the slice data is left misaligned: only
    the header is meant to be read)."""
    r = _unescape(nal)
    bits = _bits(r[1:])
    pos = 0
    for _ in range(3):  # first_mb, slice_type, pps_id
        pos = _ue_end(bits, pos)
    pos += 16  # frame_num
    assert bits[pos] == "0"  # field_pic_flag of the frame picture
    head, pos = bits[:pos] + "10", pos + 1
    p2 = _ue_end(bits, pos) + 16  # idr_pic_id, pic_order_cnt_lsb
    assert bits[p2:p2 + 3] == "010"  # delta_pic_order_cnt_bottom = se(1)
    out = head + bits[pos:p2] + bits[p2 + 3:]
    out += "0" * (-len(out) % 8)
    body = bytes(int(out[i:i + 8], 2) for i in range(0, len(out), 8))
    return _escape(r[:1] + body)


def test_cabac_field_pictures_are_unsupported(native):
    enc = high_encoder(native, 176, 144, gop=10, seed=3, interlaced=True, bframes=0)  # CABAC
    au = enc.next()
    nals = [(_frame_idr_to_top_field(bytes(n)) if (n[0] & 0x1F) == 5 else n) for n in au.nals()]
    au2 = native.AccessUnit.from_nals(nals, au.pts, au.dts, au.keyframe)
    with pytest.raises(native.UnsupportedStream, match="CABAC field pictures"):
        native.CpuDecoder().decode(au2)


def test_frame_and_field_pictures_mixed_are_unsupported(native):
    """A frame picture inside a field-coded IDR period (the surfaces hold field pairs there)."""
    fenc = paff_encoder(native, seed=3, gop=30, refs=2)
    frames = high_encoder(native, 176, 144, gop=30, seed=3, interlaced=True, cabac=False, t8x8=False,
                          bframes=0, refs=2)
    dec = native.CpuDecoder()
    for _ in range(2):  # the IDR field pair
        dec.decode(fenc.next())
    frames.next()  # (its IDR)
    p = frames.next()  # a P frame picture, same SPS / PPS ids and syntax
    with pytest.raises(native.UnsupportedStream, match="mixed"):
        dec.decode(p)


def test_paff_live_rtsp_camera(native):
    """A field-pair camera end to end (CPU backend): the loopback farm sends each field as its own
    access unit, both with the frame's RTP timestamp (paced per frame, not per field); the RTP
    depacketizer, the lazy decoder (catch-up batches merged into one job) and the runtime publish
    one frame per pair, equal to the reference decoder's frame for that capture instant."""
    live_paff_check(native, -1)


@pytest.mark.gpu
def test_paff_live_rtsp_camera_gpu(native):
    """The same on gfx950 (field slots in the camera's DPB surfaces, launch_weave on output)."""
    live_paff_check(native, 0)


def live_paff_check(native, device):
    from test_live_compressed import FPS, Live, ref_index

    c = native.SynthConfig()
    c.width, c.height, c.gop, c.fps, c.seed = 176, 144, 8, FPS, 5
    c.compressed, c.profile, c.interlaced, c.objects = True, "high", 2, 3
    n_aus = 16  # 8 frames = one GOP, looped by the farm
    enc = native.SynthH264(c)
    aus = [enc.next() for _ in range(n_aus)]
    step = 90000 // FPS
    dec, ref = native.CpuDecoder(), {}
    for k in range(n_aus * 3):  # frame j = AUs 2j, 2j + 1 (RTP time j * step)
        a = aus[k % n_aus]
        img = dec.decode(native.AccessUnit.from_nals(a.nals(), pts=(k // 2) * step, dts=k * step, keyframe=a.keyframe))
        if img is not None:
            ref[dec.last_pts // step] = img
    live = Live(native, c, n_aus, device=device)
    try:
        got = live.frames(60, max_frames=12)
        st = live.w.stats(live.cam)
    finally:
        live.close()
    assert st["errors"] == 0 and len(got) >= 12, st
    for pts, img, meta in got:
        j = pts // step
        want = ref.get(ref_index(j, n_aus // 2))
        assert want is not None and np.array_equal(img, want), f"frame {j}"
    assert st["packets"] >= 2 * st["decoded"] - 2  # two access units (fields) per decoded frame


def test_paff_corruption_never_crashes(native):
    """Bit flips anywhere in field slices (headers included: parity, frame_num, POC, lists):
    every access unit decodes or raises, nothing crashes, and the stream is bit-exact again from
    the next IDR field pair on."""
    import random

    rnd = random.Random(7)
    enc = paff_encoder(native, seed=9, gop=6, bframes=2, refs=2, coverage=True, marking=True)
    aus = [enc.next() for _ in range(36)]  # 3 GOPs of 6 frames = 12 field AUs each
    clean = native.CpuDecoder()
    want = {}
    for a in aus:
        clean.decode(a)
        for pts, (y, uv) in clean.frames():
            want[pts] = y
    for trial in range(16):
        dec = native.CpuDecoder()
        bad = rnd.randrange(1, 12)
        for i, a in enumerate(aus):
            if i == bad:
                nals = [bytearray(n) for n in a.nals()]
                k = [j for j, x in enumerate(nals) if (x[0] & 0x1F) in (1, 5)][0]
                for _ in range(rnd.randint(1, 4)):
                    pos = rnd.randrange(1, min(len(nals[k]), 12 if trial % 2 else len(nals[k])))
                    nals[k][pos] ^= 1 << rnd.randrange(8)
                a = native.AccessUnit.from_nals([bytes(x) for x in nals], a.pts, a.dts, a.keyframe)
            try:
                dec.decode(a)
                frames = dec.frames()
            except (native.NativeError, native.UnsupportedStream):
                continue
            if i >= 24:  # the third GOP: bit-exact again
                for pts, (y, uv) in frames:
                    assert np.array_equal(y, want[pts]), f"trial {trial}: AU {i}"
