"""H.265 coding tools beyond the basic Main stream, which real IP cameras use and the decoder
previously rejected: tiles (uniform and explicit spacing, loop filters across tile boundaries on
and off), wavefront parallel processing substreams (WPP), dependent slice segments, scaling lists
(default and custom, SPS and PPS), explicit weighted prediction (P and B), long-term reference
pictures (explicit and SPS candidates, with and without MSB cycles) and transquant-bypass
(lossless) CUs.

Each stream comes from the closed-loop encoder (hevc_enc.cpp) with the tool on, in coverage mode:
  * the reference CPU decoder must reproduce the encoder's reconstruction bit for bit;
  * the records-mode decoder + CPU mirror of the gfx950 kernels must equal the reference decoder
    (so the GPU kernels only have to match the mirror, tests/test_gpu_hevc_tools.py);
  * the bitstream syntax is checked independently of the decoder: entry point offsets must point
    at the substream starts, and the parameter sets must parse back to the tools' fields.
Reference behaviour: libavcodec's hevc decoder behind PyAV decodes all of these
(python/read_image.py:87); third-party parity remains unpinned (no such stream in the image).
"""
import numpy as np
import pytest

from video_edge_ai_proxy_amd import _vep as v

TOOLS = {
    "tiles_uniform": dict(tile_cols=3, tile_rows=2, width=256, height=160, log2_ctb=4),
    "tiles_explicit": dict(tile_cols=4, tile_rows=3, width=320, height=192, log2_ctb=4, seed=21, slices=2),
    "wpp": dict(wpp=True, width=256, height=160, log2_ctb=4),
    "wpp_slices": dict(wpp=True, slices=3, width=256, height=160, log2_ctb=4, seed=23),
    "tiles_wpp": dict(tile_cols=2, tile_rows=2, wpp=True, width=256, height=160, log2_ctb=4, seed=25),
    "dependent": dict(segments=3, slices=2, seed=27),
    "dependent_wpp": dict(segments=4, wpp=True, width=256, height=160, log2_ctb=4, seed=29),
    "dependent_tiles": dict(segments=3, tile_cols=2, tile_rows=2, width=256, height=160, log2_ctb=4, seed=31),
    "scaling": dict(scaling_lists=True, seed=33),
    "scaling_cov": dict(scaling_lists=True, seed=35, qp=24),
    "weighted": dict(weighted=True, bframes=2, seed=37),
    "weighted_p": dict(weighted=True, seed=39),
    "long_term": dict(long_term=True, seed=41, gop=12),
    "long_term_b": dict(long_term=True, bframes=2, seed=43, gop=12),
    "lossless": dict(lossless=True, seed=45),
    "everything": dict(tile_cols=2, tile_rows=2, wpp=True, segments=2, scaling_lists=True, weighted=True,
                       long_term=True, lossless=True, bframes=2, width=256, height=160, log2_ctb=4, seed=47,
                       gop=10),
}


def encoder(**kw):
    c = v.HevcEncConfig()
    c.width, c.height, c.gop, c.qp = 128, 96, 8, 30
    c.coverage = True
    for k, x in kw.items():
        setattr(c, k, x)
    return v.HevcEncoder(c)


def run(n=12, **kw):
    e, d, rec = encoder(**kw), v.HevcDecoder(), v.HevcRecordsDecoder()
    recon, outs, routs, aus = {}, [], [], []
    for _ in range(n):
        au = e.next()
        aus.append(au)
        y, uv = e.picture()
        recon[e.last_pts] = (y.copy(), uv.copy())
        outs += d.decode(au)
        routs += rec.decode(au)
    outs += d.flush()
    routs += rec.flush()
    return recon, outs, routs, aus, e


@pytest.mark.parametrize("name", list(TOOLS))
def test_tool_roundtrip_and_records_mirror(name):
    recon, outs, routs, _, _ = run(**TOOLS[name])
    assert len(outs) == len(recon) == len(routs)
    for (pts, poc, typ, (y, uv)), (pb, qb, tb, (yb, uvb), _slot) in zip(outs, routs):
        want_y, want_uv = recon[pts]
        assert np.array_equal(y, want_y), f"{name}: luma differs at poc {poc} ({typ}): {int((y != want_y).sum())}"
        assert np.array_equal(uv, want_uv), f"{name}: chroma differs at poc {poc} ({typ})"
        assert (pts, poc, typ) == (pb, qb, tb)
        assert np.array_equal(yb, y) and np.array_equal(uvb, uv), f"{name}: records mirror differs at poc {poc}"


def _nals(au):
    return [bytes(n) for n in au.nals()]


def _slice_nals(au):
    return [n for n in _nals(au) if ((n[0] >> 1) & 0x3F) < 32]


@pytest.mark.parametrize("name", ["wpp", "tiles_uniform", "tiles_wpp", "dependent_wpp", "everything"])
def test_entry_points_address_substreams(name):
    """Entry point offsets (emulation prevention bytes included) must land on the byte-aligned
    starts of the substreams: the CABAC data of every substream starts with a fresh arithmetic
    codeword right after the previous substream's end_of_subset_one_bit + alignment. Checked
    without the decoder: each offset must end exactly where a byte-aligned '1 0..0' stop pattern
    ends the previous substream."""
    _, _, _, aus, e = run(n=3, **TOOLS[name])
    sps, pps = e.sps_nal, e.pps_nal
    checked = 0
    for au in aus:
        for nal in _slice_nals(au):
            info = v.hevc_slice_entry_points(nal, sps, pps)
            if not info["entry_points"]:
                continue
            data_start = info["data_offset_ebsp"]
            pos = data_start
            for off in info["entry_points"]:
                pos += off
                assert pos <= len(nal)
                # the byte before a substream start ends the previous substream's alignment:
                # its lowest set bit is the alignment_bit_equal_to_one
                last = nal[pos - 1] if nal[pos - 1] != 3 or nal[pos - 2] != 0 else nal[pos - 2]
                assert last != 0, "a substream must end with its alignment bit"
                checked += 1
    assert checked > 0


def test_parameter_sets_carry_the_tools():
    e = encoder(**TOOLS["everything"])
    sps = v.parse_hevc_sps(e.sps_nal)
    pps = v.parse_hevc_pps(e.pps_nal)
    assert sps["scaling_list"] and sps["long_term_refs"]
    assert pps["tiles"] and pps["tile_cols"] == 2 and pps["tile_rows"] == 2
    assert pps["entropy_coding_sync"] and pps["dependent_slice_segments"]
    assert pps["weighted_pred"] and pps["weighted_bipred"] and pps["transquant_bypass"]


def test_scaling_list_defaults_match_spec_table():
    """Table 7-6 default 8x8 intra / inter lists (up-right diagonal order) and the up-sampled
    16x16 / 32x32 factor matrices with their DC."""
    f8 = np.array(v.hevc_scaling_factors(1, 0, None)).reshape(8, 8)
    assert f8[0, 0] == 16 and f8[7, 7] == 115 and f8[0, 7] == 24 == f8[7, 0] and f8[3, 7] == 36 == f8[7, 3]
    assert (f8 == f8.T).all()
    g8 = np.array(v.hevc_scaling_factors(1, 3, None)).reshape(8, 8)
    assert g8[7, 7] == 91 and g8[0, 7] == 24 == g8[7, 0] and g8[6, 7] == 71
    f16 = np.array(v.hevc_scaling_factors(2, 0, None)).reshape(16, 16)
    assert f16[0, 0] == 16 and f16[15, 15] == 115 and f16[14, 15] == 115 and f16[0, 1] == 16
    f4 = np.array(v.hevc_scaling_factors(0, 0, None))
    assert (f4 == 16).all()


@pytest.mark.parametrize("name", list(TOOLS) + ["coverage"])
def test_intra_edge_exchange_is_consistent(name):
    """The GPU queue kernel reconstructs every intra block of a picture in one launch; a block reads
    the reference samples other intra blocks write from their published right column / bottom row
    (GpuTu::pend). Checked on the records: every polled sample must be published by an intra block
    of a lower dependency level (a violation would be a wavefront timeout on the GPU)."""
    kw = dict(coverage=True, bframes=1, slices=2, width=200, height=120, seed=5) if name == "coverage" else TOOLS[name]
    e, rec = encoder(**kw), v.HevcRecordsDecoder()
    for _ in range(10):
        rec.decode(e.next())
    rec.flush()
    st = rec.stats
    assert st["intra_tus"] > 0 and st["exchange_violations"] == 0, st


@pytest.mark.parametrize("name", ["everything", "tiles_explicit", "scaling_cov", "long_term_b"])
def test_tool_streams_corruption_never_crashes(name):
    """Bit flips in the slice data and the parameter sets of the tool streams (tile grids,
    entry points, scaling lists, weights, long-term RPS): the reference decoder and the records
    decoder (CPU mirror of the GPU kernels, which must never index out of range) raise or
    decode; neither crashes, and a clean decoder afterwards still decodes the stream."""
    import random

    rnd = random.Random(hash(name) & 0xFFFF)
    _, _, _, aus, _ = run(n=8, **TOOLS[name])
    for trial in range(10):
        d, rec = v.HevcDecoder(), v.HevcRecordsDecoder()
        for i, au in enumerate(aus):
            nals = [bytearray(x) for x in au.nals()]
            if rnd.random() < 0.5:
                k = rnd.randrange(len(nals))
                for _ in range(rnd.randint(1, 4)):
                    pos = rnd.randrange(2, len(nals[k]))
                    nals[k][pos] ^= 1 << rnd.randrange(8)
                if rnd.random() < 0.2:
                    nals[k] = nals[k][: max(3, len(nals[k]) // 2)]
            bad = v.AccessUnit.from_nals([bytes(x) for x in nals], pts=au.pts, codec=1)
            for dec in (d, rec):
                try:
                    dec.decode(bad)
                except Exception:  # noqa: BLE001 — a NativeError / UnsupportedStream is fine
                    pass
        for dec in (d, rec):
            try:
                dec.flush()
            except Exception:  # noqa: BLE001
                pass
    clean = v.HevcDecoder()
    outs = []
    for au in aus:
        outs += clean.decode(au)
    outs += clean.flush()
    assert len(outs) == len(aus)
