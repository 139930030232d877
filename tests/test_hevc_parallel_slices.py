"""Independent slices of one H.265 picture are parsed in parallel (hevc_dec.cpp run_deferred on
the shared fan-out pool, csrc/vep/fanout.h): each slice writes its own records shard, merged in
slice order. The output must equal the sequential parse (VEP_HEVC_SLICE_THREADS=0) and the
encoder's reconstruction, record for record — for plain multi-slice pictures, slices with tiles,
and pictures whose dependent segments force the sequential path."""
import numpy as np
import pytest


def _stream(native, w, h, n, **kw):
    c = native.SynthConfig()
    c.width, c.height, c.gop, c.codec, c.compressed = w, h, 8, "h265", True
    c.bframes, c.qp = 2, 30
    for k, v in kw.items():
        setattr(c, k, v)
    s = native.SynthH264(c)
    aus, rec = [], {}
    for _ in range(n):
        aus.append(s.next())
        y, uv = s.picture()
        rec[s.last_pts] = (y.copy(), uv.copy())
    return aus, rec


def _decode(native, aus, monkeypatch, parallel, units=None):
    monkeypatch.setenv("VEP_HEVC_SLICE_THREADS", "1" if parallel else "0")
    d = native.HevcRecordsDecoder()  # records mode + the CPU mirror of the GPU kernels
    out = {}
    for au in aus:
        for pts, poc, t, (y, uv), slot in d.decode(au):
            out[pts] = (y.copy(), uv.copy())
    for pts, poc, t, (y, uv), slot in d.flush():
        out[pts] = (y.copy(), uv.copy())
    if units is not None:
        units.append(d.parallel_units)
    return out, d.stats


@pytest.mark.parametrize("kw", [dict(slices=6), dict(slices=3, tile_cols=2, tile_rows=2), dict(slices=2, segments=2),
                                dict(slices=4, coverage=True)],
                         ids=["6-slices", "slices+tiles", "dependent-segments", "coverage-4-slices"])
def test_parallel_slices_bit_exact(native, monkeypatch, kw):
    w, h = (352, 288) if kw.get("coverage") else (640, 360)
    aus, rec = _stream(native, w, h, 10, **kw)
    par, st_par = _decode(native, aus, monkeypatch, True)
    seq, st_seq = _decode(native, aus, monkeypatch, False)
    assert set(par) == set(seq) == set(rec)
    for pts in rec:
        for a, b, r in zip(par[pts], seq[pts], rec[pts]):
            assert np.array_equal(a, b) and np.array_equal(a, r[: a.shape[0], : a.shape[1]]), pts
    assert st_par == st_seq  # identical records (counts of PUs / TUs / intra TUs / levels)


@pytest.mark.parametrize("kw", [dict(tile_cols=3, tile_rows=2), dict(tile_cols=2, tile_rows=3, coverage=True, seed=5),
                                dict(tile_cols=4, tile_rows=1, bit_depth=10)],
                         ids=["1-slice-6-tiles", "coverage-tiles", "main10-tiles"])
def test_parallel_tiles_of_one_slice_bit_exact(native, monkeypatch, kw):
    """One slice, several tiles: each tile substream (found from the slice header's entry point
    offsets, emulation prevention bytes counted) is parsed as a unit of its own."""
    w, h = (352, 288) if kw.get("coverage") else (640, 360)
    aus, rec = _stream(native, w, h, 8, **kw)
    units = []
    par, st_par = _decode(native, aus, monkeypatch, True, units)
    seq, st_seq = _decode(native, aus, monkeypatch, False)
    assert set(par) == set(seq) == set(rec)
    for pts in rec:
        for a, b, r in zip(par[pts], seq[pts], rec[pts]):
            assert np.array_equal(a, b) and np.array_equal(a, r[: a.shape[0], : a.shape[1]]), pts
    assert st_par == st_seq
    tiles = kw["tile_cols"] * kw["tile_rows"]
    assert units[0] >= tiles * len(aus) // 2  # the pictures ran tile by tile


@pytest.mark.parametrize("kw", [dict(wpp=True), dict(wpp=True, slices=3, coverage=True, seed=9),
                                dict(wpp=True, bit_depth=10, bframes=1)],
                         ids=["wpp-1-slice", "wpp-3-slices-coverage", "wpp-main10"])
def test_parallel_wavefront_rows_bit_exact(native, monkeypatch, kw):
    """WPP: each CTB row (a substream at its entry point) is a unit of its own; a row waits for
    the CTBs above-left / above / above-right of each CTB it parses and takes its contexts from
    the row above's storage after that row's 2nd CTB (the two-CTB lag)."""
    w, h = (352, 288) if kw.get("coverage") else (640, 360)
    aus, rec = _stream(native, w, h, 8, **kw)
    units = []
    par, st_par = _decode(native, aus, monkeypatch, True, units)
    seq, st_seq = _decode(native, aus, monkeypatch, False)
    assert set(par) == set(seq) == set(rec)
    for pts in rec:
        for a, b, r in zip(par[pts], seq[pts], rec[pts]):
            assert np.array_equal(a, b) and np.array_equal(a, r[: a.shape[0], : a.shape[1]]), pts
    assert st_par == st_seq
    rows = (h + 31) // 32
    assert units[0] >= rows * len(aus) // 2  # the pictures ran row by row
