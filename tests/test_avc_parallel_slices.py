"""Slices of one H.264 picture are parsed in parallel (avc.cpp Decoder::parse on the shared
fan-out pool, csrc/vep/fanout.h): each slice runs the macroblock layer on its own neighbour
state — MBs of other slices are unavailable to it by definition (§6.4.11) — into its own
records shard (MbRecs + coefficient / motion / weight pools), merged in slice order with the
pool offsets rebased. The decoded pictures must equal the sequential parse
(VEP_AVC_SLICE_THREADS=0) and the encoder's reconstruction, for CABAC and CAVLC, I / P / B
slices, direct / weighted prediction and the CAVLC Baseline path."""
import numpy as np
import pytest

from conftest import high_encoder


def _decode(native, aus, monkeypatch, parallel):
    monkeypatch.setenv("VEP_AVC_SLICE_THREADS", "1" if parallel else "0")
    dec = native.CpuDecoder()
    got = {}
    for au in aus:
        dec.decode(au)
        for pts, planes in dec.frames():
            got[pts] = planes
    for pts, planes in dec.flush_frames():
        got[pts] = planes
    return got, dec


CONFIGS = {
    "high-cabac-4-slices": dict(bframes=2, slices=4),
    "high-cavlc-3-slices": dict(bframes=1, cabac=False, slices=3),
    "cov-cabac-slices-wp": dict(bframes=3, coverage=True, slices=3, weighted_b=1, weighted_p=True),
    "cov-temporal-direct-slices": dict(bframes=2, coverage=True, direct_spatial=False, slices=5, deblock_idc=2),
}


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_parallel_slices_bit_exact(native, monkeypatch, name):
    enc = high_encoder(native, 176, 144, gop=10, seed=5, **CONFIGS[name])
    aus, rec = [], {}
    for _ in range(14):
        aus.append(enc.next())
        y, uv = enc.picture()
        rec[enc.last_pts] = (y.copy(), uv.copy())
    par, dpar = _decode(native, aus, monkeypatch, True)
    seq, dseq = _decode(native, aus, monkeypatch, False)
    assert set(par) == set(seq) == set(rec)
    for pts in rec:
        for a, b, r in zip(par[pts], seq[pts], rec[pts]):
            assert np.array_equal(a, b) and np.array_equal(a, r), (name, pts)
    assert dpar.parallel_slices >= 2 * len(aus) and dseq.parallel_slices == 0
    assert dpar.mb_stats == dseq.mb_stats


def test_parallel_slices_baseline_cavlc(native, monkeypatch):
    """The Baseline CAVLC I/P path (the legacy macroblock decoder) with several slices."""
    c = native.SynthConfig()
    c.width, c.height, c.gop, c.compressed, c.profile, c.slices = 176, 144, 8, True, "baseline", 3
    s = native.SynthH264(c)
    aus, rec = [], {}
    for _ in range(10):
        aus.append(s.next())
        y, uv = s.picture()
        rec[s.last_pts] = (y.copy(), uv.copy())
    par, dpar = _decode(native, aus, monkeypatch, True)
    seq, _ = _decode(native, aus, monkeypatch, False)
    assert set(par) == set(seq)
    for pts in par:
        for a, b in zip(par[pts], seq[pts]):
            assert np.array_equal(a, b), pts
    assert dpar.parallel_slices >= 2 * len(aus)
