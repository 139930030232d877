"""Reference picture marking and list modification (§8.2.4.3, §8.2.5) through the closed loop.

The Main / High encoder's `marking` mode writes, at random, ref_pic_list_modification commands
(short-term pictures coded relative to picNumPred with wrap-around, long-term pictures by
LongTermPicNum), adaptive marking with MMCO 1 (short-term unused), 2 (long-term unused),
3 (short-term -> long-term), 4 (MaxLongTermFrameIdx), 5 (everything unused, POC / frame_num
restart; streams without B pictures) and 6 (current picture long-term), and IDR
pictures marked long-term (long_term_reference_flag). The decoder's lists (long-term pictures
after the short-term ones, by LongTermFrameIdx), its marking, temporal direct with long-term
references (mvL0 = mvCol, mvL1 = 0) and implicit weights (default weights when a long-term
picture is involved) must track the encoder's exactly for every picture to round-trip
bit-exactly. Cameras use long-term references for their static background ("smart" codecs);
libavcodec (the reference's decoder, read_image.py:87) handles all of this.
"""
import numpy as np
import pytest

from conftest import high_encoder, roundtrip

CONFIGS = {
    "p-refs4": dict(bframes=0, refs=4),
    "p-refs4-cov": dict(bframes=0, refs=4, coverage=True),
    "ibbp-pyramid": dict(bframes=2, refs=3),
    "ibbp-cov": dict(bframes=2, refs=3, coverage=True),
    "b3-temporal-cov": dict(bframes=3, refs=4, direct_spatial=False, coverage=True),
    "cavlc-implicit": dict(bframes=2, refs=3, weighted_b=2, cabac=False),
    "explicit-wp-cov": dict(bframes=1, refs=2, weighted_b=1, weighted_p=True, coverage=True),
}


@pytest.mark.parametrize("name", sorted(CONFIGS))
@pytest.mark.parametrize("seed", [3, 5])
def test_marking_and_list_modification_bit_exact(native, name, seed):
    enc = high_encoder(native, 176, 144, gop=15, seed=seed, marking=True, **CONFIGS[name])
    rec, got, dec, aus = roundtrip(native, enc, 45)
    assert set(got) == set(rec) and len(rec) == 45
    for pts in rec:
        assert np.array_equal(rec[pts][0], got[pts][0]) and np.array_equal(rec[pts][1], got[pts][1]), pts


def test_marking_covers_every_operation(native):
    """Over a few streams every MMCO the encoder writes, list modifications and long-term
    pictures actually occur (the bit-exact test above is not vacuous)."""
    total = {}
    for name, seed in [("p-refs4", 3), ("ibbp-pyramid", 5), ("b3-temporal-cov", 3), ("p-refs4-cov", 5)]:
        enc = high_encoder(native, 176, 144, gop=15, seed=seed, marking=True, **CONFIGS[name])
        _, _, dec, _ = roundtrip(native, enc, 45)
        for k, v in dec.marking_stats.items():
            total[k] = total.get(k, 0) + v
    for k in ("mmco1", "mmco2", "mmco3", "mmco4", "mmco5", "mmco6", "list_mods", "long_term_marked"):
        assert total[k] > 0, (k, total)


def test_mmco5_restarts_poc_and_frame_num(native):
    """MMCO 5 (P streams): every reference goes, the picture counts as frame_num 0 and POC 0
    from then on — for output order too (§8.2.1: the picture's POC minus tempPicOrderCnt). A
    decoder that kept its old POC would drop the following pictures as late."""
    seen = 0
    for seed in (3, 4, 5):
        enc = high_encoder(native, 176, 144, gop=30, seed=seed, marking=True, bframes=0, refs=4)
        rec, got, dec, _ = roundtrip(native, enc, 60)
        assert set(got) == set(rec) and len(rec) == 60
        for pts in rec:
            assert np.array_equal(rec[pts][0], got[pts][0]), pts
        seen += dec.marking_stats["mmco5"]
    assert seen > 0


FIELD = dict(interlaced=True, fields=True, cabac=False, t8x8=False)
FIELD_CONFIGS = {
    "fields-p-refs4": dict(bframes=0, refs=4),
    "fields-p-refs4-cov": dict(bframes=0, refs=4, coverage=True),
    "fields-ibbp": dict(bframes=2, refs=3),
    "fields-ibbp-temporal-cov": dict(bframes=2, refs=3, coverage=True, direct_spatial=False),
    "fields-ibp-implicit": dict(bframes=1, refs=2, weighted_b=2),
}


@pytest.mark.parametrize("name", sorted(FIELD_CONFIGS))
@pytest.mark.parametrize("seed", [3, 5])
def test_field_marking_and_list_modification_bit_exact(native, name, seed):
    """The same in field pictures (§8.2.4.1 field picture numbers: 2 * FrameNumWrap + 1 for the
    current parity; MMCOs mark single fields; the sliding window works on frames; the second
    field of a pair whose first field is long-term is long-term too)."""
    enc = high_encoder(native, 176, 144, gop=15, seed=seed, marking=True, **FIELD, **FIELD_CONFIGS[name])
    rec, got, dec, aus = roundtrip(native, enc, 60)
    assert set(got) == set(rec) and len(rec) == 30
    for pts in rec:
        assert np.array_equal(rec[pts][0], got[pts][0]) and np.array_equal(rec[pts][1], got[pts][1]), pts


def test_field_marking_covers_every_operation(native):
    total = {}
    for name, seed in [("fields-p-refs4", 3), ("fields-ibbp", 4), ("fields-p-refs4-cov", 5), ("fields-ibbp", 3)]:
        enc = high_encoder(native, 176, 144, gop=15, seed=seed, marking=True, **FIELD, **FIELD_CONFIGS[name])
        _, _, dec, _ = roundtrip(native, enc, 60)
        for k, v in dec.marking_stats.items():
            total[k] = total.get(k, 0) + v
    for k in ("mmco1", "mmco2", "mmco3", "mmco4", "mmco6", "list_mods", "long_term_marked"):
        assert total[k] > 0, (k, total)


def test_field_mmco5_restarts_the_pair(native):
    """MMCO 5 in the first field of a pair: every reference goes, the field counts as frame_num 0
    and POC 0, and its pair's second field follows with frame_num 0 (P field streams)."""
    seen = 0
    for seed in (4, 5):
        enc = high_encoder(native, 176, 144, gop=30, seed=seed, marking=True, **FIELD, bframes=0, refs=4)
        rec, got, dec, _ = roundtrip(native, enc, 80)
        assert set(got) == set(rec) and len(rec) == 40
        for pts in rec:
            assert np.array_equal(rec[pts][0], got[pts][0]), pts
        seen += dec.marking_stats["mmco5"]
    assert seen > 0
