"""Redundant coded pictures (redundant_pic_cnt > 0, §7.4.3): a decoder may ignore them when the
primary picture decodes, and this one does. A Main-profile CAVLC stream of the closed-loop
encoder is rewritten to carry redundant_pic_cnt: the PPS gets redundant_pic_cnt_present_flag,
every primary slice redundant_pic_cnt 0, and every access unit an extra redundant copy of each
slice (redundant_pic_cnt 1) whose slice data is garbage. The frames must equal the original
stream's, and every redundant slice must have been skipped."""
import numpy as np

from conftest import high_encoder


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


def _se_end(bits, pos):
    return _ue_end(bits, pos)


def _pack(header_byte, payload_bits):
    """RBSP from a payload bit string: the stop bit and zero padding appended."""
    bits = payload_bits + "1"
    bits += "0" * (-len(bits) % 8)
    return _escape(bytes([header_byte]) + bytes(int(bits[i:i + 8], 2) for i in range(0, len(bits), 8)))


def _payload(r):
    """Bits of an RBSP after the NAL header, without rbsp_trailing_bits."""
    bits = _bits(r[1:])
    return bits[:bits.rstrip("0").rfind("1")]


def _pps_with_redundant_cnt(nal):
    r = _unescape(nal)
    bits = _payload(r)
    pos = _ue_end(bits, 0)          # pps_id
    pos = _ue_end(bits, pos)        # sps_id
    pos += 2                        # entropy_coding_mode, bottom_field_pic_order_in_frame_present
    pos = _ue_end(bits, pos)        # num_slice_groups_minus1 (0)
    pos = _ue_end(bits, pos)        # num_ref_idx_l0_default_active_minus1
    pos = _ue_end(bits, pos)        # num_ref_idx_l1_default_active_minus1
    pos += 3                        # weighted_pred_flag, weighted_bipred_idc
    pos = _se_end(bits, pos)        # pic_init_qp_minus26
    pos = _se_end(bits, pos)        # pic_init_qs_minus26
    pos = _se_end(bits, pos)        # chroma_qp_index_offset
    pos += 2                        # deblocking_filter_control_present, constrained_intra_pred
    assert bits[pos] == "0"         # redundant_pic_cnt_present_flag
    return _pack(r[0], bits[:pos] + "1" + bits[pos + 1:])


def _slice_with_redundant_cnt(nal, cnt, garbage=False):
    """Insert redundant_pic_cnt (ue) after pic_order_cnt_lsb (log2_max_frame_num 16, POC lsb 16,
    progressive, no delta_pic_order_cnt_bottom); a redundant copy's slice data replaced by junk."""
    r = _unescape(nal)
    bits = _payload(r)
    pos = 0
    for _ in range(3):  # first_mb_in_slice, slice_type, pic_parameter_set_id
        pos = _ue_end(bits, pos)
    pos += 16  # frame_num
    if (r[0] & 0x1F) == 5:
        pos = _ue_end(bits, pos)  # idr_pic_id
    pos += 16  # pic_order_cnt_lsb
    ue = "1" if cnt == 0 else "010"
    rest = bits[pos:]
    if garbage:
        rest = ("1101001" * (len(rest) // 7 + 1))[:len(rest)]
    return _pack(r[0], bits[:pos] + ue + rest)


def test_redundant_slices_are_skipped(native):
    enc = high_encoder(native, 176, 144, gop=8, seed=9, cabac=False, t8x8=False, bframes=2, slices=2)
    aus = [enc.next() for _ in range(16)]
    ref, dec = native.CpuDecoder(), native.CpuDecoder()
    n_red = 0
    for a in aus:
        want = ref.decode(a)
        nals, red = [], []
        for n in a.nals():
            t = n[0] & 0x1F
            if t == 8:
                nals.append(_pps_with_redundant_cnt(bytes(n)))
            elif t in (1, 5):
                nals.append(_slice_with_redundant_cnt(bytes(n), 0))
                red.append(_slice_with_redundant_cnt(bytes(n), 1, garbage=True))
            else:
                nals.append(bytes(n))
        n_red += len(red)
        got = dec.decode(native.AccessUnit.from_nals(nals + red, a.pts, a.dts, a.keyframe))
        assert (got is None) == (want is None)
        if want is not None:
            assert np.array_equal(got, want)
    assert dec.marking_stats["redundant_slices_skipped"] == n_red == 32
