"""Minimal ISO-BMFF (MP4) demuxer for H.264 / H.265 video tracks.

Reads what a camera archive or a test clip holds: the first video track's decoder configuration
(avcC / hvcC parameter sets), every sample's byte range (stsz / stco / co64 / stsc), sync samples
(stss), decoding times (stts) and composition offsets (ctts). Samples are returned as lists of
NAL units (length-prefixed in the file, prefix stripped), ready for
``native.AccessUnit.from_nals``. Used by the tests to drive real encoder output (e.g. x264 High
profile clips) through the native decoder, and by ``vep synth --mp4`` to replay a clip as a
camera. Reference parity: the per-GOP MP4 segments the reference writes (python/archive.py:45-100)
are readable with it.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Iterator


@dataclass
class Mp4Track:
    codec: str = ""                 # "avc1" / "hvc1" / "hev1"
    width: int = 0
    height: int = 0
    timescale: int = 90000
    nal_len: int = 4                # NAL length prefix size
    param_sets: list[bytes] = field(default_factory=list)  # SPS/PPS (VPS) NALs
    offsets: list[int] = field(default_factory=list)
    sizes: list[int] = field(default_factory=list)
    sync: set[int] | None = None    # sample indices (0-based) that are keyframes; None = all
    dts: list[int] = field(default_factory=list)
    cts_offset: list[int] = field(default_factory=list)


def _boxes(buf: bytes, off: int, end: int) -> Iterator[tuple[bytes, int, int]]:
    while off + 8 <= end:
        size, typ = struct.unpack(">I4s", buf[off:off + 8])
        hdr = 8
        if size == 1:
            size = struct.unpack(">Q", buf[off + 8:off + 16])[0]
            hdr = 16
        elif size == 0:
            size = end - off
        if size < hdr or off + size > end:
            break
        yield typ, off + hdr, off + size
        off += size


def _find(buf: bytes, off: int, end: int, typ: bytes):
    for t, b, e in _boxes(buf, off, end):
        if t == typ:
            return b, e
    return None


def _parse_avcc(b: bytes) -> tuple[int, list[bytes]]:
    nal_len = (b[4] & 3) + 1
    n_sps = b[5] & 0x1F
    p, out = 6, []
    for _ in range(n_sps):
        ln = struct.unpack(">H", b[p:p + 2])[0]
        out.append(b[p + 2:p + 2 + ln])
        p += 2 + ln
    n_pps = b[p]
    p += 1
    for _ in range(n_pps):
        ln = struct.unpack(">H", b[p:p + 2])[0]
        out.append(b[p + 2:p + 2 + ln])
        p += 2 + ln
    return nal_len, out


def _parse_hvcc(b: bytes) -> tuple[int, list[bytes]]:
    nal_len = (b[21] & 3) + 1
    n_arrays = b[22]
    p, out = 23, []
    for _ in range(n_arrays):
        n = struct.unpack(">H", b[p + 1:p + 3])[0]
        p += 3
        for _ in range(n):
            ln = struct.unpack(">H", b[p:p + 2])[0]
            out.append(b[p + 2:p + 2 + ln])
            p += 2 + ln
    return nal_len, out


def parse(buf: bytes) -> Mp4Track:
    """The first H.264 / H.265 video track of an MP4 file."""
    moov = _find(buf, 0, len(buf), b"moov")
    if moov is None:
        raise ValueError("no moov box")
    for t, tb, te in _boxes(buf, *moov):
        if t != b"trak":
            continue
        mdia = _find(buf, tb, te, b"mdia")
        if mdia is None:
            continue
        mdhd = _find(buf, *mdia, b"mdhd")
        minf = _find(buf, *mdia, b"minf")
        stbl = _find(buf, *minf, b"stbl") if minf else None
        stsd = _find(buf, *stbl, b"stsd") if stbl else None
        if stsd is None:
            continue
        entry = None
        for et, eb, ee in _boxes(buf, stsd[0] + 8, stsd[1]):
            if et in (b"avc1", b"hvc1", b"hev1"):
                entry = (et, eb, ee)
                break
        if entry is None:
            continue
        tr = Mp4Track(codec=entry[0].decode())
        tr.width, tr.height = struct.unpack(">HH", buf[entry[1] + 24:entry[1] + 28])
        # VisualSampleEntry: 78 bytes before its child boxes
        for ct, cb, ce in _boxes(buf, entry[1] + 78, entry[2]):
            if ct == b"avcC":
                tr.nal_len, tr.param_sets = _parse_avcc(buf[cb:ce])
            elif ct == b"hvcC":
                tr.nal_len, tr.param_sets = _parse_hvcc(buf[cb:ce])
        if mdhd:
            v = buf[mdhd[0]]
            tr.timescale = struct.unpack(">I", buf[mdhd[0] + (20 if v == 1 else 12):][:4])[0]
        b = {t2: (x, y) for t2, x, y in _boxes(buf, *stbl)}
        o = b[b"stsz"][0]
        fixed, count = struct.unpack(">II", buf[o + 4:o + 12])
        tr.sizes = [fixed] * count if fixed else list(struct.unpack(f">{count}I", buf[o + 12:o + 12 + 4 * count]))
        if b"stco" in b:
            o = b[b"stco"][0]
            n = struct.unpack(">I", buf[o + 4:o + 8])[0]
            chunks = list(struct.unpack(f">{n}I", buf[o + 8:o + 8 + 4 * n]))
        else:
            o = b[b"co64"][0]
            n = struct.unpack(">I", buf[o + 4:o + 8])[0]
            chunks = list(struct.unpack(f">{n}Q", buf[o + 8:o + 8 + 8 * n]))
        o = b[b"stsc"][0]
        n = struct.unpack(">I", buf[o + 4:o + 8])[0]
        stsc = [struct.unpack(">III", buf[o + 8 + 12 * i:o + 20 + 12 * i]) for i in range(n)]
        s = 0
        for ci, off in enumerate(chunks):
            per = 0
            for first, spc, _ in stsc:
                if first - 1 <= ci:
                    per = spc
            for _ in range(per):
                if s >= count:
                    break
                tr.offsets.append(off)
                off += tr.sizes[s]
                s += 1
        if b"stss" in b:
            o = b[b"stss"][0]
            n = struct.unpack(">I", buf[o + 4:o + 8])[0]
            tr.sync = {v - 1 for v in struct.unpack(f">{n}I", buf[o + 8:o + 8 + 4 * n])}
        t0 = 0
        if b"stts" in b:
            o = b[b"stts"][0]
            n = struct.unpack(">I", buf[o + 4:o + 8])[0]
            for i in range(n):
                c, d = struct.unpack(">II", buf[o + 8 + 8 * i:o + 16 + 8 * i])
                for _ in range(c):
                    tr.dts.append(t0)
                    t0 += d
        tr.cts_offset = [0] * count
        if b"ctts" in b:
            o = b[b"ctts"][0]
            n = struct.unpack(">I", buf[o + 4:o + 8])[0]
            k = 0
            for i in range(n):
                c, d = struct.unpack(">Ii", buf[o + 8 + 8 * i:o + 16 + 8 * i])
                for _ in range(c):
                    if k < count:
                        tr.cts_offset[k] = d
                    k += 1
        return tr
    raise ValueError("no H.264/H.265 video track")


def samples(buf: bytes, tr: Mp4Track) -> Iterator[tuple[list[bytes], bool, int, int]]:
    """(NAL list, keyframe, dts, pts) per sample in decoding order; timestamps in 90 kHz."""
    for i, (off, size) in enumerate(zip(tr.offsets, tr.sizes)):
        nals, p, end = [], off, off + size
        while p + tr.nal_len <= end:
            ln = int.from_bytes(buf[p:p + tr.nal_len], "big")
            p += tr.nal_len
            nals.append(buf[p:p + ln])
            p += ln
        key = tr.sync is None or i in tr.sync
        dts = tr.dts[i] if i < len(tr.dts) else 0
        pts = dts + (tr.cts_offset[i] if i < len(tr.cts_offset) else 0)
        scale = 90000 / max(1, tr.timescale)
        yield nals, key, int(dts * scale), int(pts * scale)
