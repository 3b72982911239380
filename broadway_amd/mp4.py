"""MP4 / avcC input for the decoder.

Host-side mirror of the reference player's demuxer, Player/mp4.js:

* ``MP4Reader(data).read()`` builds the box tree the way ``MP4Reader.readBoxes``
  / ``readBox`` do (mp4.js:240-487): a box whose 4CC repeats in a parent becomes
  a list; ``trak`` boxes register a ``Track`` under their ``tkhd.trackId``;
  ``avcC`` keeps its SPS / PPS lists and requires 4-byte NAL lengths
  (``lengthSizeMinusOne == 3``, mp4.js:414-431).
* ``Track`` reproduces the sample-table arithmetic: ``sampleToSize``,
  ``sampleToChunk`` (stsc walk, mp4.js:543-611), ``chunkToOffset`` (stco),
  ``sampleToOffset`` and ``getSampleNALUnits`` (4-byte big-endian length
  prefixes stripped, mp4.js:711-722).
* ``player_nal_units(reader)`` yields the NAL units in the order
  ``MP4Player.play`` feeds them to the decoder (mp4.js:858-885): SPS[0],
  PPS[0], then every NAL of every video sample -- raw NAL units without start
  codes, which the decoder takes whole (byte_stream.c:80-236 "no start code"
  branch).

``mux_annexb`` writes the inverse: a minimal ISO-BMFF file (ftyp, moov with
one avc1 track, mdat) from an Annex-B stream, one sample per coded picture.
The reference's own MP4 fixtures (Player/mozilla_story.mp4, tree.mp4) are
not in the checkout, so tests build theirs from the seeded generator.
"""
from __future__ import annotations

import struct
from typing import Dict, Iterator, List, Optional


class MP4FormatError(ValueError):
    pass


def _assert(cond, msg="MP4 parse assertion"):
    if not cond:
        raise MP4FormatError(msg)


class _Stream:
    """Big-endian cursor over a byte range (mp4.js Bytestream)."""

    def __init__(self, data: bytes, start: int = 0, length: Optional[int] = None):
        self.data = data
        self.start = start
        self.end = len(data) if length is None else start + length
        self.pos = start

    @property
    def position(self) -> int:
        return self.pos

    @property
    def length(self) -> int:
        return self.end - self.start

    def remaining(self) -> int:
        return self.end - self.pos

    def peek32(self) -> int:
        if self.pos + 4 > self.end:
            return 0
        return struct.unpack_from(">I", self.data, self.pos)[0]

    def u8(self) -> int:
        v = self.data[self.pos]
        self.pos += 1
        return v

    def u16(self) -> int:
        v = struct.unpack_from(">H", self.data, self.pos)[0]
        self.pos += 2
        return v

    def u24(self) -> int:
        v = (self.data[self.pos] << 16) | (self.data[self.pos + 1] << 8) | self.data[self.pos + 2]
        self.pos += 3
        return v

    def u32(self) -> int:
        v = struct.unpack_from(">I", self.data, self.pos)[0]
        self.pos += 4
        return v

    def fp16(self) -> float:
        return self.u32() / 65536.0

    def fp8(self) -> float:
        return self.u16() / 256.0

    def fourcc(self) -> str:
        v = self.data[self.pos:self.pos + 4].decode("latin-1")
        self.pos += 4
        return v

    def bytes(self, n: int) -> bytes:
        v = self.data[self.pos:self.pos + n]
        self.pos += n
        return bytes(v)

    def u32_array(self, n: int) -> List[int]:
        v = list(struct.unpack_from(f">{n}I", self.data, self.pos))
        self.pos += 4 * n
        return v

    def skip(self, n: int) -> None:
        self.pos += n

    def sub(self, start: int, length: int) -> "_Stream":
        return _Stream(self.data, start, length)


class Track:
    """mp4.js Track (mp4.js:507-723): sample table lookups of one trak box."""

    def __init__(self, reader: "MP4Reader", trak: dict):
        self.file = reader
        self.trak = trak

    @property
    def stbl(self) -> dict:
        return self.trak["mdia"]["minf"]["stbl"]

    def getSampleSizeTable(self) -> List[int]:
        stsz = self.stbl["stsz"]
        if stsz.get("table") is None:           # constant sample size
            return [stsz["sampleSize"]] * stsz["count"]
        return stsz["table"]

    def getSampleCount(self) -> int:
        return len(self.getSampleSizeTable())

    def sampleToSize(self, start: int, length: int) -> int:
        table = self.getSampleSizeTable()
        return sum(table[start:start + length])

    def sampleToChunk(self, sample: int) -> dict:
        """The stsc walk of mp4.js:577-611, including its single-row shortcut."""
        table = self.stbl["stsc"]["table"]
        if len(table) == 1:
            row = table[0]
            _assert(row["firstChunk"] == 1)
            return {"index": sample // row["samplesPerChunk"], "offset": sample % row["samplesPerChunk"]}
        total = 0
        for i in range(1, len(table)):
            row, prev = table[i], table[i - 1]
            prev_chunks = row["firstChunk"] - prev["firstChunk"]
            prev_samples = prev["samplesPerChunk"] * prev_chunks
            if sample >= prev_samples:
                sample -= prev_samples
                if i == len(table) - 1:
                    return {"index": total + prev_chunks + sample // row["samplesPerChunk"],
                            "offset": sample % row["samplesPerChunk"]}
            else:
                return {"index": total + sample // prev["samplesPerChunk"],
                        "offset": sample % prev["samplesPerChunk"]}
            total += prev_chunks
        raise MP4FormatError("sample beyond the sample-to-chunk table")

    def chunkToOffset(self, chunk: int) -> int:
        return self.stbl["stco"]["table"][chunk]

    def sampleToOffset(self, sample: int) -> int:
        res = self.sampleToChunk(sample)
        return self.chunkToOffset(res["index"]) + self.sampleToSize(sample - res["offset"], res["offset"])

    def getSampleNALUnits(self, sample: int) -> List[bytes]:
        data = self.file.data
        offset = self.sampleToOffset(sample)
        end = offset + self.sampleToSize(sample, 1)
        nals = []
        while end - offset > 0:
            length = struct.unpack_from(">I", data, offset)[0]
            nals.append(bytes(data[offset + 4:offset + 4 + length]))
            offset += length + 4
        return nals

    def getTimeScale(self) -> int:
        return self.trak["mdia"]["mdhd"]["timeScale"]


class MP4Reader:
    """mp4.js MP4Reader: box tree + tracks by id."""

    def __init__(self, data: bytes):
        self.data = bytes(data)
        self.stream = _Stream(self.data)
        self.tracks: Dict[int, Track] = {}
        self.file: dict = {}

    def read(self) -> "MP4Reader":
        self._read_boxes(self.stream, self.file)
        return self

    def _read_boxes(self, stream: _Stream, parent: dict) -> None:
        while stream.peek32():
            child = self._read_box(stream)
            t = child["type"]
            if t in parent:
                old = parent[t]
                if not isinstance(old, list):
                    parent[t] = [old]
                parent[t].append(child)
            else:
                parent[t] = child

    def _read_box(self, s: _Stream) -> dict:
        box = {"offset": s.position}
        box["size"] = s.u32()
        box["type"] = s.fourcc()
        _assert(box["size"] >= 8, f"box {box['type']!r}: bad size {box['size']}")

        def remaining() -> int:
            return box["size"] - (s.position - box["offset"])

        def skip_rest() -> None:
            s.skip(remaining())

        def full_header() -> None:
            box["version"] = s.u8()
            box["flags"] = s.u24()

        def children() -> None:
            sub = s.sub(s.position, remaining())
            self._read_boxes(sub, box)
            s.skip(sub.length)

        t = box["type"]
        if t in ("moov", "mdia", "minf", "stbl", "dinf"):
            children()
        elif t == "trak":
            children()
            self.tracks[box["tkhd"]["trackId"]] = Track(self, box)
        elif t == "ftyp":
            box["majorBrand"] = s.fourcc()
            box["minorVersion"] = s.u32()
            box["compatibleBrands"] = [s.fourcc() for _ in range((box["size"] - 16) // 4)]
        elif t == "mvhd":
            full_header()
            _assert(box["version"] == 0)
            box["creationTime"], box["modificationTime"] = s.u32(), s.u32()
            box["timeScale"], box["duration"] = s.u32(), s.u32()
            skip_rest()
        elif t == "tkhd":
            full_header()
            _assert(box["version"] == 0)
            box["creationTime"], box["modificationTime"] = s.u32(), s.u32()
            box["trackId"] = s.u32()
            s.skip(4)
            box["duration"] = s.u32()
            s.skip(8)
            box["layer"], box["alternateGroup"] = s.u16(), s.u16()
            box["volume"] = s.fp8()
            s.skip(2)
            box["matrix"] = s.u32_array(9)
            box["width"], box["height"] = s.fp16(), s.fp16()
        elif t == "mdhd":
            full_header()
            _assert(box["version"] == 0)
            box["creationTime"], box["modificationTime"] = s.u32(), s.u32()
            box["timeScale"], box["duration"] = s.u32(), s.u32()
            skip_rest()
        elif t == "hdlr":
            full_header()
            s.skip(4)
            box["handlerType"] = s.fourcc()
            skip_rest()
        elif t == "stsd":
            full_header()
            box["entries"] = s.u32()
            children()
        elif t == "avc1":
            s.skip(6)
            box["dataReferenceIndex"] = s.u16()
            s.skip(16)
            box["width"], box["height"] = s.u16(), s.u16()
            s.skip(4 + 4 + 4 + 2 + 32 + 2)
            _assert(s.u16() == 0xFFFF, "avc1: color table id")
            children()
        elif t == "avcC":
            box["configurationVersion"] = s.u8()
            box["avcProfileIndication"] = s.u8()
            box["profileCompatibility"] = s.u8()
            box["avcLevelIndication"] = s.u8()
            box["lengthSizeMinusOne"] = s.u8() & 3
            _assert(box["lengthSizeMinusOne"] == 3, "avcC: only 4-byte NAL lengths (mp4.js:420)")
            box["sps"] = [s.bytes(s.u16()) for _ in range(s.u8() & 31)]
            box["pps"] = [s.bytes(s.u16()) for _ in range(s.u8())]
            skip_rest()
        elif t == "stts":
            full_header()
            n = s.u32()
            v = s.u32_array(2 * n)
            box["table"] = [{"count": v[2 * i], "delta": v[2 * i + 1]} for i in range(n)]
        elif t == "stss":
            full_header()
            box["samples"] = s.u32_array(s.u32())
        elif t == "stsc":
            full_header()
            n = s.u32()
            v = s.u32_array(3 * n)
            box["table"] = [{"firstChunk": v[3 * i], "samplesPerChunk": v[3 * i + 1],
                             "sampleDescriptionId": v[3 * i + 2]} for i in range(n)]
        elif t == "stsz":
            full_header()
            box["sampleSize"] = s.u32()
            box["count"] = s.u32()
            box["table"] = s.u32_array(box["count"]) if box["sampleSize"] == 0 else None
        elif t == "stco":
            full_header()
            box["table"] = s.u32_array(s.u32())
        else:                                   # mdat and everything else: samples are read in place
            skip_rest()
        _assert(s.position == box["offset"] + box["size"], f"box {t!r} overruns its size")
        return box

    def video_track(self) -> Track:
        """The first track whose sample description is avc1 (mp4.js uses track 1)."""
        for tid in sorted(self.tracks):
            tr = self.tracks[tid]
            if "avc1" in tr.stbl.get("stsd", {}):
                return tr
        raise MP4FormatError("no avc1 track")


def player_nal_units(reader: MP4Reader) -> Iterator[bytes]:
    """NAL units in MP4Player.play order (mp4.js:858-885): SPS[0], PPS[0],
    then every NAL unit of every video sample, without start codes."""
    video = reader.video_track()
    avcc = video.stbl["stsd"]["avc1"]["avcC"]
    yield avcc["sps"][0]
    yield avcc["pps"][0]
    for i in range(video.getSampleCount()):
        yield from video.getSampleNALUnits(i)


# ------------------------------------------------------------------ writer ---
def _nal_units_annexb(stream: bytes) -> List[bytes]:
    """NAL payloads of an Annex-B stream (start codes and trailing zeros removed)."""
    starts = []
    i, n = 0, len(stream)
    while i + 3 <= n:
        if stream[i] == 0 and stream[i + 1] == 0 and stream[i + 2] == 1:
            starts.append(i + 3)
            i += 3
        else:
            i += 1
    out = []
    for k, s0 in enumerate(starts):
        e = starts[k + 1] - 3 if k + 1 < len(starts) else n
        while e > s0 and stream[e - 1] == 0:
            e -= 1
        out.append(stream[s0:e])
    return out


def _box(t: str, payload: bytes) -> bytes:
    return struct.pack(">I", 8 + len(payload)) + t.encode("latin-1") + payload


def _full(t: str, payload: bytes, version: int = 0, flags: int = 0) -> bytes:
    return _box(t, struct.pack(">I", (version << 24) | flags) + payload)


def mux_annexb(stream: bytes, width: int, height: int, timescale: int = 30000, delta: int = 1000,
               samples_per_chunk: int = 4) -> bytes:
    """Minimal MP4 (ftyp + moov/trak/avc1/avcC + mdat) of an Annex-B H.264
    stream: SPS/PPS go to avcC, each coded picture (slices up to the next
    first_mb_in_slice == 0) becomes one sample of 4-byte length-prefixed NAL
    units, samples grouped `samples_per_chunk` to a chunk."""
    sps, pps, samples = [], [], []
    cur: List[bytes] = []
    for nal in _nal_units_annexb(stream):
        typ = nal[0] & 31
        if typ == 7:
            sps.append(nal)
        elif typ == 8:
            pps.append(nal)
        elif typ in (1, 5):
            first_mb_zero = len(nal) > 1 and (nal[1] & 0x80) != 0    # ue(v) == 0 is a single '1' bit
            if first_mb_zero and cur:
                samples.append(cur)
                cur = []
            cur.append(nal)
        # other NAL types (SEI, AUD, ...) are not carried
    if cur:
        samples.append(cur)
    if not sps or not pps or not samples:
        raise MP4FormatError("stream needs an SPS, a PPS and at least one slice")
    data = [b"".join(struct.pack(">I", len(n)) + n for n in smp) for smp in samples]
    sizes = [len(d) for d in data]
    nchunks = (len(data) + samples_per_chunk - 1) // samples_per_chunk

    s0 = sps[0]
    avcc = bytes([1, s0[1], s0[2], s0[3], 0xFC | 3, 0xE0 | len(sps)])
    avcc += b"".join(struct.pack(">H", len(x)) + x for x in sps)
    avcc += bytes([len(pps)]) + b"".join(struct.pack(">H", len(x)) + x for x in pps)
    avc1 = (b"\0" * 6 + struct.pack(">H", 1) + b"\0" * 16 + struct.pack(">HH", width, height)
            + struct.pack(">II", 0x00480000, 0x00480000) + struct.pack(">I", 0) + struct.pack(">H", 1)
            + b"\0" * 32 + struct.pack(">H", 0x18) + struct.pack(">H", 0xFFFF) + _box("avcC", avcc))
    duration = delta * len(data)

    def moov(chunk_offsets: List[int]) -> bytes:
        stsd = _full("stsd", struct.pack(">I", 1) + _box("avc1", avc1))
        stts = _full("stts", struct.pack(">III", 1, len(data), delta))
        last = len(data) - (nchunks - 1) * samples_per_chunk
        rows = [(1, samples_per_chunk)] if last == samples_per_chunk else \
            ([(1, samples_per_chunk), (nchunks, last)] if nchunks > 1 else [(1, last)])
        stsc = _full("stsc", struct.pack(">I", len(rows)) + b"".join(struct.pack(">III", fc, n, 1) for fc, n in rows))
        stsz = _full("stsz", struct.pack(">II", 0, len(sizes)) + struct.pack(f">{len(sizes)}I", *sizes))
        stco = _full("stco", struct.pack(">I", len(chunk_offsets)) + struct.pack(f">{len(chunk_offsets)}I", *chunk_offsets))
        stbl = _box("stbl", stsd + stts + stsc + stsz + stco)
        vmhd = _full("vmhd", b"\0" * 8, flags=1)
        dinf = _box("dinf", _full("dref", struct.pack(">I", 1) + _full("url ", b"", flags=1)))
        minf = _box("minf", vmhd + dinf + stbl)
        mdhd = _full("mdhd", struct.pack(">IIII", 0, 0, timescale, duration) + struct.pack(">HH", 0x55C4, 0))
        hdlr = _full("hdlr", struct.pack(">I", 0) + b"vide" + b"\0" * 12 + b"VideoHandler\0")
        mdia = _box("mdia", mdhd + hdlr + minf)
        unity = struct.pack(">9I", 0x10000, 0, 0, 0, 0x10000, 0, 0, 0, 0x40000000)
        tkhd = _full("tkhd", struct.pack(">IIIII", 0, 0, 1, 0, duration) + b"\0" * 8 + struct.pack(">HHHH", 0, 0, 0, 0)
                     + unity + struct.pack(">II", width << 16, height << 16), flags=3)
        trak = _box("trak", tkhd + mdia)
        mvhd = _full("mvhd", struct.pack(">IIII", 0, 0, timescale, duration) + struct.pack(">IH", 0x10000, 0x100)
                     + b"\0" * 10 + unity + b"\0" * 24 + struct.pack(">I", 2))
        return _box("moov", mvhd + trak)

    ftyp = _box("ftyp", b"isom" + struct.pack(">I", 0x200) + b"isomavc1")
    # two passes: the chunk offsets depend on the moov size, which does not
    # depend on the offsets' values
    size_moov = len(moov([0] * nchunks))
    base = len(ftyp) + size_moov + 8
    offs, pos = [], base
    for k in range(nchunks):
        offs.append(pos)
        pos += sum(sizes[k * samples_per_chunk:(k + 1) * samples_per_chunk])
    return ftyp + moov(offs) + _box("mdat", b"".join(data))
