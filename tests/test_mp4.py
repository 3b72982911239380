"""MP4 / avcC input (broadway_amd/mp4.py, mirror of Player/mp4.js): the
config-1 plumbing stream (640x368, 30 frames -- the stand-in for the missing
Player/mozilla_story.mp4) muxed to MP4, demuxed the way
MP4Player.play feeds the decoder, and decoded through the Decoder.js API."""
import pytest

from _golden import cases, md5s, stream
from broadway_amd import mp4

CASE = "cfg1_plumbing_640x368"


def _annexb_nals(s):
    return mp4._nal_units_annexb(s)


@pytest.mark.parametrize("spc", [1, 4, 5])
def test_mux_demux_round_trip(spc):
    """Every NAL unit comes back byte-identical and in order; the sample
    table walk (stsc with one or two rows, stco, stsz) locates all 30 samples."""
    c = cases()[CASE]
    s = stream(c)
    data = mp4.mux_annexb(s, c["width"], c["height"], samples_per_chunk=spc)
    r = mp4.MP4Reader(data).read()
    v = r.video_track()
    assert v.getSampleCount() == len(c["frames"])
    assert r.file["ftyp"]["majorBrand"] == "isom"
    avcc = v.stbl["stsd"]["avc1"]["avcC"]
    assert avcc["lengthSizeMinusOne"] == 3
    assert (v.stbl["stsd"]["avc1"]["width"], v.stbl["stsd"]["avc1"]["height"]) == (c["width"], c["height"])
    nals = [n for n in _annexb_nals(s) if n[0] & 31 in (1, 5, 7, 8)]
    assert list(mp4.player_nal_units(r)) == nals
    # sample offsets are increasing and inside mdat
    mdat = r.file["mdat"]
    offs = [v.sampleToOffset(i) for i in range(v.getSampleCount())]
    assert offs == sorted(offs) and offs[0] == mdat["offset"] + 8
    assert offs[-1] + v.sampleToSize(len(offs) - 1, 1) == mdat["offset"] + mdat["size"]


def test_sample_to_chunk_matches_mp4js_table_example():
    """The stsc example of mp4.js:560-568: chunks of 3, 3, 1, 1, 1 samples."""
    t = mp4.Track(None, {"mdia": {"minf": {"stbl": {"stsc": {"table": [
        {"firstChunk": 1, "samplesPerChunk": 3, "sampleDescriptionId": 23},
        {"firstChunk": 3, "samplesPerChunk": 1, "sampleDescriptionId": 23},
        {"firstChunk": 5, "samplesPerChunk": 1, "sampleDescriptionId": 24}]}}}}})
    got = [t.sampleToChunk(i)["index"] for i in range(5)]
    # mp4.js's walk (mp4.js:590-609) for samples 0..4 of that table
    assert got == [0, 0, 0, 1, 1]


def test_avcc_rejects_other_length_sizes():
    c = cases()[CASE]
    data = bytearray(mp4.mux_annexb(stream(c), c["width"], c["height"]))
    i = data.find(b"avcC") + 4
    data[i + 4] = 0xFC | 1            # lengthSizeMinusOne = 1
    with pytest.raises(mp4.MP4FormatError):
        mp4.MP4Reader(bytes(data)).read()


@pytest.mark.gpu
def test_mp4_player_decode_vs_reference():
    """MP4Player.play order (SPS, PPS, then raw NAL units without start
    codes) through the Decoder.js API mirror: every frame bit-exact vs the
    reference decoder's MD5s of the same stream."""
    from broadway_amd.decoder import Decoder
    c = cases()[CASE]
    r = mp4.MP4Reader(mp4.mux_annexb(stream(c), c["width"], c["height"])).read()
    got = []
    dec = Decoder()
    dec.onPictureDecoded = lambda buf, w, h, infos: got.append(bytes(buf))
    for nal in mp4.player_nal_units(r):
        dec.decode(nal)
    dec.close()
    assert md5s(got) == c["frames"]
