"""GPU parity: HIP reconstruction (libh264mi.so) against the reference
decoder's per-frame MD5s (tests/golden/golden.json) and the CPU oracle,
bit-exact (integer/byte work: no tolerance)."""
import ctypes as C
import hashlib

import pytest

import oracle as O
from _golden import cases, md5s, stream
from _swdec import swdec_decode
from broadway_amd import _lib, gen
from broadway_amd.decoder import Decoder, split_annexb
from broadway_amd.engine import Capture, Engine

pytestmark = pytest.mark.gpu
CASES = cases()
SMALL = ["small_i_6x5", "small_ip_8x6_2sl", "small_ip_11x9_cip", "small_ip_13x7_qpoff", "small_plumb_9x5",
         "poc0_inorder"]


def _js_decode(s):
    """Decoder.js semantics: one NAL per decode(), no end-of-stream flush."""
    got = []
    dec = Decoder()
    dec.onPictureDecoded = lambda buf, w, h, infos: got.append(bytes(buf))
    for nal in split_annexb(s):
        dec.decode(nal)
    dec.close()
    return got


@pytest.mark.parametrize("name", SMALL)
def test_decoder_js_api_vs_reference(name):
    c = CASES[name]
    got = md5s(_js_decode(stream(c)))
    if c["overrides"].get("poc_type", 2) == 2:
        # POC type 2: output order == decode order, every picture is emitted at once
        assert got == c["frames"]
    else:
        # POC type 0: the DPB may hold pictures that only a flush (never sent
        # by Decoder.js) would release
        assert len(got) >= len(c["frames"]) - 2 and got == c["frames"][:len(got)]


@pytest.mark.parametrize("name", ["poc0_reorder", "poc0_noreorder", "cfg1_plumbing_640x368",
                                  "cfg2_720p_ionly_s1", "cfg2_720p_ionly_idc1_s2"])
def test_swdec_api_vs_reference(name):
    """H264SwDec* C-ABI with the DecTestBench protocol (incl. DPB output
    reordering and the end-of-stream flush)."""
    c = CASES[name]
    frames, errors = swdec_decode(stream(c), no_reorder=c["no_reorder"])
    assert errors == 0
    assert md5s(frames) == c["frames"]


PICS = [n for n in CASES if "pics" in CASES[n]]


@pytest.mark.parametrize("name", PICS)
def test_swdec_damaged_and_refpic_streams_vs_reference(name):
    """Through H264SwDec* on the GPU, every output picture, picture id, IDR
    flag and nbrOfErrMBs equals the reference decoder's:
    err_*: residuals out of range, lost / truncated slices, lost pictures
    (slice un-marking slice_data.c:302-358, concealment conceal.c:125-590:
    P copies, two-pass neighbour concealment of I pictures, whole-picture
    grey / copy);  ref_*: RefPicList0 modification with aliased indices, MMCO
    1-6, long-term and non-reference pictures, gaps in frame_num
    (dpb.c:224-1350, deblocking.c:348, 402)."""
    c = CASES[name]
    frames, _, pics = swdec_decode(stream(c), no_reorder=c["no_reorder"], info=True)
    assert [list(p) for p in pics] == c["pics"]
    assert md5s(frames) == c["frames"]


def test_decoder_js_api_holds_reordered_pictures():
    """Decoder.js never flushes (Decoder.c:140): with display reordering the
    emitted pictures are a prefix of the reference output."""
    c = CASES["poc0_reorder"]
    got = md5s(_js_decode(stream(c)))
    assert 0 < len(got) < len(c["frames"]) and got == c["frames"][:len(got)]


@pytest.mark.parametrize("rpw", [None, "1", "2", "3"])
def test_engine_multistream_batch_vs_oracle_replay(rpw, monkeypatch):
    """4 streams per launch vs the oracle replay; rpw: k_wgpp rows per
    workgroup forced (H264MI_RPW; 7 rows leave a partial last group), None =
    the engine's choice by batch size."""
    if rpw:
        monkeypatch.setenv("H264MI_RPW", rpw)
    streams = [gen.generate(2, 40 + i, nframes=6, w_mbs=10, h_mbs=7, crop_bottom=0, slices=2, gop=4)
               for i in range(4)]
    caps = [Capture(s) for s in streams]
    w, h = caps[0].w_mbs, caps[0].h_mbs
    nslots = max(c.nslots for c in caps)
    eng = Engine(w, h, len(caps), nslots)
    replays = [O.Replay(w, h, nslots) for _ in caps]
    npics = min(c.npics for c in caps)
    for k in range(npics):
        pics = [c.pictures[k] for c in caps]
        eng.decode(list(range(len(caps))), pics)
        for s, p in enumerate(pics):
            replays[s].picture(p.rec, p.coef, p.cur_slot)
        for s, p in enumerate(pics):
            assert eng.read(s, p.cur_slot).tobytes() == replays[s].frame(p.cur_slot), f"stream {s} picture {k}"
    assert eng.kernel_name() == "k_wgpp"
    assert eng.errors() == 0


@pytest.mark.parametrize("rpw", [None, "3"])
def test_engine_bench_streams_vs_reference(rpw, monkeypatch):
    """The bench workload (configs[3]: 8 concurrent 1080p streams, one picture
    of each per launch), 12 pictures, every frame vs the reference MD5s; also
    with three MB rows per k_wgpp workgroup (the large-batch layout)."""
    if rpw:
        monkeypatch.setenv("H264MI_RPW", rpw)
    names = [f"bench_1080p_s{s}" for s in range(100, 108)]
    caps = []
    for n in names:
        c = CASES[n]
        s = gen.generate(c["config"], c["seed"], nframes=12)
        caps.append(Capture(s))
    w, h = caps[0].w_mbs, caps[0].h_mbs
    eng = Engine(w, h, len(caps), max(c.nslots for c in caps))
    for k in range(12):
        pics = [c.pictures[k] for c in caps]
        eng.decode(list(range(len(caps))), pics)
        for s, p in enumerate(pics):
            got = hashlib.md5(eng.read(s, p.cur_slot).tobytes()).hexdigest()
            assert got == CASES[names[s]]["frames"][k], f"stream {s} picture {k}"
    assert eng.kernel_name() == "k_wgpp"
    assert eng.errors() == 0


@pytest.mark.parametrize("rank", range(8))
def test_configs3_shard_vs_reference(rank):
    """configs[3]: 64 streams, 8 per GPU.  Rank r's shard (seeds 100+8r ..
    100+8r+7, bench.shard_seeds) through bench.py's own device-resident path
    (records in HBM, one k_prep + k_wgpp launch pair per step) and its
    verification pass: all 60 pictures of all 8 streams vs the reference
    decoder's MD5s."""
    import bench
    seeds = bench.shard_seeds(rank, 8)
    n = 60
    _, caps = bench.prepare(3, seeds, n)
    L = _lib.mi()
    d_recs, d_coef, d_pics, step_rec_bytes, nslots, _ = bench.upload(L, caps, n)
    try:
        eng = Engine(caps[0].w_mbs, caps[0].h_mbs, 8, nslots)
        def step(k):   # bench.py's step: the next step's k_prep in this launch's tail
            if k + 1 < n:
                eng.decode_device_next(8, d_recs + k * step_rec_bytes, d_coef, d_pics + k * 8 * 32,
                                       d_recs + (k + 1) * step_rec_bytes, d_coef, d_pics + (k + 1) * 8 * 32)
            else:
                eng.decode_device(8, d_recs + k * step_rec_bytes, d_coef, d_pics + k * 8 * 32)
        ok, checked, missing = bench.verify_all(eng, step, caps, seeds, 3, {}, n)
        assert (ok, checked, missing) == (True, 8 * n, 0)
        assert eng.errors() == 0
        eng.close()
    finally:
        for p in (d_recs, d_coef, d_pics):
            L.h264mi_device_free(p)


def test_2160p_vs_reference():
    c = CASES["cfg5_2160p_s200"]
    frames, errors = swdec_decode(stream(c))
    assert errors == 0 and md5s(frames) == c["frames"]


def test_broadway_glue_callbacks():
    """broadwayInit/CreateStream/PlayStream with the JS-imported callbacks
    (Decoder.c:44-162): headers once, one picture callback per frame."""
    L = _lib.mi()
    c = CASES["small_ip_8x6_2sl"]
    s = stream(c)
    got, heads = [], []

    @_lib.HEADERS_CB
    def on_headers(user):
        heads.append(1)

    @_lib.PICTURE_CB
    def on_picture(user, buf, w, h):
        got.append(C.string_at(buf, w * h * 3 // 2))

    L.broadwaySetCallbacks(on_headers, on_picture, None)
    assert L.broadwayInit() == 0
    for nal in split_annexb(s):
        p = L.broadwayCreateStream(len(nal))
        C.memmove(p, nal, len(nal))
        L.broadwayPlayStream(len(nal))
    L.broadwayExit()
    assert len(heads) >= 1
    assert md5s(got) == c["frames"]
