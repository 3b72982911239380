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


EDGE = sorted(n for n in CASES if n.startswith("edge_"))


@pytest.mark.parametrize("rpw", [None, "2", "3"])
def test_swdec_degenerate_shapes_vs_reference(rpw, monkeypatch):
    """One-MB, one-row, one-column and thin-strip pictures through H264SwDec*
    (25 % off-picture MVs, intra-heavy P pictures, constrained intra, a slice
    per MB): the row workgroup's first/last-MB, ring, hand-off and clamp
    corners; rpw forces 2 or 3 MB rows per k_wgpp workgroup (LDS hand-offs
    inside the group, partial last groups)."""
    if rpw:
        monkeypatch.setenv("H264MI_RPW", rpw)
    assert len(EDGE) >= 9
    for name in EDGE:
        c = CASES[name]
        frames, errors = swdec_decode(stream(c), no_reorder=c["no_reorder"])
        assert errors == 0, name
        assert md5s(frames) == c["frames"], name


PICS = [n for n in CASES if "pics" in CASES[n]]


def test_device_concealment_runs_and_matches_the_host_path(monkeypatch):
    """Neighbour-based concealment of I pictures with lost MBs runs on the
    device (k_conceal, h264mi_engine_conceal) by default, and the host path
    (H264MI_HOST_CONCEAL=1, a copy of the picture concealed on the CPU) gives
    the same pictures: both equal the reference decoder's."""
    L = _lib.mi()
    L.h264mi_conceal_launches.restype = C.c_ulonglong
    names = [n for n in PICS if n.startswith("err_")]
    before = L.h264mi_conceal_launches()
    for n in names:
        c = CASES[n]
        frames, _ = swdec_decode(stream(c), no_reorder=c["no_reorder"])
        assert md5s(frames) == c["frames"], n
    assert L.h264mi_conceal_launches() > before, "no damaged stream took the device concealment path"
    monkeypatch.setenv("H264MI_HOST_CONCEAL", "1")
    before = L.h264mi_conceal_launches()
    for n in names:
        c = CASES[n]
        frames, _ = swdec_decode(stream(c), no_reorder=c["no_reorder"])
        assert md5s(frames) == c["frames"], n
    assert L.h264mi_conceal_launches() == before


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


@pytest.mark.parametrize("rpw,mc", [(None, None), ("1", None), ("2", None), ("3", None), (None, "2"), (None, "3"),
                                    ("2", "2")])
def test_engine_multistream_batch_vs_oracle_replay(rpw, mc, monkeypatch):
    """4 streams per launch vs the oracle replay; rpw: k_wgpp rows per
    workgroup forced (H264MI_RPW; 7 rows leave a partial last group), None =
    the engine's choice by batch size; mc: MC waves per row forced
    (H264MI_MC_WAVES), None = per launch by intra share."""
    if rpw:
        monkeypatch.setenv("H264MI_RPW", rpw)
    if mc:
        monkeypatch.setenv("H264MI_MC_WAVES", mc)
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


@pytest.mark.parametrize("rpw,mc", [(None, None), (None, "2"), (None, "3"), ("3", None)])
def test_engine_bench_streams_vs_reference(rpw, mc, monkeypatch):
    """The bench workload (configs[3]: 8 concurrent 1080p streams, one picture
    of each per launch), 12 pictures, every frame vs the reference MD5s; also
    with three MB rows per k_wgpp workgroup (the large-batch layout), and with
    the row workgroup's MC waves forced to 2 or 3 for every launch (mc None:
    per launch, 3 for the IDR launch, 2 for the P launches)."""
    if rpw:
        monkeypatch.setenv("H264MI_RPW", rpw)
    if mc:
        monkeypatch.setenv("H264MI_MC_WAVES", mc)
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


@pytest.mark.parametrize("rank,pipe,staggered,mode",
                         [(r, 2, True, "") for r in range(8)] +
                         [(0, 1, True, ""), (1, 1, True, ""), (0, 2, False, ""), (1, 2, False, ""),
                          (0, 3, True, ""), (1, 3, True, ""), (0, 4, True, ""),
                          (0, 3, True, "cols"), (1, 2, False, "cols"), (2, 4, True, "cols")])
def test_configs3_shard_vs_reference(rank, pipe, staggered, mode, monkeypatch):
    """configs[3]: 64 streams, 8 per GPU.  Rank r's shard (seeds 100+8r ..
    100+8r+7, bench.shard_seeds) through bench.py's own device-resident path
    (bench.DeviceRun: records in HBM on the rank's engine, the next launch's
    k_prep in each launch's tail) and its verification pass.  staggered: GOP
    phases staggered over the streams, each 60-picture stream decoded
    cyclically after an untimed pre-roll -- with pipe 2 (the bench default)
    two consecutive pictures of every stream per launch (3 and 4 too), the
    phases such that an IDR is always the last picture of its launch;
    aligned: decode order from picture 0, every launch P steps
    (frame-pipelined batches).  Every picture of every
    launch vs the reference MD5s, and after the run every frame slot's last
    picture."""
    import bench
    if mode:
        monkeypatch.setenv("BENCH_DEP_MODE", mode)
    seeds = bench.shard_seeds(rank, 8)
    n = 60
    _, caps = bench.prepare(3, seeds, n)
    phases = bench.gop_phases(8, n, pipe, warmup=4) if staggered else None
    run = bench.DeviceRun(_lib.mi(), caps, 4, n - 4, pipe, phases=phases)
    try:
        assert run.P == pipe and all(d == 0 for _, d in run.placement())
        if staggered:
            steps = sum(len(x) for x in run.launches[run.n_pre:])
            assert run.n_pre == max(phases) and steps == n
            # an IDR is always the last picture of its launch (the phases)
            assert all(not run.holds_idr(x[:-1]) for x in run.launches[run.n_pre:])
            timed = run.timed_pictures()
            # stream s's IDR is at step (n - phase) % n: those in the timed window
            want = sum(1 for ph in phases if 4 <= (n - ph) % n)
            assert sum(run.is_i[k][s] for s, k in timed) == want
        else:
            assert len(run.launches) == n // pipe
        refs = [bench.golden_frames(3, sd, {}) for sd in seeds]
        ok, checked, missing, _ = run.verify(refs)
        assert (ok, checked, missing) == (True, 8 * n, 0)
        assert run.check_resident(refs)[0]
        assert run.eng.errors() == 0
        if pipe > 1:
            # configs[3]'s off-picture motion: whole rows by the bench's choice
            assert run.eng.last_deps() == {"cols": 2}.get(mode, 1)
    finally:
        run.free()


@pytest.mark.parametrize("pipe", [2, 3])
def test_realistic_motion_shard_vs_reference(pipe):
    """configs[3]'s rank-0 streams without off-picture motion (bench leg
    cfg3_realistic_motion): aligned frame-pipelined launches, whose
    dependency mode the bench picks per launch -- (MB row, MB column) cells
    here -- every picture vs the reference MD5s."""
    import bench
    seeds = bench.shard_seeds(0, 8)
    n = 60
    ov = {"offpic_pct": 0}
    _, caps = bench.prepare(3, seeds, n, ov)
    run = bench.DeviceRun(_lib.mi(), caps, pipe, 60 - pipe - (60 - pipe) % pipe, pipe)
    try:
        assert run.P == pipe
        refs = [bench.golden_frames(3, sd, ov) for sd in seeds]
        assert all(r is not None and len(r) == n for r in refs)
        ok, checked, missing, _ = run.verify(refs)
        assert run.eng.last_deps() == 2
        assert ok and missing == 0 and checked > 0
        assert run.eng.errors() == 0
    finally:
        run.free()


@pytest.mark.parametrize("pipe,staggered,check", [(1, True, False), (3, True, False), (3, False, False),
                                                   (3, True, True), (1, False, True)])
def test_no_loop_filter_shard_vs_reference(pipe, staggered, check, monkeypatch):
    """configs[3]'s rank-0 streams with the loop filter off in every slice
    (disable_deblocking_filter_idc 1: the reference's recommended `-flags
    -loop` encode, README.markdown:32-35; bench leg cfg3_no_loop_filter).  No
    MB row waits on the row above: every MB stores its own final rows 12..15
    (row_pp top_on).  Every picture vs the reference MD5s, with one and three
    pictures per launch, GOP-staggered and aligned, and under the dependency
    checker (no bit)."""
    import bench
    if check:
        monkeypatch.setenv("H264MI_CHECK", "1")
    seeds = bench.shard_seeds(0, 8)
    n = 60
    ov = {"dbf_idc1_pct": 100}
    _, caps = bench.prepare(3, seeds, n, ov)
    assert all(c.errors == 0 for c in caps)
    phases = bench.gop_phases(8, n, pipe, warmup=4) if staggered else None
    # aligned: whole launches from picture `pipe` on (as the bench leg)
    warm = 4 if staggered else pipe
    steps = n - 4 if staggered else n - pipe - (n - pipe) % pipe
    run = bench.DeviceRun(_lib.mi(), caps, warm, steps, pipe, phases=phases)
    try:
        assert run.P == pipe
        refs = [bench.golden_frames(3, sd, ov) for sd in seeds]
        assert all(r is not None and len(r) == n for r in refs)
        ok, checked, missing, _ = run.verify(refs)
        assert ok and missing == 0 and checked >= 8 * (warm + steps)
        assert run.check_resident(refs)[0]
        if check:
            assert run.eng.kernel_name() == "k_wgpp_check"
            assert run.eng.error_bits() == 0
        assert run.eng.errors() == 0
    finally:
        run.free()


@pytest.mark.parametrize("idc1,idc2,pipe", [(0, 100, 1), (0, 100, 3), (50, 50, 1), (50, 50, 2), (30, 40, 3)])
def test_slice_boundary_row_decoupling_vs_oracle(idc1, idc2, pipe):
    """Slices with the loop filter off (idc 1) or off across slice boundaries
    (idc 2), one slice per MB row or a slice boundary inside a row: MBs
    whose top edge is not filtered neither wait on nor store the row above,
    whose MBs then store their own rows 12..15.  Every picture vs the oracle's
    decode of the stream, one to three pictures per launch."""
    import bench
    w, h = 13, 9
    streams = [gen.generate(2, 80 + i, nframes=9, w_mbs=w, h_mbs=h, crop_bottom=0, slices=s, gop=5,
                            dbf_idc1_pct=idc1, dbf_idc2_pct=idc2)
               for i, s in enumerate((h, 5, 4))]
    caps = [Capture(s) for s in streams]
    refs = [O.decode(s)[0] for s in streams]
    n = min(c.npics for c in caps)
    n -= n % pipe
    run = bench.DeviceRun(_lib.mi(), caps, 0, n, pipe)
    try:
        for i, launch in enumerate(run.launches):
            run.launch(i)
            run.eng.sync()
            for step in launch:
                for s, k in enumerate(step):
                    got = run.eng.read(s, int(run.slot_of[k][s])).tobytes()
                    assert got == refs[s][k], f"stream {s} picture {k}"
        assert run.eng.errors() == 0
    finally:
        run.free()


@pytest.mark.parametrize("mode", ["rows", "cols"])
@pytest.mark.parametrize("wh,pipe", [((13, 7), 2), ((12, 9), 2), ((20, 11), 2), ((13, 7), 3), ((20, 11), 4),
                                     ((24, 7), 3), ((8, 9), 2), ((3, 5), 3)])
def test_engine_pipelined_steps_vs_oracle(wh, pipe, mode, monkeypatch):
    """Frame-pipelined launches (two to four consecutive pictures of each of
    3 streams per launch, physical slots renamed) on sizes whose luma rows do
    not end on 128-B lines (w % 8 != 0: a line holds two rows; w = 3: lines
    span more MB rows than a window, the whole-picture wait) and whose chroma
    rows are padded (H264MI_CPITCH), every picture vs the oracle's decode of
    the stream."""
    import bench
    monkeypatch.setenv("BENCH_DEP_MODE", mode)
    w, h = wh
    streams = [gen.generate(2, 70 + i, nframes=10, w_mbs=w, h_mbs=h, crop_bottom=0, slices=2, gop=5)
               for i in range(3)]
    caps = [Capture(s) for s in streams]
    refs = [O.decode(s)[0] for s in streams]
    n = min(c.npics for c in caps)
    n -= n % pipe
    run = bench.DeviceRun(_lib.mi(), caps, 0, n, pipe)
    try:
        assert run.P == pipe
        for i, launch in enumerate(run.launches):
            run.launch(i)
            run.eng.sync()
            for step in launch:
                for s, k in enumerate(step):
                    got = run.eng.read(s, int(run.slot_of[k][s])).tobytes()
                    assert got == refs[s][k], f"stream {s} picture {k}"
            assert run.eng.last_deps() == (1 if mode == "rows" else 2)
        assert run.eng.errors() == 0
    finally:
        run.free()


@pytest.mark.parametrize("share", [0, 4])
def test_swdec_concurrent_instances_vs_reference(share, monkeypatch):
    """One H264SwDec instance per thread, decoding concurrently (the
    reference's N-instance model, TestBenchMultipleInstance.c:134-305, on
    threads): four 1080p streams -- a damaged one among them, with its
    concealment and nbrOfErrMBs -- two 720p and a small damaged one.
    share = 4: instances of one picture size share one batched engine
    (h264mi_set_share; 1080p and 720p each get theirs, the small stream's
    engine is shared by nobody else).  Every output picture, picture id and
    error count equals the reference's, and the lock-step 1080p and 720p
    instances put several pictures in one launch (the batching property is
    timed with the calling threads not parsing ahead, H264MI_PARSE_HELP=0:
    parsing ahead spreads the instances' submissions; the sanitizer tests run
    shared engines with it on)."""
    import threading
    monkeypatch.setenv("H264MI_PARSE_HELP", "0")
    L = _lib.mi()
    names = ["bench_1080p_s100", "bench_1080p_s101", "bench_1080p_s102", "err_1080p_mixed",
             "leg_cfg2_720p_s1", "leg_cfg2_720p_s2", "err_range_p_11x9"]
    b0, p0 = C.c_ulonglong(), C.c_ulonglong()
    L.h264mi_share_stats(0, C.byref(b0), C.byref(p0))
    assert L.h264mi_set_share(share) == 0
    results, errors = {}, []

    def run(n):
        try:
            c = CASES[n]
            results[n] = swdec_decode(stream(c), no_reorder=c["no_reorder"], info=True)
        except Exception as ex:          # surfaced by the main thread
            errors.append((n, ex))

    try:
        th = [threading.Thread(target=run, args=(n,)) for n in names]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=240)
        assert not any(t.is_alive() for t in th), "decoder thread hung"
    finally:
        L.h264mi_set_share(0)
    assert not errors, errors
    for n in names:
        c = CASES[n]
        frames, _, pics = results[n]
        assert md5s(frames) == c["frames"], n
        if "pics" in c:
            assert [list(p) for p in pics] == c["pics"], n
    b1, p1 = C.c_ulonglong(), C.c_ulonglong()
    L.h264mi_share_stats(0, C.byref(b1), C.byref(p1))
    nb, npic = b1.value - b0.value, p1.value - p0.value
    if share:
        # a timing property of the lock-step threads (r172: 186 launches for
        # 248 pictures): batching happened, not a particular ratio
        assert npic > 0 and nb < 0.9 * npic, (nb, npic)
    else:
        assert nb == npic == 0


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


@pytest.mark.parametrize("share", [0, 2])
@pytest.mark.parametrize("k", [2, 5])
def test_device_flag_reaches_its_own_picture_under_reordering(share, k, monkeypatch):
    """A device flag (ReconArgs::err) raised for the k-th reconstruction
    (test hook H264MI_DEBUG_FLAG_PICTURE) is reported as nbrOfErrMBs = all
    MBs on exactly the output picture with picId k -- on a stream whose
    output order differs from decode order (POC type 0, MMCO, long-term),
    through the private and the shared engine -- and on no other picture;
    samples are unchanged."""
    L = _lib.mi()
    c = CASES["ref_mmco_poc0_reorder"]
    monkeypatch.setenv("H264MI_DEBUG_FLAG_PICTURE", str(k))
    assert L.h264mi_set_share(share) == 0
    try:
        frames, _, pics = swdec_decode(stream(c), no_reorder=c["no_reorder"], info=True)
    finally:
        L.h264mi_set_share(0)
    ow = c["overrides"]
    nmbs = ow["w_mbs"] * ow["h_mbs"]
    assert md5s(frames) == c["frames"]
    assert [p[0] for p in pics] == [p[0] for p in c["pics"]]
    for got, ref in zip(pics, c["pics"]):
        assert got[2] == (nmbs if got[0] == k else ref[2]), (got, ref)


def test_swdec_pooled_engines_vs_reference(monkeypatch):
    """Instances created one after another take the engine a released one left
    in the pool (H264MI_ENGINE_POOL, engine.hip engine_get / engine_put): the
    reused engine must behave as a fresh one -- cleared frame slots, no batch
    left prepped, flags of its own pictures only.  A damaged stream, a clean
    one and the damaged one again on one picture size, each equal to the
    reference; then the same with the pool off."""
    L = _lib.mi()
    names = ["err_drop_pic_gaps_11x9", "err_range_p_11x9", "err_trunc_slice_11x9", "err_drop_pic_gaps_11x9"]
    reused0, created0 = C.c_ulonglong(), C.c_ulonglong()
    L.h264mi_engine_pool_stats(C.byref(reused0), C.byref(created0))
    for n in names:
        c = CASES[n]
        frames, _, pics = swdec_decode(stream(c), no_reorder=c["no_reorder"], info=True)
        assert md5s(frames) == c["frames"] and [list(p) for p in pics] == c["pics"], n
    reused1, created1 = C.c_ulonglong(), C.c_ulonglong()
    L.h264mi_engine_pool_stats(C.byref(reused1), C.byref(created1))
    assert reused1.value - reused0.value >= len(names) - 1
    monkeypatch.setenv("H264MI_ENGINE_POOL", "0")
    for n in names[:2]:
        c = CASES[n]
        frames, _, pics = swdec_decode(stream(c), no_reorder=c["no_reorder"], info=True)
        assert md5s(frames) == c["frames"] and [list(p) for p in pics] == c["pics"], n
    reused2, created2 = C.c_ulonglong(), C.c_ulonglong()
    L.h264mi_engine_pool_stats(C.byref(reused2), C.byref(created2))
    assert reused2.value == reused1.value and created2.value - created1.value == 2
