"""Wavefront-dependency checker (the reference's compile-time
_ASSERT_USED / _RANGE_CHECK knobs, h264bsd_util.h:35-123).  With
H264MI_CHECK=1 the engine launches the CHK instantiations of k_wgpp, which
verify every hand-off at its consumer (recon_kernels.hip CHK_*): the MC
ring's slot tag and release, the partner row wave's region tag, the intra
progress words' MB index, and in frame-pipelined launches that every
reference line read from a picture of the same launch lies in (MB row, MB
column) cells already published final (the host's set_ref_rows encoding and
the kernel's dep_wait together).  Each violation sets its own bit of
the picture's error word.  Green = no bit, frames still the reference's; and
the deliberately broken hand-offs (test hooks) are caught."""
import pytest

from _golden import cases, md5s, stream
from _swdec import swdec_decode
from broadway_amd import _lib, gen
from broadway_amd.engine import Capture

pytestmark = pytest.mark.gpu
CASES = cases()
EDGE = sorted(n for n in CASES if n.startswith("edge_"))

CHK_RING, CHK_RING_WR, CHK_REGION, CHK_PROG, CHK_REFROW = 64, 128, 256, 512, 1024


@pytest.mark.parametrize("pipe,staggered,mode", [(1, True, ""), (2, False, ""), (2, True, ""), (3, True, ""),
                                                 (2, False, "cols"), (3, True, "cols")])
def test_checker_bench_shard_clean(pipe, staggered, mode, monkeypatch):
    """Rank 0's configs[3] shard (8 x 1080p, 60 pictures each) through
    bench.DeviceRun under the checker: the bench's GOP-staggered plan with 1
    to 3 steps per launch (the reference-row checks against every earlier
    step's slot), and aligned frame-pipelined launches (two pictures of
    every stream per launch).
    Every picture vs the reference MD5s, no checker bit."""
    import bench
    monkeypatch.setenv("H264MI_CHECK", "1")
    if mode:
        monkeypatch.setenv("BENCH_DEP_MODE", mode)
    seeds = bench.shard_seeds(0, 8)
    n = 60
    _, caps = bench.prepare(3, seeds, n)
    phases = bench.gop_phases(8, n, pipe, warmup=4) if staggered else None
    run = bench.DeviceRun(_lib.mi(), caps, 4, n - 4, pipe, phases=phases)
    try:
        assert run.P == pipe
        refs = [bench.golden_frames(3, sd, {}) for sd in seeds]
        ok, checked, missing, _ = run.verify(refs)
        assert run.eng.kernel_name() == "k_wgpp_check"
        bits = run.eng.error_bits()
        assert bits == 0, f"dependency checker flags {bits:#x}"
        assert (ok, checked, missing) == (True, 8 * n, 0)
    finally:
        run.free()


@pytest.mark.parametrize("rpw", [None, "2", "3"])
def test_checker_degenerate_shapes_clean(rpw, monkeypatch):
    """The edge_* set (1-MB, one-row, one-column, thin pictures, 25 % off-
    picture MVs, a slice per MB) through H264SwDec* under the checker, with
    1, 2 and 3 MB rows per workgroup: frames and error counts unchanged (a
    checker bit would reach nbrOfErrMBs)."""
    monkeypatch.setenv("H264MI_CHECK", "1")
    monkeypatch.setenv("H264MI_ENGINE_POOL", "0")
    if rpw:
        monkeypatch.setenv("H264MI_RPW", rpw)
    for name in EDGE:
        c = CASES[name]
        frames, errors = swdec_decode(stream(c), no_reorder=c["no_reorder"])
        assert errors == 0, name
        assert md5s(frames) == c["frames"], name


def test_checker_catches_a_wrong_ring_tag(monkeypatch):
    """Test hook H264MI_CHECK_INJECT=1: MB 5 of every row hands the row waves
    a wrong ring tag -- the checker must say so (CHK_RING) while the samples
    themselves stay right."""
    import bench
    monkeypatch.setenv("H264MI_CHECK", "1")
    monkeypatch.setenv("H264MI_CHECK_INJECT", "1")
    seeds = bench.shard_seeds(0, 8)[:2]
    _, caps = bench.prepare(3, seeds, 4)
    run = bench.DeviceRun(_lib.mi(), caps, 0, 4, 1)
    try:
        refs = [bench.golden_frames(3, sd, {}) for sd in seeds]
        ok, checked, _, _ = run.verify(refs)
        assert ok and checked == 8
        assert run.eng.error_bits() & CHK_RING
    finally:
        run.free()


@pytest.mark.parametrize("pipe", [2, 3])
def test_checker_catches_short_reference_columns(pipe, monkeypatch):
    """Test hook H264MI_CHECK_INJECT_REFCOLS: the host records every
    partition's last reference column 6 MB columns short, so a later picture
    of a frame-pipelined launch would read reference lines whose columns are
    not yet stored; the checker must report it (CHK_REFROW) from the loads'
    own geometry and the producers' progress granules."""
    import bench
    monkeypatch.setenv("H264MI_CHECK", "1")
    monkeypatch.setenv("BENCH_DEP_MODE", "cols")
    monkeypatch.setenv("H264MI_CHECK_INJECT_REFCOLS", "6")
    streams = [gen.generate(2, 80 + i, nframes=6, w_mbs=22, h_mbs=6, crop_bottom=0, slices=2, gop=6)
               for i in range(3)]
    caps = [Capture(s) for s in streams]
    run = bench.DeviceRun(_lib.mi(), caps, 0, 6, pipe)
    try:
        for i in range(len(run.launches)):
            run.launch(i)
        run.eng.sync()
        assert run.eng.error_bits() & CHK_REFROW
    finally:
        run.free()


def test_checker_catches_short_reference_rows(monkeypatch):
    """Test hook H264MI_CHECK_INJECT_REFROWS: the whole-row waits
    (dep_wait_rows) wait for 64 rows fewer than the host recorded, so the
    frame-pipelined launch's later pictures would read their reference
    before it is final; the checker must report it (CHK_REFROW) from the
    loads' own geometry."""
    import bench
    monkeypatch.setenv("H264MI_CHECK", "1")
    monkeypatch.setenv("BENCH_DEP_MODE", "rows")
    monkeypatch.setenv("H264MI_CHECK_INJECT_REFROWS", "64")
    streams = [gen.generate(2, 70 + i, nframes=6, w_mbs=13, h_mbs=7, crop_bottom=0, slices=2, gop=6)
               for i in range(3)]
    caps = [Capture(s) for s in streams]
    run = bench.DeviceRun(_lib.mi(), caps, 0, 6, 2)
    try:
        for i in range(len(run.launches)):
            run.launch(i)
        run.eng.sync()
        assert run.eng.error_bits() & CHK_REFROW
    finally:
        run.free()


def test_checker_intra_heavy_six_mc_waves_clean(monkeypatch):
    """Config 2 (720p I-only, 4 streams): intra-heavy one-step launches whose
    rows fit two workgroups per CU take six MC waves and the luma-first intra
    path (engine.hip launch_nmc, recon_kernels.hip mc_intra LF) -- under the
    checker, every picture vs the reference MD5s, no checker bit."""
    import bench
    monkeypatch.setenv("H264MI_CHECK", "1")
    seeds = [1, 2, 3, 4]
    _, caps = bench.prepare(1, seeds, 6)
    run = bench.DeviceRun(_lib.mi(), caps, 0, 6, 1)
    try:
        refs = [bench.golden_frames(1, sd, {}) for sd in seeds]
        ok, checked, missing, _ = run.verify(refs)
        assert run.eng.kernel_name() == "k_wgpp_check"
        assert run.eng.last_mc_waves() == 6
        assert run.eng.error_bits() == 0, f"dependency checker flags {run.eng.error_bits():#x}"
        assert (ok, checked, missing) == (True, 24, 0)
    finally:
        run.free()
