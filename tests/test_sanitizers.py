"""Host sanitizers (SURVEY.md §5 "ASan on host"): the product host path --
NAL scan, parameter sets, slice headers, CAVLC / MB layer, DPB, concealment
and the speculative parse threads (host/specparse.c) -- built with
ThreadSanitizer and with AddressSanitizer + UBSan (oracle/Makefile
`sanitize`, the oracle_dec CLI: product parser + CPU oracle reconstruction)
and run over the damaged / reference-management fixtures, a multi-slice
1080p stream and a seeded byte-fuzz set.  Clean = no sanitizer report; on the
fixtures the sanitized builds also reproduce the reference decoder's frames.

UBSan runs with -fno-sanitize=shift: left shifts of negative values are
pervasive in the reference's own CAVLC / transform arithmetic
(h264bsd_transform.c, h264bsd_cavlc.c) and in this restatement alike."""
import hashlib
import os
import random
import subprocess
import shutil
import tempfile

import pytest

import oracle
from _golden import cases, stream

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "oracle", "_build")
CASES = cases()
FIXTURES = sorted(n for n in CASES if n.startswith(("err_", "ref_", "small_")) and CASES[n]["overrides"].get("w_mbs", 0) < 100)
REPORT = ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "ERROR: LeakSanitizer")


@pytest.fixture(scope="module")
def sanitized():
    oracle.make("sanitize")
    return {k: os.path.join(BUILD, f"oracle_dec_{k}") for k in ("tsan", "asan")}


def _run(exe, data, out=None, threads="3"):
    with tempfile.NamedTemporaryFile(suffix=".h264", delete=False) as f:
        f.write(data)
        path = f.name
    try:
        env = dict(os.environ, H264MI_PARSE_THREADS=threads,
                   TSAN_OPTIONS="halt_on_error=0 report_signal_unsafe=0",
                   ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
        p = subprocess.run([exe, f"-O{out}" if out else "-Onone", path], capture_output=True, text=True,
                           timeout=300, env=env)
        return p
    finally:
        os.unlink(path)


def _frames(path, nbytes):
    with open(path, "rb") as f:
        b = f.read()
    return [hashlib.md5(b[i:i + nbytes]).hexdigest() for i in range(0, len(b), nbytes)]


def _check_clean(p, what):
    bad = [ln for ln in (p.stderr or "").splitlines() if any(r in ln for r in REPORT)]
    assert not bad, f"{what}: {bad[:3]}\n{p.stderr[-3000:]}"
    assert p.returncode in (0, 1), f"{what}: exit {p.returncode}\n{p.stderr[-2000:]}"


@pytest.mark.timeout(900)
@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_fixtures_clean_and_bitexact(sanitized, kind):
    """Every damaged / ref-management fixture (+ a 4-slice 1080p stream for
    the speculative parse threads): no sanitizer report, frames == the
    reference decoder's MD5s."""
    names = FIXTURES + ["bench_1080p_s100"]
    for n in names:
        c = CASES[n]
        s = stream(c)
        if n == "bench_1080p_s100":          # 8 pictures are enough for the slice threads
            from broadway_amd import gen
            s = gen.generate(c["config"], c["seed"], nframes=8)
        with tempfile.NamedTemporaryFile(suffix=".yuv", delete=False) as f:
            out = f.name
        try:
            p = _run(sanitized[kind], s, out)
            _check_clean(p, n)
            w = c["overrides"].get("w_mbs")
            frames = c["frames"] if n != "bench_1080p_s100" else c["frames"][:8]
            nbytes = os.path.getsize(out) // max(len(frames), 1)
            assert nbytes > 0 and _frames(out, nbytes) == frames, (n, w)
        finally:
            os.unlink(out)


def _fuzz_set(n=40, seed=1234):
    """Seeded damage on small multi-slice I+P streams: byte flips (1-8 bytes
    past the parameter sets), zeroed runs and truncation."""
    from broadway_amd import gen
    rnd = random.Random(seed)
    bases = [gen.generate(2, 40 + i, nframes=6, w_mbs=9 + i, h_mbs=5 + i, crop_bottom=0, slices=3, gop=3)
             for i in range(4)]
    out = []
    for i in range(n):
        b = bytearray(bases[i % len(bases)])
        mode = i % 3
        if mode == 0:
            for _ in range(rnd.randint(1, 8)):
                b[rnd.randrange(32, len(b))] ^= 1 << rnd.randrange(8)
        elif mode == 1:
            o, k = rnd.randrange(32, len(b) - 16), rnd.randint(2, 16)
            b[o:o + k] = bytes(k)
        else:
            b = b[:rnd.randrange(64, len(b))]
        out.append(bytes(b))
    return out


@pytest.mark.timeout(900)
@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_fuzzed_streams_clean(sanitized, kind):
    """Seeded byte-fuzzed streams: no sanitizer report (decode errors and
    concealment are expected; memory errors, UB and races are not)."""
    for i, s in enumerate(_fuzz_set(40 if kind == "asan" else 16)):
        _check_clean(_run(sanitized[kind], s), f"fuzz #{i}")


# ---------------------------------------------------------------------------
# The product's own threading: the H264Backend adapter of the HIP engine
# (broadway_amd/csrc/host/hipback.cpp -- per-GPU shared engines with their
# batch collection, 1 ms launch timeout, per-instance events and per-batch
# result ring; the pool of released engines; the pinned output-frame pool;
# blocking waits) with the product host path and the h264mi_dec CLI
# (TestBenchMultipleInstance.c's N concurrent instances, one thread each),
# built on oracle/null_device.cpp, a CPU stand-in for the GPU (HIP runtime
# calls on host memory; engines that reconstruct with the CPU oracle, so
# the output is still the reference's), under ThreadSanitizer and
# AddressSanitizer + UBSan.

NULL_SET = ["err_drop_slice_11x9", "err_trunc_slice_11x9", "err_range_p_11x9", "err_drop_pic_gaps_11x9",
            "err_range_i_9x6", "ref_mmco_lt_12x8", "ref_mod_alias_12x8", "small_ip_8x6_2sl"]
NULL_MODES = {
    # 8 instances on one 4-lane shared engine per picture size (two 11x9
    # engines' worth of instances: the extra ones take private engines)
    "share4": (["-S4"], {}),
    # private engines, released ones pooled and reused (-r2)
    "private_pool": ([], {"H264MI_ENGINE_POOL": "1"}),
    "private_nopool": ([], {"H264MI_ENGINE_POOL": "0"}),
    # device concealment off: the host path reads pictures back
    "share4_hostconceal": (["-S4"], {"H264MI_HOST_CONCEAL": "1"}),
    # no slice workers: the calling threads parse the next picture ahead
    # while they would wait for the device (H264MI_PARSE_HELP, the default),
    # and with that off too (sequential)
    "private_help_only": ([], {"H264MI_PARSE_THREADS": "0"}),
    "private_sequential": ([], {"H264MI_PARSE_THREADS": "0", "H264MI_PARSE_HELP": "0"}),
}


@pytest.fixture(scope="module")
def nulldev():
    oracle.make("nulldev")
    return {k: os.path.join(BUILD, f"h264mi_dec_null_{k}") for k in ("tsan", "asan")}


@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode", sorted(NULL_MODES))
@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_hip_backend_threads_clean(nulldev, kind, mode):
    """8 concurrent H264SwDec instances (damaged and reference-management
    streams of four picture sizes), each stream decoded twice, through the
    HIP backend adapter on the null device: no sanitizer report, every
    picture output, and the first stream's frames == the reference's."""
    flags, extra = NULL_MODES[mode]
    td = tempfile.mkdtemp(prefix="nulldev")
    try:
        paths = []
        for i, n in enumerate(NULL_SET):
            p = os.path.join(td, f"s{i}.h264")
            with open(p, "wb") as f:
                f.write(stream(CASES[n]))
            paths.append(p)
        out = os.path.join(td, "s0.yuv")
        env = dict(os.environ, H264MI_PARSE_THREADS="2", H264MI_BLOCKING_SYNC="1",
                   TSAN_OPTIONS="halt_on_error=0 report_signal_unsafe=0",
                   ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
        env.update(extra)
        p = subprocess.run([nulldev[kind], f"-O{out}", "-r2"] + flags + paths, capture_output=True, text=True,
                           timeout=600, env=env)
        _check_clean(p, f"{kind}/{mode}")
        want = 2 * sum(len(CASES[n]["frames"]) for n in NULL_SET)
        assert f"pictures {want} " in p.stdout, p.stdout
        c = CASES[NULL_SET[0]]
        assert _frames(out, c["width"] * c["height"] * 3 // 2) == c["frames"]
    finally:
        shutil.rmtree(td, ignore_errors=True)
