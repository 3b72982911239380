"""OpenMAX DL surface (include/h264mi_omx.h): every omxVCM4P10_* primitive of
libh264mi.so (computed on the GPU) against the reference's own portable C
primitives, built from Decoder/omxdl/reference by oracle/Makefile.omx into
oracle/_ref/libomxref.so (per-primitive known-answer tests).
Randomised inputs, fixed seeds; outputs, updated pair-buffer pointers and
return codes must be identical.  Argument-error cases run without a GPU."""
import ctypes as C
import os
import threading
import time

import numpy as np
import pytest

from broadway_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libomxref.so")
BADARG = -5
U8P = C.c_void_p


class Size(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int)]


def _bind(lib):
    i32, vp = C.c_int, C.c_void_p
    for n in ("omxVCM4P10_PredictIntra_4x4", "omxVCM4P10_PredictIntra_16x16", "omxVCM4P10_PredictIntraChroma_8x8"):
        getattr(lib, n).argtypes = [vp, vp, vp, vp, i32, i32, i32, i32]
    for n in ("omxVCM4P10_InterpolateLuma", "omxVCM4P10_InterpolateChroma"):
        getattr(lib, n).argtypes = [vp, i32, vp, i32, i32, i32, Size]
    for e in ("Luma_VerEdge_I", "Luma_HorEdge_I", "Chroma_VerEdge_I", "Chroma_HorEdge_I"):
        getattr(lib, "omxVCM4P10_FilterDeblocking" + e).argtypes = [vp, i32, vp, vp, vp, vp]
    lib.omxVCM4P10_TransformDequantLumaDCFromPair.argtypes = [C.POINTER(vp), vp, i32]
    lib.omxVCM4P10_TransformDequantChromaDCFromPair.argtypes = [C.POINTER(vp), vp, i32]
    lib.omxVCM4P10_DequantTransformResidualFromPairAndAdd.argtypes = [C.POINTER(vp), vp, vp, vp, i32, i32, i32, i32]
    return lib


@pytest.fixture(scope="module")
def libs():
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref/libomxref.so not built (needs /root/reference at build time)")
    ref = _bind(C.CDLL(REF_SO, mode=os.RTLD_LOCAL))
    ours = _bind(C.CDLL(os.path.join(_lib.LIB_DIR, "libh264mi.so")))
    return ours, ref


class Buf:
    """A byte buffer whose base address is 64-B aligned, and a copy of it."""

    def __init__(self, n, rng=None, data=None):
        self.raw = np.zeros(n + 64, np.uint8)
        self.off = (-self.raw.ctypes.data) % 64
        self.a = self.raw[self.off:self.off + n]
        if data is not None:
            self.a[:] = data
        elif rng is not None:
            self.a[:] = rng.integers(0, 256, n, dtype=np.uint8)

    def p(self, i=0):
        return self.a.ctypes.data + i

    def clone(self):
        return Buf(len(self.a), data=self.a)


def _both(libs, name, make_args):
    """Run primitive `name` of both libraries on identical copies; returns
    (ret_ours, ret_ref, [(ours, ref) buffer pairs]).  make_args returns the
    call's arguments and EVERY buffer they point into (the buffers must
    outlive the call)."""
    ours, ref = libs
    a_o, bufs_o = make_args()
    a_r, bufs_r = make_args()
    r_o = getattr(ours, name)(*a_o)
    r_r = getattr(ref, name)(*a_r)
    return r_o, r_r, list(zip(bufs_o, bufs_r))


def _check(r_o, r_r, pairs, what):
    assert r_o == r_r, (what, r_o, r_r)
    for bo, br in pairs:
        assert np.array_equal(bo.a, br.a), what


# ---------------------------------------------------------------- intra
I4_NEEDS = {0: 1, 1: 2, 2: 0, 3: 1, 4: 1 | 2 | 32, 5: 1 | 2 | 32, 6: 1 | 2 | 32, 7: 1, 8: 2}


def _intra_case(rng, size, mode, avail, step=64):
    src = Buf(step * 64, rng)
    dst = Buf(step * 32, rng)
    x = y = 16
    base = y * step + x

    def make():
        s, d = src.clone(), dst.clone()
        return [s.p(base - 1), s.p(base - step), s.p(base - step - 1), d.p(), step, step, mode, avail], [d, s]
    return make


@pytest.mark.gpu
def test_predict_intra_4x4_vs_reference(libs):
    rng = np.random.default_rng(1)
    for it in range(600):
        mode = it % 9
        avail = I4_NEEDS[mode] | int(rng.choice([0, 1, 2, 32, 64, 1 | 64, 1 | 2 | 32 | 64]))
        r_o, r_r, pairs = _both(libs, "omxVCM4P10_PredictIntra_4x4", _intra_case(rng, 4, mode, avail))
        _check(r_o, r_r, pairs, ("i4", mode, avail))
        assert r_o == 0


@pytest.mark.gpu
def test_predict_intra_16x16_and_chroma_vs_reference(libs):
    rng = np.random.default_rng(2)
    needs16 = {0: 1, 1: 2, 2: 0, 3: 1 | 2 | 32}
    needsc = {0: 0, 1: 2, 2: 1, 3: 1 | 2 | 32}
    for it in range(400):
        mode = it % 4
        extra = int(rng.choice([0, 1, 2, 3, 32, 35]))
        r_o, r_r, pairs = _both(libs, "omxVCM4P10_PredictIntra_16x16", _intra_case(rng, 16, mode, needs16[mode] | extra))
        _check(r_o, r_r, pairs, ("i16", mode, extra))
        assert r_o == 0
        r_o, r_r, pairs = _both(libs, "omxVCM4P10_PredictIntraChroma_8x8", _intra_case(rng, 8, mode, needsc[mode] | extra))
        _check(r_o, r_r, pairs, ("ich", mode, extra))
        assert r_o == 0


# ---------------------------------------------------------- interpolation
# The reference's armVCM4P10_InterpolateHalfVer_Luma indexes pSrc[pos - 2 *
# iSrcStep] with iSrcStep an OMX_U32: the index wraps to ~4 GiB on an LP64
# host (on its 32-bit targets the pointer wraps back), so it faults here
# (SURVEY.md §8c notes the OMX-DL build segfaulting on 64 bits).  The
# positions that use it -- dx = 0 with dy != 0, dx odd with dy = 2, dx and dy
# both odd -- are checked against the spec's formulas below instead
# (H.264 8.4.2.2.1, restated in numpy); the other seven against the
# reference itself.
REF_SAFE = {(0, 0), (1, 0), (2, 0), (3, 0), (2, 1), (2, 2), (2, 3)}


def _luma_spec(src, x0, y0, step, w, h, dx, dy):
    g = src.astype(np.int64)

    def G(x, y):
        return g[(y0 + y) * step + x0 + x]

    def tap(a, b_, c, d, e, f):
        return a - 5 * b_ + 20 * c + 20 * d - 5 * e + f

    clip = lambda v: np.clip(v, 0, 255)
    out = np.zeros((h, w), np.int64)
    for y in range(h):
        for x in range(w):
            braw = lambda xx, yy: tap(*(G(xx + k, yy) for k in range(-2, 4)))
            hraw = lambda xx, yy: tap(*(G(xx, yy + k) for k in range(-2, 4)))
            b = lambda xx, yy: clip((braw(xx, yy) + 16) >> 5)
            hh = lambda xx, yy: clip((hraw(xx, yy) + 16) >> 5)
            j = clip((tap(*(braw(x, y + k) for k in range(-2, 4))) + 512) >> 10)
            avg = lambda u, v: (u + v + 1) >> 1
            if dx == 0 and dy == 0:
                v = G(x, y)
            elif dy == 0:
                v = b(x, y) if dx == 2 else avg(b(x, y), G(x + (dx == 3), y))
            elif dx == 0:
                v = hh(x, y) if dy == 2 else avg(hh(x, y), G(x, y + (dy == 3)))
            elif dx == 2 or dy == 2:
                v = j
                if dx != 2:
                    v = avg(v, hh(x + (dx == 3), y))
                if dy != 2:
                    v = avg(v, b(x, y + (dy == 3)))
            else:
                v = avg(b(x, y + (dy == 3)), hh(x + (dx == 3), y))
            out[y, x] = v
    return out.astype(np.uint8)


# The same positions exist LP64-clean in the reference's h264bsd core
# (h264bsdPredictSamples, h264bsd_reconstruct.c:1819-1950, built with the
# reference decoder's sources into oracle/_ref/libh264bsdref.so): the numpy
# restatement above is pinned to it on all 16 positions (CPU), and the GPU
# primitive is compared with it directly (test_interpolate_luma_vs_h264bsd).
BSD_SO = os.path.join(ROOT, "oracle", "_ref", "libh264bsdref.so")
PARTS = ((16, 16), (16, 8), (8, 16), (8, 8), (8, 4), (4, 8), (4, 4))


class _Image(C.Structure):      # h264bsd_image.h:45-55 (data, width / height in MBs, ...)
    _fields_ = [("data", C.c_void_p), ("width", C.c_uint32), ("height", C.c_uint32),
                ("luma", C.c_void_p), ("cb", C.c_void_p), ("cr", C.c_void_p)]


class _Mv(C.Structure):         # h264bsd_macroblock_layer.h:119-123
    _fields_ = [("hor", C.c_int16), ("ver", C.c_int16)]


@pytest.fixture(scope="module")
def bsd():
    if not os.path.exists(BSD_SO):
        pytest.skip("oracle/_ref/libh264bsdref.so not built (needs /root/reference at build time)")
    lib = C.CDLL(BSD_SO, mode=os.RTLD_LOCAL)
    lib.h264bsdPredictSamples.argtypes = [C.c_void_p, C.POINTER(_Mv), C.POINTER(_Image)] + [C.c_uint32] * 6
    lib.h264bsdPredictSamples.restype = None
    return lib


def _bsd_luma(bsd, pic, wmb, hmb, x0, y0, w, h, dx, dy):
    """luma prediction of a w x h partition at integer (x0, y0) + (dx, dy) / 4"""
    img = _Image(pic.ctypes.data, wmb, hmb, 0, 0, 0)
    mv = _Mv(4 * x0 + dx, 4 * y0 + dy)
    data = np.zeros(384, np.uint8)
    bsd.h264bsdPredictSamples(data.ctypes.data, C.byref(mv), C.byref(img), 0, 0, 0, 0, w, h)
    return data[:256].reshape(16, 16)[:h, :w]


def test_luma_spec_restatement_pinned_to_h264bsd(bsd):
    rng = np.random.default_rng(11)
    wmb, hmb = 4, 4
    W = 16 * wmb
    pic = rng.integers(0, 256, W * 16 * hmb * 3 // 2, dtype=np.uint8)
    for w, h in PARTS:
        for dx in range(4):
            for dy in range(4):
                for _ in range(2):
                    x0 = int(rng.integers(2, W - w - 3))
                    y0 = int(rng.integers(2, 16 * hmb - h - 3))
                    want = _bsd_luma(bsd, pic, wmb, hmb, x0, y0, w, h, dx, dy)
                    got = _luma_spec(pic[:W * 16 * hmb], x0, y0, W, w, h, dx, dy)
                    assert np.array_equal(got, want), (w, h, dx, dy, x0, y0)


@pytest.mark.gpu
def test_interpolate_luma_vs_h264bsd(libs, bsd):
    ours, _ = libs
    rng = np.random.default_rng(12)
    wmb, hmb = 6, 4
    W = 16 * wmb
    for w, h in PARTS:
        for dx in range(4):
            for dy in range(4):
                pic = rng.integers(0, 256, W * 16 * hmb * 3 // 2, dtype=np.uint8)
                x0 = int(rng.integers(2, W - w - 3))
                y0 = int(rng.integers(2, 16 * hmb - h - 3))
                want = _bsd_luma(bsd, pic, wmb, hmb, x0, y0, w, h, dx, dy)
                src = Buf(pic.size, data=pic)
                dst = Buf(16 * 16)
                assert ours.omxVCM4P10_InterpolateLuma(src.p(y0 * W + x0), W, dst.p(), 16, dx, dy, Size(w, h)) == 0
                got = dst.a.reshape(16, 16)[:h, :w]
                assert np.array_equal(got, want), (w, h, dx, dy, x0, y0)


@pytest.mark.gpu
def test_interpolate_luma_vs_reference(libs):
    ours, ref = libs
    rng = np.random.default_rng(3)
    step = 64
    for w in (4, 8, 16):
        for h in (4, 8, 16):
            for dx in range(4):
                for dy in range(4):
                    src = Buf(step * 64, rng)
                    dst = Buf(step * 32, rng)

                    def make():
                        s, d = src.clone(), dst.clone()
                        return [s.p(24 * step + 24), step, d.p(), step, dx, dy, Size(w, h)], [d, s]
                    if (dx, dy) in REF_SAFE:
                        r_o, r_r, pairs = _both(libs, "omxVCM4P10_InterpolateLuma", make)
                        _check(r_o, r_r, pairs, ("luma", w, h, dx, dy))
                    else:
                        args, (d, _s) = make()
                        r_o = ours.omxVCM4P10_InterpolateLuma(*args)
                        got = d.a.reshape(32, step)[:h, :w]
                        assert np.array_equal(got, _luma_spec(src.a, 24, 24, step, w, h, dx, dy)), (w, h, dx, dy)
                    assert r_o == 0


@pytest.mark.gpu
def test_interpolate_chroma_vs_reference(libs):
    rng = np.random.default_rng(4)
    step = 32
    for w in (2, 4, 8):
        for h in (2, 4, 8):
            for dx in range(8):
                for dy in (0, 1, 3, 4, 7):
                    src = Buf(step * 32, rng)
                    dst = Buf(step * 16, rng)

                    def make():
                        s, d = src.clone(), dst.clone()
                        return [s.p(8 * step + 8), step, d.p(), step, dx, dy, Size(w, h)], [d, s]
                    r_o, r_r, pairs = _both(libs, "omxVCM4P10_InterpolateChroma", make)
                    _check(r_o, r_r, pairs, ("chroma", w, h, dx, dy))
                    assert r_o == 0


# --------------------------------------------------------------- deblocking
def _smooth(rng, n, step):
    """Samples with small steps, so that most edges pass the alpha / beta tests."""
    base = rng.integers(40, 200)
    a = base + np.cumsum(rng.integers(-3, 4, n)) % 40
    a += rng.integers(-2, 3, n) * (rng.random(n) < 0.5)
    return np.clip(a, 0, 255).astype(np.uint8)


def _bs(rng, hor):
    bs = rng.integers(0, 4, 16).astype(np.uint8)
    if rng.random() < 0.4:
        bs[:4] = 4                       # the MB edge strong (bS = 4 only on edge 0, all four)
    return bs


@pytest.mark.gpu
@pytest.mark.parametrize("edge", ["Luma_VerEdge_I", "Luma_HorEdge_I", "Chroma_VerEdge_I", "Chroma_HorEdge_I"])
def test_filter_deblocking_vs_reference(libs, edge):
    rng = np.random.default_rng(5)
    step = 32
    for it in range(300):
        img = Buf(step * 32, data=_smooth(rng, step * 32, step))
        alpha = Buf(16, data=np.array([rng.integers(0, 256), rng.integers(0, 256)] + [0] * 14, np.uint8))
        beta = Buf(16, data=np.array([rng.integers(0, 19), rng.integers(0, 19)] + [0] * 14, np.uint8))
        thr = Buf(16, data=rng.integers(0, 26, 16).astype(np.uint8))
        bs = Buf(16, data=_bs(rng, "Hor" in edge))

        def make():
            d = img.clone()
            return [d.p(8 * step + 16), step, alpha.p(), beta.p(), thr.p(), bs.p()], [d]
        r_o, r_r, pairs = _both(libs, "omxVCM4P10_FilterDeblocking" + edge, make)
        _check(r_o, r_r, pairs, (edge, it))
        assert r_o == 0


# --------------------------------------------------------- residual / DC
def _pairs(rng, n, npos):
    """A pair-buffer block (armVCM4P10_UnpackBlock4x4.c format) of n coefficients."""
    pos = rng.choice(npos, size=n, replace=False)
    out = []
    for k, p in enumerate(pos):
        v = int(rng.integers(-3000, 3000)) if rng.random() < 0.3 else int(rng.integers(-128, 128))
        last = 0x20 if k == n - 1 else 0
        if -128 <= v < 128:
            out += [int(p) | last, v & 255]
        else:
            out += [int(p) | 0x10 | last, v & 255, (v >> 8) & 255]
    return out


def _pair_call(libs, name, data, extra_args, dst_n, dst_bytes=True):
    ours, ref = libs
    res = []
    for lib in (ours, ref):
        src = Buf(len(data) + 8, data=np.array(data + [0] * 8, np.uint8))
        pp = C.c_void_p(src.p())
        dst = Buf(dst_n)
        r = getattr(lib, name)(C.byref(pp), dst.p(), *extra_args)
        res.append((r, pp.value - src.p(), dst.a.copy()))
    return res


@pytest.mark.gpu
def test_transform_dequant_dc_from_pair_vs_reference(libs):
    rng = np.random.default_rng(6)
    for it in range(400):
        qp = int(rng.integers(0, 52))
        data = _pairs(rng, int(rng.integers(1, 17)), 16)
        (ro, ao, do), (rr, ar, dr) = _pair_call(libs, "omxVCM4P10_TransformDequantLumaDCFromPair", data, [qp], 32)
        assert (ro, ao) == (rr, ar) and np.array_equal(do, dr), ("luma dc", qp)
        data = _pairs(rng, int(rng.integers(1, 5)), 4)
        (ro, ao, do), (rr, ar, dr) = _pair_call(libs, "omxVCM4P10_TransformDequantChromaDCFromPair", data, [qp], 8)
        assert (ro, ao) == (rr, ar) and np.array_equal(do, dr), ("chroma dc", qp)


@pytest.mark.gpu
def test_dequant_transform_residual_vs_reference(libs):
    ours, ref = libs
    rng = np.random.default_rng(7)
    for it in range(400):
        qp = int(rng.integers(0, 52))
        ac = int(rng.random() < 0.8)
        use_dc = (not ac) or rng.random() < 0.5
        data = _pairs(rng, int(rng.integers(1, 16)), 16)
        pred = Buf(64, rng)
        dc = np.array([rng.integers(-2000, 2000)], np.int16)
        outs = []
        for lib in (ours, ref):
            src = Buf(len(data) + 8, data=np.array(data + [0] * 8, np.uint8))
            pp = C.c_void_p(src.p())
            dst = Buf(64)
            r = lib.omxVCM4P10_DequantTransformResidualFromPairAndAdd(
                C.byref(pp), pred.p(), dc.ctypes.data if use_dc else None, dst.p(), 16, 16, qp, ac)
            outs.append((r, pp.value - src.p(), dst.a.copy()))
        assert outs[0][:2] == outs[1][:2] and np.array_equal(outs[0][2], outs[1][2]), (qp, ac, use_dc)


# ------------------------------------------------ argument errors (no GPU)
def test_argument_errors_match_reference(libs):
    """Invalid arguments return OMX_Sts_BadArgErr before any device work, as
    the reference's checks do."""
    ours, ref = libs
    src = Buf(64 * 64)
    dst = Buf(64 * 32)
    a16, b, t, bs = Buf(16), Buf(16, data=np.full(16, 30, np.uint8)), Buf(16), Buf(16)
    cases = [
        ("omxVCM4P10_PredictIntra_4x4", [src.p(1040 - 1), src.p(1040 - 64), src.p(1040 - 65), dst.p(), 64, 64, 0, 2]),
        ("omxVCM4P10_PredictIntra_4x4", [src.p(1040 - 1), src.p(1040 - 64), src.p(1040 - 65), dst.p(), 64, 64, 9, 3]),
        ("omxVCM4P10_PredictIntra_16x16", [src.p(1040 - 1), src.p(1040 - 64), src.p(1040 - 65), dst.p(), 64, 64, 3, 3]),
        ("omxVCM4P10_PredictIntraChroma_8x8", [src.p(1040 - 1), src.p(1040 - 64), src.p(1040 - 65), dst.p(1), 64, 64, 0, 0]),
        ("omxVCM4P10_InterpolateLuma", [src.p(1040), 64, dst.p(), 64, 4, 0, Size(8, 8)]),
        ("omxVCM4P10_InterpolateLuma", [src.p(1040), 64, dst.p(), 64, 0, 0, Size(12, 8)]),
        ("omxVCM4P10_InterpolateChroma", [src.p(1040), 64, dst.p(), 60, 1, 1, Size(8, 8)]),
        ("omxVCM4P10_FilterDeblockingLuma_VerEdge_I", [src.p(1040), 64, a16.p(), b.p(), t.p(), bs.p()]),
        ("omxVCM4P10_FilterDeblockingChroma_HorEdge_I", [src.p(1040), 63, a16.p(), a16.p(), t.p(), bs.p()]),
    ]
    for name, args in cases:
        assert getattr(ours, name)(*args) == getattr(ref, name)(*args) == BADARG, name


# ------------------------------------------------ the per-thread job server
def _i4_worker(libs, seed, n, pause_s, out):
    rng = np.random.default_rng(seed)
    try:
        for it in range(n):
            mode = it % 9
            avail = I4_NEEDS[mode] | int(rng.choice([0, 1, 2, 32, 64, 1 | 64, 1 | 2 | 32 | 64]))
            r_o, r_r, pairs = _both(libs, "omxVCM4P10_PredictIntra_4x4", _intra_case(rng, 4, mode, avail))
            _check(r_o, r_r, pairs, ("i4", seed, mode, avail))
            assert r_o == 0
            if pause_s:
                time.sleep(pause_s)
        out[seed] = "ok"
    except BaseException as e:  # reported by the main thread
        out[seed] = repr(e)


@pytest.mark.gpu
def test_job_server_threads_idle_exit_and_launch_mode(libs):
    """csrc/hip/omx.hip's job server: each calling thread has its own resident
    server; four threads call concurrently, one of them pausing longer than the
    server's 20 ms idle limit between calls (the server leaves and is relaunched
    from the last request it saw), and one more runs the launch-per-call mode
    (H264MI_OMX_SERVER=0, read when the thread's context is made).  Every
    result equals the reference's."""
    out = {}
    ths = [threading.Thread(target=_i4_worker, args=(libs, s, 400, 0.0, out)) for s in (11, 12, 13)]
    ths.append(threading.Thread(target=_i4_worker, args=(libs, 14, 12, 0.03, out)))
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    os.environ["H264MI_OMX_SERVER"] = "0"
    try:
        t = threading.Thread(target=_i4_worker, args=(libs, 15, 100, 0.0, out))
        t.start()
        t.join(timeout=120)
    finally:
        del os.environ["H264MI_OMX_SERVER"]
    assert out == {s: "ok" for s in (11, 12, 13, 14, 15)}, out
