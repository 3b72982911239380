"""Diagnostics (not a test): what one call of the OpenMAX DL surface costs
(csrc/hip/omx.hip: each call packs its job into pinned memory; the calling
thread's resident job server runs it, or with H264MI_OMX_SERVER=0 one k_omx
launch per call, waited for).  Times N back-to-back calls of four
primitives on aligned host buffers and prints microseconds per call, plus what
an OMXDL-configured h264bsd would spend per 1080p P picture at the call counts
of configs[3]'s MB mix.  Usage: python tools/omx_cost.py [N]"""
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from broadway_amd import _lib  # noqa: E402


class Size(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int)]


def main(n):
    lib = C.CDLL(os.path.join(_lib.LIB_DIR, "libh264mi.so"))
    i32, vp = C.c_int, C.c_void_p
    lib.omxVCM4P10_InterpolateLuma.argtypes = [vp, i32, vp, i32, i32, i32, Size]
    lib.omxVCM4P10_FilterDeblockingLuma_VerEdge_I.argtypes = [vp, i32, vp, vp, vp, vp]
    lib.omxVCM4P10_PredictIntra_4x4.argtypes = [vp, vp, vp, vp, i32, i32, i32, i32]
    lib.omxVCM4P10_DequantTransformResidualFromPairAndAdd.argtypes = [C.POINTER(vp), vp, vp, vp, i32, i32, i32, i32]
    rng = np.random.default_rng(1)

    def buf(k, data=None):
        raw = np.zeros(k + 64, np.uint8)
        off = (-raw.ctypes.data) % 64
        a = raw[off:off + k]
        a[:] = rng.integers(40, 200, k, dtype=np.uint8) if data is None else data
        return raw, a

    keep = []
    src = buf(64 * 64); dst = buf(16 * 16); img = buf(32 * 32)
    alpha = buf(16, np.array([40, 30] + [0] * 14, np.uint8)); beta = buf(16, np.array([8, 6] + [0] * 14, np.uint8))
    thr = buf(16, np.full(16, 5, np.uint8)); bs = buf(16, np.full(16, 2, np.uint8))
    pred = buf(16); pair = buf(64, np.zeros(64, np.uint8)); out4 = buf(16)
    keep += [src, dst, img, alpha, beta, thr, bs, pred, pair, out4]
    P = lambda b, i=0: b[1].ctypes.data + i
    pair[1][0] = 0x20                                   # one empty block (last-pair flag)
    ppair = C.c_void_p(P(pair))
    calls = {
        "InterpolateLuma 16x16 (dx 2, dy 2)": lambda: lib.omxVCM4P10_InterpolateLuma(P(src, 8 * 64 + 8), 64, P(dst), 16, 2, 2, Size(16, 16)),
        "FilterDeblockingLuma_VerEdge_I (one MB)": lambda: lib.omxVCM4P10_FilterDeblockingLuma_VerEdge_I(P(img, 8 * 32 + 16), 32, P(alpha), P(beta), P(thr), P(bs)),
        "PredictIntra_4x4 (DC)": lambda: lib.omxVCM4P10_PredictIntra_4x4(P(src, 16 * 64 + 15), P(src, 15 * 64 + 16), P(src, 15 * 64 + 15), P(pred), 64, 4, 2, 3),
        "DequantTransformResidualFromPairAndAdd (4x4)": lambda: (ppair.__setattr__("value", P(pair)),
                                                                 lib.omxVCM4P10_DequantTransformResidualFromPairAndAdd(C.byref(ppair), P(pred), None, P(out4), 4, 4, 28, 1))[1],
    }
    def timed(res):
        for name, f in calls.items():
            for _ in range(20):
                f()
            t = time.perf_counter()
            for _ in range(n):
                r = f()
            dt = (time.perf_counter() - t) / n * 1e6
            res[name] = {"us_per_call": round(dt, 2), "ret": int(r)}

    def in_thread(server):
        # the mode is read when a thread's context is made: one fresh thread per mode
        res = {}
        os.environ["H264MI_OMX_SERVER"] = "1" if server else "0"
        th = threading.Thread(target=timed, args=(res,))
        th.start()
        th.join()
        return res

    # the Python/ctypes floor: the same call shape rejected on the host
    # (dstStep 4 below the width 16: BadArgErr before any device work)
    bad = lambda: lib.omxVCM4P10_InterpolateLuma(P(src, 8 * 64 + 8), 64, P(dst), 4, 2, 2, Size(16, 16))
    for _ in range(20):
        bad()
    t = time.perf_counter()
    for _ in range(n):
        rb = bad()
    floor = (time.perf_counter() - t) / n * 1e6
    launch = in_thread(False)
    res = in_thread(True)
    # an OMXDL h264bsd's calls per 1080p P picture (8,160 MBs): per inter MB one
    # luma + two chroma interpolations per partition (configs[3] mix: ~2
    # partitions per MB), per MB 4 luma + 4 chroma deblocking edge calls, per
    # coded 4x4 block one residual call (~8 per MB)
    per_mb = 2 * 3 + 8 + 8
    us = np.mean([v["us_per_call"] for v in res.values()])
    us_l = np.mean([v["us_per_call"] for v in launch.values()])
    out = {"calls": res, "python_ctypes_floor_us": round(floor, 2), "floor_ret": int(rb), "calls_per_1080p_picture_est": per_mb * 8160,
           "seconds_per_1080p_picture_est": round(per_mb * 8160 * us * 1e-6, 2),
           "launch_per_call": {"calls": launch, "seconds_per_1080p_picture_est": round(per_mb * 8160 * us_l * 1e-6, 2)},
           "note": "calls: the thread's resident job server; launch_per_call: H264MI_OMX_SERVER=0. "
                   "The product path (k_wgpp) reconstructs a 1080p P picture in ~0.3 ms"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 2000)
