#!/usr/bin/env python3
"""Generate tests/golden/softavc.json: the REFERENCE decoder driven the way
the SoftAVC OMX component drives it (Decoder/SoftAVC.cpp:289-400: one NAL
unit per input buffer, picId per buffer, intraConcealmentMethod = 1 at :335,
NextPicture drained after every buffer, flushed at end of stream).

DecTestBench hardcodes intraConcealmentMethod = 0 (DecTestBench.c:211), so
the fixtures of tests/golden/golden.json never exercise SoftAVC's setting.
With method 1 a picture whose slices all fail is concealed by copying the
first available reference picture instead of grey (h264bsd_conceal.c:149-159,
177-181) -- for I pictures too.  Runs only in the build container, where
oracle/Makefile.ref builds oracle/_ref/refdec_softavc from the reference
sources and oracle/softavc_bench.c.  Stored per case: generator parameters,
stream SHA-256, frame MD5s and (picId, isIdrPicture, nbrOfErrMBs) per output
picture, for method 1 and, as the control, method 0 -- nothing from the
reference itself.

    python tests/golden/make_golden_softavc.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

_P = dict(nframes=12, w_mbs=11, h_mbs=9, crop_bottom=0)
CASES = {
    # I pictures whose slices are all truncated (whole I picture lost):
    # method 1 copies the reference, method 0 paints grey
    "sa_ionly_trunc_9x6": (1, 3, dict(nframes=8, w_mbs=9, h_mbs=6, slices=2, trunc_slice_pct=60)),
    "sa_ionly_trunc_1sl_9x6": (1, 1, dict(nframes=8, w_mbs=9, h_mbs=6, slices=1, trunc_slice_pct=60)),
    # IDR every 3 pictures, truncated / lost slices: lost I and P pictures
    "sa_ip_gop3_trunc_11x9": (2, 10, dict(_P, slices=2, gop=3, trunc_slice_pct=50)),
    "sa_ip_gop3_drop_11x9": (2, 4, dict(_P, slices=1, gop=3, trunc_slice_pct=50, drop_slice_pct=20)),
    # the DecTestBench damaged-stream fixtures, through the SoftAVC protocol
    "sa_err_range_p_11x9": (2, 6, dict(_P, slices=3, gop=6, err_range_pct=60)),
    "sa_err_drop_pic_gaps_11x9": (2, 10, dict(_P, slices=3, gop=6, drop_pic_pct=20, gaps_allowed=1)),
    "sa_err_720p_ionly_conceal": (1, 3, dict(nframes=3, drop_slice_pct=30, trunc_slice_pct=30)),
    "sa_err_1080p_mixed": (3, 300, dict(nframes=8, err_range_pct=20, drop_slice_pct=10, trunc_slice_pct=10)),
}


def one_case(item):
    from broadway_amd import gen
    import oracle as O

    name, (cfg, seed, ov) = item
    stream = gen.generate(cfg, seed, **ov)
    out = {"config": cfg, "seed": seed, "overrides": ov, "stream_sha256": hashlib.sha256(stream).hexdigest()}
    for m in (1, 0):
        frames, pics = O.refdec_softavc_frames(stream, m)
        assert frames, name
        out[f"method{m}"] = {"frames": [hashlib.md5(f).hexdigest() for f in frames], "pics": [list(p) for p in pics]}
    out["method_sensitive"] = out["method1"]["frames"] != out["method0"]["frames"]
    return name, out


def main():
    import concurrent.futures as cf

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "softavc.json")
    with cf.ProcessPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        done = dict(ex.map(one_case, CASES.items()))
    out = {"generator": "broadway_amd.gen (libh264gen.so)",
           "decoder": "reference C (Decoder/src, make.py file list) + oracle/softavc_bench.c (SoftAVC protocol), "
                      "gcc -O2",
           "protocol": "one NAL unit per H264SwDecDecode input buffer, picId per buffer, intraConcealmentMethod "
                       "1 (method0: the same with 0), NextPicture(0) after every buffer, NextPicture(1) at the end",
           "cases": {n: done[n] for n in CASES}}
    for n, c in out["cases"].items():
        print(f"{n}: {len(c['method1']['frames'])} pictures, method-sensitive {c['method_sensitive']}")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
