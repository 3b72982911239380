"""Diagnostics (not a test): reconstruct a generated stream picture by picture
on the GPU (Engine) and on the CPU oracle (Replay, the same MB records) and
list the first mismatching MBs of the first mismatching picture with their
record fields (type, prediction modes, availability, cbits).

    python tools/diff_frame.py CONFIG SEED [k=v ...]      (generator overrides)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from broadway_amd import gen  # noqa: E402
from broadway_amd.engine import Capture, Engine  # noqa: E402

cfg, seed = int(sys.argv[1]), int(sys.argv[2])
ov = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in sys.argv[3:])
cap = Capture(gen.generate(cfg, seed, **ov))
w, h = cap.w_mbs, cap.h_mbs
if os.environ.get("NODBF"):
    # deblocking off in every record (DB_LEFT | DB_TOP | DB_INNER), on both
    # sides: the raw reconstruction is compared
    import ctypes as C
    for p in cap.pictures:
        a = (C.c_uint8 * (w * h * 96)).from_address(p.rec)
        for i in range(w * h):
            a[i * 96 + 3] &= ~(16 | 32 | 64) & 255
eng = Engine(w, h, 1, cap.nslots)
rep = O.Replay(w, h, cap.nslots)
for k, p in enumerate(cap.pictures):
    eng.decode([0], [p])
    rep.picture(p.rec, p.coef, p.cur_slot)
    g = np.frombuffer(eng.read(0, p.cur_slot).tobytes(), np.uint8)
    o = np.frombuffer(rep.frame(p.cur_slot), np.uint8)
    if (g == o).all():
        continue
    W, H = w * 16, h * 16
    Y, Yo = g[:W * H].reshape(H, W), o[:W * H].reshape(H, W)
    U, Uo = g[W * H:W * H * 5 // 4].reshape(H // 2, W // 2), o[W * H:W * H * 5 // 4].reshape(H // 2, W // 2)
    V, Vo = g[W * H * 5 // 4:].reshape(H // 2, W // 2), o[W * H * 5 // 4:].reshape(H // 2, W // 2)
    recs = np.frombuffer(cap.records_bytes(k), np.uint8).reshape(h, w, 96)
    print(f"picture {k}: {int((g != o).sum())} samples differ")
    n = 0
    for my in range(h):
        for mx in range(w):
            ly = (Y[my * 16:my * 16 + 16, mx * 16:mx * 16 + 16] != Yo[my * 16:my * 16 + 16, mx * 16:mx * 16 + 16])
            cu = (U[my * 8:my * 8 + 8, mx * 8:mx * 8 + 8] != Uo[my * 8:my * 8 + 8, mx * 8:mx * 8 + 8])
            cv = (V[my * 8:my * 8 + 8, mx * 8:mx * 8 + 8] != Vo[my * 8:my * 8 + 8, mx * 8:mx * 8 + 8])
            if ly.any() or cu.any() or cv.any():
                r = recs[my, mx]
                i4 = int.from_bytes(bytes(r[16:24]), "little")
                print(f"  MB ({my},{mx}) type {r[0]} pred {r[4]:#04x} avail {r[3]:#04x} cbits {int.from_bytes(bytes(r[8:12]), 'little'):#010x}"
                      f" i4 {[(i4 >> (4 * b)) & 15 for b in range(16)] if r[0] == 2 else '-'}"
                      f" luma rows {np.nonzero(ly.any(1))[0].tolist()} cols {np.nonzero(ly.any(0))[0].tolist()}"
                      f" cb {int(cu.sum())} cr {int(cv.sum())}")
                if n == 0 and os.environ.get("DUMP"):
                    y0, x0 = my * 16, mx * 16
                    print("   GPU luma (with the row above / column left):")
                    for yy in range(max(y0 - 1, 0), y0 + 16):
                        print("   ", " ".join(f"{v:3d}" for v in Y[yy, max(x0 - 1, 0):x0 + 16]))
                    print("   oracle:")
                    for yy in range(max(y0 - 1, 0), y0 + 16):
                        print("   ", " ".join(f"{v:3d}" for v in Yo[yy, max(x0 - 1, 0):x0 + 16]))
                n += 1
                if n >= 12:
                    sys.exit(1)
    sys.exit(1)
print("all pictures match")
