"""Diagnostics (not a test): where k_wgpp's row chain spends its time.

Runs the bench workload with the profiling kernel (k_wgpp<3, true, true>) and
reads its per-MB wall-clock stamps (100 MHz; recon_kernels.hip row_pp):
  A = V(c) start (after the hdone wait and halo copy)   B = V(c) end
  C = row-above entry c in hand (H(c) starts)           D = H(c) end (hdone = c+1)
  E = entry c published (after the left-edge patch)
and prints, over the deep rows of every picture, the per-MB components
  hand-in  A(c) - D(c-1)   partner's H(c-1) done -> this wave's V(c) starts
  V        B - A
  top      C - B           waiting for the row above (0 when it was there)
  H        D - C
  patch    E - D           left-edge patch + publish of entry c
  delta    C(r,c) - E(r-1,c) for MBs whose H start waited on the row above
plus which edge of the grid gated each H start (row above vs own V).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes as C  # noqa: E402

import bench  # noqa: E402
from broadway_amd import _lib  # noqa: E402
from broadway_amd.engine import Engine  # noqa: E402

L = _lib.mi()
S = int(os.environ.get("PROF_S", "8"))
streams, caps = bench.prepare(3, [100 + i for i in range(S)], 6)
w, h = caps[0].w_mbs, caps[0].h_mbs
d_recs, d_coef, d_pics, step_rec_bytes, nslots, _ = bench.upload(L, caps, 6)
eng = Engine(w, h, S, nslots)
print("kernel", eng.kernel_name())
L.h264mi_engine_profile(eng._h, 1, None, 0)
for k in range(6):
    eng.decode_device(S, d_recs + k * step_rec_bytes, d_coef, d_pics + k * S * 32)
    eng.sync()
n = S * h * 16 + S * w * h * 4
buf = (C.c_uint64 * n)()
L.h264mi_engine_profile(eng._h, 1, buf, n)
m = np.frombuffer(buf, dtype=np.uint64)[S * h * 16:].reshape(S, h, w, 4)
lo = lambda x: (x & np.uint64(0xFFFFFFFF)).astype(np.int64)
hi = lambda x: (x >> np.uint64(32)).astype(np.int64)
Cst = lo(m[..., 0])
A, B = lo(m[..., 1]), hi(m[..., 1])
E, D = lo(m[..., 2]), hi(m[..., 2])
base = Cst[Cst > 0].min()
us = lambda x: ((x - base) % (1 << 32)) / 100.0
A, B, Cst, D, E = us(A), us(B), us(Cst), us(D), us(E)

rows = slice(8, h - 1)        # deep rows, not the last (no publish)
cols = slice(2, w - 2)
hand = (A[:, rows, cols] - D[:, rows, 1:w - 3])
V = B[:, rows, cols] - A[:, rows, cols]
top = Cst[:, rows, cols] - B[:, rows, cols]
H = D[:, rows, cols] - Cst[:, rows, cols]
patch = E[:, rows, cols] - D[:, rows, cols]
gated_top = top > 0.05
delta = (Cst[:, 8:h - 1, cols] - E[:, 7:h - 2, cols])[gated_top]


def st(name, x):
    print(f"  {name:8s} mean {x.mean():6.3f}  p10 {np.percentile(x, 10):6.3f}  p50 {np.percentile(x, 50):6.3f}"
          f"  p90 {np.percentile(x, 90):6.3f} us")


print(f"S={S}, rows 8..{h - 2}, cols 2..{w - 3}, {V.size} MBs")
st("hand-in", hand)
st("V", V)
st("top", top)
st("H", H)
st("patch", patch)
st("delta", delta)
print(f"  H start gated by the row above: {gated_top.mean() * 100:.1f} % of MBs")
per = np.diff(Cst[:, rows, :], axis=2)[:, :, 2:w - 3]
st("period", per)
