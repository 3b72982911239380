"""Diagnostics (not a test): the timeline of one frame-pipelined launch
(P steps of S streams; the profiling build of k_wgpp's DEP3 instance).
Per step: when its rows start and end (100 MHz stamps, relative to the
launch's first stamp), how long its MC waves waited on in-launch producers
(dep_wait, per MB), and how late each row started compared with the same row
of the step before.  PROF_P (3), PROF_S (8), PROF_LAUNCH (index of the
profiled launch in an aligned plan, default 2: pictures 2P..3P-1)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes as C  # noqa: E402

import bench  # noqa: E402
from broadway_amd import _lib  # noqa: E402

L = _lib.mi()
S = int(os.environ.get("PROF_S", "8"))
P = int(os.environ.get("PROF_P", "3"))
LA = int(os.environ.get("PROF_LAUNCH", "2"))
seeds = [100 + i for i in range(S)]
n = P * (LA + 1)
streams, caps = bench.prepare(3, seeds, n + 1)
w, h = caps[0].w_mbs, caps[0].h_mbs
run = bench.DeviceRun(L, caps, 0, n, P)
eng = run.eng
for i in range(LA):
    run.launch(i)
eng.sync()
L.h264mi_engine_profile(eng._h, 1, None, 0)
run.launch(LA)
eng.sync()
npics = S * P
print("kernel", eng.kernel_name(), "steps", P, "streams", S, "launch", run.launches[LA])
tot = npics * h * 16 + npics * w * h * 8
buf = (C.c_uint64 * tot)()
L.h264mi_engine_profile(eng._h, 1, buf, tot)
a = np.frombuffer(buf, dtype=np.uint64)
rows = a[:npics * h * 16].reshape(h, npics, 16)
mb = a[npics * h * 16:].reshape(npics, h, w, 8)
start = rows[:, :, 0].astype(np.int64)              # [r, p]
end = rows[:, :, 1].astype(np.int64)
base = start[start > 0].min()
st = (start - base) / 100.0
en = (end - base) / 100.0
dep = mb[..., 6].astype(np.int64) / 100.0           # [p, r, c] us
for j in range(P):
    ps = list(range(j * S, (j + 1) * S))
    print(f"step {j}: row 0 start {st[0, ps].mean():7.1f}  row 0 end {en[0, ps].mean():7.1f}  "
          f"row {h - 1} start {st[h - 1, ps].mean():7.1f}  end {en[h - 1, ps].mean():7.1f} (max {en[h - 1, ps].max():.1f})  "
          f"dep wait per MB mean {dep[ps].mean():.2f} us, sum per row {dep[ps].sum(axis=2).mean():.1f} us")
    if j:
        q = [p - S for p in ps]
        d0 = (st[:, ps] - st[:, q]).mean(axis=1)
        de = (en[:, ps] - en[:, q]).mean(axis=1)
        print(f"   vs step {j - 1}: row start later by " + " ".join(f"r{r}:{d0[r]:.0f}" for r in range(0, h, 8)))
        print(f"   vs step {j - 1}: row end later by   " + " ".join(f"r{r}:{de[r]:.0f}" for r in range(0, h, 8)))
        big = np.argwhere(dep[ps] > 20.0)
        print(f"   MBs waiting > 20 us: {len(big)}; by row band " +
              " ".join(f"{b}-{b + 7}:{int(((big[:, 1] >= b) & (big[:, 1] < b + 8)).sum())}" for b in range(0, h, 8)))
print("launch end", en[h - 1].max())

# the row chain of each step (deep rows 8..h-2, columns 2..w-3; row_pp
# stamps, as tools/prof_chain.py): per-MB period, V, the wait for the row
# above, H, the hand-off delay and the row lag
lo = lambda x: (x & np.uint64(0xFFFFFFFF)).astype(np.int64)
hi = lambda x: (x >> np.uint64(32)).astype(np.int64)
us = lambda x: ((x - base) % (1 << 32)) / 100.0
Cst = us(lo(mb[..., 0]))
A, B = us(lo(mb[..., 1])), us(hi(mb[..., 1]))
E, D = us(lo(mb[..., 2])), us(hi(mb[..., 2]))
rows_, cols_ = slice(8, h - 1), slice(2, w - 2)
for j in range(P):
    ps = slice(j * S, (j + 1) * S)
    per = np.diff(Cst[ps, rows_, :], axis=2)[:, :, 2:w - 3]
    V = (B - A)[ps, rows_, cols_]
    top = (Cst - B)[ps, rows_, cols_]
    H = (D - Cst)[ps, rows_, cols_]
    g = top > 0.05
    dl = (Cst[ps, 8:h - 1, cols_] - E[ps, 7:h - 2, cols_])[g]
    lag = (Cst[ps, 8:h - 1, 2] - Cst[ps, 7:h - 2, 2]).mean()
    print(f"step {j} chain: period {per.mean():.2f} (p50 {np.percentile(per, 50):.2f}, p90 {np.percentile(per, 90):.2f})"
          f"  V {V.mean():.2f}  top {top.mean():.2f}  H {H.mean():.2f}  delta {dl.mean() if dl.size else 0:.2f}"
          f"  lag {lag:.2f} us; MBs gated by the row above {g.mean() * 100:.0f} %")
