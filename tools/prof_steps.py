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
# PROF_OV: generator overrides, e.g. "dbf_idc1_pct=100" (rows without
# deblocking keep no row stamps: the MC stamps set the time base then)
ov = dict((k, int(v)) for k, v in (x.split("=") for x in os.environ.get("PROF_OV", "").split(",") if x))
streams, caps = bench.prepare(3, seeds, n + 1, ov or None)
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
mc3 = mb[..., 3]
base = start[start > 0].min() if (start > 0).any() else int((mc3[mc3 > 0] & np.uint64(0xFFFFFFFF)).min())
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
for j in range(P if (start > 0).any() else 0):     # (rows without deblocking have no chain)
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

# when things start: per picture, its rows' workgroup start (spread), row 0's
# MB 0 MC flag and V(0) start, and how much of row 0 waited on its own MC
# (V(c) start minus the slot flag of MB c: ~0 when the MC is what row 0 waits for)
F = us(hi(mb[..., 3]))
M0 = us(lo(mb[..., 3]))
for j in range(P):
    ps = list(range(j * S, (j + 1) * S))
    for p in ps:
        s = st[:, p]
        print(f"  pic {p}: rows start min {s.min():6.1f} p50 {np.median(s):6.1f} max {s.max():6.1f};"
              f" row 0: MC(0) start {M0[p, 0, 0]:6.1f} flag {F[p, 0, 0]:6.1f} V(0) {A[p, 0, 0]:6.1f}"
              f" end {en[0, p]:6.1f}; V(c) - flag(c) over row 0 p50 {np.median(A[p, 0, 1:] - F[p, 0, 1:]):.2f}"
              f" (< 0.2 us in {np.mean((A[p, 0, 1:] - F[p, 0, 1:]) < 0.2) * 100:.0f} % of MBs);"
              f" MC per MB row 0 {np.median(np.diff(F[p, 0, :])):.2f} us")

# MC waves, inter MBs (stamps [4] = MC start | loads landed, [5] = samples
# reconstructed, [3] hi = slot flag): load wait, compute, publish, and the gap
# from the wave's previous MB's flag to this MB's MC start (issue + ring slot)
T0, TL = us(lo(mb[..., 4])), us(hi(mb[..., 4]))
T5 = us(lo(mb[..., 5]))
inter = (mb[..., 4] != 0) & (mb[..., 5] != 0)
for name, rs in (("row 0", slice(0, 1)), ("rows 1-7", slice(1, 8)), ("rows 8-66", slice(8, h - 1))):
    m = inter[:, rs, 2:]
    ld = (TL - T0)[:, rs, 2:][m]
    cp = (T5 - TL)[:, rs, 2:][m]
    pb = (F - T5)[:, rs, 2:][m]
    gap = (T0[:, rs, 2:] - F[:, rs, :-2])[m]     # same wave two MBs earlier (NMC = 2, static walk approx.)
    print(f"MC {name}: inter MBs {m.sum()}: load wait p50 {np.median(ld):.2f} mean {ld.mean():.2f};"
          f" compute p50 {np.median(cp):.2f}; publish p50 {np.median(pb):.2f};"
          f" gap from MB c-2's flag p50 {np.median(gap):.2f} mean {gap.mean():.2f} us")

# the gap split: slot flag of the wave's previous MB -> its next MB's loads
# issued ([7]: issue start / end) -> that MB's MC start ([4] lo: claim, record
# load and ring-slot wait in between)
IS0, IS1 = us(lo(mb[..., 7])), us(hi(mb[..., 7]))
for name, rs in (("row 0", slice(0, 1)), ("rows 1-7", slice(1, 8)), ("rows 8-66", slice(8, h - 1))):
    m = inter[:, rs, 2:] & (mb[:, rs, 2:, 7] != 0)
    a1 = (IS0[:, rs, 2:] - F[:, rs, :-2])[m]
    a2 = (IS1 - IS0)[:, rs, 2:][m]
    a3 = (T0 - IS1)[:, rs, 2:][m]
    print(f"MC gap {name}: flag(c-2) -> issue start p50 {np.median(a1):.2f}; issue p50 {np.median(a2):.2f} mean {a2.mean():.2f};"
          f" issue end -> MC start p50 {np.median(a3):.2f} mean {a3.mean():.2f} us")

# [6] of a one-step launch: the issue phases (address set-up | luma loads | chroma loads)
if P == 1:
    ph = mb[..., 6]
    p0 = (ph & np.uint64(0xFFFF)).astype(np.int64) / 100.0
    p1 = ((ph >> np.uint64(16)) & np.uint64(0xFFFF)).astype(np.int64) / 100.0
    p2 = ((ph >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.int64) / 100.0
    for name, rs in (("row 0", slice(0, 1)), ("rows 8-66", slice(8, h - 1))):
        m = inter[:, rs, 2:] & (ph[:, rs, 2:] != 0)
        e = (IS1 - IS0)[:, rs, 2:][m]
        a0, a1, a2 = p0[:, rs, 2:][m], p1[:, rs, 2:][m], p2[:, rs, 2:][m]
        print(f"MC issue {name}: set-up p50 {np.median(a0):.2f}; luma loads p50 {np.median(a1 - a0):.2f};"
              f" chroma loads p50 {np.median(a2 - a1):.2f}; dbrec + residual loads p50 {np.median(e - a2):.2f} us")

# wave placement (HW_REG_HW_ID: SIMD bits 5:4, CU / SH / SE bits 8..15; XCC id):
# which SIMD each role's waves land on, and per (XCC, CU, SIMD) how many row
# waves and MC waves of the launch share it
import collections
hw = rows[:, :, 10:16].astype(np.int64)          # [r, p, k]: 10 wave 0, 11 XCC, 12.. waves 1..3
simd = lambda v: (v >> 4) & 3
cuk = lambda v, x: (x, (v >> 8) & 0xFF)
combo = collections.Counter()
occ = collections.defaultdict(lambda: [0, 0])
for r_ in range(h):
    for p_ in range(npics):
        w0, x, w1, w2, w3 = hw[r_, p_, 0], hw[r_, p_, 1], hw[r_, p_, 2], hw[r_, p_, 3], hw[r_, p_, 4]
        combo[(simd(w0), simd(w1), simd(w2), simd(w3))] += 1
        for k, v in enumerate((w0, w1, w2, w3)):
            occ[cuk(v, x) + (simd(v),)][0 if k < 2 else 1] += 1
print("SIMD of (row wave 0, row wave 1, MC wave 0, MC wave 1):", combo.most_common(6))
mix = collections.Counter(tuple(v) for v in occ.values())
print("per SIMD (row waves, MC waves) over the launch:", mix.most_common(8))

# does sharing a SIMD with another row wave slow a row's passes? per row wave:
# the row / MC waves on its SIMD (itself included), against the V / H times
# and the period of its MBs (deep rows; wave w takes the MBs c with c % 2 == w)
Vt, Ht = (B - A), (D - Cst)
per_all = np.diff(Cst, axis=2)
stat = collections.defaultdict(list)
for r_ in range(8, h - 1):
    for p_ in range(npics):
        x = hw[r_, p_, 1]
        for wv, v in ((0, hw[r_, p_, 0]), (1, hw[r_, p_, 2])):
            key = tuple(occ[cuk(v, x) + (simd(v),)])
            cs = np.arange(2 + wv, w - 2, 2)
            stat[key].append((Vt[p_, r_, cs].mean(), Ht[p_, r_, cs].mean(), per_all[p_, r_, cs - 1].mean()))
for key, vals in sorted(stat.items()):
    v = np.array(vals)
    print(f"  SIMD with (row, MC) waves {key}: {len(v)} row waves, V {v[:, 0].mean():.3f} H {v[:, 1].mean():.3f} period {v[:, 2].mean():.3f} us")
