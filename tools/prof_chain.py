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

L = _lib.mi()
S = int(os.environ.get("PROF_S", "8"))
# PROF_CONFIG=3: the bench streams (1080p I+P; picture PROF_PIC, a P picture
# by default); PROF_CONFIG=1: 720p I-only (config 2 of SURVEY §8d)
CFG = int(os.environ.get("PROF_CONFIG", "3"))
PIC = int(os.environ.get("PROF_PIC", "5"))
seeds = [(100 if CFG == 3 else 1) + i for i in range(S)]
# PROF_MIX=1: the bench's own GOP mix (IDRs staggered over the streams,
# bench.gop_phases); the profiled launch is the first one in which stream
# S-1 decodes its IDR while the others decode P pictures -- a configs[3]
# launch that holds one I picture.  Stats below then cover that I picture
# (PROF_SEL=i) or the P pictures of the launch (PROF_SEL=p)
MIX = os.environ.get("PROF_MIX") == "1"
streams, caps = bench.prepare(CFG, seeds, bench.GOP if MIX else PIC + 1)
w, h = caps[0].w_mbs, caps[0].h_mbs
if MIX:
    ph = bench.gop_phases(S, min(c.npics for c in caps))
    v_idr = (caps[0].npics - ph[S - 1]) % caps[0].npics
    run = bench.DeviceRun(L, caps, 0, v_idr + 1, 1, phases=ph)
else:
    run = bench.DeviceRun(L, caps, 0, PIC + 1, 1)
eng = run.eng
L.h264mi_engine_profile(eng._h, 1, None, 0)
for i in range(len(run.launches)):
    run.launch(i)
    eng.sync()
pics = list(run.launches[-1][0])          # picture of each stream in the profiled launch
print("kernel", eng.kernel_name(), "config", CFG, "pictures", pics,
      "types", "".join("I" if run.is_i[k][s] else "P" for s, k in enumerate(pics)))
n = S * h * 16 + S * w * h * 8
buf = (C.c_uint64 * n)()
L.h264mi_engine_profile(eng._h, 1, buf, n)
m = np.frombuffer(buf, dtype=np.uint64)[S * h * 16:].reshape(S, h, w, 8)
lo = lambda x: (x & np.uint64(0xFFFFFFFF)).astype(np.int64)
hi = lambda x: (x >> np.uint64(32)).astype(np.int64)
Cst = lo(m[..., 0])
A, B = lo(m[..., 1]), hi(m[..., 1])
E, D = lo(m[..., 2]), hi(m[..., 2])
# earliest stamp of the launch: the MC waves run ahead of the row chain
m3 = lo(m[..., 3])
base = min(Cst[Cst > 0].min(), m3[m3 > 0].min())
us = lambda x: ((x - base) % (1 << 32)) / 100.0
A, B, Cst, D, E = us(A), us(B), us(Cst), us(D), us(E)
print("per picture: row 0 end / row h-2 end (us):",
      " ".join(f"{'I' if run.is_i[k][s] else 'P'}{s}:{D[s, 0, w - 1]:.0f}/{D[s, h - 2, w - 1]:.0f}" for s, k in enumerate(pics)))
SEL = os.environ.get("PROF_SEL", "i" if MIX else "")
if SEL:
    keep = [s for s, k in enumerate(pics) if run.is_i[k][s] == (SEL == "i")]
    print(f"stats below: pictures {keep} ({'I' if SEL == 'i' else 'P'} only)")
    m = m[keep]
    A, B, Cst, D, E = A[keep], B[keep], Cst[keep], D[keep], E[keep]
    pics = [pics[s] for s in keep]
    caps = [caps[s] for s in keep]
    S = len(keep)

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

# where the hand-off tail and the period come from: by row band and by column band
print("by row band (all columns 2..w-3):")
for r0, r1 in ((1, 4), (4, 8), (8, 24), (24, 48), (48, h - 1)):
    r1 = min(r1, h - 1)
    if r1 <= r0:
        continue
    pr = np.diff(Cst[:, r0:r1, :], axis=2)[:, :, 2:w - 3]
    tp = (Cst[:, r0:r1, cols] - B[:, r0:r1, cols])
    g = tp > 0.05
    dl = (Cst[:, r0:r1, cols] - E[:, r0 - 1:r1 - 1, cols])[g]
    # row lag: H start of MB 2 of row r minus that of row r-1 (the wavefront's slope)
    lag = (Cst[:, r0:r1, 2] - Cst[:, r0 - 1:r1 - 1, 2]).mean()
    print(f"  rows {r0:2d}..{r1 - 1:2d}: lag {lag:.2f} | period mean {pr.mean():.3f} p50 {np.percentile(pr, 50):.3f}"
          f" | top mean {tp.mean():.3f} | delta mean {dl.mean() if dl.size else 0:.3f}"
          f" p90 {np.percentile(dl, 90) if dl.size else 0:.3f} | gated {g.mean() * 100:.0f} %")
print("deep rows by column band:")
for c0, c1 in ((2, 16), (16, 40), (40, 64), (64, 88), (88, w - 2)):
    c1 = min(c1, w - 2)
    if c1 <= c0:
        continue
    tp = Cst[:, rows, c0:c1] - B[:, rows, c0:c1]
    g = tp > 0.05
    dl = (Cst[:, 8:h - 1, c0:c1] - E[:, 7:h - 2, c0:c1])[g]
    pr = np.diff(Cst[:, rows, c0 - 1:c1], axis=2)
    print(f"  cols {c0:3d}..{c1 - 1:3d}: period mean {pr.mean():.3f} | top mean {tp.mean():.3f}"
          f" | delta mean {dl.mean():.3f} p50 {np.percentile(dl, 50):.3f} p90 {np.percentile(dl, 90):.3f}")
# row 0's end and the second-to-last row's (the last row publishes nothing,
# so its H end is not stamped)
print(f"  row 0 end (us, mean over pictures): {D[:, 0, w - 1].mean():.1f}; row {h - 2} end: {D[:, h - 2, w - 1].mean():.1f}")

# MC waves (stamp [3]: MC start = ring slot free, and flag set = slot final).
# For intra MBs the MC chain is a wavefront: MB (r, c) needs MB (r, c-1)'s
# slot (left, LDS flag) and the row above's unfiltered bottom row up to
# column c+1 (mailbox dwords 24..31 through L2).
M0, M1 = us(lo(m[..., 3])), us(hi(m[..., 3]))
types = np.stack([np.frombuffer(caps[s].records_bytes(pics[s]), np.uint8).reshape(h, w, 96)[..., 0] for s in range(S)])
intra = (types == 2) | (types == 3)     # I4x4 / I16x16 (I_PCM is a copy)
print(f"MC: {intra.mean() * 100:.1f} % intra MBs; MC slot-final of row 0's last MB {M1[:, 0, w - 1].mean():.1f} us, "
      f"of row {h - 1}'s {M1[:, h - 1, w - 1].mean():.1f} us")
rr, cc = slice(1, h), slice(1, w - 1)
left = M1[:, rr, 0:w - 2]
top = M1[:, 0:h - 1, 2:w]
own0 = M0[:, rr, cc]
fin = M1[:, rr, cc]
ready = np.maximum(np.maximum(left, top), own0)
im = intra[:, rr, cc]
if im.any():
    st("intra MB work (final - max(left, top-right, start))", (fin - ready)[im])
    gt = (top > left)[im]
    print(f"  intra MBs gated by the row above (top-right later than left): {gt.mean() * 100:.1f} %")
    st("intra: final - top-right final (gated by top)", (fin - top)[im][gt])
    st("intra: final - left final (gated by left)", (fin - left)[im][~gt])
    per_i = np.diff(M1, axis=2)[:, rr, 1:w - 2][intra[:, rr, 2:w - 1]]
    st("intra in-row period (slot final c-1 -> c)", per_i)
nm = ~im
if nm.any():
    st("inter MB MC (final - start)", (fin - own0)[nm])

# inside mc_intra ([4]: top loads issued | top ready, [5]: intra_tile done
# (left waits, prediction and slot writes, chroma first) | stamp written)
L0, T0 = us(lo(m[..., 4])), us(hi(m[..., 4]))
P0 = us(lo(m[..., 5]))
if im.any():
    # stamps of this launch only (a stale stamp of an earlier launch predates base)
    ok = im & (m[:, rr, cc, 4] != 0) & (L0[:, rr, cc] >= M0[:, rr, cc]) & (P0[:, rr, cc] <= M1[:, rr, cc])
    st("intra: MC start -> top loads issued (residual, record)", (L0 - M0)[:, rr, cc][ok])
    st("intra: top wait (top ready - loads issued)", (T0 - L0)[:, rr, cc][ok])
    st("intra: intra_tile (left waits + prediction + slot writes)", (P0 - T0)[:, rr, cc][ok])
    st("intra: tile done -> flag (bottom-row publish)", (M1 - P0)[:, rr, cc][ok])
    i4 = ok & (types[:, rr, cc] == 2)
    i16 = ok & (types[:, rr, cc] == 3)
    if i4.any():
        st("  I4x4 intra_tile", (P0 - T0)[:, rr, cc][i4])
    if i16.any():
        st("  I16x16 intra_tile", (P0 - T0)[:, rr, cc][i16])

# inter MBs' MC ([4] lo: MC start, hi: reference loads landed; [5] lo: samples
# reconstructed into the slot; [3] hi: flag set), top rows vs deep rows
I4lo, I4hi, I5lo = us(lo(m[..., 4])), us(hi(m[..., 4])), us(lo(m[..., 5]))
inter = ~intra & (types != 4)
for name, rs in (("rows 0..3", slice(0, 4)), ("rows 8..h-2", slice(8, h - 1))):
    sel = inter[:, rs, :] & (m[:, rs, :, 4] != 0)
    if sel.any():
        st(f"inter MC {name}: start -> loads landed", (I4hi - I4lo)[:, rs, :][sel])
        st(f"inter MC {name}: landed -> reconstructed", (I5lo - I4hi)[:, rs, :][sel])
        st(f"inter MC {name}: reconstructed -> flag", (M1 - I5lo)[:, rs, :][sel])

if os.environ.get("PROF_ROWS"):
    # per row, mean over pictures (us): MC start of MB 0, MC final of MB 2,
    # V(2) start, H(2) start, the row above's entry 2 published, last MB's H end
    print("row   mc0.start  mc2.final   V2.start   H2.start  above.E2   lag  rowend")
    for r in range(1, h):
        print(f"{r:3d} {M0[:, r, 0].mean():10.1f} {M1[:, r, 2].mean():10.1f} {A[:, r, 2].mean():10.1f}"
              f" {Cst[:, r, 2].mean():10.1f} {E[:, r - 1, 2].mean():9.1f} {(Cst[:, r, 2] - Cst[:, r - 1, 2]).mean():5.2f}"
              f" {D[:, r, w - 1].mean():7.1f}")

if os.environ.get("PROF_ROWS"):
    # placement of each row's workgroup: XCC, SE, SH, CU (HW_REG_HW_ID / XCC_ID)
    rw = np.frombuffer(buf, dtype=np.uint64)[:S * h * 16].reshape(h, S, 16)
    hwid, xcc = rw[..., 10].astype(np.int64), rw[..., 11].astype(np.int64) & 15
    cu, sh, se = (hwid >> 8) & 15, (hwid >> 12) & 1, (hwid >> 13) & 7
    print("picture 0 rows: xcc/se/sh/cu")
    print(" ".join(f"{r}:{xcc[r, 0]}/{se[r, 0]}/{sh[r, 0]}/{cu[r, 0]}" for r in range(h)))
    print("xcc per picture:", [sorted(set(xcc[:, s].tolist())) for s in range(S)])
    import collections
    for s in range(min(S, 2)):
        cnt = collections.Counter((int(se[r, s]), int(sh[r, s]), int(cu[r, s])) for r in range(h))
        print(f"picture {s}: {len(cnt)} distinct CUs, rows per CU {sorted(collections.Counter(cnt.values()).items())}")

if os.environ.get("PROF_ROWS"):
    # SIMD of each of the 5 waves of the workgroups sharing a CU (picture 0)
    simd = lambda v: (v >> 4) & 3
    by_cu = collections.defaultdict(list)
    for r in range(h):
        by_cu[(int(se[r, 0]), int(sh[r, 0]), int(cu[r, 0]))].append(r)
    for k, rs in list(by_cu.items())[:8]:
        print("CU", k, " ".join(f"row {r}: simd " + ",".join(str(int(simd(rw[r, 0, i]))) for i in (10, 12, 13, 14, 15))
                                for r in rs))

if os.environ.get("PROF_ROW0"):
    # row r's MC and deblocking per MB, mean over pictures (us): MC start /
    # final, V start (A), H end (D); MB types of picture 0
    r0 = int(os.environ.get("PROF_ROW0"))
    print(f"row {r0}: c type  mc.start  mc.final  V.start  H.end")
    for c in range(w):
        print(f"{c:3d} {int(types[0, r0, c]):2d} {M0[:, r0, c].mean():8.1f} {M1[:, r0, c].mean():8.1f} {A[:, r0, c].mean():8.1f} {D[:, r0, c].mean():8.1f}")

# the MC chain's wavefront (intra pictures): slot-final of MB (r, c) against
# (r-1, c) -- the row lag of the intra prediction -- and against (r, c-1)
if im.any():
    rl = (M1[:, 2:h, 2] - M1[:, 1:h - 1, 2])
    st("intra MC row lag (slot final, column 2)", rl.ravel())
    rlc = (M1[:, 2:h, 2:w - 2] - M1[:, 1:h - 1, 2:w - 2])
    st("intra MC row lag (all columns)", rlc.ravel())
    print(f"  MC slot-final of the last MB: {M1[:, h - 1, w - 1].mean():.1f} us; deblock row {h - 2} end {D[:, h - 2, w - 1].mean():.1f} us")
