"""Diagnostics: k_rows per-row phase clocks on the bench workload (not a test)."""
import sys, os, ctypes as C, numpy as np
os.environ.setdefault("H264MI_KERNEL", "classic")   # classic: k_rows phases; wg: k_wg (+ MC cycles per MB)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from broadway_amd import _lib
from broadway_amd.engine import Engine
L = _lib.mi()
S = int(os.environ.get("PROF_S", "8"))
streams, caps = bench.prepare(3, [100 + i for i in range(S)], 6)
w, h = caps[0].w_mbs, caps[0].h_mbs
d_recs, d_coef, d_pics, step_rec_bytes, nslots, _ = bench.upload(L, caps, 6, 1, 0)
eng = Engine(w, h, S, nslots)
L.h264mi_engine_profile(eng._h, 1, None, 0)
for k in range(6):
    eng.decode_device(S, d_recs + k * step_rec_bytes, d_coef, d_pics + k * S * 32)
    eng.sync()
    buf = (C.c_uint64 * (S * h * 16))()
    L.h264mi_engine_profile(eng._h, 1, buf, S * h * 16)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(h, S, 16).astype(np.float64)
    t0 = a[:, :, 0].min()
    st = (a[:, :, 0] - t0) / 100.0   # us
    en = (a[:, :, 1] - t0) / 100.0
    ph = a[:, :, 2:10] / w           # cycles per MB
    print(f"pic {k}: span {en.max():.1f} us; row start  r0 {st[0].mean():.1f} r1 {st[1].mean():.1f} r10 {st[10].mean():.1f} r67 {st[-1].mean():.1f}; "
          f"row dur r0 {(en[0]-st[0]).mean():.1f} r34 {(en[34]-st[34]).mean():.1f} r67 {(en[-1]-st[-1]).mean():.1f}")
    print("   cycles/MB  pre(+intra wait) %.0f  V %.0f  H %.0f  publish %.0f  stores %.0f  top-wait %.0f  intra+unf %.0f ring-wait %.0f" % tuple(ph.mean(axis=(0, 1))))
    if os.environ["H264MI_KERNEL"] == "wg":
        mbuf = (C.c_uint64 * (S * h * 16 + S * w * h * 4))()
        L.h264mi_engine_profile(eng._h, 1, mbuf, len(mbuf))
        mc = np.frombuffer(mbuf, dtype=np.uint64)[S * h * 16:].reshape(S, h, w, 4)[:, :, :, 3].astype(np.float64)
        print("   MC wave cycles/MB mean %.0f p50 %.0f p90 %.0f max %.0f" % (mc.mean(), np.percentile(mc, 50), np.percentile(mc, 90), mc.max()))
        mph = np.frombuffer(mbuf, dtype=np.uint64)[S * h * 16:].reshape(S, h, w, 4)[:, :, :, 1]
        parts = [((mph >> np.uint64(16 * i)) & np.uint64(0xFFFF)).astype(np.float64) for i in range(4)]
        parts = [x[mph > 0] for x in parts]
        print("   MC phases (mean cycles): dbrec %.0f residual %.0f windows %.0f interp %.0f" % tuple(x.mean() for x in parts))
    print("   row0 cycles/MB", " ".join("%.0f" % x for x in ph[0].mean(axis=0)), " row40", " ".join("%.0f" % x for x in ph[40].mean(axis=0)))

# per-MB hand-off timing of the last picture batch (100 MHz clock -> us)
buf = (C.c_uint64 * (S * h * 16 + S * w * h * 4))()
L.h264mi_engine_profile(eng._h, 1, buf, len(buf))
m = np.frombuffer(buf, dtype=np.uint64)[S * h * 16:].reshape(S, h, w, 4).astype(np.float64) / 100.0
p0 = m[0]
for r in (1, 2, 20, 40):
    for c in (10, 60):
        start, valid, pub = p0[r, c, 0], p0[r, c, 1], p0[r - 1, c + 1, 2]
        print(f"row {r} col {c}: consumer start {start - p0[r-1, c, 0]:.2f}us after producer's start of same col; "
              f"producer published entry {c} at +{pub - p0[r-1, c+1, 0]:.2f}us into its iter {c+1}; "
              f"consumer saw it {valid - pub:.2f}us after publish; iter len {p0[r, c+1, 0] - p0[r, c, 0]:.2f}us")

# per-row: duration, summed top-wait, own work (cycles/MB) for picture 0 of the last batch
a = np.frombuffer(buf, dtype=np.uint64)[:S * h * 16].reshape(h, S, 16).astype(np.float64)
t0 = a[:, :, 0].min()
for r in range(h):
    st = (a[r, 0, 0] - t0) / 100; en = (a[r, 0, 1] - t0) / 100
    ph = a[r, 0, 2:10] / w
    own = ph.sum() - ph[5]
    xcc = ""
    print(f"r{r:02d} start {st:7.1f} end {en:7.1f} dur {en-st:7.1f}  own {own:6.0f} cyc/MB  wait {ph[5]:6.0f}  [pre {ph[0]:.0f} intra+unf {ph[6]:.0f} V {ph[1]:.0f} H {ph[2]:.0f} pub {ph[3]:.0f} st {ph[4]:.0f}]")

# row progress timeline of picture 0 of the last batch (us since the first row started)
t0m = m[0, :, 0, 0].min()
print("row: t(c=0) t(c=30) t(c=60) t(c=90) t(c=119) | per-row delta at c=60")
prev = None
for r in range(0, h, 4):
    ts = [m[0, r, c, 0] - t0m for c in (0, 30, 60, 90, w - 1)]
    d = "" if prev is None else f"{(ts[2] - prev) / 4:.2f}/row"
    print(f"r{r:02d} " + " ".join(f"{x:7.1f}" for x in ts) + "  " + d)
    prev = ts[2]

# k_wgpp hand-off latency: row r's arrival of entry c (stamp 0) minus row r-1's
# publish of entry c (stamp 2 of its MB c+1), deep rows, picture 0 of the last batch
if os.environ.get("H264MI_WG_PP", "1") != "0":
    d = []
    for r in range(20, h):
        for c in range(4, w - 2):
            d.append(m[0, r, c, 0] - m[0, r - 1, c, 2])     # k_wgpp: stamp 2 of MB c = entry c published
    d = np.array(d)
    print("hand-off arrival-publish (us): min %.2f p10 %.2f p50 %.2f p90 %.2f" % (d.min(), np.percentile(d, 10), np.percentile(d, 50), np.percentile(d, 90)))
    per = np.diff(m[0, 40, :, 0])
    print("row 40 H-start period (us): p10 %.2f p50 %.2f p90 %.2f" % (np.percentile(per, 10), np.percentile(per, 50), np.percentile(per, 90)))
    pubs = m[0, 40, :, 2] - m[0, 40, :, 0]
    print("row 40 H(c) start -> publish(c) (us): p10 %.2f p50 %.2f p90 %.2f" % (np.percentile(pubs, 10), np.percentile(pubs, 50), np.percentile(pubs, 90)))
