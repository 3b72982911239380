"""Diagnostics (not a test): wall time per step of the bench workload with and
without the per-launch timing events, to price the markers between launches."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from broadway_amd import _lib  # noqa: E402
from broadway_amd.engine import Engine  # noqa: E402

L = _lib.mi()
S, N = 8, 24
streams, caps = bench.prepare(3, [100 + i for i in range(S)], N)
w, h = caps[0].w_mbs, caps[0].h_mbs
d_recs, d_coef, d_pics, step_rec_bytes, nslots, _ = bench.upload(L, caps, N)
eng = Engine(w, h, S, nslots)


def run(k0, k1):
    for k in range(k0, k1):
        eng.decode_device(S, d_recs + k * step_rec_bytes, d_coef, d_pics + k * S * 32)


run(0, 4)
eng.sync()
for rep in range(2):
    for timed in (False, True):
        # restart from picture 4 each time (P pictures reference the previous
        # slot; the timing is what is measured here, not the output)
        if timed:
            eng.set_timing(N - 4)
        t0 = time.perf_counter()
        run(4, N)
        eng.sync()
        dt = (time.perf_counter() - t0) / (N - 4)
        extra = ""
        if timed:
            _, rows_us, nb = eng.timing_report()
            extra = f" kernel {rows_us / max(nb, 1):.1f} us"
            eng.set_timing(0)
        print(f"timing events {'on ' if timed else 'off'}: {dt * 1e6:.1f} us per step{extra}")
