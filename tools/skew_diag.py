"""Diagnostics (not a test): time single k_wgpp launches of the bench's
streams (configs[3], S streams, P steps) one by one with the engine's error
bits after each, for a study build (H264MI_LIB_DIR).  Usage:
python tools/skew_diag.py [S] [P] [launches]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from broadway_amd import _lib  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1
P = int(sys.argv[2]) if len(sys.argv) > 2 else 1
NL = int(sys.argv[3]) if len(sys.argv) > 3 else 4
L = _lib.mi()
seeds = [100 + i for i in range(S)]
streams, caps = bench.prepare(3, seeds, P * (NL + 1) + 1)
run = bench.DeviceRun(L, caps, 0, P * NL, P)
for i in range(min(NL, len(run.launches))):
    t = time.perf_counter()
    run.launch(i)
    run.eng.sync()
    print(f"launch {i} ({len(run.launches[i])} steps): {(time.perf_counter() - t) * 1e3:.2f} ms,"
          f" error bits {run.eng.error_bits():#x}, errors {run.eng.errors()}", flush=True)
