"""Frame-pipelined launches vs the oracle: mismatch summary per configuration
(size, streams, steps per launch).  GPU box: python tools/pipe_diag.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import bench  # noqa: E402
import oracle as O  # noqa: E402
from broadway_amd import _lib, gen  # noqa: E402
from broadway_amd.engine import Capture  # noqa: E402


def run(w, h, S, pipe, preset=2, nf=10):
    streams = [gen.generate(preset, 70 + i, nframes=nf, w_mbs=w, h_mbs=h, crop_bottom=0, slices=2, gop=5)
               for i in range(S)]
    caps = [Capture(s) for s in streams]
    refs = [O.decode(s)[0] for s in streams]
    n = min(c.npics for c in caps)
    n -= n % 2
    r = bench.DeviceRun(_lib.mi(), caps, 0, n, pipe)
    bad = []
    try:
        for i, (k0, P) in enumerate(r.sched):
            r.launch(i)
            r.eng.sync()
            for k in range(k0, k0 + P):
                for s in range(S):
                    got = np.frombuffer(r.eng.read(s, int(r.cur_slots[k][s])).tobytes(), np.uint8)
                    ref = np.frombuffer(refs[s][k], np.uint8)
                    d = np.nonzero(got != ref)[0]
                    if len(d):
                        ysz = w * h * 256
                        y = d[d < ysz]
                        c = d[d >= ysz] - ysz
                        mbs = sorted(set(((int(o) // (w * 16)) // 16, (int(o) % (w * 16)) // 16) for o in y[:2000]))
                        cmbs = sorted(set((((int(o) % (w * h * 64)) // (w * 8)) // 8, ((int(o) % (w * h * 64)) % (w * 8)) // 8)
                                          for o in c[:2000]))
                        bad.append((s, k, len(y), len(c), mbs[:8], cmbs[:8]))
        print(f"{w}x{h} S={S} pipe={pipe} P={r.P} launches={len(r.sched)} errors={r.eng.errors()} "
              f"bad={len(bad)}", flush=True)
        for b in bad[:6]:
            print("   stream %d pic %d luma %d chroma %d luma MBs %s chroma MBs %s" % b, flush=True)
    finally:
        r.free()


if __name__ == "__main__":
    for args in [(13, 7, 3, 1), (13, 7, 3, 2), (13, 7, 8, 2), (12, 9, 3, 2), (16, 8, 3, 2), (16, 8, 8, 2),
                 (120, 68, 3, 2)]:
        run(*args)
