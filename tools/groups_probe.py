"""Diagnostics (not the bench): the configs[3] workload (8 x 1080p streams on
one GPU) split over K engines of 8/K streams each, every engine on its own
HIP stream, launches issued round-robin.  A launch then waits only for its
own group's previous pictures instead of the slowest of all 8, and the
groups' launches overlap.  Prints frames/s per K and verifies every picture
against the reference MD5s (bench.verify_all per group).

    python tools/groups_probe.py [K ...]      (default: 1 2 4)
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

WARMUP, STEPS, S = 4, 56, 8


def main(ks):
    import torch
    from broadway_amd import _lib
    L = _lib.mi()
    seeds = bench.shard_seeds(0, S)
    streams, caps = bench.prepare(3, seeds, WARMUP + STEPS, {})
    for k in ks:
        g = S // k
        runs = [bench.DeviceRun(L, caps[i * g:(i + 1) * g], WARMUP, STEPS, 1) for i in range(k)]
        nwarm = sum(1 for k0, _ in runs[0].sched if k0 < WARMUP)
        for i in range(nwarm):
            for r in runs:
                r.launch(i)
        for r in runs:
            r.eng.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(nwarm, len(runs[0].sched)):
            for r in runs:
                r.launch(i)
        for r in runs:
            r.eng.sync()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ok_all, n_all = True, 0
        for i, r in enumerate(runs):
            ok, n, _ = bench.verify_all(r.eng, r.launch, r.sched, caps[i * g:(i + 1) * g],
                                        seeds[i * g:(i + 1) * g], 3, {}, r.cur_slots)
            ok_all &= bool(ok)
            n_all += n
        print(f"K={k} engines x {g} streams: {S * STEPS / dt:.1f} frames/s, {dt / STEPS * 1e6:.1f} us per step, "
              f"bit-exact {ok_all} ({n_all} frames)", flush=True)
        for r in runs:
            r.free()


if __name__ == "__main__":
    main([int(x) for x in sys.argv[1:]] or [1, 2, 4])
