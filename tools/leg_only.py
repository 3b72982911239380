#!/usr/bin/env python3
"""Run one bench.py config leg on its own (GPU box), for A/B work:
    python tools/leg_only.py noloop [pipe [mc]] # cfg3 streams, loop filter off
    python tools/leg_only.py cfg3 [pipe]        # the same streams as configs[3]
    python tools/leg_only.py offpic0 [pipe]     # configs[3] without off-picture MVs
    python tools/leg_only.py cfg2 | cfg5        # 720p I-only x4 / 2160p x1
Prints the leg's JSON dict (bench.run_leg)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch
    from broadway_amd import _lib
    which = sys.argv[1] if len(sys.argv) > 1 else "noloop"
    pipe = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    nmc = int(sys.argv[3]) if len(sys.argv) > 3 else 2     # MC waves per row workgroup (one-step launches)
    L = _lib.mi()
    seeds = list(range(100, 108))
    steps, warm = (54, 3) if pipe == 3 else (56, 4)
    if which == "noloop":
        r = bench.run_leg(L, torch, 3, seeds, steps, warm, overrides={"dbf_idc1_pct": 100}, pipe=pipe, mc_waves=nmc)
    elif which == "cfg3":
        r = bench.run_leg(L, torch, 3, seeds, steps, warm, pipe=pipe, mc_waves=2)
    elif which == "offpic0":
        r = bench.run_leg(L, torch, 3, seeds, steps, warm, overrides={"offpic_pct": 0}, pipe=pipe, mc_waves=2)
    elif which == "cfg2":
        r = bench.run_leg(L, torch, 1, [1, 2, 3, 4], 20, 4, mc_waves=0)
    elif which == "cfg2s1":
        r = bench.run_leg(L, torch, 1, [1], 20, 4, mc_waves=0)
    elif which == "cfg5":
        r = bench.run_leg(L, torch, 4, [100], 21, 3, pipe=3)
    else:
        raise SystemExit(f"unknown leg {which}")
    print(json.dumps({"leg": which, "pipe": pipe, **r}))


if __name__ == "__main__":
    main()
