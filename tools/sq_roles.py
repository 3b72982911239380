"""Workload for the SQ role split (tools/sq_roles.sh), not a test: the bench's
8 1080p streams, pictures 0..N-1 (PICS, default 12; P pictures after the
IDR) through the profiling k_wgpp (k_wgpp<3, true, ...>), H264MI_PROF_MODE
from the environment: 0 = normal, 1 = row waves only drain the MC ring.
rocprofv3's SQ counters of the two runs, launch for launch, differ by what
the row waves execute (the MC waves and tail k_prep workgroups do the same
work in both).

    python tools/sq_roles.py            (under rocprofv3 --pmc ...)
    python tools/sq_roles.py report DIR0 DIR1   (per-MB table from two captures)
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

S, W, H = 8, 120, 68


def run():
    import bench
    from broadway_amd import _lib
    n = int(os.environ.get("PICS", "12"))
    L = _lib.mi()
    _, caps = bench.prepare(3, [100 + i for i in range(S)], n)
    r = bench.DeviceRun(L, caps, 0, n, 1)
    L.h264mi_engine_profile(r.eng._h, 1, None, 0)
    for i in range(len(r.launches)):
        r.launch(i)
    r.eng.sync()
    r.free()


def counters(d):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "k_wgpp" in row["Kernel_Name"]:
                acc[(row["Counter_Name"], int(row.get("Dispatch_Id", 0)))].append(float(row["Counter_Value"]))
    per = collections.defaultdict(list)
    for (name, disp), v in sorted(acc.items()):
        per[name].append(sum(v))
    # the first k_wgpp launch follows the standalone k_prep: keep launches 2..
    return {k: sum(v[1:]) / max(len(v) - 1, 1) for k, v in per.items()}


def report(d0, d1):
    a, b = counters(d0), counters(d1)
    mbs = S * W * H
    keys = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
            "SQ_INSTS_SMEM", "SQ_WAVES"]
    keys += sorted(k for k in a if k not in keys)     # cycle counters (quad-cycles, summed over waves)
    out = {"mbs_per_launch": mbs, "method": "SQ counters per k_wgpp launch (profiling build), normal run minus a run "
                                            "whose row waves only drain the MC ring; per MB of the launch"}
    for k in keys:
        if k in a and k in b:
            out[k] = {"all_per_mb": round(a[k] / mbs, 1), "mc_and_tail_prep_per_mb": round(b[k] / mbs, 1),
                      "row_waves_per_mb": round((a[k] - b[k]) / mbs, 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "report":
        report(sys.argv[2], sys.argv[3])
    else:
        run()
