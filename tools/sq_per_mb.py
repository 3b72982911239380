#!/usr/bin/env python3
"""Per-MB view of a tools/pmc_sq.sh capture (SQ counters of k_wgpp / k_prep).

Usage: python tools/sq_per_mb.py gpurun_out/<tag>/sqN MBS_PER_LAUNCH > profiles/<tag>_sq_sN.json

k_wgpp launches after the first carry the NEXT batch's k_prep as tail
workgroups; its per-MB cost is taken from the one standalone k_prep launch
(the first batch) and subtracted, so `k_wgpp_rows` is the row workgroups
alone.  SQ_*_CYCLES counters are in quad-cycles (4 clocks); waves per CU =
SQ_WAVE_CYCLES * 4 / (launch duration * 2.4 GHz * 256 CUs).
"""
import collections
import csv
import glob
import json
import sys

src, mbs = sys.argv[1], int(sys.argv[2])
acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in glob.glob(f"{src}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].split("<")[0].split()[-1]
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for f in glob.glob(f"{src}/**/*kernel_trace.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].split("<")[0].split()[-1]
        dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
mean = lambda v: sum(v) / len(v)
res = {"source": src, "mbs_per_launch": mbs, "note": __doc__.strip().splitlines()[0]}
per = {}
for k in ("k_wgpp", "k_prep"):
    if k not in acc:
        continue
    c = {n: mean(v) for n, v in acc[k].items()}
    d = mean(dur[k][1:] if len(dur[k]) > 2 else dur[k])
    per[k] = c
    res[k] = {
        "launches": len(acc[k]["SQ_WAVES"]), "avg_launch_us": round(d * 1e6, 1),
        "waves": round(c["SQ_WAVES"]),
        "valu_per_mb": round(c["SQ_INSTS_VALU"] / mbs, 1), "salu_per_mb": round(c["SQ_INSTS_SALU"] / mbs, 1),
        "lds_per_mb": round(c["SQ_INSTS_LDS"] / mbs, 1),
        "vmem_per_mb": round((c["SQ_INSTS_VMEM_RD"] + c["SQ_INSTS_VMEM_WR"]) / mbs, 1),
        "branch_per_mb": round(c["SQ_INSTS_BRANCH"] / mbs, 1),
        "waves_per_cu": round(c["SQ_WAVE_CYCLES"] * 4 / (d * 2.4e9 * 256), 2),
        "wave_time_frac": {
            "issuing": round(c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"], 3),
            "parked_waitcnt_barrier": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 3),
            "issue_stalled": round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 3),
            "lds_issue_stalled": round(c["SQ_WAIT_INST_LDS"] / c["SQ_WAVE_CYCLES"], 3)},
        "SQ_BUSY_CYCLES": round(c["SQ_BUSY_CYCLES"]),
        "valu_simd_busy_frac": round(c["SQ_ACTIVE_INST_VALU"] * 4 / (d * 2.4e9 * 1024), 3),
    }
if "k_wgpp" in per and "k_prep" in per:
    w, p = per["k_wgpp"], per["k_prep"]
    res["k_wgpp_rows"] = {n: round((w[i] - p[i]) / mbs, 1) for n, i in
                          (("valu_per_mb", "SQ_INSTS_VALU"), ("salu_per_mb", "SQ_INSTS_SALU"),
                           ("lds_per_mb", "SQ_INSTS_LDS"), ("branch_per_mb", "SQ_INSTS_BRANCH"),
                           ("vmem_rd_per_mb", "SQ_INSTS_VMEM_RD"), ("vmem_wr_per_mb", "SQ_INSTS_VMEM_WR"))}
print(json.dumps(res, indent=1))
