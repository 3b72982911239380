#!/usr/bin/env python3
"""Summarise a gpu_round.sh session into profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats of the bench command
  profiles/<tag>_pmc.json           FETCH_SIZE / WRITE_SIZE per launch (separate passes)
  profiles/traffic.json             HBM bytes per reconstruction step (k_wgpp + k_prep),
                                    read by bench.py for roofline.traffic

Units and corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE / WRITE_SIZE are
KiB; on gfx950 FETCH_SIZE counts 64 B per 128-B request, so it is doubled.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kname(full):
    """'void k_wgpp<3, false, true, 1>(ReconArgs)' -> 'k_wgpp'"""
    n = full.split("(")[0].split("<")[0]
    return n.split()[-1]


def per_launch(path, counter):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            d[kname(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in d.items()}


def calibration(src):
    """FETCH_SIZE per kernel of tools/ubench/fetch_calib vs the bytes it reads
    (printed by the program): factor = bytes / (FETCH_SIZE KiB * 1024)."""
    log, cc = os.path.join(src, "calib.log"), os.path.join(src, "calib", "calib_counter_collection.csv")
    if not (os.path.exists(log) and os.path.exists(cc)):
        return None
    want = {}
    for line in open(log):
        f = line.split()
        if len(f) >= 3 and f[0].startswith("k_") and f[1] == "bytes":
            want[f[0]] = int(f[2])
    got = per_launch(cc, "FETCH_SIZE")
    return {k: {"bytes": b, "FETCH_SIZE_KiB": round(got[k][0], 1), "factor": round(b / (got[k][0] * 1024), 3)}
            for k, b in want.items() if k in got}


def trace_window(src):
    """k_wgpp durations of the bench's timed window in the rocprofv3 kernel
    trace of the same command (bench line kernels.k_wgpp.trace_window /
    trace_sampled: dispatch indices in trace order), beside the bench's own
    HIP-event average"""
    tr, bj = os.path.join(src, "prof", "bench_kernel_trace.csv"), os.path.join(src, "prof_bench.json")
    if not (os.path.exists(tr) and os.path.exists(bj)):
        return None
    line = json.loads(open(bj).read().strip().splitlines()[-1])
    k = line["kernels"]["k_wgpp"]
    if "trace_window" not in k:
        return None
    rows = [r for r in csv.DictReader(open(tr)) if kname(r["Kernel_Name"]) == "k_wgpp"]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    a, b = k["trace_window"]
    win = dur[a:b]
    ts = k["trace_sampled"]
    smp = win if ts == "all" else [dur[i] for i in ts if i < len(dur)]
    return {"k_wgpp_dispatches_in_trace": len(dur), "timed_window": [a, b],
            "rocprof_timed_window_avg_us": round(sum(win) / max(len(win), 1), 2),
            "rocprof_sampled_avg_us": round(sum(smp) / max(len(smp), 1), 2),
            "bench_hip_event_avg_us": k["avg_launch_us"],
            "note": "the stats CSV's k_wgpp average also counts pre-roll / warmup launches (IDR-heavy) "
                    "and the P-only leg's; this is the timed window alone"}


def window_bytes(src, counter, sub):
    """Counter values of the k_wgpp dispatches of the bench's timed window
    (kernels.k_wgpp.trace_window of prof_bench.json, the same command as the
    --pmc passes), in dispatch order, and the steps each of those launches
    holds (trace_steps; one step each when the line predates it)."""
    bj = os.path.join(src, "prof_bench.json")
    cc = os.path.join(src, sub, "bench_counter_collection.csv")
    if not (os.path.exists(bj) and os.path.exists(cc)):
        return None
    k = json.loads(open(bj).read().strip().splitlines()[-1])["kernels"]["k_wgpp"]
    if "trace_window" not in k:
        return None
    rows = [r for r in csv.DictReader(open(cc)) if kname(r["Kernel_Name"]) == "k_wgpp" and r["Counter_Name"] == counter]
    if rows and "Dispatch_Id" in rows[0]:
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    a, b = k["trace_window"]
    vals = [float(r["Counter_Value"]) for r in rows][a:b]
    steps = k.get("trace_steps") or [1] * len(vals)
    return vals, steps[:len(vals)]


def _counters(path):
    """{kernel: {counter: (mean per launch, launches)}} of one counter-collection CSV"""
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        d[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: (sum(v) / len(v), len(v)) for c, v in cs.items()} for k, cs in d.items()}


def exact_bytes(src, prefix, prog):
    """Memory-side bytes per launch from the L2's request-size counters
    (tools/pmc_bytes.sh): read = 32 n32 + 64 n64 + 128 n128 (TCC_EA0_RDREQ_*B),
    split by destination with the 32-B-unit counters RDREQ_{DRAM,GMI,IO}_32B;
    write = 32 x WRREQ_WRITE_{DRAM,GMI,IO}_32B.  None when the passes are absent."""
    paths = {p: os.path.join(src, f"bytes_{prefix}_{p}", f"{prog}_counter_collection.csv") for p in ("rd", "src", "wr")}
    if not all(os.path.exists(p) for p in paths.values()):
        return None
    c = {p: _counters(q) for p, q in paths.items()}
    out = {}
    for k in c["rd"]:
        rd, sr, wr = c["rd"][k], c["src"].get(k, {}), c["wr"].get(k, {})
        g = lambda t, n: t.get(n, (0.0, 0))[0]
        n32, n64, n128 = g(rd, "TCC_EA0_RDREQ_32B_sum"), g(rd, "TCC_EA0_RDREQ_64B_sum"), g(rd, "TCC_EA0_RDREQ_128B_sum")
        out[k] = {"launches": rd["TCC_EA0_RDREQ_sum"][1],
                  "rdreq": {"all": g(rd, "TCC_EA0_RDREQ_sum"), "32B": n32, "64B": n64, "128B": n128},
                  "read_bytes": int(32 * n32 + 64 * n64 + 128 * n128),
                  "read_bytes_dram": int(32 * g(sr, "TCC_EA0_RDREQ_DRAM_32B_sum")),
                  "read_bytes_gmi": int(32 * g(sr, "TCC_EA0_RDREQ_GMI_32B_sum")),
                  "read_bytes_io": int(32 * g(sr, "TCC_EA0_RDREQ_IO_32B_sum")),
                  "write_bytes_dram": int(32 * g(wr, "TCC_EA0_WRREQ_WRITE_DRAM_32B_sum")),
                  "write_bytes_gmi": int(32 * g(wr, "TCC_EA0_WRREQ_WRITE_GMI_32B_sum")),
                  "write_bytes_io": int(32 * g(wr, "TCC_EA0_WRREQ_WRITE_IO_32B_sum"))}
    return out


def bytes_report(tag, src, dst):
    """profiles/<tag>_bytes.json from tools/pmc_bytes.sh: the calibration
    program's known byte counts against the request-size accounting, and the
    bench's bytes per reconstruction step (k_wgpp + the standalone k_prep
    spread over the k_wgpp launches, as main() does); the request-size
    figures are added to profiles/traffic.json beside the FETCH_SIZE one"""
    rep = {"tag": tag, "method": "tools/pmc_bytes.sh: rocprofv3 --pmc, three passes of <= 4 TCC counters "
                                 "(TCC_EA0_RDREQ_{32B,64B,128B}, RDREQ_{DRAM,GMI,IO}_32B, "
                                 "WRREQ_WRITE_{DRAM,GMI,IO}_32B); bytes per launch"}
    want = {}
    log = os.path.join(src, "bytes_calib.log")
    if os.path.exists(log):
        for line in open(log):
            f = line.split()
            if len(f) >= 3 and f[0].startswith("k_") and f[1] == "bytes":
                want[f[0]] = int(f[2])
    cal = exact_bytes(src, "calib", "calib") or {}
    rep["calibration"] = {k: {"bytes_read_by_program": b, "request_size_bytes": cal[k]["read_bytes"],
                              "ratio": round(cal[k]["read_bytes"] / b, 3),
                              "dram_32B_unit_bytes": cal[k]["read_bytes_dram"], "rdreq": cal[k]["rdreq"]}
                          for k, b in want.items() if k in cal}
    ex = exact_bytes(src, "bench", "bench")
    rep["kernels"] = ex
    main_k = "k_wgpp"
    n = ex[main_k]["launches"]
    keys = ("read_bytes", "read_bytes_dram", "read_bytes_gmi", "read_bytes_io",
            "write_bytes_dram", "write_bytes_gmi", "write_bytes_io")
    step = {k: sum(ex[kk][k] * ex[kk]["launches"] for kk in ex if kk in ("k_wgpp", "k_prep")) / n for k in keys}
    step = {k: int(v) for k, v in step.items()}
    step["dram_bytes"] = step["read_bytes_dram"] + step["write_bytes_dram"]
    step["all_bytes"] = step["read_bytes"] + step["write_bytes_dram"] + step["write_bytes_gmi"] + step["write_bytes_io"]
    rep["per_step"] = step
    json.dump(rep, open(os.path.join(dst, f"{tag}_bytes.json"), "w"), indent=1)
    tp = os.path.join(dst, "traffic.json")
    t = json.load(open(tp)) if os.path.exists(tp) else {}
    t["request_size_accounting"] = {"source": f"profiles/{tag}_bytes.json (tools/pmc_bytes.sh)",
                                    "dram_bytes_per_step": step["dram_bytes"],
                                    "all_bytes_per_step": step["all_bytes"],
                                    "read_bytes_per_step": step["read_bytes"],
                                    "write_bytes_dram_per_step": step["write_bytes_dram"]}
    json.dump(t, open(tp, "w"), indent=1)
    print(json.dumps(rep, indent=1))


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    if not os.path.exists(os.path.join(src, "prof")):         # tools/pmc_bytes.sh alone
        return bytes_report(tag, src, dst)
    shutil.copy(os.path.join(src, "prof", "bench_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    fetch = per_launch(os.path.join(src, "pmc_fetch", "bench_counter_collection.csv"), "FETCH_SIZE")
    write = per_launch(os.path.join(src, "pmc_write", "bench_counter_collection.csv"), "WRITE_SIZE")
    kernels = {}
    step = 0.0
    step_kernels = ("k_wgpp",) + (("k_prep",) if "k_prep" in fetch else ())
    for k in step_kernels:
        f_kib, n = fetch[k]
        w_kib, _ = write[k]
        hbm = (2 * f_kib + w_kib) * 1024
        kernels[k] = {"launches": n, "FETCH_SIZE_KiB": round(f_kib, 1), "WRITE_SIZE_KiB": round(w_kib, 1),
                      "read_bytes_corrected": int(2 * f_kib * 1024), "write_bytes": int(w_kib * 1024),
                      "hbm_bytes": int(hbm)}
        step += hbm * n
    # a step is one launch of the main kernel; the standalone k_prep launch
    # (the pipeline's first step) is spread over them
    step /= kernels[step_kernels[0]]["launches"]
    # (every launch of the main kernel averaged -- pre-roll, warmup and the
    # untimed legs included; the timed window's own bytes are timed_window)
    out = {"tag": tag, "kernels": kernels, "hbm_bytes_per_launch_all_launches": int(step),
           "note": "FETCH_SIZE doubled per the gfx950 correction; the factor 2.0 is measured for this kernel's 4-, 8-, 12- and 16-B per-lane loads (tools/ubench/fetch_calib.hip, profiles/r34_fetch_calib.json)"}
    json.dump(out, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
    json.dump({"source": f"profiles/{tag}_pmc.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)",
               "hbm_bytes_per_launch_all_launches": int(step)}, open(os.path.join(dst, "traffic.json"), "w"), indent=1)
    tw = trace_window(src)
    if tw:
        out["trace_window"] = tw
        json.dump(out, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
    # the bench's timed launches alone (a launch holds 1 or 2 steps): bytes
    # per timed launch -- roofline.traffic, the unit of roofline.achieved --
    # and per step
    fw, ww = window_bytes(src, "FETCH_SIZE", "pmc_fetch"), window_bytes(src, "WRITE_SIZE", "pmc_write")
    if fw and ww and fw[0] and len(fw[0]) == len(ww[0]):
        tot = sum((2 * f + w) * 1024 for f, w in zip(fw[0], ww[0]))
        win = {"launches": len(fw[0]), "steps": sum(fw[1]),
               "hbm_bytes_per_timed_launch": int(tot / len(fw[0])),
               "hbm_bytes_per_timed_step": int(tot / max(sum(fw[1]), 1))}
        out["timed_window"] = win
        json.dump(out, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
        t = json.load(open(os.path.join(dst, "traffic.json")))
        t.update(win)
        json.dump(t, open(os.path.join(dst, "traffic.json"), "w"), indent=1)
    cal = calibration(src)
    if cal:
        json.dump(cal, open(os.path.join(dst, f"{tag}_fetch_calib.json"), "w"), indent=1)
        print(json.dumps(cal, indent=1))
    for extra in ("chain_s8.log", "chain_s1.log"):
        if os.path.exists(os.path.join(src, extra)):
            shutil.copy(os.path.join(src, extra), os.path.join(dst, f"{tag}_{extra}"))
    if os.path.exists(os.path.join(src, "bench.json")):
        shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, f"{tag}_bench.json"))
    print(json.dumps(out, indent=1))
    if os.path.exists(os.path.join(src, "bytes_bench_rd")):
        bytes_report(tag, src, dst)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
