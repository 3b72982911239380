#!/usr/bin/env python3
"""CPU-comparator and end-to-end table of SURVEY.md §8d configs 1, 2, 3 and 5
(BASELINE.md §3).  Per config, on the machine it runs on:
  reference CPU   oracle/_ref/refdec (the reference C, built from
                  /root/reference by oracle/Makefile.ref): 1 process on one
                  stream, and 8 processes on 8 streams in parallel (one core each)
  end-to-end      broadway_amd/lib/h264mi_dec (the product H264SwDec* C-ABI:
                  host parse + H2D + kernels + D2H), same 1 / 8 process models,
                  only when a GPU is visible
Prints one JSON object.  Usage: python tools/config_table.py [--no-gpu]"""
import concurrent.futures as cf
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {   # name -> (generator preset, seeds of the 8-process run, frames)
    "1_640x368_plumbing": (0, list(range(1, 9)), 60),
    "2_720p_ionly": (1, list(range(1, 9)), 24),
    "3_1080p_ip": (3, list(range(100, 108)), 60),
    "5_2160p_ip": (4, list(range(100, 108)), 24),
}


def timed(cmds):
    """run the commands in parallel; wall seconds of the whole set"""
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(max_workers=len(cmds)) as ex:
        rs = list(ex.map(lambda c: subprocess.run(c, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True), cmds))
    dt = time.perf_counter() - t0
    for r in rs:
        if r.returncode != 0:
            raise RuntimeError(r.stderr[-300:])
    return dt, rs


def main():
    from broadway_amd import gen
    refdec = os.path.join(ROOT, "oracle", "_ref", "refdec")
    e2e = os.path.join(ROOT, "broadway_amd", "lib", "h264mi_dec")
    gpu = "--no-gpu" not in sys.argv
    try:
        cpu_model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        cpu_model = "unknown"
    out = {"host": cpu_model, "cpus_visible": os.cpu_count(), "configs": {}}
    td = tempfile.mkdtemp(prefix="cfgtab")
    for name, (preset, seeds, n) in CONFIGS.items():
        paths = []
        for s in seeds:
            p = os.path.join(td, f"{name}_{s}.h264")
            with open(p, "wb") as f:
                f.write(gen.generate(preset, s, nframes=n))
            paths.append(p)
        row = {"frames_per_stream": n, "seeds": seeds}
        if os.path.exists(refdec):
            t1, _ = timed([[refdec, "-Onone", paths[0]]])
            t8, _ = timed([[refdec, "-Onone", p] for p in paths])
            row["reference_cpu_1core_fps"] = round(n / t1, 1)
            row["reference_cpu_8x8_fps"] = round(8 * n / t8, 1)
        if gpu and os.path.exists(e2e):
            reps = 3 if n <= 60 and preset != 4 else 1
            # -T: the process's own decode-loop time (HIP start-up excluded)
            def e2e_rate(ps):
                _, rs = timed([[e2e, "-Onone", f"-r{reps}", "-T", p] for p in ps])
                secs = [float(l.split()[1]) for r in rs for l in r.stdout.splitlines() if l.startswith("decode_seconds")]
                return round(len(ps) * n * reps / max(secs), 1)
            row["e2e_1proc_fps"] = e2e_rate(paths[:1])
            row["e2e_8proc_fps"] = e2e_rate(paths)
        out["configs"][name] = row
        print(name, row, file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
