#!/usr/bin/env python3
"""Host cost of the drop-in decode loop without the GPU, on the box's host
cores (diagnostics): tools/ubench/parse_null (the product decoder core over a
backend that reconstructs nothing) on the configs[3] rank-0 streams,
  - one process alone, without and with speculative-parse workers;
  - 8 processes at once (one per stream, as bench.end_to_end), pinned to the
    same NUMA-local core share the end-to-end leg uses, with PN_COPY=0 / 1
    (1: each picture's records and coefficients copied to a staging buffer,
    as the HIP backend copies them into pinned memory).
Prints CPU ms per picture and pictures/s for each, one JSON line."""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

EXE = os.path.join(ROOT, "tools", "ubench", "parse_null")


def run(paths, threads, passes, cpus=None, copy=0, l3=False):
    env = dict(os.environ, H264MI_PARSE_THREADS=str(threads), PN_COPY=str(copy))
    per = bench.process_cpus(cpus, len(paths)) if cpus and l3 else [cpus] * len(paths)
    pre = lambda i: ["taskset", "-c", bench.format_cpulist(per[i])] if per[i] else []
    t0 = time.monotonic()
    procs = [subprocess.Popen(pre(i) + [EXE, p, str(passes)], stdout=subprocess.PIPE, text=True, env=env)
             for i, p in enumerate(paths)]
    outs = [pr.communicate(timeout=600)[0] for pr in procs]
    wall = time.monotonic() - t0
    pics = cpu = 0.0
    for o in outs:
        f = o.split()
        n = int(f[f.index("pictures") + 1])
        pics += n
        cpu += float(f[f.index("cpu") + 1]) * n
    return {"processes": len(paths), "parse_threads": threads, "staging_copy": copy, "one_l3_per_process": l3,
            "cpu_ms_per_picture": round(cpu / pics, 3), "pictures_per_s": round(pics / wall, 1)}


def main():
    import torch
    cpus, _ = bench.e2e_core_plan(0, [bench.gpu_numa_node(torch, 0)], os.sched_getaffinity(0))
    td = tempfile.mkdtemp(prefix="hpp")
    streams, _ = bench.prepare(3, [100 + i for i in range(8)], bench.GOP)
    paths = []
    for i, s in enumerate(streams):
        p = os.path.join(td, f"s{i}.h264")
        open(p, "wb").write(s)
        paths.append(p)
    res = {"cpus": bench.format_cpulist(cpus), "host_cores": len(cpus),
           "one_sequential": run(paths[:1], 0, 6), "one_spec2": run(paths[:1], 2, 6),
           "eight_sequential": run(paths, 0, 6, cpus), "eight_spec2": run(paths, 2, 6, cpus),
           "eight_spec2_copy": run(paths, 2, 6, cpus, 1),
           "eight_spec2_l3": run(paths, 2, 6, cpus, 0, True), "eight_spec3_l3": run(paths, 3, 6, cpus, 0, True),
           "one_spec2_l3": run(paths[:1], 2, 6, cpus, 0, True),
           "l3_groups": [bench.format_cpulist(g) for g in bench.l3_groups(cpus)]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
