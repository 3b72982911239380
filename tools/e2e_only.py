"""The bench's end-to-end leg alone (bench.end_to_end: 8 h264mi_dec processes,
host parse + H2D + kernels + D2H of every picture), for A/B of host-side
changes: H264MI_LIB_DIR picks the build.  Prints one JSON line.

    python tools/e2e_only.py [reps]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
# E2E_PIN=1: pin the processes to GPU 0's NUMA-local cores (bench.e2e_core_plan)
cpus = None
if os.environ.get("E2E_PIN") == "1":
    import torch
    cpus, _ = bench.e2e_core_plan(0, [bench.gpu_numa_node(torch, 0)], os.sched_getaffinity(0))
streams, _ = bench.prepare(3, [100 + i for i in range(8)], bench.GOP)
r = bench.end_to_end(streams, bench.GOP, reps=reps, cpus=cpus)
print(json.dumps({k: r[k] for k in ("value", "host_cpu_ms_per_picture", "host_cores_busy", "cpus", "per_picture_ms")}))
