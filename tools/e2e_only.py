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
streams, _ = bench.prepare(3, [100 + i for i in range(8)], bench.GOP)
print(json.dumps(bench.end_to_end(streams, bench.GOP, reps=reps)))
