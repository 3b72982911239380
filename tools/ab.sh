#!/bin/bash
# A/B timing of library builds in one GPU call (box-to-box clock variation
# is larger than most kernel changes).  tools/ab_build.sh puts builds into
# abtest/<name>/; this runs the bench ROUNDS times per build, interleaved.
# Usage (GPU box): ROUNDS=3 bash tools/ab.sh A B [C ...]
set -o pipefail
mkdir -p gpurun_out/ab
for i in $(seq 1 ${ROUNDS:-3}); do
  for v in "$@"; do
    H264MI_LIB_DIR=abtest/$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-verify --steps 30 > gpurun_out/ab/b.log 2>&1 || { tail -20 gpurun_out/ab/b.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab/b.log').read().strip().splitlines()[-1]);k=next(iter(d['kernels']));print(sys.argv[1], d['value'], k, d['kernels'][k]['avg_launch_us'])" "$v"
  done
done
