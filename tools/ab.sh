#!/bin/bash
# A/B timing of library builds in one GPU call (box-to-box clock variation
# is larger than most kernel changes).  tools/ab_build.sh puts builds into
# abtest/<name>/; this runs the bench ROUNDS times per build, interleaved,
# and prints per run: the GOP-mix frames/s, its k_wgpp us per launch, and the
# P-only (aligned GOPs) frames/s and us per launch.
# Usage (GPU box): ROUNDS=3 bash tools/ab.sh A B [C ...]
set -o pipefail
mkdir -p gpurun_out/ab
for i in $(seq 1 ${ROUNDS:-3}); do
  for v in "$@"; do
    H264MI_LIB_DIR=abtest/$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-verify --no-legs --no-rgba $BENCH_ARGS > gpurun_out/ab/b.log 2>&1 || { tail -20 gpurun_out/ab/b.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab/b.log').read().strip().splitlines()[-1]);p=d.get('p_only') or {};print(sys.argv[1], d['value'], d['kernels']['k_wgpp']['avg_launch_us'], p.get('value'), p.get('avg_launch_kernel_us'))" "$v"
  done
done
