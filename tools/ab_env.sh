#!/bin/bash
# A/B timing of environment settings of one build in one GPU call.
# Usage (GPU box): ROUNDS=2 BENCH_ARGS="--streams 8" bash tools/ab_env.sh "H264MI_RPW=1" "H264MI_RPW=3"
set -o pipefail
mkdir -p gpurun_out/ab
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-legs --no-rgba --steps 30 $BENCH_ARGS > gpurun_out/ab/e.log 2>&1 || { tail -20 gpurun_out/ab/e.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab/e.log').read().strip().splitlines()[-1]);k=next(iter(d['kernels']));print(sys.argv[1], d['value'], k, d['kernels'][k]['avg_launch_us'], (d.get('bitexact_check') or {}).get('ok'))" "$v"
  done
done
