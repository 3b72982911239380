#!/bin/bash
# bench at a given --streams for several environment settings (experiments)
set -o pipefail
S=$1; shift
mkdir -p gpurun_out/sweep
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-verify --steps 20 --streams $S > gpurun_out/sweep/b.log 2>&1 || { tail -20 gpurun_out/sweep/b.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/sweep/b.log').read().strip().splitlines()[-1]);k=next(iter(d['kernels']));print('S=$S', repr(sys.argv[1]), d['value'], d['ms_per_step'], k, d['kernels'][k]['avg_launch_us'])" "$cfg"
done
