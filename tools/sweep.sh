#!/bin/bash
# GPU experiment helper: parity tests, then one short bench per environment
# setting given as arguments ("VAR=x VAR2=y" per argument; "" = defaults).
# Usage (GPU box, repo root): bash tools/sweep.sh "" "H264MI_WG_PP=0"
set -o pipefail
mkdir -p gpurun_out/sweep
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep/t.log 2>&1 || { tail -30 gpurun_out/sweep/t.log; exit 1; }
tail -1 gpurun_out/sweep/t.log
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/sweep/b.log 2>&1 || { tail -20 gpurun_out/sweep/b.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/sweep/b.log').read().strip().splitlines()[-1]);k=next(iter(d['kernels']));print(repr(sys.argv[1]), d['value'], d['ms_per_step'], k, d['kernels'][k]['avg_launch_us'], d['bitexact_check']['ok'])" "$cfg"
done
if [ -n "$PROF" ]; then H264MI_KERNEL=wg timeout -k 10 200 python tools/prof_rows.py > gpurun_out/sweep/prof.log 2>&1; fi
