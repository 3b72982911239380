#!/bin/bash
# A/B of the tail-prep start (H264MI_PREP_AT, % of a launch's rows done) in one
# GPU call; bench without the CPU / end-to-end legs.  Usage: bash tools/prep_at.sh 20 35 50
set -o pipefail
mkdir -p gpurun_out/prepat
for i in 1 2; do
  for v in "$@"; do
    H264MI_PREP_AT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-rgba --steps 30 > gpurun_out/prepat/b.log 2>&1 || { tail -20 gpurun_out/prepat/b.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/prepat/b.log').read().strip().splitlines()[-1]);print('PREP_AT', sys.argv[1], d['value'], d['ms_per_step'], d['kernels']['k_wgpp']['avg_launch_us'], d['bitexact_check']['ok'], d['bitexact_check']['frames_checked'])" "$v"
  done
done
