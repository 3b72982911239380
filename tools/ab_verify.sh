#!/bin/bash
# A/B of library builds (abtest/<name>/, tools/ab_build.sh) in one GPU call, each
# run verified bit-exact.  Usage (GPU box): ROUNDS=2 bash tools/ab_verify.sh A B [C ...]
set -o pipefail
mkdir -p gpurun_out/ab
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    H264MI_LIB_DIR=abtest/$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-legs --no-rgba $BENCH_ARGS > gpurun_out/ab/b.log 2>&1 || { tail -20 gpurun_out/ab/b.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab/b.log').read().strip().splitlines()[-1]);k=next(iter(d['kernels']));print(sys.argv[1], d['value'], k, d['kernels'][k]['avg_launch_us'], d['bitexact_check']['ok'], d['bitexact_check']['frames_checked'])" "$v"
  done
done
