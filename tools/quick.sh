#!/bin/bash
# quick GPU iteration: parity tests + bench (no CPU baseline) [+ extra bench args]
set -o pipefail
mkdir -p gpurun_out/q
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q/t.log 2>&1 || { tail -30 gpurun_out/q/t.log; exit 1; }
tail -2 gpurun_out/q/t.log
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/q/b.log 2>&1 || { tail -20 gpurun_out/q/b.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/q/b.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['bitexact_check'])"
if [ -n "$PROF" ]; then timeout -k 10 200 python tools/prof_chain.py > gpurun_out/q/prof.log 2>&1 && tail -12 gpurun_out/q/prof.log; fi
