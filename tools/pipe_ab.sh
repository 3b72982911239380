#!/bin/bash
# Frame-pipelined launches, A/B on the bench workload and on the same streams
# without off-picture MVs (offpic_pct=0): bench kernel leg at P = 1 and P = 2.
# Usage (GPU box, repo root): bash tools/pipe_ab.sh TAG
set -o pipefail
TAG=${1:-pipe_ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for G in "" "offpic_pct=0"; do
  for P in 1 2; do
    F=$OUT/bench_p${P}_${G:-default}.json
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e --no-legs --no-rgba --pipe $P ${G:+--gen $G} > $F 2> $F.err || { tail -20 $F.err; exit 1; }
    python -c "import json;d=json.load(open('$F'));print('P=$P gen=${G:-default}', d['value'], d['ms_per_step'], d['kernels']['k_wgpp']['avg_launch_us'], d['bitexact_check'])"
  done
done
