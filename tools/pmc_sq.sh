#!/bin/bash
# SQ instruction/cycle counters per kernel (two PMC passes), bench workload.
# Usage (GPU box, repo root): bash tools/pmc_sq.sh TAG [bench args...]
set -o pipefail
TAG=${1:-sq}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o sq -- python3 bench.py --no-cpu-baseline --no-verify --no-e2e --no-legs --steps 8 --warmup 2 "$@" > $OUT/p$i.log 2>&1 || { tail -20 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_sq_report.py $OUT
