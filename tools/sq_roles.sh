#!/bin/bash
# SQ instruction counters of the final k_wgpp split by wave role (row vs MC):
# tools/sq_roles.py under rocprofv3, normal and ring-drain modes, two counter
# passes each.  Usage (GPU box, repo root): bash tools/sq_roles.sh TAG
set -o pipefail
TAG=${1:-sqroles}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
P2="SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"
# where the cycles go (quad-cycles): issuing, parked in s_waitcnt / barrier /
# s_sleep, or ready but not issued (VALU dependency, arbitration)
P3="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
for m in 0 1; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    H264MI_PROF_MODE=$m timeout -s KILL 150 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/m$m -o p$i -- python3 tools/sq_roles.py > $OUT/m${m}_p$i.log 2>&1 || { tail -20 $OUT/m${m}_p$i.log; exit 1; }
  done
done
python3 tools/sq_roles.py report $OUT/m0 $OUT/m1 > $OUT/sq_roles.json && cat $OUT/sq_roles.json
