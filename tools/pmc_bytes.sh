#!/bin/bash
# Exact memory-side bytes from the L2's request-size counters (gfx950 lists
# them; FETCH_SIZE's formula counts 128-B requests through TCC_BUBBLE, which
# is why it reads 1/2 of a streaming read here).  Three passes of <= 4 TCC
# counters each, on the FETCH_SIZE calibration program (known byte counts)
# and on the bench command of gpu_round.sh's PMC passes:
#   rd: RDREQ_32B / _64B / _128B / all   -> 32 n32 + 64 n64 + 128 n128
#   src: RDREQ_{DRAM,GMI,IO}_32B (32-B units, a 64-B request counts 2, 128-B 4), RDREQ_DRAM
#   wr: WRREQ_WRITE_{DRAM,GMI,IO}_32B (32-B units), WRREQ_64B
# Usage (GPU box, repo root): bash tools/pmc_bytes.sh TAG; then
# python3 tools/pmc_traffic.py TAG (here) summarises gpurun_out/TAG/bytes_*.
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P_RD="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"
P_SRC="TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_GMI_32B_sum TCC_EA0_RDREQ_IO_32B_sum TCC_EA0_RDREQ_DRAM_sum"
P_WR="TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_GMI_32B_sum TCC_EA0_WRREQ_WRITE_IO_32B_sum TCC_EA0_WRREQ_64B_sum"
for p in rd src wr; do
  case $p in rd) C=$P_RD;; src) C=$P_SRC;; wr) C=$P_WR;; esac
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/bytes_calib_$p -o calib -- tools/ubench/fetch_calib > $OUT/bytes_calib.log 2>&1 || { tail -20 $OUT/bytes_calib.log; exit 1; }
  echo "calib pass $p done"
done
for p in rd src wr; do
  case $p in rd) C=$P_RD;; src) C=$P_SRC;; wr) C=$P_WR;; esac
  timeout -s KILL 400 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/bytes_bench_$p -o bench -- python3 bench.py --no-cpu-baseline --no-verify --no-e2e --no-legs --no-rgba > /dev/null 2> $OUT/bytes_bench_$p.err || { tail -20 $OUT/bytes_bench_$p.err; exit 1; }
  echo "bench pass $p done"
done
