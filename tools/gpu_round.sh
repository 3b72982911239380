#!/bin/bash
# One GPU session: parity tests, bench (with CPU baseline), rocprofv3 kernel
# stats of the bench command, and the two PMC passes for HBM traffic.
# Usage (from the repo root, on the GPU box): bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -c 400 $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-e2e --no-legs --no-rgba --no-verify > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o bench -- python3 bench.py --no-cpu-baseline --no-verify --no-e2e --no-legs --no-rgba > /dev/null 2> $OUT/pmc_fetch.err || { tail -20 $OUT/pmc_fetch.err; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o bench -- python3 bench.py --no-cpu-baseline --no-verify --no-e2e --no-legs --no-rgba > /dev/null 2> $OUT/pmc_write.err || { tail -20 $OUT/pmc_write.err; exit 1; }
bash tools/pmc_bytes.sh $TAG || exit 1
find $OUT -name "*.csv" | head -20
# FETCH_SIZE calibration for this kernel's access widths (tools/ubench/fetch_calib.hip)
if [ -x tools/ubench/fetch_calib ]; then
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/calib -o calib -- tools/ubench/fetch_calib > $OUT/calib.log 2>&1 || { tail -20 $OUT/calib.log; exit 1; }
fi
# row-chain decomposition of the profiling kernel (tools/prof_chain.py)
timeout -k 10 200 python tools/prof_chain.py > $OUT/chain_s8.log 2>&1 || { tail -20 $OUT/chain_s8.log; exit 1; }
PROF_S=1 timeout -k 10 200 python tools/prof_chain.py > $OUT/chain_s1.log 2>&1 || { tail -20 $OUT/chain_s1.log; exit 1; }
