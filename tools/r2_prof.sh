#!/bin/bash
# Profiles of the default bench command: rocprofv3 kernel stats, the two PMC
# passes (FETCH_SIZE / WRITE_SIZE, separate runs), then a 2-rank rehearsal of
# the multi-GPU path on this one GPU (BENCH_ONE_DEVICE=1).
# Usage (GPU box, repo root): bash tools/r2_prof.sh TAG; then tools/pmc_traffic.py TAG here
set -o pipefail
TAG=${1:-r2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-e2e --no-legs > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o bench -- python3 bench.py --no-cpu-baseline --no-verify --no-e2e --no-legs --no-rgba > /dev/null 2> $OUT/pmc_fetch.err || { tail -20 $OUT/pmc_fetch.err; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o bench -- python3 bench.py --no-cpu-baseline --no-verify --no-e2e --no-legs --no-rgba > /dev/null 2> $OUT/pmc_write.err || { tail -20 $OUT/pmc_write.err; exit 1; }
find $OUT -name "*.csv" | head -20
BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 bench.py --gpus 2 --no-cpu-baseline --no-e2e --no-legs --no-rgba > $OUT/rehearsal_2ranks.json 2> $OUT/rehearsal.err || { tail -20 $OUT/rehearsal.err; exit 1; }
tail -c 600 $OUT/rehearsal_2ranks.json
