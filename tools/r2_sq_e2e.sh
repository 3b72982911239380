#!/bin/bash
# e2e leg with the per-picture time split (with and without parse threads),
# then SQ counters of k_wgpp at 8 and 32 streams (bench workload only).
set -o pipefail
OUT=gpurun_out/${TAG:-r19}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-legs --no-rgba > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
H264MI_PARSE_THREADS=0 timeout -k 10 300 python3 -c "import bench,json;print(json.dumps(bench.end_to_end(bench.prepare(3, bench.shard_seeds(0,8), 60)[0], 60)))" > $OUT/e2e_nothreads.json 2> $OUT/e2e0.err || { tail -20 $OUT/e2e0.err; exit 1; }
[ -n "$NO_SQ" ] && { echo done; exit 0; }
bash tools/pmc_sq.sh ${TAG:-r19}/sq8 > $OUT/sq8.txt 2>&1 || { tail -20 $OUT/sq8.txt; exit 1; }
bash tools/pmc_sq.sh ${TAG:-r19}/sq32 --streams 32 > $OUT/sq32.txt 2>&1 || { tail -20 $OUT/sq32.txt; exit 1; }
echo done
