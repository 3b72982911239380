#!/bin/bash
# SURVEY §8d config 5 (one 3840x2160 stream) and config 2 (720p I-only):
# bench lines, rocprofv3 kernel stats and the two HBM PMC passes, plus the
# CPU / end-to-end table (tools/config_table.py).  Usage: bash tools/cfg5_profile.sh TAG
set -o pipefail
TAG=${1:-cfg5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B4="bench.py --config 4 --streams 1 --steps 20 --warmup 4 --no-cpu-baseline --no-e2e --no-rgba --no-legs"
B2="bench.py --config 1 --streams 4 --steps 20 --warmup 4 --no-cpu-baseline --no-e2e --no-rgba --no-legs"
timeout -k 10 300 python3 $B4 > $OUT/bench_cfg5.json 2> $OUT/b5.err || { tail -20 $OUT/b5.err; exit 1; }
timeout -k 10 300 python3 $B2 > $OUT/bench_cfg2.json 2> $OUT/b2.err || { tail -20 $OUT/b2.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof5 -o bench -- python3 $B4 > /dev/null 2> $OUT/prof5.err || { tail -20 $OUT/prof5.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o bench -- python3 $B4 --no-verify > /dev/null 2> $OUT/pf.err || { tail -20 $OUT/pf.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o bench -- python3 $B4 --no-verify > /dev/null 2> $OUT/pw.err || { tail -20 $OUT/pw.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof2 -o bench -- python3 $B2 > /dev/null 2> $OUT/prof2.err || { tail -20 $OUT/prof2.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc2_fetch -o bench -- python3 $B2 --no-verify > /dev/null 2> $OUT/pf2.err || { tail -20 $OUT/pf2.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc2_write -o bench -- python3 $B2 --no-verify > /dev/null 2> $OUT/pw2.err || { tail -20 $OUT/pw2.err; exit 1; }
[ "${CFG_TABLE:-1}" = 1 ] || { echo done; exit 0; }
timeout -k 10 600 python3 tools/config_table.py > $OUT/config_table.json 2> $OUT/config_table.err || { tail -20 $OUT/config_table.err; exit 1; }
echo done
