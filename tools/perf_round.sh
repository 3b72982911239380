#!/bin/bash
# Kernel iteration on the GPU box: parity subset, bench (kernel legs only),
# rocprofv3 kernel stats and the two HBM PMC passes of the bench command.
# Usage: bash tools/perf_round.sh TAG
set -o pipefail
TAG=${1:-perf}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "engine or configs3_shard_vs_reference[0] or swdec_api or damaged_and_refpic" > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print('BENCH', d['value'], d['ms_per_step'], d['kernels']['k_wgpp']['avg_launch_us'], d['bitexact_check']['ok'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-e2e --no-rgba > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o bench -- python3 bench.py --no-cpu-baseline --no-verify --no-e2e --no-rgba > /dev/null 2> $OUT/pmc_fetch.err || { tail -20 $OUT/pmc_fetch.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o bench -- python3 bench.py --no-cpu-baseline --no-verify --no-e2e --no-rgba > /dev/null 2> $OUT/pmc_write.err || { tail -20 $OUT/pmc_write.err; exit 1; }
echo done
