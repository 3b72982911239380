#!/bin/bash
# Round-2 GPU step: parity tests, then the default bench (driver contract).
# Usage (GPU box, repo root): bash tools/r2_gpu.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-r2}; K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -c 1500 $OUT/bench.json
