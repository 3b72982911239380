#!/bin/bash
# One GPU call: the OMX GPU tests, a verified bench of build $2, and the A/B
# of builds $1 vs $2 (tools/ab.sh).  Usage: bash tools/ab_session.sh BASE VARIANT
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_omx.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/omx.log 2>&1 || { tail -20 gpurun_out/ab/omx.log; exit 1; }
tail -1 gpurun_out/ab/omx.log
H264MI_LIB_DIR=abtest/$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-legs --no-rgba > gpurun_out/ab/verify_$2.json 2> gpurun_out/ab/verify_$2.err || { tail -20 gpurun_out/ab/verify_$2.err; exit 1; }
ROUNDS=${ROUNDS:-3} bash tools/ab.sh $1 $2
