#!/bin/bash
# One GPU call: the GPU test suite on the working tree's build, then an A/B of
# abtest builds/envs over the bench configs (tools/gpu_ab_cfgs.sh).
#   bash tools/gpu_ab_tests.sh "prev:" "new:"
set -o pipefail
mkdir -p gpurun_out/abt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abt/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/abt/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/abt/pytest_gpu.log
ROUNDS=${ROUNDS:-2} bash tools/gpu_ab_cfgs.sh "$@"
