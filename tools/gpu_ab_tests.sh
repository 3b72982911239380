set -o pipefail
mkdir -p gpurun_out/r48
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r48/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r48/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r48/pytest_gpu.log
ROUNDS=2 bash tools/ab_env.sh "prevc:" "noc:"
BENCH_ARGS="--config 1 --streams 4 --steps 20 --warmup 4" ROUNDS=1 bash tools/ab_env.sh "prevc:" "noc:"
