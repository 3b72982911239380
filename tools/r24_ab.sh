set -o pipefail
mkdir -p gpurun_out/r24
export TMPDIR=/tmp
ROUNDS=2 bash tools/ab_verify.sh base midpoll midpoll_nosleep > gpurun_out/r24/ab.txt 2>&1 || { cat gpurun_out/r24/ab.txt; exit 1; }
cat gpurun_out/r24/ab.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r24/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r24/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r24/pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/r24/bench.json 2> gpurun_out/r24/bench.err || { tail -20 gpurun_out/r24/bench.err; exit 1; }
tail -c 300 gpurun_out/r24/bench.json
