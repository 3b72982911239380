set -o pipefail
mkdir -p gpurun_out/r44
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r44/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r44/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r44/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-legs --no-rgba > gpurun_out/r44/verify.json 2> gpurun_out/r44/verify.err || { tail -20 gpurun_out/r44/verify.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r44/verify.json').read().strip().splitlines()[-1]);print('verify', d['value'], d['kernels']['k_wgpp']['avg_launch_us'], d['p_only']['avg_launch_kernel_us'], d['bitexact_check']['ok'])"
ROUNDS=2 bash tools/ab_env.sh "dyn4:" "auto:"
