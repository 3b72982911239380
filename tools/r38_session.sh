set -o pipefail
mkdir -p gpurun_out/r38
H264MI_LIB_DIR=abtest/dyn5 timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-legs --no-rgba > gpurun_out/r38/verify_dyn5.json 2> gpurun_out/r38/verify.err || { tail -20 gpurun_out/r38/verify.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r38/verify_dyn5.json').read().strip().splitlines()[-1]);print('verify', d['value'], d['kernels']['k_wgpp']['avg_launch_us'], d['bitexact_check']['ok'])"
PROF_ROWS=1 H264MI_LIB_DIR=abtest/dyn5 timeout -k 10 200 python tools/prof_chain.py > gpurun_out/r38/chain_rows_dyn5.log 2>&1 || { tail -20 gpurun_out/r38/chain_rows_dyn5.log; exit 1; }
ROUNDS=3 bash tools/ab.sh cur dyn5
