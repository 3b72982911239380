set -o pipefail
mkdir -p gpurun_out/r36
timeout -k 10 200 python tools/prof_chain.py > gpurun_out/r36/chain_s8.log 2>&1 || { tail -20 gpurun_out/r36/chain_s8.log; exit 1; }
H264MI_NO_TAIL_PREP=1 timeout -k 10 200 python tools/prof_chain.py > gpurun_out/r36/chain_s8_notail.log 2>&1 || { tail -20 gpurun_out/r36/chain_s8_notail.log; exit 1; }
for i in 1 2; do
  for v in 0 1; do
    H264MI_NO_TAIL_PREP=$v H264MI_LIB_DIR=abtest/cur timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-verify --no-legs --no-rgba > gpurun_out/r36/b.log 2>&1 || { tail -20 gpurun_out/r36/b.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/r36/b.log').read().strip().splitlines()[-1]);p=d.get('p_only') or {};print('notail', sys.argv[1], d['value'], d['kernels']['k_wgpp']['avg_launch_us'], p.get('value'), p.get('avg_launch_kernel_us'))" "$v"
  done
done
