set -o pipefail
mkdir -p gpurun_out/r40
for i in 1 2; do
  for v in cur dyn5; do
    for m in 2 3; do
      H264MI_MC_WAVES=$m H264MI_LIB_DIR=abtest/$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-verify --no-legs --no-rgba > gpurun_out/r40/b.log 2>&1 || { tail -20 gpurun_out/r40/b.log; exit 1; }
      python3 -c "import json,sys;d=json.loads(open('gpurun_out/r40/b.log').read().strip().splitlines()[-1]);p=d.get('p_only') or {};print(sys.argv[1], 'mc', sys.argv[2], d['value'], d['kernels']['k_wgpp']['avg_launch_us'], p.get('value'), p.get('avg_launch_kernel_us'))" $v $m
    done
  done
done
