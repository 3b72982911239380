#!/bin/bash
# A/B of (library build, environment) pairs in one GPU call, interleaved:
#   ROUNDS=2 bash tools/ab_env.sh "cur:" "dyn4p:H264MI_MC_WAVES=2" ...
# prints per run: label, GOP-mix frames/s, k_wgpp us, P-only frames/s, us
set -o pipefail
mkdir -p gpurun_out/ab
for i in $(seq 1 ${ROUNDS:-2}); do
  for spec in "$@"; do
    lib=${spec%%:*}; envs=${spec#*:}
    env $envs H264MI_LIB_DIR=abtest/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-verify --no-legs --no-rgba $BENCH_ARGS > gpurun_out/ab/b.log 2>&1 || { tail -20 gpurun_out/ab/b.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab/b.log').read().strip().splitlines()[-1]);p=d.get('p_only') or {};r=d['roofline'];print(sys.argv[1], d['value'], d['kernels']['k_wgpp']['avg_launch_us'], p.get('value'), p.get('avg_launch_kernel_us'), 'idr', (r.get('launches_with_idr') or {}).get('avg_launch_kernel_us'), 'p', (r.get('launches_p_only') or {}).get('avg_launch_kernel_us'), 'per-step', r.get('avg_kernel_us_per_step'))" "$spec"
  done
done
