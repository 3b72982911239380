set -o pipefail
mkdir -p gpurun_out/e2
for S in 1 2 4 8 16; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-verify --streams $S --steps 20 > gpurun_out/e2/b$S.log 2>&1 || { tail -20 gpurun_out/e2/b$S.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/e2/b$S.log').read().strip().splitlines()[-1]);print('S=$S', d['value'], d['ms_per_step'], d['kernels']['k_wg']['avg_launch_us'])"
done
