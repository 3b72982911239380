set -o pipefail
mkdir -p gpurun_out/e3
for N in 2 3 4; do
  H264MI_WG_NMC=$N timeout -k 10 300 python bench.py --no-cpu-baseline --no-verify --steps 20 > gpurun_out/e3/b$N.log 2>&1 || { tail -20 gpurun_out/e3/b$N.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/e3/b$N.log').read().strip().splitlines()[-1]);print('NMC=$N', d['value'], d['ms_per_step'], d['kernels']['k_wg']['avg_launch_us'])"
done
H264MI_WG_NMC=4 H264MI_KERNEL=wg timeout -k 10 200 python tools/prof_rows.py > gpurun_out/e3/prof4.log 2>&1
