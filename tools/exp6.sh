set -o pipefail
mkdir -p gpurun_out/e6
for cfg in "H264MI_WG_NMC=2" "H264MI_WG_NMC=3"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/e6/b.log 2>&1 || { tail -20 gpurun_out/e6/b.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/e6/b.log').read().strip().splitlines()[-1]);print(sys.argv[1], d['value'], d['ms_per_step'], d['kernels']['k_wg']['avg_launch_us'], d['bitexact_check']['ok'])" "$cfg"
done
H264MI_WG_NMC=3 H264MI_KERNEL=wg timeout -k 10 200 python tools/prof_rows.py > gpurun_out/e6/prof.log 2>&1
