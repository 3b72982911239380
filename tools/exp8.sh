set -o pipefail
mkdir -p gpurun_out/e8
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e8/t.log 2>&1 || { tail -30 gpurun_out/e8/t.log; exit 1; }
tail -2 gpurun_out/e8/t.log
for cfg in "H264MI_WG_CH=1" "H264MI_WG_CH=0"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/e8/b.log 2>&1 || { tail -20 gpurun_out/e8/b.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/e8/b.log').read().strip().splitlines()[-1]);print(sys.argv[1], d['value'], d['ms_per_step'], d['kernels']['k_wg']['avg_launch_us'], d['bitexact_check']['ok'])" "$cfg"
done
H264MI_KERNEL=wg timeout -k 10 200 python tools/prof_rows.py > gpurun_out/e8/prof.log 2>&1
