set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
run() {
  timeout -k 10 300 env $1 python bench.py --no-cpu-baseline $2 > gpurun_out/pe.log 2>&1 || { tail -20 gpurun_out/pe.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/pe.log').read().strip().splitlines()[-1]);print(sys.argv[1], d['value'], d['roofline']['achieved'], d['kernels']['k_wg']['avg_launch_us'], d['bitexact_check'])" "$1 $2"
}
run "H264MI_WG_NMC=3" ""
H264MI_KERNEL=wg timeout -k 10 120 python tools/prof_rows.py > gpurun_out/prof_wg.log 2>&1
