set -o pipefail
mkdir -p gpurun_out/e9
run() {
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/e9/b.log 2>&1 || { tail -20 gpurun_out/e9/b.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/e9/b.log').read().strip().splitlines()[-1]);print(sys.argv[1], d['value'], d['ms_per_step'], d['kernels']['k_wg']['avg_launch_us'], d['bitexact_check']['ok'])" "$1"
}
run base
H264MI_WG_PP=0 run single
cp broadway_amd/lib_uni/libh264mi.so broadway_amd/lib/libh264mi.so
run uniform
H264MI_WG_PP=0 run uniform-single
H264MI_KERNEL=wg timeout -k 10 200 python tools/prof_rows.py > gpurun_out/e9/prof.log 2>&1
