set -o pipefail
mkdir -p gpurun_out/r46
for i in 1 2; do
  for v in e2eold e2enew; do
    H264MI_LIB_DIR=abtest/$v timeout -k 10 300 python tools/e2e_only.py > gpurun_out/r46/e.json 2> gpurun_out/r46/e.err || { tail -20 gpurun_out/r46/e.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/r46/e.json').read().strip().splitlines()[-1]);print(sys.argv[1], d['value'], d['host_cpu_ms_per_picture'], d['per_picture_ms'])" $v
  done
done
