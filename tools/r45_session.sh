set -o pipefail
mkdir -p gpurun_out/r45
export TMPDIR=/tmp
H264MI_LIB_DIR=abtest/nt timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-legs --no-rgba > gpurun_out/r45/verify_nt.json 2> gpurun_out/r45/v.err || { tail -20 gpurun_out/r45/v.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r45/verify_nt.json').read().strip().splitlines()[-1]);print('verify nt', d['value'], d['kernels']['k_wgpp']['avg_launch_us'], d['bitexact_check']['ok'])"
ROUNDS=2 bash tools/ab_env.sh "base:" "nt:"
for v in base nt; do
  for c in FETCH_SIZE WRITE_SIZE; do
    H264MI_LIB_DIR=abtest/$v timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/r45/${v}_${c} -o p -- python3 bench.py --no-cpu-baseline --no-verify --no-e2e --no-legs --no-rgba > /dev/null 2> gpurun_out/r45/pmc.err || { tail -20 gpurun_out/r45/pmc.err; exit 1; }
    python3 - $v $c gpurun_out/r45/${v}_${c}/p_counter_collection.csv <<'PY'
import csv, sys
v, c, f = sys.argv[1:4]
vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "k_wgpp" in r["Kernel_Name"] and r["Counter_Name"] == c]
print(v, c, "KiB per k_wgpp launch", round(sum(vals) / len(vals), 1), "launches", len(vals))
PY
  done
done
