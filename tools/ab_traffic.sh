#!/bin/bash
# Speed and memory-side traffic of environment variants in one GPU call:
#   ROUNDS=2 bash tools/ab_traffic.sh "base:" "lead16:H264MI_MC_LEAD0=16" ...
# per variant and round: GOP-mix frames/s and k_wgpp us (bench, no verify);
# then one FETCH_SIZE and one WRITE_SIZE pass (k_wgpp average per launch, KiB:
# read = 2 x FETCH_SIZE on gfx950, profiles/r54_bytes.json); VERIFY=1 adds a
# verified bench run per variant (480 frames vs the reference MD5s); NO_PMC=1
# skips the counter passes.
set -o pipefail
mkdir -p gpurun_out/abt
export TMPDIR=/tmp
for i in $(seq 1 ${ROUNDS:-2}); do
  for spec in "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    ( [ -n "$envs" ] && export $envs; timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-verify --no-legs --no-rgba > gpurun_out/abt/b.log 2>&1 ) || { tail -20 gpurun_out/abt/b.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/abt/b.log').read().strip().splitlines()[-1]);print(sys.argv[1], d['value'], d['kernels']['k_wgpp']['avg_launch_us'], flush=True)" "$spec"
  done
done
for spec in "$@"; do
  [ -n "$NO_PMC" ] && break
  name=${spec%%:*}; envs=${spec#*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    ( [ -n "$envs" ] && export $envs; timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/abt/${name}_$c -o bench -- python3 bench.py --no-cpu-baseline --no-verify --no-e2e --no-legs --no-rgba > /dev/null 2> gpurun_out/abt/pmc.err ) || { tail -20 gpurun_out/abt/pmc.err; exit 1; }
  done
  python3 - "$name" <<'EOF'
import csv, sys
name = sys.argv[1]
v = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    xs = [float(r["Counter_Value"]) for r in csv.DictReader(open(f"gpurun_out/abt/{name}_{c}/bench_counter_collection.csv"))
          if r["Counter_Name"] == c and "k_wgpp" in r["Kernel_Name"]]
    v[c] = sum(xs) / len(xs)
print(name, "k_wgpp MB/launch: read", round(2 * v["FETCH_SIZE"] * 1024 / 1e6, 1), "write", round(v["WRITE_SIZE"] * 1024 / 1e6, 1),
      "total", round((2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024 / 1e6, 1), flush=True)
EOF
done
if [ -n "$VERIFY" ]; then
  for spec in "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    ( [ -n "$envs" ] && export $envs; timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-legs --no-rgba > gpurun_out/abt/v.log 2>&1 ) || { tail -20 gpurun_out/abt/v.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/abt/v.log').read().strip().splitlines()[-1]);b=d['bitexact_check'];print(sys.argv[1], 'verified', d['value'], b['ok'], b['frames_checked'], b['frames_expected'], flush=True)" "$spec"
  done
fi
