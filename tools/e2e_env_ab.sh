#!/bin/bash
# A/B of the end-to-end leg (bench.end_to_end: one h264mi_dec process per
# stream through the H264SwDec C-ABI), interleaved.  A variant is a list of
# environment settings; LIB=<name> in it swaps in abtest/<name>/libh264mi.so
# (h264mi_dec loads broadway_amd/lib/libh264mi.so through its rpath).
# Usage (GPU box): ROUNDS=2 bash tools/e2e_env_ab.sh "LIB=a H264MI_PARSE_THREADS=3" "LIB=b"
set -o pipefail
cp broadway_amd/lib/libh264mi.so /tmp/libh264mi.so.orig
restore() { cp /tmp/libh264mi.so.orig broadway_amd/lib/libh264mi.so; }
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    envs=""
    restore
    for t in $v; do
      case $t in
        LIB=*) cp abtest/${t#LIB=}/libh264mi.so broadway_amd/lib/libh264mi.so ;;
        *) envs="$envs $t" ;;
      esac
    done
    env $envs timeout -k 10 200 python -c "
import bench, sys, json
streams, caps = bench.prepare(3, [100 + i for i in range(8)], 60)
r = bench.end_to_end(streams, 60)
print(sys.argv[1], r['value'], json.dumps(r.get('per_picture_ms')), r.get('host_cpu_ms_per_picture'), r.get('host_cores_busy'))" "$v" 2>gpurun_out/e2e_env.err || { tail -5 gpurun_out/e2e_env.err; restore; exit 1; }
  done
done
restore
