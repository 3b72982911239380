#!/bin/bash
# End-to-end leg (bench.end_to_end: 8 processes, plus one process x 8 threads
# on a shared engine) under host-side settings.  GPU box: bash tools/e2e_env_sweep.sh "ENV=.. ENV2=.." ...
set -o pipefail
for v in "$@"; do
  env $v timeout -k 10 200 python -c "
import bench, sys, json
streams, caps = bench.prepare(3, [100 + i for i in range(8)], 60)
r = bench.end_to_end(streams, 60)
sh = r.get('one_process_shared_engine') or {}
print(repr(sys.argv[1]), r['value'], r.get('host_cpu_ms_per_picture'), r.get('host_cores_busy'), json.dumps(r.get('per_picture_ms')), '| shared', sh.get('value'), sh.get('pictures_per_launch'), sh.get('host_cpu_ms_per_picture'))" "$v" 2>>gpurun_out/e2e_sweep.err || { tail -5 gpurun_out/e2e_sweep.err; exit 1; }
done
