#!/bin/bash
# A/B of the end-to-end leg (host parse + H2D + kernels + D2H through the
# H264SwDec C-ABI, bench.end_to_end) for library builds in abtest/<name>/:
# h264mi_dec loads broadway_amd/lib/libh264mi.so (rpath), so each build is
# copied there in turn.  Usage (GPU box): ROUNDS=3 bash tools/e2e_ab.sh A B
set -o pipefail
cp broadway_amd/lib/libh264mi.so /tmp/libh264mi.so.orig
for i in $(seq 1 ${ROUNDS:-3}); do
  for v in "$@"; do
    cp abtest/$v/libh264mi.so broadway_amd/lib/libh264mi.so
    timeout -k 10 200 python -c "
import bench, sys
streams, caps = bench.prepare(3, [100 + i for i in range(8)], 60)
r = bench.end_to_end(streams, 60)
print(sys.argv[1], r['value'])" "$v" 2>/dev/null || { cp /tmp/libh264mi.so.orig broadway_amd/lib/libh264mi.so; exit 1; }
  done
done
cp /tmp/libh264mi.so.orig broadway_amd/lib/libh264mi.so
