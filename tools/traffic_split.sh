#!/bin/bash
# Memory-side traffic of k_wgpp split by source, on tools/sq_roles.py's
# workload (8 x 1080p, 12 pictures, profiling k_wgpp): FETCH_SIZE (x2, gfx950)
# and WRITE_SIZE per launch in four runs --
#   full      normal launches
#   drain     row waves only drain the MC ring (H264MI_PROF_MODE=1): no
#             deblocking, mailboxes, frame stores
#   notail    every batch's k_prep as its own launch (H264MI_NO_TAIL_PREP=1)
#   drain_nt  both
# full - drain = the row waves' bytes; full - notail = the tail k_prep's;
# drain_nt = MC waves alone (records, k_prep outputs, reference windows,
# intra mailbox reads).  Usage (GPU box): bash tools/traffic_split.sh TAG
set -o pipefail
TAG=${1:-split}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for spec in "full:" "drain:H264MI_PROF_MODE=1" "notail:H264MI_NO_TAIL_PREP=1" "drain_nt:H264MI_PROF_MODE=1 H264MI_NO_TAIL_PREP=1"; do
  name=${spec%%:*}; envs=${spec#*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    ( [ -n "$envs" ] && export $envs; timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/${name}_$c -o p -- python3 tools/sq_roles.py > $OUT/${name}_$c.log 2>&1 ) || { tail -20 $OUT/${name}_$c.log; exit 1; }
  done
  echo "$name done"
done
python3 - $OUT <<'EOF'
import csv, json, sys
out = sys.argv[1]
rep = {}
for name in ("full", "drain", "notail", "drain_nt"):
    r = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        per = {}
        for row in csv.DictReader(open(f"{out}/{name}_{c}/p_counter_collection.csv")):
            if row["Counter_Name"] != c:
                continue
            k = row["Kernel_Name"].split("(")[0].split("<")[0].split()[-1]
            per.setdefault(k, []).append(float(row["Counter_Value"]) * 1024 * (2 if c == "FETCH_SIZE" else 1))
        r[c] = {k: (round(sum(v) / len(v) / 1e6, 2), len(v)) for k, v in per.items()}
    rep[name] = {"k_wgpp_read_MB": r["FETCH_SIZE"]["k_wgpp"][0], "k_wgpp_write_MB": r["WRITE_SIZE"]["k_wgpp"][0],
                 "k_wgpp_launches": r["FETCH_SIZE"]["k_wgpp"][1],
                 "k_prep": {"read_MB": r["FETCH_SIZE"].get("k_prep", (0, 0)), "write_MB": r["WRITE_SIZE"].get("k_prep", (0, 0))}}
json.dump(rep, open(f"{out}/traffic_split.json", "w"), indent=1)
print(json.dumps(rep, indent=1))
EOF
