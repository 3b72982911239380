"""Summarise tools/pmc_sq.sh counter CSVs: per kernel, counters per dispatch and per wave."""
import csv, glob, sys, collections

out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(f"{out}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0]
        acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[(k, row["Counter_Name"])].add(row["Dispatch_Id"])
for k, cs in acc.items():
    waves = cs.get("SQ_WAVES", 0)
    print(k)
    for c, v in sorted(cs.items()):
        n = len(disp[(k, c)])
        print(f"   {c:22s} per-dispatch {v / n:14.1f}   per-wave {v / max(waves / max(len(disp[(k, 'SQ_WAVES')]), 1) * n, 1):10.1f}")
