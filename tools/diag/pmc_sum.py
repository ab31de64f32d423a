#!/usr/bin/env python3
"""Per-launch averages of PMC counters for one kernel from pmc_dec.sh output."""
import csv, glob, sys, collections
d = sys.argv[1]; pat = sys.argv[2] if len(sys.argv) > 2 else "k_decode"
acc = collections.defaultdict(list)
for f in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        if pat not in r.get("Kernel_Name", ""): continue
        per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, v in per.items():
        acc[c].append(sum(v.values()) / len(v))
for c in sorted(acc):
    print("%-28s %16.4g" % (c, sum(acc[c]) / len(acc[c])))
