#!/bin/bash
# WRITE_SIZE per k_decode launch for the three output layouts of
# tools/diag/write_layout.py (one PMC counter group, --kernel-trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/wl; rm -rf $O; mkdir -p $O
timeout -k 10 120 python3 tools/diag/write_layout.py > $O/plain.log 2>&1 || { echo "plain run failed"; tail -5 $O/plain.log; exit 1; }
tail -1 $O/plain.log
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/p -o run --output-format csv -- python3 tools/diag/write_layout.py > $O/pmc.log 2>&1 || { echo "pmc run failed"; tail -5 $O/pmc.log; exit 1; }
python3 - <<'PY'
import csv, glob
from collections import defaultdict
per, names, order = defaultdict(float), {}, []
for f in glob.glob("gpurun_out/wl/p/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d = int(r["Dispatch_Id"])
        if r["Counter_Name"] == "WRITE_SIZE":
            per[d] += float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
auto = [per[d] for d in sorted(per) if names[d].startswith("void k_decode<true>")]
false = [per[d] for d in sorted(per) if names[d].startswith("void k_decode<false>")]
k = len(auto)
for tag, v in (("auto", auto), ("slots", false[:k]), ("tight", false[k:])):
    print("%-5s launches %d  WRITE_SIZE %.1f MB per launch" % (tag, len(v), sum(v) / max(1, len(v)) * 1024 / 1e6))
PY
