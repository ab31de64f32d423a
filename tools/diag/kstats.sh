#!/bin/bash
# Kernel-trace stats of a driver script (per-kernel average duration).
# Usage: kstats.sh OUTDIR driver.py args...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=$1; shift
rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 "$@" > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("%-60s %6s %12.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1000))
PY
