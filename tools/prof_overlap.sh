#!/bin/bash
# Kernel trace of the bench's two-stream pipeline (config 3) and of the one-
# stream run: per-kernel stats, and from the two-stream trace how the steps'
# kernels overlap (tools/trace_overlap.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/ovl}; mkdir -p $O
rm -rf $O/s2 $O/s1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary --steps 30 --warmup 5 --config 3 > $O/s2.log 2>&1 || { tail -5 $O/s2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary --streams 1 --steps 30 --warmup 5 --config 3 > $O/s1.log 2>&1 || { tail -5 $O/s1.log; exit 1; }
python3 tools/trace_overlap.py $O/s2 | tee $O/overlap.txt
for d in s1 s2; do echo "== $d"; python3 -c "
import csv
for r in csv.DictReader(open('$O/$d/run_kernel_stats.csv')):
    print('%-70s %6s %10.1f us' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1000))
"; done
