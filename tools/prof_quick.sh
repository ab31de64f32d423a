#!/bin/bash
# Kernel-trace stats of a short bench run per config (no counters).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for c in ${CFGS:-2 3}; do
  rm -rf gpurun_out/pq$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pq$c -o run --output-format csv \
     -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 --config $c > gpurun_out/pq$c.log 2>&1 || { tail -5 gpurun_out/pq$c.log; exit 1; }
  echo "== config $c"; tail -1 gpurun_out/pq$c.log | cut -c1-200
  python3 -c "
import csv,sys
for r in csv.DictReader(open('gpurun_out/pq$c/run_kernel_stats.csv')):
    print('%-60s %6s %10.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1000))
"
done
