#!/bin/bash
# Round-5 closing record: FETCH/WRITE PMC passes (configs 2, 3, 5) for
# profiles/traffic.json, then the driver's bench command three times, then
# config 4 at N = 1.  Every GPU step has its own limit; a failing step ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT_DIR:-gpurun_out/r5f}; mkdir -p $O; export TMPDIR=/tmp
run() {
  local name=$1; shift; local t=$1; shift
  echo "== $name (limit ${t}s)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 1 "$O/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
for c in 2 3 5; do
  rm -rf $O/pmc_c$c
  run pmc_c${c}_fetch 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_c$c/p1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary --steps 5 --warmup 2 --config $c
  run pmc_c${c}_write 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_c$c/p2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary --steps 5 --warmup 2 --config $c
done
for r in 1 2 3; do run driver_cmd_$r 300 python3 bench.py --gpus 1 --steps 20 --warmup 5; done
run config4_n1 600 python3 bench.py --config 4 --no-cpu-baseline
echo "all steps done"
