#!/bin/bash
# Round-6 closing record: FETCH/WRITE PMC passes (configs 2, 3, 5) for
# profiles/traffic.json, SQ issue/wait counters of the config-3 decode,
# rocprof kernel stats of configs 3 / 2 / 5 on one stream, then the driver's
# bench command three times, config 5, and config 4 at N = 1.  Every GPU step
# has its own limit; a failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT_DIR:-gpurun_out/r6f}; mkdir -p $O; export TMPDIR=/tmp
run() {
  local name=$1; shift; local t=$1; shift
  echo "== $name (limit ${t}s)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 1 "$O/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
B="python3 bench.py --no-cpu-baseline --no-secondary"
for c in 2 3 5; do
  rm -rf $O/pmc_c$c
  run pmc_c${c}_fetch 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_c$c/p1 -o run --output-format csv -- $B --steps 5 --warmup 2 --config $c
  run pmc_c${c}_write 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_c$c/p2 -o run --output-format csv -- $B --steps 5 --warmup 2 --config $c
done
rm -rf $O/pmc_issue
run pmc_issue_a 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/pmc_issue/a -o run --output-format csv -- $B --steps 5 --warmup 2 --config 3
run pmc_issue_b 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT -d $O/pmc_issue/b -o run --output-format csv -- $B --steps 5 --warmup 2 --config 3
for c in 3 2 5; do
  rm -rf $O/ks_c$c
  run kstats_c$c 300 rocprofv3 --kernel-trace --stats -d $O/ks_c$c -o run --output-format csv -- $B --streams 1 --steps 100 --warmup 20 --config $c
done
for r in 1 2 3; do run driver_cmd_$r 300 python3 bench.py --gpus 1 --steps 20 --warmup 5; done
run bench100 300 python3 bench.py --steps 100 --no-cpu-baseline
run config5 300 python3 bench.py --config 5
run config4_n1 600 python3 bench.py --config 4 --no-cpu-baseline
echo "all steps done"
