#!/bin/bash
# One GPU-box session: parity tests, smoke, bench (default = config 3 with
# the config-2 secondary; config 5), kernel-trace stats.  Every GPU step has
# its own time limit; a failure ends the script (no GPU step after a fault).
# Usage: STEPS="pytest smoke bench bench5 prof" OUT=gpurun_out/r2a tools/gpu_r2.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r2}
mkdir -p "$O"
run() {
  local name=$1; shift; local t=$1; shift
  echo "== $name (limit ${t}s)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 4 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
for s in ${STEPS:-pytest smoke bench bench5 prof}; do
  case $s in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 600 python bench.py ;;
    bench2) run bench2 600 python bench.py --config 2 --no-cpu-baseline ;;
    bench5) run bench5 600 python bench.py --config 5 ;;
    bench4) run bench4 900 python bench.py --config 4 --no-cpu-baseline --steps 5 --warmup 2 ;;
    host)   run bench_host 600 python bench.py --host-resident --no-cpu-baseline --no-secondary ;;
    prof)   for c in 3 2 5; do
              rm -rf $O/prof$c
              # --streams 1: launches never overlap, so the per-kernel averages
              # are the isolated durations the roofline uses
              run prof$c 300 rocprofv3 --kernel-trace --stats -d $O/prof$c -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary --streams 1 --config $c
            done ;;
    pmc)    for c in ${PMC_CFGS:-3 2 5}; do
              rm -rf $O/pmc_c$c
              run pmc_c${c}_fetch 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_c$c/p1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary --steps 5 --warmup 2 --streams 1 --config $c
              run pmc_c${c}_write 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_c$c/p2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary --steps 5 --warmup 2 --streams 1 --config $c
            done ;;
    variants) run variants 600 python tools/diag/time_variants.py ${VCFG:-3} ;;
  esac
done
echo "all steps done"
