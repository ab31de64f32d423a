#!/bin/bash
# One GPU-box session for the round's record: parity tests, smoke, bench
# (configs 2, 3 and host-resident), kernel-trace stats, FETCH/WRITE PMC
# passes (configs 2, 3).  Every GPU step has its own time limit; a fault /
# abort / timeout (exit status other than 0 or 1) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/round
export TMPDIR=/tmp
O=gpurun_out/round
run() {
  local name=$1; shift; local t=$1; shift
  echo "== $name (limit ${t}s)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
for s in ${STEPS:-pytest smoke bench bench3 host prof pmc names}; do
  case $s in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 600 python bench.py ;;
    bench3) run bench3 600 python bench.py --config 3 --no-cpu-baseline ;;
    host)   run bench_host 600 python bench.py --host-resident --no-cpu-baseline ;;
    prof)   rm -rf $O/prof2 $O/prof3 $O/prof2s1 $O/prof3s1
            # --streams 1: launches never overlap, so the per-kernel averages
            # are the isolated durations the roofline uses
            run prof2s1 300 rocprofv3 --kernel-trace --stats -d $O/prof2s1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --streams 1
            run prof3s1 300 rocprofv3 --kernel-trace --stats -d $O/prof3s1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --streams 1 --config 3
            run prof2 300 rocprofv3 --kernel-trace --stats -d $O/prof2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline
            run prof3 300 rocprofv3 --kernel-trace --stats -d $O/prof3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --config 3 ;;
    pmc)    for c in 2 3; do
              rm -rf gpurun_out/pmc_c$c
              run pmc_c${c}_fetch 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_c$c/p1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --config $c
              run pmc_c${c}_write 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_c$c/p2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --config $c
            done ;;
    names)  rm -rf $O/prof_names
            run rows_names 300 python tools/bench_rows.py names_short names
            run prof_names 300 rocprofv3 --kernel-trace --stats -d $O/prof_names -o run --output-format csv -- python3 tools/bench_rows.py names ;;
  esac
done
echo "all steps done"
