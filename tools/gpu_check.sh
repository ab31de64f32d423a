#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel stats.
# Each GPU step has its own time limit; a fault / abort / timeout (any exit
# status other than 0 or 1) ends the script before the next GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-pytest smoke bench prof}"
run() {
  local name=$1; shift; local t=$1; shift
  echo "== $name (limit ${t}s): $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 120 --timeout-method thread ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 600 python bench.py ${BENCH_ARGS:-} ;;
    bench3) run bench3 600 python bench.py --config 3 --no-cpu-baseline ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run \
              --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} ;;
  esac
done
echo "all steps done"
