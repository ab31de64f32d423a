#!/bin/bash
# Round-5 record on one GPU box: parity suite, smoke, bench (configs 3 + 2,
# 5, host-resident), kernel-trace stats (one stream), FETCH/WRITE PMC passes (configs 2, 3),
# the 8(f) rows (emit, inflate, names) with their kernel stats.  Every GPU
# step has its own limit; a failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT_DIR:-gpurun_out/r5}; mkdir -p $O; export TMPDIR=/tmp
run() {
  local name=$1; shift; local t=$1; shift
  echo "== $name (limit ${t}s)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
for s in ${STEPS:-pytest smoke bench bench5 host prof pmc issue rows}; do
  case $s in
    pytest) run pytest_gpu 1100 python -u -m pytest tests -m gpu -v -s -rf --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 600 python bench.py ;;
    bench5) run bench5 600 python bench.py --config 5 ;;
    host)   run bench_host 600 python bench.py --host-resident --no-cpu-baseline ;;
    prof)   rm -rf $O/prof3s1 $O/prof2s1
            run prof3s1 300 rocprofv3 --kernel-trace --stats -d $O/prof3s1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary --streams 1 --config 3
            run prof2s1 300 rocprofv3 --kernel-trace --stats -d $O/prof2s1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --streams 1 --config 2
            run prof5s1 300 rocprofv3 --kernel-trace --stats -d $O/prof5s1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --streams 1 --config 5 ;;
    issue)  OUT=$O/pmc_issue CFGS="3 2 5" timeout -k 10 600 bash tools/diag/pmc_dec2.sh > $O/pmc_issue.log 2>&1 || { echo "stopping: issue"; exit 1; }
            OUT=$O/pmc_issue_enc timeout -k 10 300 bash tools/diag/pmc_enc2.sh > $O/pmc_issue_enc.log 2>&1 || { echo "stopping: issue_enc"; exit 1; } ;;
    pmc)    for c in 2 3 5; do
              rm -rf $O/pmc_c$c
              run pmc_c${c}_fetch 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_c$c/p1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary --steps 5 --warmup 2 --config $c
              run pmc_c${c}_write 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_c$c/p2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary --steps 5 --warmup 2 --config $c
            done ;;
    rows)   rm -rf $O/prof_rows
            run rows 300 python tools/bench_rows.py emit emit3 inflate inflate_index names
            run prof_rows 300 rocprofv3 --kernel-trace --stats -d $O/prof_rows -o run --output-format csv -- python3 tools/bench_rows.py emit emit3 names ;;
  esac
done
echo "all steps done"
