#!/bin/bash
# Round-5 check after the decoder map change and the pipelined inflate:
# GPU tests, smoke, decode A/B (HEAD vs tree), inflate vs CPU port, bench,
# overlap trace.  Every GPU step has its own limit; a failing step ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT_DIR:-gpurun_out/r5b}; mkdir -p $O; export TMPDIR=/tmp
run() {
  local name=$1; shift; local t=$1; shift
  echo "== $name (limit ${t}s)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
for s in ${STEPS:-pytest smoke ab infl bench ovl}; do
  case $s in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -v -s -rf --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    ab)     run ab 400 env ROUNDS=12 python -u tools/diag/ab_libs.py 3 2 5 ;;
    infl)   run infl 300 python tools/bench_rows.py inflate_alt inflate_alt_index ;;
    bench)  run bench 600 python bench.py ;;
    ovl)    run ovl 600 env OUT=$O/ovl bash tools/prof_overlap.sh ;;
  esac
done
echo "all steps done"
