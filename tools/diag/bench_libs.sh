#!/bin/bash
# bench.py (no CPU baseline, no secondary rows) with each whole-library
# variant tools/diag/full_<name>.so, alternated ROUNDS times, order rotated.
# Usage: LIBS="cur iw13" ROUNDS=3 ARGS="--steps 100" bench_libs.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=${OUT:-gpurun_out/benchlibs}; mkdir -p $O
set -- ${LIBS:-cur}
for r in $(seq 1 ${ROUNDS:-3}); do
  for k in "$@"; do
    NGHTTP2_AMD_LIB=$PWD/tools/diag/full_$k.so timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-secondary ${ARGS:-} > $O/${k}_$r.json 2> $O/${k}_$r.err || { tail -5 $O/${k}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/${k}_$r.json').read().strip().splitlines()[-1]); f=d['roofline']
print('$k', $r, d['value'], d['ms_per_step'], f['launch_ms'], f['enc_ms'])" | tee -a $O/summary.txt
  done
  set -- "${@:2}" "$1"
done
