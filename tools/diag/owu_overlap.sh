#!/bin/bash
# Round 6: the one-wave pack units
# (patches/r5_encode_one_wave_units.patch, EC_WGW=1, full_owu.so) against the
# tree (full_cur.so) in the pipelined two-stream bench itself: bench_libs
# alternations, then a two-stream kernel trace of each (trace_overlap.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/owu}; mkdir -p $O
LIBS="cur owu" ROUNDS=${ROUNDS:-3} ARGS="--steps 100" OUT=$O/bench bash tools/diag/bench_libs.sh || exit 1
for k in cur owu; do
  rm -rf $O/tr_$k
  NGHTTP2_AMD_LIB=$PWD/tools/diag/full_$k.so timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_$k -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary --steps 30 --warmup 5 > $O/tr_$k.log 2>&1 || { tail -5 $O/tr_$k.log; exit 1; }
  echo "== $k" >> $O/overlap.txt
  python3 tools/trace_overlap.py $O/tr_$k >> $O/overlap.txt
done
cat $O/overlap.txt
