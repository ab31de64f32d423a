#!/bin/bash
# bench.py (config 3, 2 streams, no CPU baseline) with the product library
# and with each tools/diag/lib_*.so (NGHTTP2_AMD_LIB), interleaved, twice.
# Usage: OUT=gpurun_out/abb tools/diag/ab_bench_libs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=${OUT:-gpurun_out/abb}; mkdir -p $O
for rep in 1 2; do
  for v in cur $(cd tools/diag && ls lib_*.so 2>/dev/null | sed 's/^lib_//; s/\.so$//'); do
    if [ $v = cur ]; then L=""; else L=$PWD/tools/diag/lib_$v.so; fi
    NGHTTP2_AMD_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/b_${v}_$rep.json 2>$O/b_${v}_$rep.err || exit $?
    echo "$rep $v $(python -c "import json; d=json.loads(open('$O/b_${v}_$rep.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['enc_ms'])")"
  done
done
