#!/bin/bash
# The inflate_alt row (tools/bench_rows.py) with tools/diag/full_base.so (a
# full library built from an earlier revision) and the in-tree library,
# alternated, the order swapped every run.
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/infab
for r in ${RUNS:-1 2 3 4 5 6}; do
  if [ $((r % 2)) = 1 ]; then ORDER="base cur"; else ORDER="cur base"; fi
  for m in $ORDER; do
    if [ $m = base ]; then export NGHTTP2_AMD_LIB=$PWD/tools/diag/full_base.so; else unset NGHTTP2_AMD_LIB; fi
    timeout -k 10 200 python3 tools/bench_rows.py inflate_alt > gpurun_out/infab/${m}_$r.json 2>/dev/null || exit 1
    python3 -c "
import json; v=json.load(open('gpurun_out/infab/${m}_$r.json'))['inflate_alt']; print('$m', $r, v['c_wire_MBps'], v['cpu_port_16t_wire_MBps'], v['ratio_front_end_over_cpu16'])"
  done
done
