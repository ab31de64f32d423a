#!/bin/bash
# The inflate row's phases (NGHTTP2_AMD_TRACE=1) with the pinned pools
# coherent (default) or not, and with copies instead of zero-copy input.
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/inpin
for v in "" "NGHTTP2_AMD_PIN_NONCOHERENT=1" "NGHTTP2_AMD_INFLATE_ZC=0" "NGHTTP2_AMD_PIN_NONCOHERENT=1 NGHTTP2_AMD_INFLATE_ZC=0"; do
  echo "== ${v:-default}"
  env $v NGHTTP2_AMD_TRACE=1 timeout -k 10 200 python3 tools/bench_rows.py inflate > gpurun_out/inpin/r.json 2> gpurun_out/inpin/trace.txt || exit 1
  grep "nghttp2_amd inflate" gpurun_out/inpin/trace.txt | tail -2
  env $v timeout -k 10 200 python3 tools/bench_rows.py inflate_alt > gpurun_out/inpin/a.json 2>/dev/null || exit 1
  python3 -c "
import json; v=json.load(open('gpurun_out/inpin/a.json'))['inflate_alt']; print(v['c_wire_MBps'], v['cpu_port_16t_wire_MBps'], v['ratio_front_end_over_cpu16'])"
done
