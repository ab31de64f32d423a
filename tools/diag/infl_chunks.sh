#!/bin/bash
# The inflate front-end's C call at 1, 2 and 4 literal chunks (phase traces).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/inflc; mkdir -p $O
for k in 1 2 4 1 2 4; do
  NGHTTP2_AMD_INFLATE_CHUNKS=$k NGHTTP2_AMD_TRACE=1 timeout -k 10 200 python tools/bench_rows.py inflate > $O/k$k.json 2> $O/k$k.log || exit 1
  python -c "import json;d=json.load(open('$O/k$k.json'))['inflate'];print('chunks',$k,d['c_wire_MBps'],'cpu16',d['cpu_port_16t_wire_MBps'])"
  grep "nghttp2_amd inflate" $O/k$k.log | tail -2
done
