#!/bin/bash
# The inflate front-end: zero-copy decode against device copies, with phase
# traces, then the alternating comparison with the 16-thread CPU port.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/inflzc; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "inflate or reference or drivers" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for zc in 2 0 1 2 0 1; do
  NGHTTP2_AMD_INFLATE_ZC=$zc NGHTTP2_AMD_TRACE=1 timeout -k 10 200 python tools/bench_rows.py inflate > $O/zc$zc.json 2> $O/zc$zc.log || exit 1
  python -c "import json;d=json.load(open('$O/zc$zc.json'))['inflate'];print('zc',$zc,d['c_wire_MBps'],'cpu16',d['cpu_port_16t_wire_MBps'])"
  grep "nghttp2_amd inflate" $O/zc$zc.log | tail -2
done
timeout -k 10 300 python tools/bench_rows.py inflate_alt inflate_alt_index > $O/alt.json 2>/dev/null || exit 1
python -c "
import json
d=json.load(open('$O/alt.json'))
for k,v in d.items(): print(k, v['c_wire_MBps'], v['cpu_port_16t_wire_MBps'], v['ratio_front_end_over_cpu16'])"
