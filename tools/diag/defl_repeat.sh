#!/bin/bash
# deflatehd on one connection file several times, fused encode and two-pass:
# are the outputs stable?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=${OUT:-gpurun_out/defl2}; rm -rf $O; mkdir -p $O
python3 -c "
import json
src = json.load(open('tests/golden/config1_cases.json'))['cases']
json.dump({'cases': src[450:600 + 51]}, open('$O/conn3.json', 'w'))"
B=nghttp2_amd/bin/deflatehd
for i in ${RUNS:-1 2 3 4}; do
  timeout -k 10 60 $B $O/conn3.json > $O/f$i.json 2>/dev/null || exit 1
  NGHTTP2_AMD_ENCODE_TWO_PASS=1 timeout -k 10 60 $B $O/conn3.json > $O/t$i.json 2>/dev/null || exit 1
done
md5sum $O/*.json
