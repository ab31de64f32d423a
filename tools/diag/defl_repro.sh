#!/bin/bash
# test_drivers_many_connections by hand: 5 connections batched vs alone,
# fused encode (default) and two-pass; prints where the outputs differ.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=${OUT:-gpurun_out/defl}; rm -rf $O; mkdir -p $O/in $O/b $O/b2
python3 - "$O" <<'PY'
import json, sys, os
O = sys.argv[1]
src = json.load(open("tests/golden/config1_cases.json"))["cases"]
for k in range(5):
    json.dump({"cases": src[k * 150:(k + 1) * 150 + 17 * k]}, open("%s/in/conn%d.json" % (O, k), "w"))
PY
B=nghttp2_amd/bin/deflatehd
timeout -k 10 60 $B -o $O/b $O/in/conn*.json || exit 1
NGHTTP2_AMD_ENCODE_TWO_PASS=1 timeout -k 10 60 $B -o $O/b2 $O/in/conn*.json || exit 1
for k in 0 1 2 3 4; do
  timeout -k 10 60 $B $O/in/conn$k.json > $O/alone$k.json || exit 1
  NGHTTP2_AMD_ENCODE_TWO_PASS=1 timeout -k 10 60 $B $O/in/conn$k.json > $O/alone2_$k.json || exit 1
  for f in $O/b/conn$k.json $O/b2/conn$k.json $O/alone2_$k.json; do cmp -s $f $O/alone$k.json || echo "conn$k: $f differs from fused alone"; done
done
echo done
