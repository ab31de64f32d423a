#!/bin/bash
# Phase times of the batched front-ends under the drivers: 64 connections of
# the config-1 set, host threads 1 and default (NGHTTP2_AMD_TRACE=1).
set -e
cd "$(dirname "$0")/../.."
T=$(mktemp -d)
for k in $(seq -w 0 63); do cp tests/golden/config1_cases.json $T/c$k.json; done
mkdir -p $T/w $T/h
for th in 1 16; do
  echo "== threads $th"
  NGHTTP2_AMD_HOST_THREADS=$th NGHTTP2_AMD_TRACE=1 timeout -k 5 60 nghttp2_amd/bin/deflatehd --timing --repeat 3 -o $T/w $T/c*.json 2>&1 | grep -v Overall | tail -3
  NGHTTP2_AMD_HOST_THREADS=$th NGHTTP2_AMD_TRACE=1 timeout -k 5 60 nghttp2_amd/bin/inflatehd --timing --repeat 3 -o $T/h $T/w/c*.json 2>&1 | tail -3
  NGHTTP2_AMD_HOST_THREADS=$th NGHTTP2_AMD_TRACE=1 timeout -k 5 60 nghttp2_amd/bin/deflatehd --timing --repeat 3 tests/golden/config1_cases.json 2>&1 >/dev/null | grep -v Overall | tail -2
  NGHTTP2_AMD_HOST_THREADS=$th NGHTTP2_AMD_TRACE=1 timeout -k 5 60 nghttp2_amd/bin/inflatehd --timing --repeat 3 $T/w/c00.json 2>&1 >/dev/null | tail -2
done
rm -rf $T
