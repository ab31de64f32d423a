#!/bin/bash
# Build whole-library variants (every C-ABI symbol, so bench.py and the tests
# can load them through NGHTTP2_AMD_LIB) into tools/diag/full_<name>.so.
# Usage: build_full.sh name:"-DFLAG=1 ..." ...   (built from a copy of the tree)
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$HERE/../..
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}; [ "$name" = "$spec" ] && flags=""
  T=$(mktemp -d)
  mkdir -p $T/nghttp2_amd
  cp -rp $ROOT/nghttp2_amd/csrc $ROOT/nghttp2_amd/Makefile $ROOT/nghttp2_amd/drivers $ROOT/nghttp2_amd/tools $T/nghttp2_amd/
  cp -rp $ROOT/include $T/
  make -s -j8 -C $T/nghttp2_amd $T/nghttp2_amd/lib/libnghttp2_amd_hd.so \
    HIPFLAGS="-O3 -std=c++17 -fPIC -Wall -fvisibility=hidden --offload-arch=gfx950 $flags"
  cp $T/nghttp2_amd/lib/libnghttp2_amd_hd.so $HERE/full_$name.so
  rm -rf $T
  echo $HERE/full_$name.so
done
