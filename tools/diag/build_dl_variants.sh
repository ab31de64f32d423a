#!/bin/bash
# Builds lane-decoder variants of the library into tools/diag/lib_<name>.so:
#   build_dl_variants.sh name1 "-DFLAG=.." name2 "-DFLAG=.." ...
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
C=$R/nghttp2_amd/csrc
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  (cd /tmp && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -fvisibility=hidden --offload-arch=gfx950 $flags \
     -o $R/tools/diag/lib_$name.so $C/hd_huff.hip $C/hd_huff_compat.hip $C/hd_names.hip $C/hd_inflate.cpp $C/hd_deflate.cpp 2>&1 | grep -v warning || true) &
done
wait
ls -la $R/tools/diag/lib_*.so
