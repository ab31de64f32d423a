#!/bin/bash
# Build ablation variants of the engine library into tools/diag/ (built in
# the container; the .so files travel to the GPU box with the snapshot).
# Usage: build_variants.sh name:"-DFLAG=1 -DX=2" ...   (name "cur" = no flags)
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
C=$HERE/../../nghttp2_amd/csrc
SRC=$C/hd_huff.hip
# FULL=1: the whole library (every source), so that bench.py can load it
if [ "${FULL:-0}" = 1 ]; then SRC="$C/hd_huff.hip $C/hd_huff_compat.hip $C/hd_names.hip $C/hd_inflate.cpp $C/hd_deflate.cpp"; fi
rm -f $HERE/lib_*.so
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}; [ "$name" = "$spec" ] && flags=""
  (cd /tmp && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -fvisibility=hidden --offload-arch=gfx950 $flags -o $HERE/lib_$name.so $SRC) &
done
wait
ls $HERE/lib_*.so
