#!/bin/bash
# Decoder scheduler variants of the working tree: lib_<name>.so with the
# decode translation unit built under each flag set (name:"flags" ...).
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
SRC=$HERE/../../nghttp2_amd/csrc/hd_huff.hip
F="-O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950"
rm -f $HERE/lib_*.so
O=$(mktemp -d)
(cd /tmp && /opt/rocm/bin/hipcc $F -DHD_PART_ENC -c -o $O/e.o $SRC)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}; [ "$name" = "$spec" ] && flags=""
  ( (cd /tmp && /opt/rocm/bin/hipcc $F $flags -DHD_PART_DEC -c -o $O/d_$name.o $SRC) &&
    (cd /tmp && /opt/rocm/bin/hipcc $F -shared -o $HERE/lib_$name.so $O/e.o $O/d_$name.o) ) &
done
wait
rm -rf $O
ls $HERE/lib_*.so
