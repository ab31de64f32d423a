#!/bin/bash
# A/B library pair for ab_libs.py: lib_base.so from git revision $1 (default
# HEAD), lib_cur.so from the working tree (engine sources only).
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
REV=${1:-HEAD}
T=$(mktemp -d)
(cd $HERE/../.. && git archive $REV nghttp2_amd/csrc include | tar -x -C $T)
rm -f $HERE/lib_*.so
F="-O3 -std=c++17 -fPIC -shared -fvisibility=hidden --offload-arch=gfx950"
(cd /tmp && /opt/rocm/bin/hipcc $F -o $HERE/lib_base.so $T/nghttp2_amd/csrc/hd_huff.hip) &
(cd /tmp && /opt/rocm/bin/hipcc $F ${CUR_FLAGS:-} -o $HERE/lib_cur.so $HERE/../../nghttp2_amd/csrc/hd_huff.hip) &
wait
rm -rf $T
ls -la $HERE/lib_*.so
